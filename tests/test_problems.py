"""CPU checks of the problem generators' numpy side (hgmres/problems.py), no GPU.

* The parallel-beam Siddon projector after the round-5 refactor (_siddon_chunk -> the generic
  _siddon_rays) reproduces the committed fixtures' raw operators bit for bit.
* The fan-beam (curved detector) projector, the 'fancurved' geometry of run_2D_phantom.m:12-13
  (parity unpinned against PRtomo_mismatched, which the reference does not vendor; checked
  against its own definition): every row sums to the chord of its ray through the N x N square
  (the intersection lengths partition the chord), entries are positive and at most sqrt(2), the
  fan covers every pixel from every source position, and a quarter turn of the sources is a
  quarter turn of the image.
"""
import math

import numpy as np
import pytest

from conftest import golden_problem
from hgmres.problems import fan_geometry, fanbeam_projector, siddon_projector, tomo_problem


def test_parallel_refactor_keeps_fixture_bits():
    A, _, _, _, g = golden_problem("tomo24_matched.npz")
    S = siddon_projector(24, 12)
    assert np.array_equal(S.indptr, A.indptr)
    assert np.array_equal(S.indices, A.indices)
    assert np.array_equal(S.data, A.data)


def _chords(N, x0, y0, ux, uy):
    """Length of each ray's intersection with the square [-N/2, N/2]^2 (slab method)."""
    h = N / 2.0
    with np.errstate(divide="ignore", invalid="ignore"):
        tx = np.sort(np.stack([(-h - x0) / ux, (h - x0) / ux]), axis=0)
        ty = np.sort(np.stack([(-h - y0) / uy, (h - y0) / uy]), axis=0)
    lo = np.maximum(tx[0], ty[0])
    hi = np.minimum(tx[1], ty[1])
    return np.maximum(hi - lo, 0.0)


@pytest.mark.parametrize("N,na", [(32, 90), (48, 37), (64, 16)])
def test_fanbeam_rows_partition_their_chords(N, na):
    A = fanbeam_projector(N, na)
    p, x0, y0, ux, uy = fan_geometry(N, na)
    assert A.shape == (p * na, N * N)
    assert np.all(A.data > 0) and np.all(A.data <= math.sqrt(2.0) + 1e-12)
    rs = np.asarray(A.sum(axis=1)).ravel()
    ch = _chords(N, x0, y0, ux, uy)
    assert np.max(np.abs(rs - ch)) < 1e-9 * N
    # the fan spans the circumscribed circle: every source position's fan meets pixels in every
    # quadrant, and over the turn every pixel is crossed (no empty column)
    Ac = A.tocoo()
    q = (Ac.col // N >= N // 2) * 2 + (Ac.col % N >= N // 2)
    seen = np.zeros((na, 4), dtype=bool)
    seen[Ac.row // p, q] = True
    assert seen.all()
    assert np.all(np.diff(A.tocsc().indptr) > 0)
    # entries of a row are along the ray, so each row's pixels are distinct
    for r in range(0, A.shape[0], 97):
        cols = A.indices[A.indptr[r]:A.indptr[r + 1]]
        assert cols.size == np.unique(cols).size


def test_fanbeam_quarter_turn_symmetry():
    """Sources a and a + na/4 see the image rotated by 90 degrees: A rows of the shifted source
    equal A rows of the rotated image (up to the rounding of the libm angles)."""
    N, na = 32, 16
    A = fanbeam_projector(N, na).toarray()
    p = A.shape[0] // na
    img = np.arange(N * N, dtype=np.float64).reshape(N, N, order="F")   # x(:) column-major, row 0 = top
    # a source a quarter turn on sees the image turned a quarter back: the columns of its rows
    # are those of source a under the image rotation np.rot90 (counter-clockwise)
    rot = np.rot90(img, k=1)
    perm = rot.ravel(order="F").astype(np.int64)
    for a in range(na - na // 4):
        R0 = A[a * p:(a + 1) * p]
        R1 = A[(a + na // 4) * p:(a + na // 4 + 1) * p]
        assert np.max(np.abs(R1 - R0[:, perm])) < 1e-9


def test_fan_problem_and_refusals():
    P = tomo_problem(32, 16, geometry_kind="fan")
    assert P.A.shape == (fan_geometry(32, 16)[0] * 16, 32 * 32)
    assert np.allclose(P.B.toarray(), P.A.toarray().T)
    with pytest.raises(ValueError):
        tomo_problem(32, 16, backprojector="pixel", geometry_kind="fan")
    with pytest.raises(ValueError):
        tomo_problem(32, 16, geometry_kind="cone")
