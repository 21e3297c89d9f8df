"""Synthetic 2-D parallel-beam tomography problems (the input side of the hot path).

The reference's only 2-D case comes from the un-vendored ``PRtomo_mismatched``
(``run_2D_phantom.m:12-15``) and its ``generate_test_problem.m:1-11`` only
dispatches to 1-D Regularization-Tools problems, so the operators for the
BASELINE configs are built here:

* ``A``  – ray-driven Siddon line-integral projector, CSR, one row per ray
  (ray-major), ``m = p * n_angles`` rows with ``p = ceil(sqrt(2) N)``
  detectors of unit spacing; ``n = N*N`` pixels of unit size, pixel index in
  MATLAB column-major order ``col*N + row``.
* ``B``  – the back-projector: ``A^T`` (matched, pixel-major CSR) or an
  unmatched pixel-driven linear-interpolation back-projector (the classic
  ray-driven/pixel-driven mismatched pair the reference studies).
* ``x_true`` – modified Shepp–Logan phantom, ``b = A x_true + e`` with
  ``||e|| = eta ||A x_true||`` (as ``run_2D_phantom.m:18-20``).

Detector positions are offset by a quarter spacing so no ray runs exactly
along a pixel boundary (keeps pixel assignment well defined for every
implementation of the generator).

This module is host (numpy) code: it produces the operands that the C-ABI
library uploads; it is not part of the timed path.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

DETECTOR_OFFSET = 0.25

# BASELINE.json configs -> (N, n_angles)   (SURVEY.md §8(d) "Synthetic inputs")
CONFIGS = {
    "c1": (64, 90),      # 64^2, m=8,190,  nnz~4.7e5 (CPU plumbing case)
    "c2": (512, 30),     # 512^2, m=21,750, nnz~1.0e7 (hybrid_ab_gmres_rtp, 1 GPU)
    "c3": (2048, 19),    # 2048^2, m=55,043, nnz~1.0e8 (BA-GMRES + GCV, MGS vs CGS2)
    "c4": (4096, 47),    # 4096^2, m=272,271, nnz~1.0e9 (AB-GMRES, 8 GPUs)
}


def geometry(N: int, n_angles: int):
    """Parallel-beam geometry: detector count, angles, detector offsets."""
    p = int(math.ceil(math.sqrt(2.0) * N))
    theta = np.arange(n_angles, dtype=np.float64) * (np.pi / n_angles)
    s = np.arange(p, dtype=np.float64) - (p - 1) / 2.0 + DETECTOR_OFFSET
    return p, theta, s


def _siddon_chunk(N, cos_t, sin_t, s):
    """Siddon ray tracing for a chunk of parallel rays (direction (cos_t, sin_t), signed
    detector offset s from the centre).  Returns (counts, cols, vals) with the entries of each
    ray ordered along the ray (increasing t)."""
    return _siddon_rays(N, -s * sin_t, s * cos_t, cos_t, sin_t)


def _siddon_rays(N, x0, y0, cos_t, sin_t):
    """Siddon ray tracing for a chunk of rays x(t) = (x0, y0) + t (cos_t, sin_t) (unit direction)
    over the N x N grid of unit pixels centred on the origin.  Returns (counts, cols, vals)
    with the entries of each ray ordered along the ray (increasing t).  Mirrored by the device
    generators' ray_geom / siddon_walk (csrc/ops.hip)."""
    half = N / 2.0
    grid = np.arange(N + 1, dtype=np.float64) - half
    eps = 1e-12
    cx = np.abs(cos_t) > eps
    cy = np.abs(sin_t) > eps
    with np.errstate(divide="ignore", invalid="ignore"):
        tx = (grid[None, :] - x0[:, None]) / np.where(cx, cos_t, 1.0)[:, None]
        ty = (grid[None, :] - y0[:, None]) / np.where(cy, sin_t, 1.0)[:, None]
    inf = np.inf
    txmin = np.where(cx, np.minimum(tx[:, 0], tx[:, N]), np.where(np.abs(x0) < half, -inf, inf))
    txmax = np.where(cx, np.maximum(tx[:, 0], tx[:, N]), np.where(np.abs(x0) < half, inf, -inf))
    tymin = np.where(cy, np.minimum(ty[:, 0], ty[:, N]), np.where(np.abs(y0) < half, -inf, inf))
    tymax = np.where(cy, np.maximum(ty[:, 0], ty[:, N]), np.where(np.abs(y0) < half, inf, -inf))
    tmin = np.maximum(txmin, tymin)
    tmax = np.minimum(txmax, tymax)
    hit = tmin < tmax
    tx = np.where(cx[:, None], tx, inf)
    ty = np.where(cy[:, None], ty, inf)
    T = np.concatenate([tx, ty, tmin[:, None], tmax[:, None]], axis=1)
    lo = tmin[:, None]
    hi = tmax[:, None]
    T = np.where((T >= lo) & (T <= hi) & hit[:, None], T, inf)
    T.sort(axis=1)
    t0 = T[:, :-1]
    t1 = T[:, 1:]
    with np.errstate(invalid="ignore"):
        L = t1 - t0
    valid = np.isfinite(t1) & (L > 1e-10)
    mid = 0.5 * (t0 + t1)
    with np.errstate(invalid="ignore"):
        xm = x0[:, None] + mid * cos_t[:, None]
        ym = y0[:, None] + mid * sin_t[:, None]
    ix = np.clip(np.floor(np.where(valid, xm, 0.0) + half), 0, N - 1).astype(np.int64)
    iy = np.clip(np.floor(np.where(valid, ym, 0.0) + half), 0, N - 1).astype(np.int64)
    col = ix * N + (N - 1 - iy)          # column-major pixel index, row 0 = top
    counts = valid.sum(axis=1)
    return counts, col[valid].astype(np.int32), L[valid]


def siddon_projector(N: int, n_angles: int, chunk_elems: int = 1 << 24) -> sp.csr_matrix:
    """Ray-major CSR of the parallel-beam line-integral operator (m x N^2).
    Entries of each row are in along-ray order (increasing t), exactly as the
    device generator ``hgm_mat_create_siddon`` emits them."""
    p, theta, s = geometry(N, n_angles)
    # C-libm cos/sin (math module), identical to the device generator's host-side geometry
    cos_t = np.array([math.cos(t) for t in theta])
    sin_t = np.array([math.sin(t) for t in theta])
    m = p * n_angles
    rays_per_chunk = max(1, chunk_elems // (2 * N + 4))
    counts_all, cols_all, vals_all = [], [], []
    ray = 0
    while ray < m:
        r1 = min(m, ray + rays_per_chunk)
        idx = np.arange(ray, r1)
        a = idx // p
        d = idx % p
        cnt, col, val = _siddon_chunk(N, cos_t[a], sin_t[a], s[d])
        counts_all.append(cnt)
        cols_all.append(col)
        vals_all.append(val)
        ray = r1
    counts = np.concatenate(counts_all)
    indptr = np.zeros(m + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    A = sp.csr_matrix((np.concatenate(vals_all), np.concatenate(cols_all), indptr), shape=(m, N * N))
    A.has_sorted_indices = False
    return A


FAN_R = 2.0          # source-to-centre distance in units of N (this repository's choice; see fan_geometry)


def fan_geometry(N: int, n_angles: int, R: float = FAN_R, span: float | None = None,
                 det_offset: float = DETECTOR_OFFSET):
    """Fan-beam, curved (equiangular) detector geometry standing in for the CTtype 'fancurved' of
    run_2D_phantom.m:12-13.  PRtomo_mismatched is not vendored by the reference and no fixture of
    it exists, so this geometry is the repository's OWN choice, modelled on a curved-detector fan
    beam; parity with PRtomo_mismatched / AIR Tools II fanbeamtomo is UNPINNED.  Its
    departures from fanbeamtomo as commonly documented (unverifiable offline): p = ceil(sqrt(2) N)
    rays per source (fanbeamtomo reportedly rounds), a fan span fitted to the circumscribed circle
    rather than a user angle, and source angles equispaced over a full turn.  The geometry:
    * source angles beta_a = a * 2 pi / n_angles (a full turn), the source at distance D = R N
      from the centre, S_a = D (cos beta_a, sin beta_a);
    * p = ceil(sqrt(2) N) rays per source position at fan angles
      omega_d = ((d - (p-1)/2) + det_offset) * span / p, d = 0..p-1 (equiangular bins: a curved
      detector on an arc around the source);
    * span (radians) defaults to the fan that just covers the image's circumscribed circle,
      2 asin(1 / (sqrt(2) R));
    * ray (a, d) leaves S_a towards the centre rotated by omega_d: direction
      u = -(cos(beta + omega), sin(beta + omega)), formed by the angle-addition formula from the
      C-libm cos / sin of beta and omega (the same IEEE operations on the host and the device).
    Row index a * p + d (source-angle-major, as the parallel geometry).  Returns
    (p, x0, y0, ux, uy) per ray."""
    p = int(math.ceil(math.sqrt(2.0) * N))
    if span is None:
        span = 2.0 * math.asin(1.0 / (math.sqrt(2.0) * R))
    D = R * N
    dom = span / p
    cb = np.array([math.cos(a * (2.0 * math.pi / n_angles)) for a in range(n_angles)])
    sb = np.array([math.sin(a * (2.0 * math.pi / n_angles)) for a in range(n_angles)])
    om = [((d - (p - 1) / 2.0) + det_offset) * dom for d in range(p)]
    co = np.array([math.cos(w) for w in om])
    so = np.array([math.sin(w) for w in om])
    cbr, sbr = np.repeat(cb, p), np.repeat(sb, p)
    cor, sor = np.tile(co, n_angles), np.tile(so, n_angles)
    x0 = D * cbr
    y0 = D * sbr
    ux = -(cbr * cor - sbr * sor)
    uy = -(sbr * cor + cbr * sor)
    return p, x0, y0, ux, uy


def fanbeam_projector(N: int, n_angles: int, R: float = FAN_R, span: float | None = None,
                      det_offset: float = DETECTOR_OFFSET, chunk_elems: int = 1 << 24) -> sp.csr_matrix:
    """Ray-major CSR of the fan-beam (curved detector) line-integral operator (fan_geometry),
    entries of each row in along-ray order; bit-identical to the device generator
    ``hgm_mat_create_fanbeam``."""
    p, x0, y0, ux, uy = fan_geometry(N, n_angles, R, span, det_offset)
    m = p * n_angles
    rays_per_chunk = max(1, chunk_elems // (2 * N + 4))
    counts_all, cols_all, vals_all = [], [], []
    for r0 in range(0, m, rays_per_chunk):
        sl = slice(r0, min(m, r0 + rays_per_chunk))
        cnt, col, val = _siddon_rays(N, x0[sl], y0[sl], ux[sl], uy[sl])
        counts_all.append(cnt)
        cols_all.append(col)
        vals_all.append(val)
    counts = np.concatenate(counts_all)
    indptr = np.zeros(m + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    A = sp.csr_matrix((np.concatenate(vals_all), np.concatenate(cols_all), indptr), shape=(m, N * N))
    A.has_sorted_indices = False
    return A


def pixel_driven_backprojector(N: int, n_angles: int) -> sp.csr_matrix:
    """Unmatched back-projector B (n x m, pixel-major CSR): for every pixel
    centre and angle, linear interpolation between the two nearest detector
    bins.  Weights per (pixel, angle) sum to 1, the scale of A^T."""
    p, theta, s = geometry(N, n_angles)
    half = N / 2.0
    n = N * N
    pix = np.arange(n, dtype=np.int64)
    c = pix // N
    r = pix % N
    xc = c - half + 0.5
    yc = (N - 1 - r) - half + 0.5
    rows, cols, vals = [], [], []
    for a in range(n_angles):
        sa = -xc * math.sin(float(theta[a])) + yc * math.cos(float(theta[a]))
        df = sa + (p - 1) / 2.0 - DETECTOR_OFFSET
        d0 = np.floor(df).astype(np.int64)
        w1 = df - d0
        for dd, w in ((d0, 1.0 - w1), (d0 + 1, w1)):
            ok = (dd >= 0) & (dd < p) & (w > 0)
            rows.append(pix[ok])
            cols.append((a * p + dd[ok]).astype(np.int64))
            vals.append(w[ok])
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    vals = np.concatenate(vals)
    B = sp.csr_matrix((vals, (rows, cols)), shape=(n, p * n_angles))
    B.sum_duplicates()
    B.sort_indices()
    return B


def shepp_logan(N: int) -> np.ndarray:
    """Modified (Toft) Shepp–Logan phantom on an N x N grid, values in [0, 1].
    Row 0 is the top of the image (y = +1)."""
    E = [  # intensity, a, b, x0, y0, phi(deg)
        (1.0, 0.69, 0.92, 0.0, 0.0, 0.0),
        (-0.8, 0.6624, 0.8740, 0.0, -0.0184, 0.0),
        (-0.2, 0.1100, 0.3100, 0.22, 0.0, -18.0),
        (-0.2, 0.1600, 0.4100, -0.22, 0.0, 18.0),
        (0.1, 0.2100, 0.2500, 0.0, 0.35, 0.0),
        (0.1, 0.0460, 0.0460, 0.0, 0.1, 0.0),
        (0.1, 0.0460, 0.0460, 0.0, -0.1, 0.0),
        (0.1, 0.0460, 0.0230, -0.08, -0.605, 0.0),
        (0.1, 0.0230, 0.0230, 0.0, -0.606, 0.0),
        (0.1, 0.0230, 0.0460, 0.06, -0.605, 0.0),
    ]
    g = (np.arange(N) + 0.5) / N * 2.0 - 1.0
    X, Y = np.meshgrid(g, -g)          # Y[0, :] = top row
    P = np.zeros((N, N))
    for I, a, b, x0, y0, phi in E:
        ph = math.radians(phi)
        xr = (X - x0) * math.cos(ph) + (Y - y0) * math.sin(ph)
        yr = -(X - x0) * math.sin(ph) + (Y - y0) * math.cos(ph)
        P[(xr / a) ** 2 + (yr / b) ** 2 <= 1.0] += I
    return np.clip(P, 0.0, 1.0)


@dataclass
class TomoProblem:
    N: int
    n_angles: int
    p: int
    A: sp.csr_matrix          # m x n, ray-major
    B: sp.csr_matrix          # n x m, pixel-major back-projector
    b: np.ndarray             # noisy sinogram (m)
    b_exact: np.ndarray
    x_true: np.ndarray        # phantom, column-major (n)

    @property
    def m(self):
        return self.A.shape[0]

    @property
    def n(self):
        return self.A.shape[1]


def tomo_problem(N: int, n_angles: int, noise: float = 1e-2, seed: int = 0,
                 backprojector: str = "matched", geometry_kind: str = "parallel") -> TomoProblem:
    """Build (A, B, b, x_true).  ``backprojector`` is ``"matched"`` (B = A^T)
    or ``"pixel"`` (unmatched pixel-driven B, parallel beam only).  ``geometry_kind``:
    ``"parallel"`` (Siddon, angles over [0, pi)) or ``"fan"`` (curved-detector fan beam over a
    full turn, :func:`fan_geometry`)."""
    if geometry_kind == "fan":
        if backprojector != "matched":
            raise ValueError("the fan-beam geometry pairs with the matched back-projector only")
        A = fanbeam_projector(N, n_angles)
    elif geometry_kind == "parallel":
        A = siddon_projector(N, n_angles)
    else:
        raise ValueError("geometry_kind must be 'parallel' or 'fan'")
    p = geometry(N, n_angles)[0]
    x_true = shepp_logan(N).ravel(order="F")
    b_exact = A @ x_true
    rng = np.random.default_rng(seed)
    e = rng.standard_normal(A.shape[0])
    e = e / np.linalg.norm(e) * noise * np.linalg.norm(b_exact)
    b = b_exact + e
    if backprojector == "matched":
        B = A.T.tocsr()
        B.sort_indices()
    elif backprojector == "pixel":
        B = pixel_driven_backprojector(N, n_angles)
    else:
        raise ValueError("backprojector must be 'matched' or 'pixel'")
    return TomoProblem(N, n_angles, p, A, B, b, b_exact, x_true)


def config_problem(name: str, **kw) -> TomoProblem:
    N, na = CONFIGS[name]
    return tomo_problem(N, na, **kw)
