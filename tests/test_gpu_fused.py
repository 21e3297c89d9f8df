"""The one-pass m-space operator A*(B*q) (csrc/fused.hip; HGM_OPT_FUSED_AB).

For the AB solvers (ABgmres_*_bounds.m:25, m-space Arnoldi on A*B) with B = A' value for value,
B*q (the kept column) and A*(B*q) come out of one pass over B's pixel-major entries.  The sums run
in another fixed order than the two-pass kernels', so:
  * against the two-pass path and the oracle: H, x and the histories within 1e-10 (north_star),
  * repeated solves: bitwise equal (no atomics),
  * B*q itself (the kept column, read by x = (B*Q) y): within rounding of the two-pass product,
  * pixel grids whose side is not a multiple of the region, several region sizes, and a region
    crossed by more rays than the LDS holds (the plan is refused: the two-pass path runs).
Two kernels do the pass (HGM_OPT_FUSED_KIND): the sub-chunk pass (kind 0) and the row-wave pass
(kind 1, the default); both are held to the same bars over several region shapes, waves and row
batches.
The full-size check (C4, 1e9 nnz, 20 iterations vs the oracle fixture) is
tests/test_gpu_fullsize.py::test_c4_ab_gmres_full_size, which runs with the fused pass on (default).
"""
import numpy as np
import pytest

import hgmres
from hgmres.problems import shepp_logan, tomo_problem
from oracle import restatement as R

pytestmark = pytest.mark.gpu

TOL = 1e-10


def rel(a, b):
    return float(np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(b), 1e-300))


def hist_dev(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b)) / np.abs(np.asarray(b))))


def _device_problem(ctx, N, na, seed=0):
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx)          # tiled pixel order (fused-eligible)
    xt = shepp_logan(N).ravel(order="F")
    b0 = A @ xt
    e = np.random.default_rng(seed).standard_normal(A.shape[0])
    return A, A.T, b0 + e / np.linalg.norm(e) * 1e-2 * np.linalg.norm(b0), xt


# (N, angles, kind, region, waves, rows per batch, ring depth, pairs): kind 0 the sub-chunk pass
# (fused_region), kind 1 the row-wave pass (fused_wregion / _waves / _group / _depth / _pairs);
# the row-wave variants other than the default (8 rows, depth 2, pairs) exist for 4 waves and
# <= 1,984 rays per region (the 32 x 32 regions at 47 angles)
CASES = [(512, 30, 0, 64, 0, 0, 0, 0), (100, 17, 0, 64, 0, 0, 0, 0), (256, 47, 0, 32, 0, 0, 0, 0),
         (256, 47, 0, 16, 0, 0, 0, 0), (128, 90, 0, 24, 0, 0, 0, 0),
         (512, 30, 1, 32, 4, 8, 2, 1), (100, 17, 1, 32, 4, 8, 2, 1), (256, 47, 1, 24, 4, 8, 2, 1),
         (256, 47, 1, 16, 1, 8, 2, 1), (256, 47, 1, 32, 2, 8, 2, 1), (128, 90, 1, 16, 2, 8, 2, 1),
         (200, 60, 1, 20, 1, 8, 2, 1), (256, 47, 1, 32, 4, 4, 3, 1), (256, 47, 1, 32, 4, 8, 3, 1),
         (256, 47, 1, 32, 4, 4, 2, 1), (256, 47, 1, 32, 4, 8, 2, 0), (256, 47, 1, 32, 4, 4, 2, 0)]


def _experiments():
    from hgmres import _lib as L
    return bool(L.load().hgm_experiments())


def _variant_only_in_experiments(is_variant):
    """Measured variants of the one-pass kernel (kind 0, other wave / batch / depth / pairing
    shapes, row-pair modes 1-3) are compiled into the experiments build only (HGM_EXPERIMENTS=1;
    run these cases with HGM_LIB pointing at it); the default library refuses their option values."""
    if is_variant and not _experiments():
        pytest.skip("measured variant of the one-pass kernel: experiments build only")


def _fused_opts(kind, region, waves=4, group=8, depth=2, pairs=1):
    if kind == 0:
        return dict(fused_ab=1, fused_kind=0, fused_region=region)
    return dict(fused_ab=1, fused_kind=1, fused_wregion=region, fused_waves=waves, fused_group=group,
                fused_depth=depth, fused_pairs=pairs)


@pytest.mark.parametrize("N,na,kind,region,waves,group,depth,pairs", CASES)
def test_fused_ab_matches_two_pass_and_oracle(gpu_ctx, N, na, kind, region, waves, group, depth, pairs):
    _variant_only_in_experiments(kind == 0 or (waves, group, depth, pairs) != (4, 8, 2, 1))
    A, B, b, xt = _device_problem(gpu_ctx, N, na)
    k = 20
    with gpu_ctx.options(fused_ab=0):
        ref2 = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
    with gpu_ctx.options(**_fused_opts(kind, region, waves, group, depth, pairs)):
        out = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
        again = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
        hyb = hgmres.ABgmres_hybrid_bounds(A, B, b, xt, 0.0, k, 1e-2, ctx=gpu_ctx, return_H=True)
        if kind == 0:
            # the workgroup-size variant keeps the summation order: the same bits
            with gpu_ctx.options(fused_bs=512):
                o2 = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
            assert all(np.array_equal(np.asarray(a_), np.asarray(b_)) for a_, b_ in zip(out, o2))
    with gpu_ctx.options(fused_ab=0):
        hyb2 = hgmres.ABgmres_hybrid_bounds(A, B, b, xt, 0.0, k, 1e-2, ctx=gpu_ctx, return_H=True)
    for a_, b_ in zip(out, again):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))               # bitwise reproducible
    dH = float(np.max(np.abs(out[-1] - ref2[-1])) / np.max(np.abs(ref2[-1])))
    print(f"[fused N={N} angles={na} kind={kind} region={region} waves={waves} group={group} depth={depth} "
          f"pairs={pairs}] "
          f"|dH| vs two-pass {dH:.1e}, x {rel(out[0], ref2[0]):.1e}")
    assert dH <= TOL and rel(out[0], ref2[0]) <= TOL
    assert hist_dev(out[1], ref2[1]) <= TOL and hist_dev(out[2], ref2[2]) <= TOL
    assert rel(hyb[0], hyb2[0]) <= TOL and hist_dev(hyb[2], hyb2[2]) <= TOL
    # the oracle on the downloaded operator (reference pixel order)
    As = A.to_scipy()
    Bs = As.T.tocsr()
    xo, eo, ro, ko, Ho = R.ABgmres_nonhybrid_bounds(As, Bs, b, xt, 0.0, k, return_H=True)
    assert ko == out[3] == k
    assert float(np.max(np.abs(out[-1] - Ho)) / np.max(np.abs(Ho))) <= TOL
    assert rel(out[0], xo) <= TOL and hist_dev(out[1], eo) <= TOL and hist_dev(out[2], ro) <= TOL


@pytest.mark.parametrize("N,na,dtype", [(2048, 19, None), (1024, 47, "f32")])
def test_fused_pass_stress_repeat_bitwise(gpu_ctx, N, na, dtype):
    """The row-wave pass adds into LDS accumulators without atomicity (ds_add_f64 into a wave-private
    array, fp32 read-add-write); its determinism rests on the in-order execution of one wave's DS
    instructions and distinct slots per instruction (fused.hip lds_add).  Stress it:
    60 back-to-back passes over an operator with thousands of regions in flight must all return the
    same bits as the first, for both outputs."""
    from hgmres import _lib as L
    dt = L.HGM_F32 if dtype else L.HGM_F64
    A = hgmres.SparseOperator.siddon(N, na, ctx=gpu_ctx, dtype=dt)
    B = A.T
    q = np.random.default_rng(11).standard_normal(A.shape[0])
    if dtype:
        q = q.astype(np.float32)
    with gpu_ctx.options(fused_ab=1):
        hgmres.fused_plan_info(A, B)                     # the one pass is taken
        bq0, ab0 = hgmres.spmv_ab(A, B, q)
        for i in range(60):
            bq, ab = hgmres.spmv_ab(A, B, q)
            assert np.array_equal(ab, ab0) and np.array_equal(bq, bq0), i
    A.close()
    B.close()


@pytest.mark.parametrize("kind", [0, 1])
def test_fused_region_overflow_falls_back(gpu_ctx, kind):
    """A 128 x 128 region at 47 angles is crossed by ~7,700 rays (> the 3,968 LDS accumulators of
    the sub-chunk pass); a 64 x 64 region by ~3,900 (> the 1,984 ray slots of four row waves):
    the plan is refused and the two-pass path gives the result, bit for bit."""
    _variant_only_in_experiments(kind == 0)
    A, B, b, xt = _device_problem(gpu_ctx, 256, 47)
    with gpu_ctx.options(fused_ab=0):
        ref = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True)
    if kind == 1:
        # the row-wave plan retries a refused region with half its side (round 5): 64 -> 32, the
        # default plan, bit for bit
        with gpu_ctx.options(**_fused_opts(1, 64)):
            out = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True)
        with gpu_ctx.options(**_fused_opts(1, 32)):
            dflt = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True)
        for a_, b_ in zip(out, dflt):
            assert np.array_equal(np.asarray(a_), np.asarray(b_))
        # refused at every size: 24 x 24 regions at 180 angles (~5,600 rays) and 12 < 16 -> two passes
        A, B, b, xt = _device_problem(gpu_ctx, 256, 180)
        with gpu_ctx.options(fused_ab=0):
            ref = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True)
        with gpu_ctx.options(**_fused_opts(1, 24)):
            with pytest.raises((ValueError, hgmres.HgmError)):   # HGM_E_ARG: no plan for the pair
                hgmres.fused_plan_info(A, B)
            out = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True)
    else:
        with gpu_ctx.options(**_fused_opts(0, 128)):
            out = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True)
    for a_, b_ in zip(out, ref):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))


@pytest.mark.parametrize("N,na", [(512, 30), (256, 47), (100, 17)])
def test_fused_pending_normalisation_is_bitwise(gpu_ctx, N, na):
    """Round 6 (HGM_OPT_PEND_NORM = 2, opt-in): on the m-space side the one pass over B stages
    q_k = v_k / H(k,k-1) itself (every wave re-reduces the previous sweep's norm partials in
    k_mgs_normalize's order) and the MGS
    sweep writes q_k back, so the sweep has no scale pass.  The divisions are the same IEEE
    operations on the same operands, so every output is bit for bit the scale-pass solve's: H, x,
    both histories, the hybrid (PTR) variant, the shortest pipeline, and a tol stop mid-solve
    (the speculative steps then hold a pending column that is discarded)."""
    with pytest.raises((ValueError, hgmres.HgmError)):     # 0, 1 or 2
        gpu_ctx.set_option("pend_norm", 3)
    A, B, b, xt = _device_problem(gpu_ctx, N, na)
    k = 20
    runs = {}
    for pn in (0, 1, 2):                                # 2: the m-space pending normalisation
        with gpu_ctx.options(fused_ab=1, pend_norm=pn):
            r = [hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True),
                 hgmres.ABgmres_hybrid_bounds(A, B, b, xt, 0.0, k, 1e-2, ctx=gpu_ctx, return_H=True)]
            with gpu_ctx.options(pipe_depth=1):
                r.append(hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True))
            for kk in (1, 2):
                r.append(hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, kk, ctx=gpu_ctx, return_H=True))
            res = r[0][2]
            tol = 0.5 * (res[6] + res[7])               # stops after iteration 8 (1-based)
            r.append(hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, tol, k, ctx=gpu_ctx, return_H=True))
            runs[pn] = r
    assert runs[2][-1][3] == runs[1][-1][3] == runs[0][-1][3] == 8
    for pn in (1, 2):
        for a, b_ in zip(runs[pn], runs[0]):
            for x1, x0 in zip(a, b_):
                assert np.array_equal(np.asarray(x1), np.asarray(x0))
    print(f"[pending normalisation N={N} angles={na}] 6 solves bitwise equal to the scale-pass solves")


def test_fused_not_taken_for_unmatched_or_reference_order(gpu_ctx):
    """Unmatched B (not A' value for value) and reference-order operators keep the two-pass path:
    the option changes nothing there."""
    P = tomo_problem(32, 16, noise=1e-2, seed=0, backprojector="pixel")
    outs = []
    for f, kd in ((0, 1), (1, 1)) + (((1, 0),) if _experiments() else ()):
        with gpu_ctx.options(fused_ab=f, fused_kind=kd):
            outs.append(hgmres.ABgmres_nonhybrid_bounds(P.A, P.B, P.b, P.x_true, 0.0, 8, ctx=gpu_ctx, return_H=True))
    for o in outs[1:]:
        for a_, b_ in zip(outs[0], o):
            assert np.array_equal(np.asarray(a_), np.asarray(b_))


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("world", [2, 4])
def test_fused_on_pixel_shards(gpu_ctx, world, kind):
    _variant_only_in_experiments(kind == 0)
    """The multi-GPU path (bench.py build_shard, DESIGN.md §5): rank g holds B_g = B(P_g,:), whole
    tile columns of the tiled pixels, and A_g = B_g'.  The one-pass A_g*(B_g*q) on each shard (its
    regions laid over the shard's window of pixel columns) matches the two-pass shard product, repeats
    bitwise, and the shards' partials sum to the full operator's A*(B*q) (the all-reduce)."""
    from hgmres.dist import tile_column_shards
    N, na = 256, 47
    A = hgmres.SparseOperator.siddon(N, na, ctx=gpu_ctx)
    B = A.T
    Nn, tile, sup = A.pixel_order("cols")
    q = np.random.default_rng(1).standard_normal(A.shape[0])
    with gpu_ctx.options(fused_ab=0):
        _, full = hgmres.spmv_ab(A, B, q)
    total = np.zeros(A.shape[0])
    for lo, hi in tile_column_shards(N, world, tile):
        B_g = B.row_slice(lo, hi)
        A_g = B_g.T
        with gpu_ctx.options(fused_ab=0):
            bq2, ab2 = hgmres.spmv_ab(A_g, B_g, q)
        with gpu_ctx.options(fused_ab=1, fused_kind=kind):
            bq1, ab1 = hgmres.spmv_ab(A_g, B_g, q)
            bq1b, ab1b = hgmres.spmv_ab(A_g, B_g, q)
        assert np.array_equal(ab1, ab1b) and np.array_equal(bq1, bq1b)
        assert rel(bq1, bq2) <= 1e-14 and rel(ab1, ab2) <= 1e-13
        total += ab1
        A_g.close()
        B_g.close()
    assert rel(total, full) <= 1e-13


# ---------------------------------------------------------------------------------------------
# One pass per Golub-Kahan iteration: with At = A' value for value on the tiled
# grid, lsqr_solver / lsmr_solver form v_hat = A'*u - beta*v and A*v_hat in one pass over At (the
# row epilogue of the row-wave kernel), alpha^2 as its side sum, and A*v_{k+1} = (A*v_hat)/alpha.
# That differs from A*(v_hat/alpha) by rounding only; the Golub-Kahan recurrences amplify rounding
# about tenfold per iteration, so the bars are those of the production GKB tests:
# 1e-10 against the oracle over the first iterations, bitwise repeats, and fp32 against the fp32
# oracle within the fp32 envelope.
# ---------------------------------------------------------------------------------------------
def _gkb_pair(ctx, N, na, dtype=None):
    from hgmres import _lib as L
    A64, _, b, xt = _device_problem(ctx, N, na)
    if dtype is None:
        return A64, A64.T, b, xt
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=L.HGM_F32)
    return A, A.T, b, xt


@pytest.mark.parametrize("N,na", [(256, 47), (512, 30), (100, 17)])
def test_fused_gkb_fp64_matches_two_pass_and_oracle(gpu_ctx, N, na):
    A, At, b, xt = _gkb_pair(gpu_ctx, N, na)
    with gpu_ctx.options(fused_ab=1):
        hgmres.fused_plan_info(A, At)                    # the one pass is taken (a plan exists)
    k = 8
    with gpu_ctx.options(fused_ab=0):
        q2 = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m2 = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
    with gpu_ctx.options(fused_ab=1):
        q1 = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        q1b = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m1 = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m1b = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
    for a_, b_ in list(zip(q1, q1b)) + list(zip(m1, m1b)):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))               # bitwise reproducible
    As = A.to_scipy()
    xo, eo, ro, ko = R.lsqr_solver(As, b, xt, 0.0, k)
    mo = R.lsmr_solver(As, b, xt, 0.0, k)
    def devs(q, mm):
        return dict(lsqr_x=rel(q[0], xo), lsqr_res=hist_dev(q[2], ro), lsqr_err=hist_dev(q[1], eo),
                    lsmr_x=rel(mm[0], mo[0]), lsmr_res=hist_dev(mm[2], mo[2]), lsmr_err=hist_dev(mm[1], mo[1]),
                    lsmr_ar=hist_dev(mm[3], mo[3]))
    dev, dev2 = devs(q1, m1), devs(q2, m2)
    print(f"[fused gkb fp64 N={N} angles={na} k={k}] " + " ".join(f"{a}={v:.1e}" for a, v in dev.items()) +
          " | two-pass: " + " ".join(f"{a}={v:.1e}" for a, v in dev2.items()))
    assert q1[3] == m1[4] == k
    # the one-pass solve holds the production bar: 1e-10 against the oracle, or (where the two-pass
    # production solve itself is past 1e-10 at k = 8: GKB rounding growth) within 3x of its deviation
    for key in dev:
        assert dev[key] <= max(TOL, 3 * dev2[key]), key


@pytest.mark.parametrize("N,na", [(256, 47), (512, 30)])
def test_fused_gkb_fp32_matches_oracle(gpu_ctx, N, na):
    """configs[4]'s path at test size: the fp32 one-pass LSQR / LSMR against the fp32 restatement
    (oracle/restatement.py lsqr_solver_f32 / lsmr_solver_f32) and the fp32 two-pass solve.  The
    fp32 rows sum in another order, so the bar is the production fp32 envelope:
    1e-5 on every history entry through iteration 4."""
    A, At, b, xt = _gkb_pair(gpu_ctx, N, na, dtype="f32")
    with gpu_ctx.options(fused_ab=1):
        hgmres.fused_plan_info(A, At)                    # the fp32 one pass is taken
    k = 4
    with gpu_ctx.options(fused_ab=0):
        q2 = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m2 = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
    with gpu_ctx.options(fused_ab=1):
        q1 = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        q1b = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m1 = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
    for a_, b_ in zip(q1, q1b):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))
    As = A.to_scipy()                              # fp32 values (exact in float64)
    xo, eo, ro, ko = R.lsqr_solver_f32(As, b, xt, 0.0, k)
    mo = R.lsmr_solver_f32(As, b, xt, 0.0, k)
    dev = dict(lsqr_x=rel(q1[0], xo), lsqr_res=hist_dev(q1[2], ro), lsqr_err=hist_dev(q1[1], eo),
               lsmr_x=rel(m1[0], mo[0]), lsmr_res=hist_dev(m1[2], mo[2]), lsmr_err=hist_dev(m1[1], mo[1]),
               two_pass_lsqr_x=rel(q2[0], xo), vs_two_pass_lsqr_x=rel(q1[0], q2[0]),
               vs_two_pass_lsmr_x=rel(m1[0], m2[0]))
    print(f"[fused gkb fp32 N={N} angles={na} k={k}] " + " ".join(f"{a}={v:.1e}" for a, v in dev.items()))
    for key in ("lsqr_res", "lsqr_err", "lsmr_res", "lsmr_err"):
        assert dev[key] <= 1e-5, key
    for key in ("lsqr_x", "lsmr_x", "vs_two_pass_lsqr_x", "vs_two_pass_lsmr_x"):
        assert dev[key] <= 1e-4, key


@pytest.mark.parametrize("dtype", [None, "f32"])
def test_lsmr_device_scalars_match_host_loop(gpu_ctx, dtype):
    """lsmr_solver's device-resident scalars (HGM_OPT_LSQR_DEV): the rotations
    lsmr_solver.m:42-67 in one device thread and the stop test :76 on the device against the host
    loop (lsqr_dev = 0) -- the same iterations, histories and x up to the last bits of hypot (device
    against host libm); with tol between two residuals the solve stops at the same iteration
    (inside the first batch of 8), and the iterations enqueued past the stop leave x as it was."""
    A, At, b, xt = _gkb_pair(gpu_ctx, 256, 47, dtype=dtype)
    bar = 1e-12 if dtype is None else 1e-5
    with gpu_ctx.options(fused_ab=1):
        hgmres.fused_plan_info(A, At)
        full = {}
        for dev_ in (1, 0):
            with gpu_ctx.options(lsqr_dev=dev_):
                full[dev_] = hgmres.lsmr_solver(A, b, xt, 0.0, 12, ctx=gpu_ctx, At=At)
        d, h = full[1], full[0]
        assert d[4] == h[4] == 12
        for i in range(1, 4):
            assert hist_dev(d[i], h[i]) <= bar, i
        assert rel(d[0], h[0]) <= bar
        res = np.asarray(h[2])
        tol = 0.5 * (res[4] + res[5])                  # stops at iteration 6 (1-based): res[5] < tol
        assert res[5] < tol <= res[4]
        stopped = {}
        for dev_ in (1, 0):
            with gpu_ctx.options(lsqr_dev=dev_):
                stopped[dev_] = hgmres.lsmr_solver(A, b, xt, tol, 12, ctx=gpu_ctx, At=At)
        sd, sh = stopped[1], stopped[0]
        assert sd[4] == sh[4] == 6
        for i in range(1, 4):
            assert len(sd[i]) == 6 and hist_dev(sd[i], sh[i]) <= bar, i
        assert rel(sd[0], sh[0]) <= bar


@pytest.mark.parametrize("dtype", [None, "f32"])
def test_lsqr_one_pass_scalars_and_tol_stop(gpu_ctx, dtype):
    """lsqr_solver's one-pass path: device-resident scalars (k_lsqr_rot, the stop test
    lsqr_solver.m:44-46 on the device, read once per batch of 8) against the same pass with host
    scalars (lsqr_dev = 0: beta^2 / alpha^2 read back, the rotation :31-38 on the host) -- the same
    double arithmetic, so the same bits up to sqrt; with tol between two residuals both stop at
    the same iteration inside the first batch, with the iterations enqueued past the stop leaving
    x and w as they were; against the two-pass solve and (fp64) the oracle, niters equal and the
    histories at 1e-10 (fp32: the fp32 envelope, 1e-5, against the fp32 restatement)."""
    A, At, b, xt = _gkb_pair(gpu_ctx, 256, 47, dtype=dtype)
    bar = 1e-12 if dtype is None else 1e-5
    with gpu_ctx.options(fused_ab=1):
        hgmres.fused_plan_info(A, At)                  # the one pass is taken
        full = {}
        for dev_ in (1, 0):
            with gpu_ctx.options(lsqr_dev=dev_):
                full[dev_] = hgmres.lsqr_solver(A, b, xt, 0.0, 12, ctx=gpu_ctx, At=At)
    d, h = full[1], full[0]
    assert d[3] == h[3] == 12
    for i in (1, 2):
        assert hist_dev(d[i], h[i]) <= bar, i
    assert rel(d[0], h[0]) <= bar
    res = np.asarray(h[2])
    tol = 0.5 * (res[4] + res[5])                      # :46 (<=) stops at iteration 6 (1-based)
    assert res[5] <= tol < res[4]
    stopped = {}
    with gpu_ctx.options(fused_ab=1):
        for dev_ in (1, 0):
            with gpu_ctx.options(lsqr_dev=dev_):
                stopped[dev_] = hgmres.lsqr_solver(A, b, xt, tol, 12, ctx=gpu_ctx, At=At)
    with gpu_ctx.options(fused_ab=0):
        two = hgmres.lsqr_solver(A, b, xt, tol, 12, ctx=gpu_ctx, At=At)
    As = A.to_scipy()
    ref = (R.lsqr_solver(As, b, xt, tol, 12) if dtype is None else R.lsqr_solver_f32(As, b, xt, tol, 12))
    sd, sh = stopped[1], stopped[0]
    assert sd[3] == sh[3] == two[3] == ref[3] == 6
    devs = dict(dev_vs_host=max(hist_dev(sd[1], sh[1]), hist_dev(sd[2], sh[2]), rel(sd[0], sh[0])),
                vs_two_pass=max(hist_dev(sd[1], two[1]), hist_dev(sd[2], two[2]), rel(sd[0], two[0])),
                vs_oracle=max(hist_dev(sd[1], ref[1]), hist_dev(sd[2], ref[2]), rel(sd[0], ref[0])))
    print(f"[lsqr one pass tol stop {dtype or 'f64'}] k={sd[3]} " + " ".join(f"{a}={v:.1e}" for a, v in devs.items()))
    assert devs["dev_vs_host"] <= bar
    # the exact final residual (lsqr_solver.m:52) from the kept A*x image against one more SpMV
    # (lsqr_res_img = 0): the same x, the last residual within the image's rounding
    with gpu_ctx.options(fused_ab=1, lsqr_res_img=0):
        expl = hgmres.lsqr_solver(A, b, xt, tol, 12, ctx=gpu_ctx, At=At)
    assert np.array_equal(np.asarray(expl[0]), np.asarray(sd[0]))
    assert np.array_equal(np.asarray(expl[2])[:-1], np.asarray(sd[2])[:-1])
    dres = abs(expl[2][-1] - sd[2][-1]) / expl[2][-1]
    print(f"[lsqr final residual image vs SpMV {dtype or 'f64'}] {dres:.1e}")
    assert dres <= (1e-12 if dtype is None else 1e-4)
    # fp32: iterations 5-6 are past the fp32 envelope's 1e-5 (1e-3 from iteration 5)
    assert devs["vs_two_pass"] <= (TOL if dtype is None else 1e-3)
    assert devs["vs_oracle"] <= (TOL if dtype is None else 1e-3)


def test_fused_spmv_ab_fp32(gpu_ctx):
    """hgm_spmv_ab on an fp32 pair runs the fp32 one-pass kernel: within fp32 rounding of the
    two-pass product, bitwise repeatable."""
    A, At, b, xt = _gkb_pair(gpu_ctx, 256, 47, dtype="f32")
    B = At
    q = np.random.default_rng(3).standard_normal(A.shape[0]).astype(np.float32)
    with gpu_ctx.options(fused_ab=0):
        bq2, ab2 = hgmres.spmv_ab(A, B, q)
    with gpu_ctx.options(fused_ab=1):
        bq1, ab1 = hgmres.spmv_ab(A, B, q)
        bq1b, ab1b = hgmres.spmv_ab(A, B, q)
    assert np.array_equal(ab1, ab1b) and np.array_equal(bq1, bq1b)
    Bs = B.to_scipy()
    ref_bq = Bs @ q.astype(np.float64)
    ref_ab = Bs.T @ ref_bq
    print(f"[fused spmv_ab fp32] bq {rel(bq1, ref_bq):.1e} (two-pass {rel(bq2, ref_bq):.1e}), "
          f"ab {rel(ab1, ref_ab):.1e} (two-pass {rel(ab2, ref_ab):.1e})")
    assert rel(bq1, ref_bq) <= 1e-6 and rel(ab1, ref_ab) <= 1e-6


def test_fused_failed_plan_is_retried_with_other_options(gpu_ctx):
    """a refused plan (70 x 70 regions at 47 angles: ~3,400 rays, and ~2,100 at the
    35 x 35 half it is retried with, past the 1,984 ray slots of four row waves) is remembered for
    THAT option tuple only; the default options then plan and run the one pass on the same operator
    (kernel timing sees the fused class)."""
    A, B, b, xt = _device_problem(gpu_ctx, 256, 47)
    q = np.random.default_rng(2).standard_normal(A.shape[0])
    with gpu_ctx.options(fused_ab=0):
        _, ref = hgmres.spmv_ab(A, B, q)
    with gpu_ctx.options(**_fused_opts(1, 70)):
        with pytest.raises((ValueError, hgmres.HgmError)):
            hgmres.fused_plan_info(A, B)
        _, r64 = hgmres.spmv_ab(A, B, q)                  # refused: the two-pass product
    assert np.array_equal(r64, ref)
    gpu_ctx.kernel_timing(True)
    try:
        _, r32 = hgmres.spmv_ab(A, B, q)                  # defaults: the one pass
        ms, calls, _ = gpu_ctx.kernel_timing_read(3)
    finally:
        gpu_ctx.kernel_timing(False)
    assert calls == 1 and rel(r32, ref) <= 1e-13


def test_fused_dbg_refused_by_solvers(gpu_ctx):
    """fused_dbg (phase-skipping timing variants, wrong results) is refused by every
    solver; hgm_spmv_ab keeps it for scripts/fused_micro.py in the experiments build.  The default
    library refuses the option value itself."""
    A, B, b, xt = _device_problem(gpu_ctx, 64, 17)
    if not _experiments():
        with pytest.raises((ValueError, hgmres.HgmError), match="experiments build"):
            gpu_ctx.set_option("fused_dbg", 1)
        assert gpu_ctx.get_option("fused_dbg") == 0
        return
    with gpu_ctx.options(fused_dbg=1):
        with pytest.raises(ValueError, match="fused_dbg"):
            hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 4, ctx=gpu_ctx)
        with pytest.raises(ValueError, match="fused_dbg"):
            hgmres.lsqr_solver(A, b, xt, 0.0, 4, ctx=gpu_ctx, At=B)


@pytest.mark.parametrize("N,na,dtype,world", [(256, 47, None, 1), (512, 30, None, 1), (100, 17, None, 1),
                                              (256, 47, "f32", 1), (256, 47, None, 2)])
def test_fused_plan_device_build_matches_host(gpu_ctx, N, na, dtype, world):
    """VERDICT r3 "Next" #5: the row-wave plan's ray sets and slots built on the device (an LDS
    bitmap per region, fused.hip k_plan_count / k_plan_fill) are the host build's byte for byte
    (checksum over every plan array), and the products are bitwise equal.  world = 2: rank 0's
    pixel shard (bench.py build_shard)."""
    from hgmres import _lib as L
    A = hgmres.SparseOperator.siddon(N, na, ctx=gpu_ctx, dtype=L.HGM_F32 if dtype else L.HGM_F64)
    B = A.T
    if world > 1:
        from hgmres.dist import tile_column_shards
        Nn, tile, sup = A.pixel_order("cols")
        lo, hi = tile_column_shards(N, world, tile)[0]
        B = B.row_slice(lo, hi)
        A = B.T
    q = np.random.default_rng(4).standard_normal(A.shape[0])
    info, outs = {}, {}
    for dev in (0, 1):
        with gpu_ctx.options(fused_ab=1, fused_plan_dev=dev):
            info[dev] = hgmres.fused_plan_info(A, B)
            outs[dev] = hgmres.spmv_ab(A, B, q)
    print(f"[plan N={N} angles={na} {dtype or 'f64'} world={world}] host {info[0]['build_s']:.3f} s, "
          f"device {info[1]['build_s']:.3f} s, {info[1]['nslot']} slots")
    assert info[1]["device_built"] and not info[0]["device_built"]
    assert info[0]["checksum"] == info[1]["checksum"] and info[0]["nslot"] == info[1]["nslot"]
    assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,na,dtype", [(256, 47, None), (512, 30, None), (256, 47, "f32"), (100, 17, None)])
def test_fused_reduce_by_band_is_bitwise(gpu_ctx, N, na, dtype):
    """The partial reduction by ray band (runs of consecutive slots, HGM_OPT_FUSED_REDUCE = 1)
    forms exactly the sums of the per-ray reduction through the slot list (= 0, the default):
    products, the AB-GMRES solve and the one-pass LSQR bit for bit.  The fewer-lanes-per-ray
    variants (2, 3, 4: another fixed order, measured slower) are refused by the default library."""
    from hgmres import _lib as L
    A = hgmres.SparseOperator.siddon(N, na, ctx=gpu_ctx, dtype=L.HGM_F32 if dtype else L.HGM_F64)
    B = A.T
    q = np.random.default_rng(5).standard_normal(A.shape[0])
    xt = shepp_logan(N).ravel(order="F")
    b = (A @ xt).astype(np.float64)
    outs = {}
    for red in (0, 1):
        with gpu_ctx.options(fused_ab=1, fused_reduce=red):
            hgmres.fused_plan_info(A, B)
            o = list(hgmres.spmv_ab(A, B, q))
            o += list(hgmres.lsqr_solver(A, b, xt, 0.0, 6, ctx=gpu_ctx, At=B)[:3])
            if dtype is None:
                o += list(hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, 8, ctx=gpu_ctx, return_H=True))
            outs[red] = o
    for a_, b_ in zip(outs[0], outs[1]):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))
    if not _experiments():
        for red in (2, 3, 4):
            with pytest.raises((ValueError, hgmres.HgmError), match="experiments build"):
                gpu_ctx.set_option("fused_reduce", red)
        assert gpu_ctx.get_option("fused_reduce") == 0


# ---------------------------------------------------------------------------------------------
# Row pairs (HGM_OPT_FUSED_ROWPAIR, k_fused_rw RP, round 5): two consecutive pixel rows per
# 128-entry chunk, each row parity into its own private accumulator array per wave.  Another
# fixed summation order: the same bars as the default pass (two-pass and oracle at 1e-10,
# bitwise repeats; GKB in its production envelope), on geometries whose pairs overflow a chunk
# (the plan cuts those runs) and ones that never do.
# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("N,na,rp", [(256, 47, 1), (256, 47, 2), (256, 47, 3), (256, 47, 4), (512, 30, 4),
                                     (100, 17, 4), (200, 60, 4), (2048, 19, 4)])
def test_fused_rowpair_gmres_matches_oracle(gpu_ctx, N, na, rp):
    _variant_only_in_experiments(rp in (1, 2, 3))
    A, B, b, xt = _device_problem(gpu_ctx, N, na)
    k = 20
    with gpu_ctx.options(fused_ab=0):
        ref2 = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
    with gpu_ctx.options(fused_ab=1, fused_rowpair=rp):
        info = hgmres.fused_plan_info(A, B)
        out = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
        again = hgmres.ABgmres_nonhybrid_bounds(A, B, b, xt, 0.0, k, ctx=gpu_ctx, return_H=True)
        bq1, ab1 = hgmres.spmv_ab(A, B, b)
    with gpu_ctx.options(fused_ab=1, fused_rowpair=0):
        bq0, ab0 = hgmres.spmv_ab(A, B, b)

    for a_, b_ in zip(out, again):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))
    dH = float(np.max(np.abs(out[-1] - ref2[-1])) / np.max(np.abs(ref2[-1])))
    print(f"[rowpair {rp} N={N} angles={na}] slots {info['nslot']}: |dH| vs two-pass {dH:.1e}, x {rel(out[0], ref2[0]):.1e}, "
          f"A(Bq) vs default pass {rel(ab1, ab0):.1e}, Bq {rel(bq1, bq0):.1e}")
    assert rel(bq1, bq0) <= 1e-14 and rel(ab1, ab0) <= 1e-14
    assert dH <= TOL and rel(out[0], ref2[0]) <= TOL
    As = A.to_scipy()
    xo, eo, ro, ko, Ho = R.ABgmres_nonhybrid_bounds(As, As.T.tocsr(), b, xt, 0.0, k, return_H=True)
    assert float(np.max(np.abs(out[-1] - Ho)) / np.max(np.abs(Ho))) <= TOL
    assert rel(out[0], xo) <= TOL and hist_dev(out[1], eo) <= TOL and hist_dev(out[2], ro) <= TOL


@pytest.mark.parametrize("rp", [1, 2, 3, 4])
@pytest.mark.parametrize("dtype", [None, "f32"])
def test_fused_rowpair_gkb_matches_oracle(gpu_ctx, dtype, rp):
    _variant_only_in_experiments(rp in (1, 2, 3))
    A, At, b, xt = _gkb_pair(gpu_ctx, 256, 47, dtype=dtype)
    k = 8 if dtype is None else 4
    with gpu_ctx.options(fused_ab=1, fused_rowpair=rp):
        hgmres.fused_plan_info(A, At)
        q1 = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        q1b = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m1 = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
    with gpu_ctx.options(fused_ab=1, fused_rowpair=0):
        q0 = hgmres.lsqr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
        m0 = hgmres.lsmr_solver(A, b, xt, 0.0, k, ctx=gpu_ctx, At=At)
    for a_, b_ in zip(q1, q1b):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))
    As = A.to_scipy()
    if dtype is None:
        qo, mo = R.lsqr_solver(As, b, xt, 0.0, k), R.lsmr_solver(As, b, xt, 0.0, k)
    else:
        qo, mo = R.lsqr_solver_f32(As, b, xt, 0.0, k), R.lsmr_solver_f32(As, b, xt, 0.0, k)
    dev = dict(lsqr_x=rel(q1[0], qo[0]), lsqr_res=hist_dev(q1[2], qo[2]), lsmr_x=rel(m1[0], mo[0]),
               lsmr_res=hist_dev(m1[2], mo[2]), lsmr_ar=hist_dev(m1[3], mo[3]))
    dev0 = dict(lsqr_x=rel(q0[0], qo[0]), lsqr_res=hist_dev(q0[2], qo[2]), lsmr_x=rel(m0[0], mo[0]),
                lsmr_res=hist_dev(m0[2], mo[2]), lsmr_ar=hist_dev(m0[3], mo[3]))
    print(f"[rowpair {rp} gkb {dtype or 'f64'} k={k}] " + " ".join(f"{a}={v:.1e}" for a, v in dev.items()) +
          " | default pass: " + " ".join(f"{a}={v:.1e}" for a, v in dev0.items()))
    bar = TOL if dtype is None else 1e-5
    for key in dev:
        assert dev[key] <= max(bar, 3 * dev0[key]), key


# ---------------------------------------------------------------------------------------------
# The fp32 one pass (C5's kernels) against the fp32 oracle within the oracle's OWN fp32 rounding
# envelope (at 4096^2 the fp32 production histories are held to fixed bars
# through iteration 5 only, test_gpu_fullsize.py).  _Rounded32 is the dot-product rounding model at
# fp32 eps: a stand-in for any other correct fp32 summation order.  Every history entry and x of a
# 12-iteration solve at 512^2 / 47 angles must lie within max(1e-6, 100 x the largest deviation of
# 4 such oracle runs): the Golub-Kahan recurrences amplify any rounding ~10x per iteration, and the
# device may not do worse than a differently-rounded oracle by more than that factor.
# ---------------------------------------------------------------------------------------------
class _Rounded32:
    dtype = np.float32

    def __init__(self, M, rng, c=4.0, absM=None):
        import scipy.sparse as sp
        self.M, self.rng, self.c = sp.csr_matrix(M, dtype=np.float32), rng, c
        self.absM = abs(self.M) if absM is None else absM
        self.shape = self.M.shape

    def __matmul__(self, v):
        v = np.asarray(v, dtype=np.float32)
        y = (self.M @ v).astype(np.float64)
        y += self.c * 5.96e-8 * (self.absM @ np.abs(v)).astype(np.float64) * self.rng.standard_normal(y.shape)
        return y.astype(np.float32)

    @property
    def T(self):
        return _Rounded32(self.M.T.tocsr(), self.rng, self.c, self.absM.T.tocsr())

    @property
    def val(self):                                   # (lsmr_solver_f32's norm(A, 'fro'))
        return self.M.data


@pytest.mark.parametrize("solver", ["lsqr", "lsmr"])
def test_fp32_one_pass_within_fp32_oracle_envelope(gpu_ctx, solver):
    import scipy.sparse as sp
    from hgmres import _lib as L
    N, na, K, kfac = 512, 47, 12, 100.0
    A, At, b, xt = _gkb_pair(gpu_ctx, N, na, dtype="f32")
    with gpu_ctx.options(fused_ab=1):
        info = hgmres.fused_plan_info(A, At)            # the one pass runs
    Ar = hgmres.SparseOperator.siddon(N, na, ctx=gpu_ctx, dtype=L.HGM_F32, order="reference")
    As = Ar.to_scipy()
    A32 = sp.csr_matrix((As.data.astype(np.float32), As.indices, As.indptr), shape=As.shape)
    fn = {"lsqr": R.lsqr_solver_f32, "lsmr": R.lsmr_solver_f32}[solver]
    gfn = {"lsqr": hgmres.lsqr_solver, "lsmr": hgmres.lsmr_solver}[solver]
    nh = 2 if solver == "lsqr" else 3
    ref = fn(A32, b, xt, 0.0, K)
    with gpu_ctx.options(fused_ab=1):
        out = gfn(A, b, xt, 0.0, K, ctx=gpu_ctx, At=At)
    sx, sh = 0.0, [np.zeros(K) for _ in range(nh)]
    for seed in range(1, 5):
        p = fn(_Rounded32(A32, np.random.default_rng(seed)), b, xt, 0.0, K)
        sx = max(sx, rel(p[0].astype(np.float64), ref[0].astype(np.float64)))
        for i in range(nh):
            sh[i] = np.maximum(sh[i], np.abs(p[1 + i] - ref[1 + i]) / np.abs(ref[1 + i]))
    dx = rel(out[0], ref[0].astype(np.float64))
    ratios = []
    for i in range(nh):
        d = np.abs(np.asarray(out[1 + i]) - ref[1 + i]) / np.abs(ref[1 + i])
        tol = np.maximum(1e-6, kfac * sh[i])
        ratios.append((float(np.max(d)), float(np.max(d / tol)), float(np.max(sh[i]))))
        assert np.all(d <= tol), (i, np.max(d / tol))
    print(f"[fp32 envelope {solver} {N}^2/{na} k={K} slots {info['nslot']}] x dev {dx:.2e} (oracle spread {sx:.2e}); "
          f"histories: " + "; ".join(f"max dev {a:.1e}, {f_:.3f} of the bar (oracle spread up to {m_:.1e})"
                                     for a, f_, m_ in ratios))
    assert dx <= max(1e-6, kfac * sx), (dx, sx)
    Ar.close()


def test_lsmr_fused_step_monitor_is_bitwise(gpu_ctx):
    """HGM_OPT_LSMR_FUSE_NMON: the fp32 one-pass LSMR's n-space step and n-space monitor in one
    launch give the two launches' bits (x and every history)."""
    A, At, b, xt = _gkb_pair(gpu_ctx, 512, 47, dtype="f32")
    outs = {}
    for f in (0, 1):
        with gpu_ctx.options(fused_ab=1, lsmr_fuse_nmon=f):
            outs[f] = hgmres.lsmr_solver(A, b, xt, 0.0, 10, ctx=gpu_ctx, At=At)
    for a_, b_ in zip(outs[0], outs[1]):
        assert np.array_equal(np.asarray(a_), np.asarray(b_))


@pytest.mark.parametrize("maxit", [20, 100, 200])
def test_lsqr_res_img_fp32_long_runs(gpu_ctx, maxit):
    """HGM_OPT_LSQR_RES_IMG (on by default) replaces lsqr_solver.m:52's exact final
    residual norm(b - A*x) by the norm of b minus a double-precision image of A*x kept alongside
    the fp32 x.  Held at the bench's 20 iterations and far past them (100, 200) on the fp32
    one-pass path: the image's value against the true residual of the RETURNED x (b - A*x in
    float64 over the fp32 operator's values, on the host) within 1e-4 relative, and no worse than
    1.5 x the explicit fp32 evaluation (lsqr_res_img = 0: one fp32 SpMV of x, whose own rounding
    in the cancellation b - A*x is ~ eps32 ||b|| / ||r||).  The iterates are the same bits
    either way."""
    A, At, b, xt = _gkb_pair(gpu_ctx, 512, 47, dtype="f32")
    with gpu_ctx.options(fused_ab=1, lsqr_res_img=1):
        xi, ei, ri, ki = hgmres.lsqr_solver(A, b, xt, 0.0, maxit, ctx=gpu_ctx, At=At)
        assert gpu_ctx.solve_path()["one_pass"] == 1
    with gpu_ctx.options(fused_ab=1, lsqr_res_img=0):
        xe, ee, re, ke = hgmres.lsqr_solver(A, b, xt, 0.0, maxit, ctx=gpu_ctx, At=At)
    assert np.array_equal(xi, xe) and np.array_equal(ri[:-1], re[:-1]) and np.array_equal(ei, ee)
    As = A.to_scipy()                                   # fp32 values, held in float64
    true = float(np.linalg.norm(b - As @ xi) / np.linalg.norm(b))
    d_img, d_exp = abs(ri[-1] - true) / true, abs(re[-1] - true) / true
    print(f"[lsqr res img fp32 k={maxit}] true {true:.9e}: image {ri[-1]:.9e} (dev {d_img:.1e}), "
          f"explicit fp32 {re[-1]:.9e} (dev {d_exp:.1e})")
    assert d_img <= 1e-4 and d_img <= max(1.5 * d_exp, 1e-6), (d_img, d_exp)
