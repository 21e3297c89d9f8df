"""Generate the committed golden fixtures under tests/golden/.

The reference (MATLAB) cannot run in this image or on the GPU box and ships no
fixtures, so these vectors are produced by the CPU restatement in
``oracle/restatement.py`` on small synthetic tomography problems.  Inputs are
stored raw (CSR arrays, b, x_true); outputs are the reference-semantics
solver results.  Regenerate with:  python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "hybrid-gmres_amd"))
sys.path.insert(0, ROOT)

from hgmres.problems import tomo_problem  # noqa: E402
from oracle import restatement as R       # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def csr_hash(M):
    """sha256 over indptr (int64), indices (int32), data (float64), without copying the arrays
    (the C4 operator is 12 GB)."""
    h = hashlib.sha256()
    for a, dt in ((M.indptr, np.int64), (M.indices, np.int32), (M.data, np.float64)):
        a = np.ascontiguousarray(a, dtype=dt).reshape(-1)
        step = 1 << 24
        for i in range(0, a.size, step):
            h.update(memoryview(a[i:i + step]))
    return h.hexdigest()


def dump(name, P, maxit, lam, tol=0.0, store_raw=True):
    A, B, b, xt = P.A, P.B, P.b, P.x_true
    d = {"maxit": maxit, "lam": lam, "tol": tol, "N": P.N, "n_angles": P.n_angles,
         "A_sha256": csr_hash(A), "B_sha256": csr_hash(B), "b": b, "x_true": xt}
    if store_raw:
        d.update(A_indptr=A.indptr.astype(np.int64), A_indices=A.indices.astype(np.int32), A_data=A.data.copy(),
                 B_indptr=B.indptr.astype(np.int64), B_indices=B.indices.astype(np.int32), B_data=B.data.copy(),
                 shape=np.array(A.shape))
    x, e, r, k, H = R.hybrid_ab_gmres_rtp(A, B, b, xt, tol, maxit, lam, return_H=True)
    d.update(hab_x=x, hab_err=e, hab_res=r, hab_k=k, hab_H=H)
    x, e, r, k, H = R.hybrid_ba_gmres_rtp(A, B, b, xt, tol, maxit, lam, return_H=True)
    d.update(hba_x=x, hba_err=e, hba_res=r, hba_k=k, hba_H=H)
    for tag, f, args in (("abp", R.ABgmres_hybrid_bounds, (lam,)), ("abn", R.ABgmres_nonhybrid_bounds, ()),
                         ("bap", R.BAgmres_hybrid_bounds, (lam,)), ("ban", R.BAgmres_nonhybrid_bounds, ())):
        x, e, r, k, H = f(A, B, b, xt, tol, maxit, *args, return_H=True)
        d.update({f"{tag}_x": x, f"{tag}_err": e, f"{tag}_res": r, f"{tag}_k": k, f"{tag}_H": H})
    x, e, r, k = R.lsqr_solver(A, b, xt, tol, maxit)
    d.update(lsqr_x=x, lsqr_err=e, lsqr_res=r, lsqr_k=k)
    x, e, r, a, k = R.lsmr_solver(A, b, xt, tol, maxit)
    d.update(lsmr_x=x, lsmr_err=e, lsmr_res=r, lsmr_ar=a, lsmr_k=k)
    x, e, r, k = R.hybrid_lsqr_solver(A, b, xt, tol, maxit, lam)
    d.update(hlsqr_x=x, hlsqr_err=e, hlsqr_res=r, hlsqr_k=k)
    x, e, r, k = R.hybrid_lsmr_solver(A, b, xt, tol, maxit, lam)
    d.update(hlsmr_x=x, hlsmr_err=e, hlsmr_res=r, hlsmr_k=k)
    m = A.shape[0]
    for typ in ("ab", "ba"):
        H, beta = R.arnoldi(A, B, b, maxit, typ)
        d[f"gcv_{typ}_H"] = H
        d[f"gcv_{typ}_beta"] = beta
        d[f"gcv_{typ}_vals"] = np.array([R.gcv_function(l, A, B, b, m, maxit, typ) for l in (1e-6, 1e-4, 1e-2)])
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name, {k: (v.shape if hasattr(v, "shape") else v) for k, v in d.items() if "sha" in k or k == "shape"})


def dump_c3(name="c3_2048.npz", k=20):
    """BASELINE configs[2] at full size (2048^2, 19 angles, nnz 1.01e8) at the bench's iteration
    counts (bench.py WORKLOADS["c3gcv"]): BA-GMRES (hybrid_ba_gmres_rtp, 20 iterations, lambda 1e-2)
    with MGS (the reference's orthogonalisation, hybrid_ba_gmres_rtp.m:20-23) and with CGS2 (the
    config's alternative), and the 20-step GCV Arnoldi (gcv_function.m:18-33) with the lambda that
    fminbnd picks on it over the bench's bounds [1e-8, 1] (TolX 1e-10, analyze_regularization.m:39-46).
    The lambda search is the oracle's own: scipy's fminbound (the Forsythe-Malcolm-Moler search
    MATLAB documents for fminbnd) over the restatement's gcv_from_H -- not the product's
    hgm_gcv_fminbnd, which the full-size test checks against it.
    The operator is pinned by its CSR hash (the device generator reproduces it bitwise); x is stored
    as its norm plus every 997th entry.  SpMVs run on the host's OpenMP threads (oracle/parallel.py:
    bitwise scipy's csr_matvec)."""
    import scipy.optimize as so
    from oracle import parallel as OP
    P = tomo_problem(2048, 19, noise=1e-2, seed=0, backprojector="matched")
    A, B, b, xt = P.A, P.B.tocsr(), P.b, P.x_true
    OP.build()
    PA, PB = OP.ParallelCSR(A), OP.ParallelCSR(B)
    gcv = dict(lo=1e-8, hi=1.0, tolx=1e-10)
    d = {"maxit": k, "lam": 1e-2, "N": 2048, "n_angles": 19, "A_sha256": csr_hash(A), "b": b,
         "sample_stride": 997, "gcv_k": k, "gcv_lo": gcv["lo"], "gcv_hi": gcv["hi"], "gcv_tolx": gcv["tolx"]}
    for orth in ("mgs", "cgs2"):
        x, e, r, kk, H = R.hybrid_ba_gmres_rtp(PA, PB, b, xt, 0.0, k, 1e-2, return_H=True, orth=orth)
        d.update({f"hba_{orth}_H": H, f"hba_{orth}_err": e, f"hba_{orth}_res": r, f"hba_{orth}_k": kk,
                  f"hba_{orth}_xnorm": np.linalg.norm(x), f"hba_{orth}_xs": x[::997].copy()})
        Hg, beta = R.arnoldi(PA, PB, b, k, "ba", orth=orth)
        lam, g, _, _ = so.fminbound(lambda l: R.gcv_from_H(Hg, beta, l, A.shape[1]), gcv["lo"], gcv["hi"],
                                    xtol=gcv["tolx"], full_output=True)
        lam, g = float(lam), float(g)
        d.update({f"gcv_{orth}_H": Hg, f"gcv_{orth}_beta": beta, f"gcv_{orth}_lam": lam, f"gcv_{orth}_val": g})
        # the solve at the GCV lambda: the c3gcv bench step (hybrid_ba_gmres_rtp at lambda_GCV)
        x, e, r, kk, H = R.hybrid_ba_gmres_rtp(PA, PB, b, xt, 0.0, k, lam, return_H=True, orth=orth)
        d.update({f"hbg_{orth}_H": H, f"hbg_{orth}_err": e, f"hbg_{orth}_res": r, f"hbg_{orth}_k": kk,
                  f"hbg_{orth}_xnorm": np.linalg.norm(x), f"hbg_{orth}_xs": x[::997].copy()})
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name, "MGS vs CGS2 |dH|/|H| =",
          np.max(np.abs(d["hba_mgs_H"] - d["hba_cgs2_H"])) / np.max(np.abs(d["hba_mgs_H"])),
          "lambda_GCV", d["gcv_mgs_lam"], d["gcv_cgs2_lam"])


def dump_c4(name="c4_4096.npz", k=20):
    """BASELINE configs[3] at full size (4096^2, 47 angles, nnz 1.004e9): the bench's AB-GMRES
    (ABgmres_nonhybrid_bounds.m, m-space Arnoldi on A*B, B = A') through all 20 iterations.
    Inputs: b (stored: the device forms A*x_true in another summation order), the operator pinned
    by the sha256 of its CSR (reference pixel order).  Outputs: H (21 x 20), the histories, x as its
    norm plus every 997th entry.  SpMVs on the host's OpenMP threads (bitwise scipy).  Needs ~45 GB
    of host memory and ~10 minutes on 8 cores."""
    import gc
    from oracle import parallel as OP
    from hgmres.problems import siddon_projector, shepp_logan
    A = siddon_projector(4096, 47)
    h = csr_hash(A)
    xt = shepp_logan(4096).ravel(order="F")
    OP.build()
    PA = OP.ParallelCSR(A)
    del A
    gc.collect()
    b_exact = PA @ xt
    e = np.random.default_rng(0).standard_normal(PA.shape[0])
    b = b_exact + e / np.linalg.norm(e) * 1e-2 * np.linalg.norm(b_exact)
    PB = PA.T                                     # scipy M.T.tocsr(): rows keep increasing column order
    x, err, res, kk, H = R.ABgmres_nonhybrid_bounds(PA, PB, b, xt, 0.0, k, return_H=True)
    d = {"maxit": k, "N": 4096, "n_angles": 47, "A_sha256": h, "b": b, "sample_stride": 997,
         "abn_H": H, "abn_err": err, "abn_res": res, "abn_k": kk, "abn_xnorm": np.linalg.norm(x),
         "abn_xs": x[::997].copy()}
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name, "k", kk, "res", res[-1], "err", err[-1])


class _Ordered32:
    """The fp32 operator with every product summed in ANOTHER fixed order (oracle/spmv_omp.c
    oracle_csr_matvec_f32_order: row entries forward or backward over `ways` round-robin
    accumulators combined by a pairwise tree -- the shape of a lane-parallel GPU row sum).  Each is
    a correct fp32 implementation of the same products; the spread of the solves over such orders
    is the fp32 oracle's own rounding envelope."""
    dtype = np.float32

    def __init__(self, PM, ways, rev):
        self.PM, self.ways, self.rev = PM, ways, rev
        self.shape = PM.shape

    def __matmul__(self, v):
        return self.PM.matvec_f32_order(v, self.ways, self.rev)

    @property
    def T(self):
        return _Ordered32(self.PM.T, self.ways, self.rev)

    @property
    def val(self):
        return self.PM.val


# the alternative orders of dump_c5: SpMV rows (accumulators, reversed) and the fp32 sums of
# squares (chunk, reversed; restatement.fsum32_order) -- the device sums both in other orders.
# The chunks keep the sums as accurate as the documented order's (<= 4,096 values in the last,
# sequential level at n = 16.7M, as chunk 64 has): 64, 128, 256 and 512, forwards and reversed.
C5_ORDERS = ((1, 1, 128, 1), (2, 0, 256, 0), (4, 1, 512, 1), (8, 0, 64, 1), (16, 1, 128, 0), (32, 0, 256, 1),
             (64, 1, 512, 0), (128, 0, 64, 0))


def csr_hash32(M):
    """sha256 of the fp32 operator: indptr (int64), indices (int32), data (float32)."""
    h = hashlib.sha256()
    for a, dt in ((M.indptr, np.int64), (M.indices, np.int32), (M.data, np.float32)):
        a = np.ascontiguousarray(a, dtype=dt).reshape(-1)
        for i in range(0, a.size, 1 << 24):
            h.update(memoryview(a[i:i + (1 << 24)]))
    return h.hexdigest()


def dump_c5(name="c5_4096.npz", k=20, stride=197):
    """BASELINE configs[4] at full size: lsqr_solver / lsmr_solver on the 4096^2 / 47-angle operator
    in fp32 (the restatement's lsqr_solver_f32 / lsmr_solver_f32: float32 operator, vectors and
    fixed-order sums), all 20 iterations of the bench, with the fixture's b (c4_4096.npz, the
    fp64 operator's A x_true + 1 % noise).  Plus the oracle's OWN fp32 rounding spread: the same
    solves with every SpMV and every fp32 sum of squares summed in each of the 8 other orders of
    C5_ORDERS (_Ordered32, restatement.fsum32_order); per history entry the largest relative
    deviation from the documented-order run, and for x the largest normwise deviation over the
    samples x[::stride].  The production test holds the device within 100 x
    that spread at every iteration (VERDICT r5 "Next" #2).  The fp32 operator is pinned by the
    sha256 of (indptr, indices, float32 data) in reference pixel order.  ~40 GB, ~40 min on 8 cores."""
    import gc
    import time
    import scipy.sparse as sp
    from oracle import parallel as OP
    from hgmres.problems import siddon_projector, shepp_logan
    g = np.load(os.path.join(OUT, "c4_4096.npz"))
    b = np.ascontiguousarray(g["b"])
    A = siddon_projector(4096, 47)
    h64 = csr_hash(A)
    assert h64 == str(g["A_sha256"]), "generator drifted from the C4 fixture's operator"
    A32 = sp.csr_matrix((A.data.astype(np.float32), A.indices, A.indptr), shape=A.shape)
    del A
    gc.collect()
    h32 = csr_hash32(A32)
    xt = shepp_logan(4096).ravel(order="F")
    OP.build()
    PA = OP.ParallelCSR(A32)
    del A32
    gc.collect()
    PA.T                                           # formed once, shared by every run
    d = {"maxit": k, "N": 4096, "n_angles": 47, "A_sha256": h64, "A32_sha256": h32, "sample_stride": stride,
         "orders": np.array(C5_ORDERS)}
    for tag, fn, nh in (("lsqr", R.lsqr_solver_f32, 2), ("lsmr", R.lsmr_solver_f32, 3)):
        t0 = time.time()
        ref = fn(PA, b, xt, 0.0, k)
        print(f"{tag} fixed order: {time.time() - t0:.0f} s, res {ref[2][-1]:.6e}", flush=True)
        xs = ref[0][::stride].astype(np.float64)
        sx, sh = 0.0, [np.zeros(k) for _ in range(nh)]
        for ways, rev, ch, nrev in C5_ORDERS:
            t0 = time.time()
            with R.fsum32_order(ch, nrev):
                p = fn(_Ordered32(PA, ways, rev), b, xt, 0.0, k)
            ps = p[0][::stride].astype(np.float64)
            sx = max(sx, float(np.linalg.norm(ps - xs) / np.linalg.norm(xs)))
            for i in range(nh):
                sh[i] = np.maximum(sh[i], np.abs(p[1 + i] - ref[1 + i]) / np.abs(ref[1 + i]))
            print(f"  order {ways}/{rev}/{ch}/{nrev}: {time.time() - t0:.0f} s, spread x {sx:.2e} hist "
                  + " ".join(f"{float(np.max(s)):.1e}" for s in sh), flush=True)
        hn = ["err", "res", "ar"][:nh]
        d.update({f"{tag}_k": int(ref[-1]), f"{tag}_xs": ref[0][::stride].copy(), f"{tag}_xnorm":
                  float(np.linalg.norm(ref[0].astype(np.float64))), f"{tag}_spread_xs": sx})
        for i, nm in enumerate(hn):
            d[f"{tag}_{nm}"] = np.asarray(ref[1 + i], dtype=np.float64)
            d[f"{tag}_spread_{nm}"] = sh[i]
        np.savez_compressed(os.path.join(OUT, name), **d)     # partial file after LSQR
    print("wrote", name)


def dump_c2(name="c2_512.npz", k=20):
    """BASELINE configs[1] at full size and at the bench's count (bench.py WORKLOADS["c2"]):
    hybrid_ab_gmres_rtp (hybrid_ab_gmres_rtp.m:1-43), 512^2, 30 angles, nnz 1.0e7, lambda 1e-2,
    all 20 iterations (the reference re-forms A*Qk each iteration, :28-36: 210 host SpMVs).
    Inputs: b stored (the host's A*x_true + 1 % noise, numpy default_rng(0)); A and B = A' pinned
    by the sha256 of their CSR in reference pixel order.  Outputs: H (21 x 20), both histories,
    x as its norm plus every 97th entry."""
    from oracle import parallel as OP
    P = tomo_problem(512, 30, noise=1e-2, seed=0, backprojector="matched")
    A, B, b, xt = P.A, P.B, P.b, P.x_true
    OP.build()
    PA, PB = OP.ParallelCSR(A), OP.ParallelCSR(B)
    x, e, r, kk, H = R.hybrid_ab_gmres_rtp(PA, PB, b, xt, 0.0, k, 1e-2, return_H=True)
    st = 97
    d = {"maxit": k, "lam": 1e-2, "N": 512, "n_angles": 30, "A_sha256": csr_hash(A), "B_sha256": csr_hash(B),
         "b": b, "sample_stride": st, "hab_H": H, "hab_err": e, "hab_res": r, "hab_k": kk,
         "hab_xnorm": np.linalg.norm(x), "hab_xs": x[::st].copy()}
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name, "k", kk, "res", r[-1], "err", e[-1])


def dump_c4u(name="c4u_2048.npz", k=20):
    """The C4 unmatched line's path (bench.py --unmatched: ABgmres_nonhybrid_bounds with the
    pixel-driven back-projector B != A', run_2D_phantom.m:13-15 / analyze_regularization.m B_pert)
    at a quarter of C4's pixels with C4's 47 angles, so the device kernels are the ones C4 takes
    (column-banded A, the paged streaming B kernel for its 94-entry rows over an L2-resident x):
    2048^2, nnz(A) 2.5e8, nnz(B) 3.9e8, 20 iterations.  Operators pinned by CSR hash; b stored;
    x as its norm plus every 997th entry."""
    import gc
    from oracle import parallel as OP
    from hgmres.problems import pixel_driven_backprojector, shepp_logan, siddon_projector
    A = siddon_projector(2048, 47)
    hA = csr_hash(A)
    xt = shepp_logan(2048).ravel(order="F")
    OP.build()
    PA = OP.ParallelCSR(A)
    del A
    gc.collect()
    b_exact = PA @ xt
    e = np.random.default_rng(0).standard_normal(PA.shape[0])
    b = b_exact + e / np.linalg.norm(e) * 1e-2 * np.linalg.norm(b_exact)
    B = pixel_driven_backprojector(2048, 47)
    hB = csr_hash(B)
    PB = OP.ParallelCSR(B)
    del B
    gc.collect()
    x, err, res, kk, H = R.ABgmres_nonhybrid_bounds(PA, PB, b, xt, 0.0, k, return_H=True)
    d = {"maxit": k, "N": 2048, "n_angles": 47, "A_sha256": hA, "B_sha256": hB, "b": b, "sample_stride": 997,
         "abn_H": H, "abn_err": err, "abn_res": res, "abn_k": kk, "abn_xnorm": np.linalg.norm(x),
         "abn_xs": x[::997].copy()}
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name, "k", kk, "res", res[-1], "err", err[-1])


def dump_shaw_pipeline(name="shaw32_pipeline.npz"):
    """analyze_regularization.m on shaw(32) (restated, hgmres.regtools) with numpy noise and
    mismatch (MATLAB's randn stream cannot be reproduced): inputs, the oracle's outputs in the
    default (LAPACK/BLAS) order with dense operands as the reference has them, and the same
    pipeline in the fixed summation order.  Their difference is the pipeline's own rounding
    sensitivity (it is large: the 32-step Arnoldi on shaw(32) runs far past the numerical rank),
    stored as `spread_<key>` (normwise: max|default - fixed| / max|fixed|) for the production-path
    test's envelope."""
    import warnings
    import scipy.sparse as sp
    from hgmres.analysis import regularization_problem
    from oracle import pipeline
    P = regularization_problem(32)
    d = {"A": P.A, "b": P.b, "b_exact": P.b_exact, "x_true": P.x_true, "E": P.E}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        o = pipeline.analyze_regularization(P.A, P.b, P.x_true, P.B_pert, P.DeltaM_AB, P.DeltaM_BA)
        with R.fixed_order():
            f = pipeline.analyze_regularization(sp.csr_matrix(P.A), P.b, P.x_true, sp.csr_matrix(P.B_pert),
                                                P.DeltaM_AB, P.DeltaM_BA, bounds_outputs=False, explicit_BA=False)
    for k, v in o.items():
        d[f"out_{k}"] = np.asarray(v)
    for k, v in f.items():
        a, b = np.asarray(o[k], dtype=np.float64), np.asarray(v, dtype=np.float64)
        d[f"spread_{k}"] = np.max(np.abs(a - b), initial=0.0) / max(np.max(np.abs(b), initial=0.0), 1e-300)
    np.savez_compressed(os.path.join(OUT, name), **d)
    print("wrote", name, {k: float(np.max(v)) for k, v in d.items() if k.startswith("spread_")})


if __name__ == "__main__":
    if sys.argv[1:] == ["c3"]:
        dump_c3()
        sys.exit(0)
    if sys.argv[1:] == ["c2"]:
        dump_c2()
        sys.exit(0)
    if sys.argv[1:] == ["c4u"]:
        dump_c4u()
        sys.exit(0)
    if sys.argv[1:] == ["c4"]:
        dump_c4()
        sys.exit(0)
    if sys.argv[1:] == ["c5"]:
        dump_c5()
        sys.exit(0)
    if sys.argv[1:] == ["shaw"]:
        dump_shaw_pipeline()
        sys.exit(0)
    # matched back-projector B = A^T (run_equivalence_plots.m:5 style), 24^2 phantom, 12 angles
    dump("tomo24_matched.npz", tomo_problem(24, 12, noise=1e-2, seed=0, backprojector="matched"), maxit=12, lam=1e-2)
    # unmatched pixel-driven back-projector (the reference's B != A^T setting)
    dump("tomo24_pixel.npz", tomo_problem(24, 12, noise=1e-2, seed=1, backprojector="pixel"), maxit=12, lam=1e-2)
    # C1 geometry (64^2, 90 angles): operator regenerated from the generator, pinned by hash
    dump("tomo64_c1.npz", tomo_problem(64, 90, noise=1e-2, seed=0, backprojector="matched"), maxit=20, lam=1e-2,
         store_raw=False)
