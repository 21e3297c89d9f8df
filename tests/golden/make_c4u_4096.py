"""Fixture tests/golden/c4u_4096.npz: the C4 unmatched line at full size.

bench.py --workload c4 --unmatched runs ABgmres_nonhybrid_bounds (ABgmres_nonhybrid_bounds.m:24-40)
on the 4096^2 / 47-angle Siddon A with the pixel-driven back-projector B != A'
(run_2D_phantom.m:13-15 / analyze_regularization.m B_pert).  The oracle is the CPU restatement
(oracle/restatement.py) on operators pinned by CSR hash:

* A = the device Siddon operator, downloaded; its hash must equal tests/golden/c4_4096.npz's, the
  numpy generator's (make_golden.py c4);
* B = the device pixel-driven back-projector, downloaded; its hash must equal the numpy generator's
  (hgmres.problems.pixel_driven_backprojector(4096, 47)), computed here first.

The host side needs ~100 GB at the peak (1.6e9-entry B in numpy, both operators downloaded), so it
runs on the GPU box, as test infrastructure (the device only generates and downloads the
operators):
    gpurun -- 'python tests/golden/make_c4u_4096.py gpurun_out/c4u_4096.npz'
then copy the file to tests/golden/.  A heartbeat line every 30 s keeps the run visibly alive."""
import gc
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT, os.path.join(ROOT, "tests", "golden")]
from make_golden import csr_hash  # noqa: E402


def main(out, k=20, N=4096, na=47):
    t0 = time.time()
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"  ... {time.time() - t0:.0f} s", flush=True)

    threading.Thread(target=beat, daemon=True).start()
    from hgmres.problems import pixel_driven_backprojector, shepp_logan
    Bn = pixel_driven_backprojector(N, na)
    hB_np = csr_hash(Bn)
    print(f"numpy B: nnz {Bn.nnz}, {time.time() - t0:.0f} s", flush=True)
    del Bn
    gc.collect()
    import torch  # noqa: F401  (the HIP runtime before libhgmres)
    import hgmres
    from oracle import parallel as OP
    from oracle import restatement as R
    ctx = hgmres.Context(0)
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx)
    As = A.to_scipy()
    A.close()
    hA = csr_hash(As)
    g4 = np.load(os.path.join(ROOT, "tests", "golden", "c4_4096.npz"))
    assert hA == str(g4["A_sha256"]), "device A != the numpy generator's"
    OP.build()
    PA = OP.ParallelCSR(As)
    del As
    gc.collect()
    B = hgmres.SparseOperator.pixel_backprojector(N, na, ctx=ctx)
    Bs = B.to_scipy()
    B.close()
    hB = csr_hash(Bs)
    assert hB == hB_np, "device B != the numpy generator's"
    PB = OP.ParallelCSR(Bs)
    del Bs
    gc.collect()
    print(f"operators pinned: {time.time() - t0:.0f} s", flush=True)
    xt = shepp_logan(N).ravel(order="F")
    b_exact = PA @ xt
    e = np.random.default_rng(0).standard_normal(PA.shape[0])
    b = b_exact + e / np.linalg.norm(e) * 1e-2 * np.linalg.norm(b_exact)
    x, err, res, kk, H = R.ABgmres_nonhybrid_bounds(PA, PB, b, xt, 0.0, k, return_H=True)
    st = 997
    np.savez_compressed(out, maxit=k, N=N, n_angles=na, A_sha256=hA, B_sha256=hB, b=b, sample_stride=st,
                        abn_H=H, abn_err=err, abn_res=res, abn_k=kk, abn_xnorm=np.linalg.norm(x),
                        abn_xs=x[::st].copy())
    stop.set()
    print(f"wrote {out}: k {kk} res {res[-1]:.6e} err {err[-1]:.6e}, {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "tests", "golden", "c4u_4096.npz"))
