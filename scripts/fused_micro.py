"""Micro-benchmark of the m-space operator A*(B*q) (hgm_spmv_ab) at a BASELINE geometry: the
one-pass kernel (fused.hip) against the two SpMVs, and phase-skip timing variants (fused_dbg:
results wrong, timing only).  Prints one JSON line per variant.  Run on the GPU box:
    python scripts/fused_micro.py [N angles reps [variants]]
HGM_MICRO_F32=1: the fp32 operator (BASELINE configs[4]; the fp32 one-pass kernel)."""
import ctypes as C
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402

N, na, reps = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (4096, 47, 20)))
variants = sys.argv[4].split(",") if len(sys.argv) > 4 else ["two", "f1024", "f512", "d1", "d2", "d4", "d8", "d15"]
ctx = hgmres.Context(0)
lib = L.load()
f32 = os.environ.get("HGM_MICRO_F32", "0") == "1"
A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=L.HGM_F32 if f32 else L.HGM_F64)
B = A.T
m, n = A.shape
dev = torch.device("cuda", 0)
tdt = torch.float32 if f32 else torch.float64
q = torch.from_numpy(np.random.default_rng(0).standard_normal(m)).to(dev).to(tdt)
bq = torch.empty(n, dtype=tdt, device=dev)
abq = torch.empty(m, dtype=tdt, device=dev)
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
s_ = 4.0 if f32 else 8.0
two = 2 * (s_ + 4) * A.nnz + 8.0 * (m + 1) + 8.0 * (n + 1) + 2 * s_ * (m + n)
ref = None
for vname in variants:
    # two | f<threads>[x<depth>][r<region>] (fused, pipeline depth [2], region side [64])
    # | d<bits> (phase-skip timing)
    mf = re.fullmatch(r"f(\d+)(?:x(\d))?(?:r(\d+))?", vname)
    # row-wave pass: waves, region, rows per batch, ring depth, pairs
    mw = re.fullmatch(r"w(\d)r(\d+)(?:g(\d+))?(?:d(\d))?(?:p(\d))?(?:a(\d))?(?:q(\d))?", vname)
    if vname.startswith("e"):                                   # row-wave pass, phase-skip timing
        o = dict(fused_ab=1, fused_kind=1, fused_dbg=int(vname[1:]), fused_acc32=1)
    elif mw:
        o = dict(fused_ab=1, fused_kind=1, fused_waves=int(mw.group(1)), fused_wregion=int(mw.group(2)),
                 fused_group=int(mw.group(3) or 8), fused_depth=int(mw.group(4) or 2),
                 fused_pairs=int(mw.group(5) or 1), fused_acc32=int(mw.group(6) or 1),
                 fused_rowpair=int(mw.group(7) or 0))
    elif vname == "two":
        o = dict(fused_ab=0)
    elif mf:
        o = dict(fused_ab=1, fused_kind=0, fused_bs=int(mf.group(1)), fused_pf=int(mf.group(2) or 2),
                 fused_region=int(mf.group(3) or 64))
    else:
        o = dict(fused_ab=1, fused_kind=0, fused_dbg=int(vname[1:]))
    with ctx.options(**o):
        lib.hgm_spmv_ab(ctx.handle, A._h, B._h, P(q), P(bq), P(abq))      # plan / warm-up
        ctx.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            rc = lib.hgm_spmv_ab(ctx.handle, A._h, B._h, P(q), P(bq), P(abq))
        ctx.synchronize()
        dt = (time.perf_counter() - t0) / reps
    assert rc == 0
    out = abq.cpu().numpy()
    if vname == "two":
        ref = (bq.cpu().numpy(), out)
    dev_ = None if ref is None else float(np.linalg.norm(out - ref[1]) / np.linalg.norm(ref[1]))
    devz = None if ref is None else float(np.linalg.norm(bq.cpu().numpy() - ref[0]) / np.linalg.norm(ref[0]))
    print(json.dumps({"variant": vname, "N": N, "angles": na, "dtype": "f32" if f32 else "f64", "ms": round(dt * 1e3, 4),
                      "effective_GBps_two_pass": round(two / dt / 1e9, 1), "rel_dev_vs_two_pass": dev_, "bq_rel_dev": devz}), flush=True)
