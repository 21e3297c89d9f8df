"""Per-rank cost of the AB step of the pixel-sharded C4 solve (bench.py --gpus N), measured on one
GPU: rank 0's shard for world = 1, 2, 4, 8 built exactly as bench.py builds it (build_shard), and
its local A_g*(B_g*q) timed two-pass and one-pass (hgm_spmv_ab; fused.hip on a shard of whole tile
columns).  The all-reduce of the m-vector that follows on a real communicator is not included.
usage: python scripts/shard_fused.py [reps] [worlds, e.g. 1,2,4,8] [extra fused region sides, e.g. 32,48]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    worlds = [int(w) for w in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
    ctx = hgmres.Context(0)
    lib = L.load()
    dev = torch.device("cuda", 0)
    P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    for world in worlds:
        A_g, B_g, _, _, (lo, hi), _ = bench.build_shard(ctx, bench.WORKLOADS["c4"], 0, world)
        m, n = A_g.shape
        q = torch.from_numpy(np.random.default_rng(0).standard_normal(m)).to(dev)
        bq = torch.empty(n, dtype=torch.float64, device=dev)
        abq = torch.empty(m, dtype=torch.float64, device=dev)
        out = {"world": world, "shard": [lo, hi], "nnz": A_g.nnz}
        res = {}
        regions = [int(r) for r in sys.argv[3].split(",")] if len(sys.argv) > 3 else []
        runs = [("two", dict(fused_ab=0)), ("fused", dict(fused_ab=1)), ("two_b", dict(fused_ab=0)),
                ("fused_b", dict(fused_ab=1))] + [(f"fused_r{r}", dict(fused_ab=1, fused_region=r)) for r in regions]
        for name, o in runs:
            with ctx.options(**o):
                assert lib.hgm_spmv_ab(ctx.handle, A_g._h, B_g._h, P(q), P(bq), P(abq)) == 0   # plan / warm-up
                ctx.synchronize()
                t0 = time.perf_counter()
                for _ in range(reps):
                    lib.hgm_spmv_ab(ctx.handle, A_g._h, B_g._h, P(q), P(bq), P(abq))
                ctx.synchronize()
                out[name + "_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
            res[name] = (bq.cpu().numpy().copy(), abq.cpu().numpy().copy())
        out["rel_dev_ABq"] = float(np.linalg.norm(res["fused"][1] - res["two"][1]) / np.linalg.norm(res["two"][1]))
        out["rel_dev_Bq"] = float(np.linalg.norm(res["fused"][0] - res["two"][0]) / np.linalg.norm(res["two"][0]))
        out["fused_bitwise_repeat"] = bool(np.array_equal(res["fused"][1], res["fused_b"][1]))
        print(json.dumps(out), flush=True)
        A_g.close()
        B_g.close()


if __name__ == "__main__":
    main()
