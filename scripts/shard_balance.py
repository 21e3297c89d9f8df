"""Per-shard cost of the one-pass A_g*(B_g*q) across ALL ranks of a C4 cut (the step time of a
sharded solve is the slowest rank's): for world W, every rank's shard as bench.py build_shard
cuts it (or an explicit list of tile-column boundaries), its nnz, the one-pass plan's partial
slots, and the pass time (HIP events, kernel class 3 = k_fused_rw + k_fused_reduce).
usage: python scripts/shard_balance.py [world] [reps] [bounds as comma-separated stored positions, or -]
       [options name=value,... (hgm_ctx_set_option)] [ranks, e.g. 0,3]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import hgmres  # noqa: E402
from hgmres.dist import tile_column_shards  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    ctx = hgmres.Context(0)
    N, na = 4096, 47
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx)
    B = A.T
    Nn, tile, sup = A.pixel_order("cols")
    for kv in (sys.argv[4].split(",") if len(sys.argv) > 4 and sys.argv[4] != "-" else []):
        k_, v_ = kv.split("=")
        ctx.set_option(k_, float(v_))
    only = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else None
    if len(sys.argv) > 3 and sys.argv[3] != "-":
        bnd = [int(v) for v in sys.argv[3].split(",")]
        cuts = list(zip(bnd[:-1], bnd[1:]))
    else:
        cuts = tile_column_shards(N, world, tile)
    q = np.random.default_rng(3).standard_normal(A.shape[0])
    rows = []
    for r, (lo, hi) in enumerate(cuts):
        if only is not None and r not in only:
            continue
        B_g = B.row_slice(lo, hi)
        A_g = B_g.T
        A_g.set_bands(64 * N, 0)
        info = hgmres.fused_plan_info(A_g, B_g)
        for _ in range(3):
            hgmres.spmv_ab(A_g, B_g, q)
        ctx.kernel_timing(True)
        for _ in range(reps):
            hgmres.spmv_ab(A_g, B_g, q)
        ms, calls, by = ctx.kernel_timing_read(3)
        ctx.kernel_timing(False)
        rec = {"opts": sys.argv[4] if len(sys.argv) > 4 else "-", "rank": r, "lo": lo, "hi": hi, "nnz": int(B_g.nnz), "nslot": int(info["nslot"]),
               "pass_us": round(ms / calls * 1e3, 2)}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
        A_g.close()
        B_g.close()
    t = [r_["pass_us"] for r_ in rows]
    print(json.dumps({"world": world, "max_us": max(t), "mean_us": round(float(np.mean(t)), 2),
                      "imbalance": round(max(t) / float(np.mean(t)), 4)}))


if __name__ == "__main__":
    main()
