"""Which fp32 production formulation leaves the fp32 oracle's rounding envelope at 4096^2?
Runs lsqr_solver / lsmr_solver (20 iterations, configs[4] operator, tiled order) under option
sets and prints, per iteration, the deviation from tests/golden/c5_4096.npz over its bar
max(1e-5, 100 x the oracle's spread over 8 SpMV summation orders).
usage: python scripts/c5_envelope_probe.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT, os.path.join(ROOT, "tests")]
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402
from hgmres.problems import shepp_logan  # noqa: E402
from conftest import load_golden  # noqa: E402

VARIANTS = {"default": {}, "host_scalars": dict(lsqr_dev=0), "two_pass": dict(fused_ab=0),
            "two_pass_host": dict(fused_ab=0, lsqr_dev=0), "no_res_img": dict(lsqr_res_img=0)}


def main():
    g5 = load_golden("c5_4096.npz")
    b = load_golden("c4_4096.npz")["b"]
    xt = shepp_logan(4096).ravel(order="F")
    st = int(g5["sample_stride"])
    ctx = hgmres.Context(0)
    A = hgmres.SparseOperator.siddon(4096, 47, ctx=ctx, dtype=L.HGM_F32)
    At = A.T
    for name, nh in (("lsqr", 2), ("lsmr", 3)):
        fn = hgmres.lsqr_solver if name == "lsqr" else hgmres.lsmr_solver
        for vn, opts in VARIANTS.items():
            if vn == "no_res_img" and name == "lsmr":
                continue
            with ctx.options(**opts):
                out = fn(A, b, xt, 0.0, 20, ctx=ctx, At=At)
            rec = {"solver": name, "variant": vn, "path": ctx.solve_path()["one_pass"]}
            for i, nm in enumerate(["err", "res", "ar"][:nh]):
                ref, spr = g5[f"{name}_{nm}"], g5[f"{name}_spread_{nm}"]
                d = np.abs(np.asarray(out[1 + i]) - ref) / np.abs(ref)
                rec[f"{nm}_dev"] = [float(f"{v:.2e}") for v in d]
                rec[f"{nm}_ratio"] = [round(float(v), 2) for v in d / np.maximum(1e-5, 100 * spr)]
            xs = g5[f"{name}_xs"].astype(np.float64)
            rec["x_dev"] = float(np.linalg.norm(out[0][::st] - xs) / np.linalg.norm(xs))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
