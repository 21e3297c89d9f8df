"""Pages of x per 4096-entry chunk of the banded ray-major A (64-column strips of the 4 x 4-tiled
order), per projection angle: which chunks exceed the LDS page budget (256 pages fp64, 512 fp32)
and fall back to 32-bit gathers.  Host-only; N = 2048 with C4's 47 angles (a chunk's page count
depends on the strip width and the angle, not on N).  --dual: the dual strips (HGM_OPT_BAND_DUAL,
csrc/ops.hip BandKey): rays whose pixel-row span exceeds their pixel-column span are banded in
64-pixel-row strips (18.8 % -> 3.2 % of the fp64 chunks over 256 pages).
usage: python scripts/page_stats_angles.py [--dual]"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
from hgmres.problems import _siddon_chunk, geometry  # noqa: E402

CH, PAGE = 4096, 16


def main():
    dual = "--dual" in sys.argv
    N, na = 2048, 47
    bands = (8, 16, 24)                      # strips of 64 pixel columns (tile columns 16b..16b+15)
    p, theta, s = geometry(N, na)
    st_cols = 64 * N
    tot = {128: 0, 256: 0, 512: 0}
    tot_e = {128: 0, 256: 0, 512: 0}
    allc = 0
    for a in range(na):
        c, sn = math.cos(theta[a]), math.sin(theta[a])
        segs = {b: [] for b in bands}
        for r0 in range(0, p, 256):
            d = np.arange(r0, min(p, r0 + 256))
            cnt, col, _ = _siddon_chunk(N, np.full(d.size, c), np.full(d.size, sn), s[d])
            pc, pr = col // N, col % N
            stored = ((pc // 4) * (N // 4) + pr // 4) * 16 + (pc % 4) * 4 + pr % 4
            b = stored // st_cols
            if dual and col.size:
                rid = np.repeat(np.arange(d.size), cnt)
                span = []
                for v in (pr, pc):
                    hi_, lo_ = np.full(d.size, -1), np.full(d.size, 1 << 30)
                    np.maximum.at(hi_, rid, v)
                    np.minimum.at(lo_, rid, v)
                    span.append(hi_ - lo_)
                steep = span[0] > span[1]
                b = np.where(steep[rid], (stored % (4 * N)) // 256, b)
            for bb in bands:
                segs[bb].append(stored[b == bb])       # ray order, then along-ray order
        for bb in bands:
            e = np.concatenate(segs[bb])
            nch = e.size // CH
            if nch == 0:
                continue
            pg = (e[: nch * CH] // PAGE).reshape(nch, CH)
            sp_ = np.sort(pg, axis=1)
            npg = (sp_[:, 1:] != sp_[:, :-1]).sum(axis=1) + 1
            pg32 = np.sort((e[: nch * CH] // (2 * PAGE)).reshape(nch, CH), axis=1)
            npg32 = (pg32[:, 1:] != pg32[:, :-1]).sum(axis=1) + 1
            allc += nch
            for lim in tot:
                tot[lim] += int((npg > lim).sum())
                tot_e[lim] += int((npg32 > lim).sum())
            if bb == bands[1]:
                print(f"angle {a:2d} ({math.degrees(theta[a]):6.1f} deg): chunks {nch:4d} pages mean {npg.mean():6.1f} "
                      f"max {npg.max():5d}  >256: {(npg > 256).mean():5.2f}", flush=True)
    print("fp64 pages (16 values):", {f">{lim}": round(tot[lim] / allc, 4) for lim in tot}, "chunks", allc)
    print("fp32 pages (32 values):", {f">{lim}": round(tot_e[lim] / allc, 4) for lim in tot_e})


if __name__ == "__main__":
    main()
