# LDS bank-load model of the row-wave pass: for sampled 32 x 32 regions of a
# 256^2, 47-angle operator (the C4 geometry at a smaller N), the worst per-bank count of distinct dword
# addresses per q-read instruction (pairs layout, one row, dummy lanes) under several slot numberings.
import sys, numpy as np
sys.path[:0] = ['hybrid-gmres_amd']
from hgmres.problems import tomo_problem
N, na, R = 256, 47, 32
P = tomo_problem(N, na, noise=0, seed=0)
B = P.A.T.tocsr()            # rows = pixels (column-major pixel index), cols = rays
MAXR = 2048
rng = np.random.default_rng(0)

def region_of(p):
    x, y = p // N, p % N      # column-major: p = x*N + y
    return (x // R) * (N // R) + (y // R)

pix = np.arange(N * N)
reg = np.array([region_of(p) for p in pix])
def cycles(slots):
    # slots: lane -> 8-byte slot index; dword banks 2s, 2s+1 mod 64; distinct addresses per bank
    banks = {}
    for s in slots:
        for d in (2 * s, 2 * s + 1):
            banks.setdefault(d % 64, set()).add(d)
    return max(len(v) for v in banks.values())

def simulate(perm_fn, nreg=24):
    tot = 0; cnt = 0
    for g in rng.choice(reg.max() + 1, nreg, replace=False):
        rows = np.nonzero(reg == g)[0]
        rays = np.unique(np.concatenate([B.indices[B.indptr[r]:B.indptr[r + 1]] for r in rows]))
        nr = len(rays)
        rank = {r: i for i, r in enumerate(rays)}
        perm = perm_fn(nr)
        for r in rows:
            ent = np.sort(B.indices[B.indptr[r]:B.indptr[r + 1]])
            off = rng.integers(0, 2)
            L = len(ent)
            for e in (0, 1):
                slots = []
                for ln in range(64):
                    pos = 2 * ln - off + e
                    if 0 <= pos < L:
                        slots.append(perm[rank[ent[pos]]])
                    else:
                        slots.append(MAXR - 64 + ln)
                tot += cycles(slots); cnt += 1
    return tot / cnt

ident = lambda nr: np.arange(nr)
def xor_sw(nr):
    s = np.arange(nr)
    out = s ^ ((s >> 5) & 31)
    return out if len(np.unique(out)) == nr and out.max() < MAXR - 64 else s
def rnd(nr):
    return np.random.default_rng(1).permutation(nr)
def mul(c):
    def f(nr):
        return (np.arange(nr) * c) % nr if np.gcd(c, nr) == 1 else np.arange(nr)
    return f
for name, f in [("rank", ident), ("xor", xor_sw), ("random", rnd), ("mul17", mul(17)), ("mul33", mul(33)), ("mul41", mul(41))]:
    print(name, round(simulate(f), 3), flush=True)
# dummies: one shared slot (broadcast) instead of per lane
def simulate2(perm_fn, nreg=24, shared=True):
    tot = 0; cnt = 0
    rng2 = np.random.default_rng(0)
    for g in rng2.choice(reg.max() + 1, nreg, replace=False):
        rows = np.nonzero(reg == g)[0]
        rays = np.unique(np.concatenate([B.indices[B.indptr[r]:B.indptr[r + 1]] for r in rows]))
        rank = {r: i for i, r in enumerate(rays)}
        perm = perm_fn(len(rays))
        for r in rows:
            ent = np.sort(B.indices[B.indptr[r]:B.indptr[r + 1]])
            off = rng2.integers(0, 2)
            L = len(ent)
            for e in (0, 1):
                slots = []
                for ln in range(64):
                    pos = 2 * ln - off + e
                    if 0 <= pos < L: slots.append(perm[rank[ent[pos]]])
                    elif shared: slots.append(MAXR - 64)
                tot += cycles(slots) if slots else 1; cnt += 1
    return tot / cnt
print("rank shared-dummy", round(simulate2(ident), 3))
print("rank no-dummy-lanes(exec)", round(simulate2(ident, shared=False), 3))
