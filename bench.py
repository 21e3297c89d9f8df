#!/usr/bin/env python3
"""Benchmark: GMRES iterations/s + SpMV GB/s (% HBM roofline) on a synthetic 2-D phantom.

Default workload = BASELINE.json configs[3], the configuration the metric's
"1/2/4/8 GPU" and north_star's ">= 60 % ... at nnz ~ 1e9" are quoted on, which fits
one MI355X:  AB-GMRES (ABgmres_nonhybrid_bounds.m, m-space Arnoldi on A*B), fp64,
4096x4096 Shepp-Logan phantom, parallel-beam Siddon A (47 angles, 5793 detectors:
m = 272,271 rays, n = 16,777,216 pixels, nnz(A) = 1.0e9), matched B = A', maxit = 20,
tol = 0 (all 20 iterations run).  One "step" = one complete 20-iteration solve.
Inputs (A, B, b, x_true) are resident in HBM before the timed region.
`--workload c2|c3|c3gcv|c5|c5m` runs the other BASELINE configs as side lines.

Multi-GPU (one process per GPU): under torch.distributed.run WORLD_SIZE must equal --gpus;
`python bench.py --gpus N` without a launcher spawns the N ranks itself (torch.distributed.run
as a child process, before any GPU call).  By default ONE global solve of the same
operator, pixel-sharded by nnz across the ranks: rank g holds
A(:,P_g) and B(P_g,:), and the only data-path collective is an RCCL all-reduce of
the m-vector partial A_g*(B_g*q) per Arnoldi step (strong scaling; value = GMRES
iterations of the global solve / max rank time).  `--replicas` instead runs one
independent solve per GPU (weak scaling, no collective).

Extra fields: "roofline" for the dominant SpMV kernel (algorithmic bytes per
launch / average launch duration from HIP events recorded on the library's
stream during the timed region), "kernels" (both SpMV classes and MGS),
"cpu_baseline" (the oracle restatement timed on the host cores, rank 0, N=1: the process's
OMP_NUM_THREADS share of the cores through oracle/spmv_omp.c -- 16 on the 1-GPU box -- plus a
one-core scipy leg; thread count, its reason, nproc and CPU model stated).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

# cpu_iters: iterations of the oracle timed for cpu_baseline (a bounded 10-30 s sample: the full maxit
# where the per-iteration cost grows with k, a few iterations where the SpMVs dominate)
WORKLOADS = {
    "c2": dict(N=512, angles=30, solver="hybrid_ab_gmres_rtp", maxit=20, lam=1e-2, cpu_iters=20),
    "c3": dict(N=2048, angles=19, solver="hybrid_ba_gmres_rtp", maxit=20, lam=1e-2, cpu_iters=20),
    # BASELINE configs[2]: GCV lambda selection (k_gcv Arnoldi steps once, fminbnd on the
    # cached H: analyze_regularization.m:39-46) + the BA-GMRES solve at the chosen lambda
    "c3gcv": dict(N=2048, angles=19, solver="hybrid_ba_gmres_rtp", maxit=20, lam=1e-2, cpu_iters=20,
                  gcv=dict(k=20, lo=1e-8, hi=1.0, tolx=1e-10)),
    "c4": dict(N=4096, angles=47, solver="ABgmres_nonhybrid_bounds", maxit=20, lam=0.0, cpu_iters=4,
               cpu_iters_single=1),
    # BASELINE configs[4]: the Golub-Kahan path on the 4096^2 operator in fp32
    "c5": dict(N=4096, angles=47, solver="lsqr_solver", maxit=20, lam=0.0, f32=True, cpu_iters=4,
               cpu_iters_single=1),
    "c5m": dict(N=4096, angles=47, solver="lsmr_solver", maxit=20, lam=0.0, f32=True, cpu_iters=4,
                cpu_iters_single=1),
}
UNITS = {"lsqr_solver": "LSQR iters/s", "lsmr_solver": "LSMR iters/s"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node, one rank each: under torch.distributed.run WORLD_SIZE must equal it; "
                         "without a launcher N > 1 spawns the N ranks itself")
    ap.add_argument("--dry-run", action="store_true",
                    help="print the planned world and every rank's pixel shard (JSON) without touching a GPU")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--orth", default="mgs", choices=["mgs", "cgs2"])
    ap.add_argument("--tune-a", default="", help="experiment: SpMV variant:group for A (default: auto)")
    ap.add_argument("--tune-b", default="", help="experiment: SpMV variant:group for B (default: auto)")
    ap.add_argument("--explicit-residual", action="store_true",
                    help="monitor norm(b - A*x) with an explicit SpMV (default: b - (A*Q) y)")
    ap.add_argument("--unmatched", action="store_true",
                    help="GMRES workloads: B = the unmatched pixel-driven back-projector instead of A'")
    ap.add_argument("--replicas", action="store_true",
                    help="N>1: one independent solve per GPU (weak scaling) instead of one pixel-sharded solve")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                    help="sharded-solve transport: RCCL, or the host all-reduce hook (single-device emulation)")
    ap.add_argument("--same-device", action="store_true", help="run every rank on GPU 0 (shard emulation)")
    ap.add_argument("--shard1", action="store_true",
                    help="N=1: the sharded code path on a one-rank RCCL communicator (transport rehearsal)")
    ap.add_argument("--shard-of", type=int, default=1, metavar="N",
                    help="with --shard1: solve rank 0's pixel shard of an N-way cut (per-rank kernel costs at "
                         "N GPUs, without the transport; the solve is then of that shard alone)")
    ap.add_argument("--shard-rank", type=int, default=0, metavar="R",
                    help="with --shard1 --shard-of N: solve rank R's shard instead of rank 0's (rank 0's shard of "
                         "an 8-way C4 cut is all background, x_true = 0 there, which sends the shard's own error "
                         "monitor to the x-forming reconstruction on the step stream: not the global solve's path)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="experiment: per-context numerics option (hgm_ctx_set_option), e.g. mgs_fused=0")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP-event timing")
    # default A: the roofline kernel; timing both classes costs ~11% of the C2 step, A alone ~4%
    ap.add_argument("--time-classes", default="A", choices=["A", "B", "AB", "MGS", "ALL"],
                    help="kernel classes timed with HIP events in the timed region (roofline: A)")
    ap.add_argument("--cpu-iters", type=int, default=0, help="oracle iterations of the all-core cpu_baseline leg "
                                                             "(0 = the workload's default)")
    ap.add_argument("--no-cpu-single", action="store_true", help="skip the one-core cpu_baseline leg")
    ap.add_argument("--time-every", type=int, default=4,
                    help="HIP-event timing on every Nth timed step (all its launches of the timed classes); "
                         "events ride in the dispatch packets and cost ~3%% of a C2 step when on every step")
    return ap.parse_args()


def build_problem(ctx, wl, seed):
    """A generated on the device (bit-identical to hgmres.problems.siddon_projector),
    B = A' by the device transpose, b = A x_true + noise."""
    import hgmres
    from hgmres import _lib as L
    from hgmres.problems import shepp_logan
    N, na = wl["N"], wl["angles"]
    A = hgmres.SparseOperator.siddon(N, na, ctx=ctx)
    x_true = shepp_logan(N).ravel(order="F")
    b_exact = A @ x_true                      # fp64 data even for the fp32 operator
    if wl.get("f32"):
        A.close()
        A = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=L.HGM_F32)
    B = A.T
    rng = np.random.default_rng(seed)
    e = rng.standard_normal(A.shape[0])
    e = e / np.linalg.norm(e) * 1e-2 * np.linalg.norm(b_exact)
    return A, B, b_exact + e, x_true


def build_shard(ctx, wl, rank, world):
    """Rank `rank`'s pixel shard of the device-generated operator: B_g = B(P_g,:) by a
    device row slice of B = A', A_g = A(:,P_g) as its device transpose.  The operator keeps
    its 4 x 4-tiled pixel storage and P_g is a contiguous range of STORED positions made of
    whole tile columns (hgm_mat_row_slice on tiled rows), so every shard keeps the tiled
    gather locality and the 64-column bands of the single-GPU kernels.  Parallel-beam nnz per
    pixel is uniform: equal pixel counts balance nnz to 0.02 % at 8 shards (512^2 check).
    x_true (and the returned x) are the shard's stored-order pixels; b (replicated) is formed
    from the full operator before it is released.  fp32 workloads (configs[4]): b from the fp64
    operator, as build_problem does, then the shards are cut from the fp32 operator and its
    fp32 transpose (the solve's dtype is the shards')."""
    import hgmres
    from hgmres import _lib as L
    from hgmres.core import stored_pixel_index
    from hgmres.problems import shepp_logan
    from hgmres.dist import tile_column_shards
    N, na = wl["N"], wl["angles"]
    Af = hgmres.SparseOperator.siddon(N, na, ctx=ctx)
    Nn, tile, sup = Af.pixel_order("cols")
    x_true = shepp_logan(N).ravel(order="F")
    b_exact = Af @ x_true
    rng = np.random.default_rng(0)                         # same noise on every rank
    e = rng.standard_normal(Af.shape[0])
    e = e / np.linalg.norm(e) * 1e-2 * np.linalg.norm(b_exact)
    if wl.get("f32"):
        Af.close()
        Af = hgmres.SparseOperator.siddon(N, na, ctx=ctx, dtype=L.HGM_F32)
    Bf = Af.T
    n = Af.shape[1]
    lo, hi = tile_column_shards(N, world, tile)[rank]     # whole tile columns of stored pixels
    B_g = Bf.row_slice(lo, hi)
    A_g = B_g.T
    if Nn and sup == 0 and A_g.shape[1] * 8 > 4 * 1024 * 1024:
        A_g.set_bands(64 * N, 0)                           # the tiled operators' 64-column strips
    xs = np.empty(n)
    xs[stored_pixel_index(N, tile, sup) if Nn else np.arange(n)] = x_true
    full = Af.shape
    Af.close()
    Bf.close()
    return A_g, B_g, b_exact + e, xs, (lo, hi), full


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`--gpus N` without a launcher: start N rank processes (torch.distributed.run, one per
    GPU, rendezvous on 127.0.0.1) as CHILDREN of this process, which has not touched the GPU,
    and return their exit code.  Rank 0 prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def wl_dtype(wl):
    """The arithmetic type of the workload's operator and vectors (the line's `dtype`)."""
    return "f32" if wl.get("f32") else "f64"


def plan(args, world):
    """What a rank will run: the workload, the world and every rank's pixel shard (stored
    positions, whole tile columns).  Host only."""
    from hgmres.core import auto_pixel_order
    from hgmres.dist import tile_column_shards
    wl = WORKLOADS[args.workload]
    N = wl["N"]
    shard = (world > 1 and not args.replicas) or args.shard1
    tile = auto_pixel_order(N)[0]
    return {"workload": args.workload, "solver": wl["solver"], "N": N, "angles": wl["angles"], "world": world,
            "dtype": wl_dtype(wl),
            "mode": "pixel-sharded" if shard else ("replicas" if world > 1 else "single GPU"),
            "shards": tile_column_shards(N, world, tile) if shard else [(0, N * N)] * world}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # one process per GPU: spawn the ranks before anything initialises the GPU (never exec)
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    if args.dry_run:
        # the launch plumbing without a GPU: every rank reports the shard it would hold
        p = plan(args, world)
        got = [None] * world
        if world > 1:
            dist.all_gather_object(got, {"rank": rank, "local_rank": local, "shard": p["shards"][rank]})
            dist.destroy_process_group()
        else:
            got = [{"rank": 0, "local_rank": local, "shard": p["shards"][0]}]
        if rank == 0:
            print(json.dumps({"dry_run": True, **p, "ranks": got}))
        return
    if args.same_device:
        local = 0                      # shard emulation: every rank on GPU 0
    torch.cuda.set_device(local)
    import ctypes as C
    import hgmres
    from hgmres import _lib as L
    from hgmres.core import _check

    wl = WORKLOADS[args.workload]
    shard = (world > 1 and not args.replicas) or args.shard1
    if shard:
        # one global problem, pixel-sharded: RCCL context (or the host
        # all-reduce hook for the single-device emulation)
        from hgmres.dist import host_allreduce_context, init_context
        if args.comm == "host":
            ctx = host_allreduce_context(local, rank, world)
        else:
            ctx = init_context(local, rank, world, one_rank_comm=args.shard1)
        cut = args.shard_of if args.shard1 else world
        if args.same_device and world > 1:
            # shard emulation on one GPU: the ranks build one after the other (each build holds the
            # full operator, its transpose and the sort scratch for a moment: ~50 GB at C4)
            for turn in range(world):
                if turn == rank:
                    A, B, b, x_true, (lo, hi), full = build_shard(ctx, wl, rank, cut)
                    torch.cuda.synchronize()
                dist.barrier()
        else:
            A, B, b, x_true, (lo, hi), full = build_shard(ctx, wl, args.shard_rank if args.shard1 else rank, cut)
    else:
        ctx = hgmres.Context(local)
        A, B, b, x_true = build_problem(ctx, wl, seed=rank)
        if args.unmatched and wl["solver"] not in UNITS:
            B.close()
            B = hgmres.SparseOperator.pixel_backprojector(wl["N"], wl["angles"], ctx=ctx, dtype=A.dtype)
        lo, hi, full = 0, A.shape[1], A.shape
    # the line's dtype is the operator's: a workload's fp32 must reach the shards / operator it solves
    got = "f32" if A.dtype == L.HGM_F32 else "f64"
    if got != wl_dtype(wl) or B.dtype != A.dtype:
        raise RuntimeError(f"bench.py: {args.workload} is {wl_dtype(wl)} but the operators are {got}/{B.dtype}")
    for o in args.opt:
        name, val = o.split("=", 1)
        ctx.set_option(name, float(val))
        if name == "band_dual":        # read when an operator is banded: re-band A
            A.set_bands(64 * wl["N"] if shard else -1)
    for M, t in ((A, args.tune_a), (B, args.tune_b)):
        if t:
            v, g = t.split(":")
            M.tune(int(v), int(g))
    m, n = A.shape
    dev = torch.device("cuda", local)
    b_d = torch.from_numpy(b).to(dev)
    xt_d = torch.from_numpy(np.ascontiguousarray(x_true[lo:hi])).to(dev)
    x_d = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    maxit, lam = wl["maxit"], wl["lam"]
    err = np.zeros(maxit)
    res = np.zeros(maxit)
    it = C.c_int(0)
    o = L.hgm_opts()
    o.flags = L.HGM_DEVICE_PTRS | (L.HGM_EXPLICIT_RESIDUAL if args.explicit_residual else 0)
    o.orth = L.HGM_CGS2 if args.orth == "cgs2" else L.HGM_MGS
    o.H_out = None
    lib = L.load()
    dptr = lambda t: C.cast(C.c_void_p(t.data_ptr()), L.dp)   # noqa: E731
    arh = np.zeros(maxit)                      # lsmr_solver's ar_hist
    ep, rp, aph = err.ctypes.data_as(L.dp), res.ctypes.data_as(L.dp), arh.ctypes.data_as(L.dp)

    gcv = wl.get("gcv")
    if gcv:
        kg = gcv["k"]
        Hg = np.zeros((kg + 1) * kg)
        beta_g, kdone, lam_c, g_c = C.c_double(), C.c_int(), C.c_double(), C.c_double()
        o_orth = L.HGM_CGS2 if args.orth == "cgs2" else L.HGM_MGS
    chosen = {}

    # the solver call's pointer arguments, formed once (the timed loop measures the solves, not
    # ctypes argument conversion)
    pb, pxt, px, po_, pit = dptr(b_d), dptr(xt_d), dptr(x_d), C.byref(o), C.byref(it)

    def step():
        nonlocal lam
        if gcv:
            _check(lib.hgm_arnoldi(ctx.handle, A._h, B._h, b.ctypes.data_as(L.dp), kg, L.HGM_SIDE_BA, 1e-12, o_orth,
                                   Hg.ctypes.data_as(L.dp), C.byref(beta_g), C.byref(kdone)), ctx)
            # k = size(H,2) = k_gcv (gcv_function.m:33): the columns past a breakdown are zero.
            # trace term n (gcv_function.m:46-50, 'ba'): the GLOBAL pixel count, not the shard's
            rc = lib.hgm_gcv_fminbnd(Hg.ctypes.data_as(L.dp), kg, beta_g.value, float(full[1]), gcv["lo"],
                                     gcv["hi"], gcv["tolx"], C.byref(lam_c), C.byref(g_c))
            if rc != 0:
                raise RuntimeError(f"hgm_gcv_fminbnd failed ({rc})")
            lam = lam_c.value
            chosen.update(lam=lam, gcv=g_c.value, k_gcv=kdone.value)
        if wl["solver"] == "hybrid_ab_gmres_rtp":
            rc = lib.hgm_hybrid_ab_gmres_rtp_ex(ctx.handle, po_, A._h, B._h, pb, pxt, 0.0, maxit, lam, px, ep, rp,
                                                pit)
        elif wl["solver"] == "hybrid_ba_gmres_rtp":
            rc = lib.hgm_hybrid_ba_gmres_rtp_ex(ctx.handle, po_, A._h, B._h, pb, pxt, 0.0, maxit, lam, px, ep, rp,
                                                pit)
        elif wl["solver"] == "lsqr_solver":        # B = A' is the transpose operand At
            rc = lib.hgm_lsqr_solver_ex(ctx.handle, po_, A._h, B._h, pb, pxt, 0.0, maxit, px, ep, rp, pit)
        elif wl["solver"] == "lsmr_solver":
            rc = lib.hgm_lsmr_solver_ex(ctx.handle, po_, A._h, B._h, pb, pxt, 0.0, maxit, px, ep, rp, aph, pit)
        else:
            rc = lib.hgm_gmres_bounds_ex(ctx.handle, po_, A._h, B._h, pb, pxt, 0.0, maxit, lam, L.HGM_SIDE_AB, 0, px,
                                         ep, rp, pit)
        _check(rc, ctx)
        if it.value != maxit:
            raise RuntimeError(f"solver stopped at {it.value} != {maxit}")

    for _ in range(args.warmup):
        step()
    timing = not args.no_timing
    # HGM_TIMING_CLASSES: every timed launch carries HIP events, so time only what the line reports
    # (the one-pass A*(B*q) kernel of the AB solvers, class 3, is timed with A: it replaces A and B)
    mask = {"A": 0b1001, "B": 0b0010, "AB": 0b1011, "MGS": 0b0100, "ALL": 0b1111}[args.time_classes]
    ctx.kernel_timing(0x100 | mask if timing else 0)

    def barrier():
        if world > 1:
            dist.barrier()

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if timing:
            ctx.kernel_timing_pause(i % max(1, args.time_every) != 0)
        step()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    kern = {}
    names = {0: "spmv_A_raymajor", 1: "spmv_B_pixelmajor", 2: "mgs_pass_sweep", 3: "spmv_AB_fused"}
    if timing:
        for cls, nm in names.items():
            ms, calls, by = ctx.kernel_timing_read(cls)
            if calls:
                avg_s = ms / calls / 1e3
                kern[nm] = {"calls": calls, "avg_us": avg_s * 1e6, "bytes_per_launch": by / calls,
                            "GBps": by / calls / avg_s / 1e9, "total_ms": ms}
        ctx.kernel_timing(False)
    iters = args.steps * maxit * (1 if shard else world)   # sharded: one global solve
    value = iters / dt
    roof = None
    spmv = {k: v for k, v in kern.items() if k.startswith("spmv")}
    if spmv:
        dom_name = max(spmv, key=lambda k: spmv[k]["total_ms"])
        d = spmv[dom_name]
        traffic = None
        tf = os.path.join(ROOT, "profiles", f"traffic_{args.workload}{'_unmatched' if args.unmatched else ''}.json")
        # the committed PMC traffic is the single-GPU operator's: not a shard's
        if os.path.exists(tf) and not shard:
            try:
                traffic = json.load(open(tf)).get(dom_name)
            except Exception:   # noqa: BLE001
                traffic = None
        if dom_name == "spmv_AB_fused":
            # the one pass replaces the two SpMVs B*q and A*(B*q): their algorithmic bytes (SURVEY
            # §8(d)) over the same time give the effective rate of the pair it replaces (this
            # rank's operator: a shard's local shape with its own nnz)
            mm, nn, nz = A.shape[0], A.shape[1], A.nnz
            s = 4.0 if got == "f32" else 8.0
            two = (((s + 4) * nz + 8.0 * (nn + 1) + s * mm + s * nn) +
                   ((s + 4) * nz + 8.0 * (mm + 1) + s * nn + s * mm))
            if wl["solver"] in UNITS:
                two += s * nn      # the Golub-Kahan B product's epilogue read of v (A'*u - beta*v)
            d["two_pass_bytes"] = two
            d["effective_GBps_two_pass"] = two / (d["avg_us"] * 1e-6) / 1e9
        roof = {"bound": "hbm", "kernel": dom_name, "achieved": round(d["GBps"], 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(d["GBps"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_per_launch": d["bytes_per_launch"], "avg_launch_us": round(d["avg_us"], 2),
                "sample": f"{d['calls']} launches: HIP events on every {max(1, args.time_every)}th of the "
                          f"{args.steps} timed steps"}
        if traffic:
            # the counter-byte rate next to the nominal one (VERDICT r4 "Next" #4): the kernels that
            # read compressed indices (2-B slots, 16-bit page indices) move fewer bytes than the
            # nominal CSR count, so `frac` alone would overstate how close they are to HBM peak
            at = traffic / (d["avg_us"] * 1e-6) / 1e9
            roof.update(achieved_traffic=round(at, 1), frac_traffic=round(at / HBM_PEAK_GBS, 4),
                        traffic_ratio=round(traffic / d["bytes_per_launch"], 4),
                        traffic_source=f"profiles/{os.path.basename(tf)}: HBM bytes per launch of this kernel on "
                                       f"this workload, (2 x FETCH_SIZE + WRITE_SIZE) from separate rocprofv3 --pmc "
                                       f"passes (gfx950 wide-read correction), committed -- not counters of this "
                                       f"run; frac_traffic = traffic / avg_launch_us / peak")

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(A, B, b, x_true, wl, args.cpu_iters or wl["cpu_iters"],
                           0 if args.no_cpu_single else wl.get("cpu_iters_single", wl["cpu_iters"]))

    if rank == 0:
        line = {
            "metric": "GMRES iters/sec + SpMV GB/s (% HBM roofline), 2-D phantom A, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": UNITS.get(wl["solver"], "GMRES iters/s"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            # the default --gpus N series solves ONE global problem (pixel-sharded for N > 1):
            # total work is fixed, so the N = 1 line of that series is strong scaling too
            "scaling": "weak" if args.replicas else "strong",
            "vs_baseline": None,
            "dtype": got,
            "data": "synthetic (Siddon parallel-beam A generated on device, Shepp-Logan phantom, 1% noise"
                    + (", unmatched pixel-driven B" if args.unmatched and wl["solver"] not in UNITS else ", B = A'")
                    + ")",
            "config": {
                "workload": f"{args.workload}: {wl['solver']} {wl['N']}x{wl['N']} phantom, {wl['angles']} angles, "
                            f"m={full[0]}, n={full[1]}, nnz(A)={A.nnz if not shard else 'sharded'}, maxit={maxit}, "
                            f"tol=0, lambda={lam}, orth={args.orth}, "
                            f"residual={'explicit A*x' if args.explicit_residual else '(A*Q)*y'}",
                "global_batch": 1 if shard else world,
                "parallelism": (f"rank {args.shard_rank}'s shard of a {args.shard_of}-way pixel cut on a one-rank communicator "
                                f"(per-rank kernel costs; not a global solve)" if args.shard1 and args.shard_of > 1 else
                                f"pixel-sharded over {world} ranks ({args.comm} all-reduce of the m-vector)"
                                if shard else
                                "replicas: one independent slice per GPU" if world > 1 else "single GPU"),
                "step": (f"GCV lambda selection ({gcv['k']} Arnoldi steps + fminbnd on the cached H) and one "
                         f"complete {maxit}-iteration solve at that lambda" if gcv else
                         f"one complete {maxit}-iteration solve"),
            },
            "roofline": roof,
            "kernels": kern,
            "cpu_baseline": cpu,
            # last solve's monitors (identical across ranks / sharding up to rounding)
            "monitors": {"residual_norm_last": float(res[maxit - 1]), "error_norm_last": float(err[maxit - 1]),
                         **({"gcv_lambda": chosen["lam"], "gcv_value": chosen["gcv"], "k_gcv": chosen["k_gcv"]}
                            if chosen else {})},
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _host_cores():
    """CPUs this process may run on (the box's share, not the machine's count)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:   # pragma: no cover
        return os.cpu_count() or 1


def cpu_baseline(A, B, b, x_true, wl, iters, iters_single):
    """The oracle restatement (the reference algorithm) on the same operator, timed on the
    host: the process's OMP_NUM_THREADS cores (oracle/spmv_omp.c row-block SpMV, BLAS
    unrestricted; the products are bitwise those of the one-core scipy leg) and, if
    iters_single > 0, one core (scipy CSR SpMV, BLAS limited to one thread).  fp32 workloads run
    the fp32 restatement (lsqr_solver_f32 / lsmr_solver_f32: float32 operator and vectors, the
    GPU's arithmetic type).  The restatement's iteration clock (oracle/restatement.py
    iteration_clock) splits each timed solve into its setup (r0, norms: before the first
    iteration) and its iterations; `value` is iterations / iteration time, the setup is stated
    apart.  GMRES samples run the workload's full maxit where the per-iteration cost grows with k
    (the MGS sweep, hybrid_ab_gmres_rtp's A*Qk), a few iterations where the SpMVs dominate (C4's
    m-space basis is 2.2 MB a column)."""
    import scipy.sparse as sp
    from oracle import parallel as OP
    from oracle import restatement as R
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:   # pragma: no cover
        threadpool_limits = None
    import contextlib
    f32 = bool(wl.get("f32"))
    fn = getattr(R, wl["solver"] + ("_f32" if f32 else ""))
    gkb = wl["solver"] in UNITS
    gcv = wl.get("gcv")
    unit = UNITS.get(wl["solver"], "GMRES iters/s")
    As, Bs = A.to_scipy(), B.to_scipy()
    if f32:
        As = sp.csr_matrix((As.data.astype(np.float32), As.indices, As.indptr), shape=As.shape)
        Bs = sp.csr_matrix((Bs.data.astype(np.float32), Bs.indices, Bs.indptr), shape=Bs.shape)

    def run(Aop, Bop, k):
        """(iterations, setup s, iteration s) of one timed step of the workload on the oracle."""
        n = Aop.shape[1]
        t0 = time.perf_counter()
        with R.iteration_clock() as clk:
            lam = wl["lam"]
            if gcv:   # the c3gcv step: GCV on one Arnoldi, fminbnd, the solve at that lambda
                import scipy.optimize as so
                Hg, beta = R.arnoldi(Aop, Bop, b, gcv["k"], "ba")
                lam = float(so.fminbound(lambda l_: R.gcv_from_H(Hg, beta, l_, n), gcv["lo"], gcv["hi"],
                                         xtol=gcv["tolx"]))
            if gkb:   # the restatement applies A' itself (lsqr_solver.m:10); here B = A' (device transpose)
                args = (Aop, b, x_true, 0.0, k)
            else:
                args = (Aop, Bop, b, x_true, 0.0, k) + ((lam,) if wl["solver"] != "ABgmres_nonhybrid_bounds" else ())
            out = fn(*args)
            t1 = time.perf_counter()
            ticks = list(clk)
        kk = out[-1] if wl["solver"] == "lsmr_solver" else out[3]
        # (c3gcv: the setup is the GCV Arnoldi's r0; the solve's own setup counts as step work)
        return kk, ticks[0] - t0, t1 - ticks[0]

    OP.build()
    threads = OP.num_threads()
    PB = OP.ParallelCSR(Bs)
    PA = OP.ParallelCSR(As, T=PB if gkb else None)
    k_all, su, it_s = run(PA, PB, iters)
    what = (f"one c3gcv step (the {gcv['k']}-step GCV Arnoldi, fminbnd, and a {k_all}-iteration solve)" if gcv else
            f"a {k_all}-iteration solve" + (" (the workload's full maxit)" if k_all == wl["maxit"] else ""))
    res = {"value": round(k_all / it_s, 4), "unit": unit, "cores": threads, "kind": "port",
           "setup_s": round(su, 2), "iteration_s": round(it_s, 2),
           "nproc": _host_cores(), "cpu_model": _cpu_model(),
           "cores_reason": f"OpenMP threads = OMP_NUM_THREADS ({os.environ.get('OMP_NUM_THREADS', 'unset')}): the "
                           "host-core share of this process (the 1-GPU box grants 16 cores; nproc counts the whole "
                           "machine's CPUs, which other boxes' jobs use)",
           "sample": f"oracle/restatement.py {fn.__name__} on the same {wl['N']}^2 operator, {what}: setup "
                     f"{su:.1f} s (before the first iteration, not in value) + iterations {it_s:.1f} s; CSR SpMV on "
                     f"{threads} OpenMP threads (oracle/spmv_omp.c, bitwise = scipy), numpy BLAS unrestricted"}
    if iters_single > 0:
        with (threadpool_limits(limits=1) if threadpool_limits else contextlib.nullcontext()):
            k1, su1, it1 = run(As, Bs, iters_single)
        res["single_core"] = {"value": round(k1 / it1, 4), "unit": unit, "cores": 1, "setup_s": round(su1, 2),
                              "sample": f"same solver, {k1}-iteration solve: setup {su1:.1f} s apart, iterations "
                                        f"{it1:.1f} s; scipy CSR SpMV + numpy on 1 thread"}
    return res


if __name__ == "__main__":
    main()
