"""Worker for the multi-rank tests: test_gpu_parity.py::test_shard_emulation_two_ranks,
test_gpu_fullsize.py::test_c4_c5_sharded_vs_oracle (world 2, 4, 8) and, through solve_all,
test_gpu_rccl.py's one-rank RCCL run.

Runs the pixel-sharded solvers as ``world`` processes on ONE device with the
cross-rank sums routed through the library's host all-reduce hook (a fixed-order
sum over local sockets: rank 0 adds the ranks' arrays in rank order and sends the
sum back), i.e. the same C++ code path as RCCL mode with a different transport.
usage: _shard_worker.py RANK WORLD PORT OUTDIR [c4]
"""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]

import hgmres  # noqa: E402
from hgmres.dist import plan_pixel_shards, shard_operators  # noqa: E402
from hgmres.problems import tomo_problem  # noqa: E402


class Hub:
    """Fixed-order all-reduce of ``world`` processes over local sockets.  Rank 0 listens and
    accepts the other ranks (each announces its rank); a sum is ((r0 + r1) + r2) + ... in rank
    order, formed on rank 0 and sent back to every rank, so every rank gets the same bits (as
    RCCL's all-reduce gives every rank the same result)."""

    def __init__(self, rank, world, port):
        from multiprocessing.connection import Client, Listener
        self.rank, self.world, self.conns = rank, world, {}
        if world == 1:
            return
        if rank == 0:
            lst = Listener(("127.0.0.1", port), authkey=b"hgm", backlog=world)
            lst._listener._socket.settimeout(240.0)      # (a rank that never starts fails the test)
            for _ in range(world - 1):
                c = lst.accept()
                self.conns[int(c.recv())] = c
            print(f"[hub] rank 0 connected to {sorted(self.conns)}", flush=True)
            lst.close()
        else:
            c = None
            for _ in range(1200):
                try:
                    c = Client(("127.0.0.1", port), authkey=b"hgm")
                    break
                except (ConnectionRefusedError, OSError):
                    time.sleep(0.1)
            assert c is not None, "no hub"
            c.send(rank)
            self.conns[0] = c

    def allreduce(self, arr):
        if self.world == 1:
            return
        if self.rank == 0:
            s = np.array(arr, dtype=arr.dtype, copy=True)
            for r in range(1, self.world):
                other = self._recv(r)
                if other.shape != s.shape:    # a collective-sequence mismatch between ranks: fail loudly
                    raise RuntimeError(f"rank {r} sent {other.shape} while rank 0 reduces {s.shape}")
                s = s + other
            for r in range(1, self.world):
                self.conns[r].send(s)
            arr[:] = s
        else:
            self.conns[0].send(np.array(arr, copy=True))
            arr[:] = self._recv(0)

    def _recv(self, r, timeout=240.0):
        # (a rank that died or stalls fails the collective instead of blocking the others forever)
        if not self.conns[r].poll(timeout):
            raise TimeoutError(f"rank {self.rank}: nothing from rank {r} for {timeout:.0f} s")
        return self.conns[r].recv()

    def barrier(self):
        self.allreduce(np.zeros(1))

    def close(self):
        for c in self.conns.values():
            c.close()


def run_rank(rank, world, port, out, mode):
    """One rank: its own context on device 0, the hub, the solves, rank{r}_of{world}.npz."""
    ctx = hgmres.Context(0)
    hub = Hub(rank, world, port)
    try:
        if world > 1:
            ctx.set_host_allreduce(rank, world, hub.allreduce)
        res = solve_c4(ctx, rank, world, hub) if mode == "c4" else solve_all(ctx, rank, world)
        np.savez(os.path.join(out, f"rank{rank}_of{world}.npz"), **res)
    finally:
        hub.close()
        ctx.close()


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    # a stuck rank reports where it is (every 60 s) and exits after 5 minutes instead of hanging
    # the test run (a world-8 C4/C5 run takes ~1 minute): the parent kills the others and fails
    import faulthandler
    faulthandler.dump_traceback_later(60, repeat=True)
    watchdog = threading.Timer(300.0, lambda: os._exit(3))
    watchdog.daemon = True
    watchdog.start()
    run_rank(rank, world, port, out, sys.argv[5] if len(sys.argv) > 5 else "all")


def _abn_device(ctx, A_g, B_g, b, xt, maxit):
    import ctypes as C
    import torch
    from hgmres import _lib as L
    from hgmres.core import _ops
    ctx_, Ao, Bo = _ops(A_g, B_g, ctx)
    dev = torch.device("cuda", 0)
    b_d = torch.from_numpy(np.ascontiguousarray(b, dtype=np.float64)).to(dev)
    xt_d = torch.from_numpy(np.ascontiguousarray(xt, dtype=np.float64)).to(dev)
    x_d = torch.zeros(Ao.shape[1], dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    err, res = np.zeros(maxit), np.zeros(maxit)
    it = C.c_int(0)
    o = L.hgm_opts()
    o.flags = L.HGM_DEVICE_PTRS
    o.orth = L.HGM_MGS
    o.H_out = None
    dp = lambda t: C.cast(C.c_void_p(t.data_ptr()), L.dp)   # noqa: E731
    rc = L.load().hgm_gmres_bounds_ex(ctx_.handle, C.byref(o), Ao._h, Bo._h, dp(b_d), dp(xt_d), 0.0, maxit, 0.0,
                                      L.HGM_SIDE_AB, 0, dp(x_d), err.ctypes.data_as(L.dp), res.ctypes.data_as(L.dp),
                                      C.byref(it))
    assert rc == 0, rc
    k = it.value
    return dict(abnd_x=x_d.cpu().numpy(), abnd_err=err[:k].copy(), abnd_res=res[:k].copy())


def solve_all(ctx, rank, world):
    """Every sharded solve of the test on rank `rank`'s shard; returns the arrays by tag."""
    P = tomo_problem(64, 90, noise=1e-2, seed=0)
    lo, hi = plan_pixel_shards(P.A, world, P.B)[rank]
    A_g, B_g = shard_operators(P.A, P.B, lo, hi)
    xt = P.x_true[lo:hi]
    res = {}
    x, e, r, k, H = hgmres.hybrid_ba_gmres_rtp(A_g, B_g, P.b, xt, 0.0, 15, 1e-2, ctx=ctx, return_H=True)
    res.update(hba_x=x, hba_res=r, hba_err=e, hba_H=H)
    x, e, r, k = hgmres.lsqr_solver(A_g, P.b, xt, 0.0, 10, ctx=ctx, At=B_g)
    res.update(lsqr_x=x, lsqr_res=r, lsqr_err=e)
    out_ = hgmres.ABgmres_hybrid_bounds(A_g, B_g, P.b, xt, 0.0, 12, 1e-2, ctx=ctx)
    res.update(abp_x=out_[0], abp_res=out_[2], abp_err=out_[1])
    # configs[3]'s AB-GMRES (m-space Arnoldi, replicated basis, one all-reduce per A*(B*q))
    out_ = hgmres.ABgmres_nonhybrid_bounds(A_g, B_g, P.b, xt, 0.0, 12, ctx=ctx, return_H=True)
    res.update(abn_x=out_[0], abn_res=out_[2], abn_err=out_[1], abn_H=out_[-1])
    # the same solve with device inputs / outputs (HGM_DEVICE_PTRS, bench.py's hand-over): the
    # setup norms take another branch there (||x_true||^2 must still be summed over the shards)
    res.update(_abn_device(ctx, A_g, B_g, P.b, xt, 12))
    x, e, r, k, H = hgmres.hybrid_ab_gmres_rtp(A_g, B_g, P.b, xt, 0.0, 12, 1e-2, ctx=ctx, return_H=True)
    res.update(hab_x=x, hab_res=r, hab_err=e, hab_H=H)
    # configs[4]: the Golub-Kahan path on fp32 shards
    A32 = hgmres.SparseOperator.from_scipy(A_g, ctx, dtype=1)
    B32 = hgmres.SparseOperator.from_scipy(B_g, ctx, dtype=1)
    x, e, r, k = hgmres.lsqr_solver(A32, P.b, xt, 0.0, 4, ctx=ctx, At=B32)
    res.update(lsqr32_x=x, lsqr32_res=r, lsqr32_err=e)
    # the device-generated 4 x 4-tiled operator sharded in STORED order (bench.py build_shard):
    # B_g = hgm_mat_row_slice of the tiled B over whole tile columns, A_g its transpose
    from hgmres.core import stored_pixel_index
    Af = hgmres.SparseOperator.siddon(64, 90, ctx=ctx, order=(4, 0))
    n, col = Af.shape[1], 4 * 64
    bounds = [0] + [int(round(g * (n // col) / world)) * col for g in range(1, world)] + [n]
    tlo, thi = bounds[rank], bounds[rank + 1]
    B2 = Af.T.row_slice(tlo, thi)
    A2 = B2.T
    A2.set_bands(16 * 64, 0)       # 16-column strips; steep rays in the shard's dual row strips
    A2.tune(8 | 2 | 4 | 16, 4)     # the paged streaming kernel of the C4 shards
    xs = np.empty(n)
    xs[stored_pixel_index(64, 4, 0)] = P.x_true
    out_ = hgmres.ABgmres_nonhybrid_bounds(A2, B2, P.b, xs[tlo:thi], 0.0, 12, ctx=ctx, return_H=True)
    res.update(tabn_x=out_[0], tabn_res=out_[2], tabn_err=out_[1], tabn_H=out_[-1])
    x, e, r, k, H = hgmres.hybrid_ba_gmres_rtp(A2, B2, P.b, xs[tlo:thi], 0.0, 15, 1e-2, ctx=ctx, return_H=True)
    res.update(thba_x=x, thba_res=r, thba_err=e, thba_H=H)
    # the one-pass LSQR on these shards with a tol stop inside the first batch of 8:
    # tol between the 5th and 6th residual estimates of a tol = 0 run (the same on every rank)
    r0 = hgmres.lsqr_solver(A2, P.b, xs[tlo:thi], 0.0, 12, ctx=ctx, At=B2)[2]
    tol = 0.5 * (r0[4] + r0[5])
    x, e, r, k = hgmres.lsqr_solver(A2, P.b, xs[tlo:thi], tol, 12, ctx=ctx, At=B2)
    res.update(tlsqrtol_x=x, tlsqrtol_res=r, tlsqrtol_err=e, tlsqrtol_k=k, tlsqrtol_tol=tol)
    # configs[2]'s GCV on pixel shards: the n-space Arnoldi (sharded basis) once, fminbnd on the
    # cached H with the GLOBAL pixel count as the trace term (gcv_function.m:46-50; bench.py c3gcv),
    # and the one-call gcv_function (the library all-reduces n itself)
    Hg, beta_g, kd = hgmres.arnoldi(A_g, B_g, P.b, 20, "ba", ctx=ctx)
    lam, gval = hgmres.gcv_fminbnd(Hg, beta_g, float(P.A.shape[1]), 1e-8, 1.0, 1e-10)
    gfix = hgmres.gcv_function(1e-3, A_g, B_g, P.b, P.A.shape[0], 20, "ba", ctx=ctx)
    res.update(gcv_H=Hg, gcv_beta=beta_g, gcv_lam=lam, gcv_val=gval, gcv_fix=gfix)
    # configs[4] as bench.py build_shard cuts it: fp32 tiled shards of the fp32 operator (one pass
    # per Golub-Kahan iteration on each shard, A*v_hat all-reduced with alpha^2 riding along)
    from hgmres import _lib as L
    Af32 = hgmres.SparseOperator.siddon(64, 90, ctx=ctx, order=(4, 0), dtype=L.HGM_F32)
    B32s = Af32.T.row_slice(tlo, thi)
    A32s = B32s.T
    x, e, r, k = hgmres.lsqr_solver(A32s, P.b, xs[tlo:thi], 0.0, 6, ctx=ctx, At=B32s)
    res.update(tlsqr32_x=x, tlsqr32_res=r, tlsqr32_err=e)
    res.update(tlsqr32_path=ctx.solve_path()["one_pass"])
    x, e, r, a, k = hgmres.lsmr_solver(A32s, P.b, xs[tlo:thi], 0.0, 6, ctx=ctx, At=B32s)
    res.update(tlsmr32_x=x, tlsmr32_res=r, tlsmr32_err=e, tlsmr32_ar=a, tlsmr32_path=ctx.solve_path()["one_pass"])
    # a one-pass plan refused on ONE rank only (HGM_OPT_FUSED_AB off on the last rank;
    # a fan-beam cut can refuse the centre shards' plans alone): the ranks agree on the two-pass
    # path (solvers.cpp agreed_gk_plan) instead of issuing different collective sequences, so the
    # solve equals the one with the pass off on every rank, bit for bit
    for tag, off in (("tmix", rank == world - 1), ("toff", True)):
        with ctx.options(fused_ab=0 if off else 1):
            x, e, r, k = hgmres.lsqr_solver(A32s, P.b, xs[tlo:thi], 0.0, 6, ctx=ctx, At=B32s)
            pq = ctx.solve_path()["one_pass"]
            xm_, em_, rm_, am_, km_ = hgmres.lsmr_solver(A32s, P.b, xs[tlo:thi], 0.0, 6, ctx=ctx, At=B32s)
            pm = ctx.solve_path()["one_pass"]
        res.update({f"{tag}q_x": x, f"{tag}q_res": r, f"{tag}q_err": e, f"{tag}q_path": pq,
                    f"{tag}m_x": xm_, f"{tag}m_res": rm_, f"{tag}m_ar": am_, f"{tag}m_path": pm})
    res.update(lo=lo, hi=hi, tlo=tlo, thi=thi)
    return res


def solve_c4(ctx, rank, world, hub):
    """BASELINE configs[3] and [4] at full size, cut exactly as bench.py build_shard cuts them
    for --gpus `world` (device-generated 4096^2 / 47-angle operator, 4 x 4-tiled, whole tile
    columns of stored pixels, B_g = row slice of A', A_g its transpose, 64-column bands), with the
    fixture's b (tests/golden/c4_4096.npz) in place of the device-formed one.  The ranks build
    their shards one after the other (each build holds the full operator, its transpose and the
    sort's scratch for a moment), so the peak HBM of `world` ranks on one device is one build plus
    the shards:
    * ABgmres_nonhybrid_bounds, 20 iterations, fp64 (the one pass per shard + the m-vector
      all-reduce), with the per-iteration monitor path (Gram form or x formed) of every rank;
    * lsqr_solver / lsmr_solver on the fp32 shards, the bench's 20 iterations, with the path."""
    import bench
    from conftest import load_golden
    g = load_golden("c4_4096.npz")
    b = np.ascontiguousarray(g["b"])
    res = {}
    for wl, tag in (("c4", "abn"), ("c5", "f32")):
        for turn in range(world):
            if turn == rank:
                fr, tot = ctx.mem_info()
                print(f"[rank {rank}/{world}] {wl} shard: building ({fr / 2**30:.0f} of {tot / 2**30:.0f} GiB free)",
                      flush=True)
                t0 = time.time()
                A_g, B_g, _, xs, (lo, hi), full = bench.build_shard(ctx, bench.WORKLOADS[wl], rank, world)
                ctx.synchronize()
                print(f"[rank {rank}/{world}] {wl} shard [{lo}, {hi}) built in {time.time() - t0:.1f} s", flush=True)
            hub.barrier()
        xt = np.ascontiguousarray(xs[lo:hi])
        t0 = time.time()
        if tag == "abn":
            out_ = hgmres.ABgmres_nonhybrid_bounds(A_g, B_g, b, xt, 0.0, 20, ctx=ctx, return_H=True)
            res.update(abn_x=out_[0], abn_err=out_[1], abn_res=out_[2], abn_k=out_[3], abn_H=out_[-1],
                       abn_path=np.array(ctx.solve_path()["gram_monitor"]), abn_xt_zero=bool(np.all(xt == 0)))
        else:
            x, e, r, k = hgmres.lsqr_solver(A_g, b, xt, 0.0, 20, ctx=ctx, At=B_g)
            res.update(lsqr32_x=x, lsqr32_err=e, lsqr32_res=r, lsqr32_k=k, lsqr32_path=ctx.solve_path()["one_pass"])
            x, e, r, a, k = hgmres.lsmr_solver(A_g, b, xt, 0.0, 20, ctx=ctx, At=B_g)
            res.update(lsmr32_x=x, lsmr32_err=e, lsmr32_res=r, lsmr32_ar=a, lsmr32_k=k,
                       lsmr32_path=ctx.solve_path()["one_pass"])
        print(f"[rank {rank}/{world}] {wl} solves {time.time() - t0:.1f} s", flush=True)
        res.update({f"{tag}_lo": lo, f"{tag}_hi": hi})
        A_g.close()
        B_g.close()
        hub.barrier()
    return res


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    main()
