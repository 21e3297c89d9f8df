"""Host-side mirror of the reference's MATLAB solver interface over libhgmres.

Every public solver keeps the reference's name, positional arguments and
output tuple (the MATLAB ``[x, error_norm, residual_norm, niters] = f(...)``
becomes a Python tuple), with histories truncated to ``1:niters`` exactly as
the ``.m`` files do.  Operators may be scipy sparse matrices, dense arrays, or
:class:`SparseOperator` handles already resident in HBM.

Reference signatures mirrored (file:line):
  hybrid_ab_gmres_rtp.m:1, hybrid_ba_gmres_rtp.m:1, lsqr_solver.m:1,
  lsmr_solver.m:1 (defaults :3,5), hybrid_lsqr_solver.m:1,
  hybrid_lsmr_solver.m:1, gcv_function.m:1, ABgmres_hybrid_bounds.m:1-2,
  ABgmres_nonhybrid_bounds.m:1-2, BAgmres_hybrid_bounds.m:1-2,
  BAgmres_nonhybrid_bounds.m:1-2.
Error behaviour: MATLAB errors (dimension mismatch, unassigned output) raise
ValueError / :class:`OutputNotAssigned`; Krylov breakdown is not an error.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import threading

import numpy as np
import scipy.sparse as sp

from . import _lib as L


class HgmError(RuntimeError):
    pass


class OutputNotAssigned(HgmError):
    """MATLAB: 'Output argument "x" not assigned during call'."""


def _check(rc, ctx=None):
    if rc == L.HGM_OK:
        return
    msg = ""
    if ctx is not None and ctx._h:
        msg = L.load().hgm_last_error(ctx._h).decode(errors="replace")
    if rc == L.HGM_E_ARG:
        raise ValueError(msg or "invalid argument")
    if rc == L.HGM_E_NOT_ASSIGNED:
        raise OutputNotAssigned(msg)
    raise HgmError(f"libhgmres status {rc}: {msg}")


def _dp(a):
    return a.ctypes.data_as(L.dp) if a is not None else None


def _f64(v, n=None, name="vector"):
    a = np.ascontiguousarray(np.asarray(v, dtype=np.float64).reshape(-1))
    if n is not None and a.shape[0] != n:
        raise ValueError(f"{name} has length {a.shape[0]}, expected {n}")
    return a


class Context:
    """One HIP device + stream (``hgm_ctx``).  ``world > 1`` contexts are made
    by :func:`hgmres.dist.init_context`."""

    def __init__(self, device: int = 0, _handle=None):
        lib = L.load()
        self.device = device
        if _handle is None:
            h = C.c_void_p()
            rc = lib.hgm_ctx_create(device, C.byref(h))
            if rc != L.HGM_OK:
                n, paths = L.runtime_check(lib)
                if n > 1:
                    raise HgmError(f"hgm_ctx_create refused: two HIP runtimes are mapped ({paths})")
                raise HgmError(f"hgm_ctx_create(device={device}) failed with status {rc} (is a GPU visible?)")
            _handle = h
        self._h = _handle
        self._keep = []          # callbacks kept alive

    @property
    def handle(self):
        return self._h

    def rank_world(self):
        r, w = C.c_int(), C.c_int()
        _check(L.load().hgm_ctx_rank(self._h, C.byref(r), C.byref(w)), self)
        return r.value, w.value

    def release_workspace(self):
        """Free this context's device workspace (hgm_ctx_release_workspace); returns the bytes freed."""
        b = C.c_int64()
        _check(L.load().hgm_ctx_release_workspace(self._h, C.byref(b)), self)
        return b.value

    def mem_info(self):
        """(free, total) bytes of device memory on this context's GPU (all processes)."""
        f, t = C.c_int64(), C.c_int64()
        _check(L.load().hgm_mem_info(self._h, C.byref(f), C.byref(t)), self)
        return f.value, t.value

    def solve_path(self):
        """Path decisions of the last solve on this context (``hgm_ctx_solve_path``):
        ``{"gram_monitor": [0/1 per GMRES iteration], "one_pass": 0/1 or None}``."""
        lib = L.load()
        out = {}
        for what, key in ((0, "gram_monitor"), (1, "one_pass")):
            n = C.c_int()
            _check(lib.hgm_ctx_solve_path(self._h, what, None, 0, C.byref(n)), self)
            buf = (C.c_int * max(n.value, 1))()
            _check(lib.hgm_ctx_solve_path(self._h, what, buf, n.value, C.byref(n)), self)
            out[key] = list(buf[:n.value])
        out["one_pass"] = out["one_pass"][0] if out["one_pass"] else None
        return out

    def set_option(self, name, value):
        """Per-context numerics option (``hgm_ctx_set_option``; names in ``_lib.OPTIONS``),
        e.g. ``ctx.set_option("parity", 1)``.  Returns the previous value."""
        prev = self.get_option(name)
        _check(L.load().hgm_ctx_set_option(self._h, L.OPTIONS[name], float(value)), self)
        return prev

    def get_option(self, name):
        v = C.c_double()
        _check(L.load().hgm_ctx_get_option(self._h, L.OPTIONS[name], C.byref(v)), self)
        return v.value

    def options(self, **kw):
        """Context manager: set options for a block, restore them after."""
        import contextlib

        @contextlib.contextmanager
        def _cm():
            prev = {k: self.set_option(k, v) for k, v in kw.items()}
            try:
                yield self
            finally:
                for k, v in prev.items():
                    self.set_option(k, v)
        return _cm()

    def synchronize(self):
        _check(L.load().hgm_ctx_synchronize(self._h), self)

    def stream(self):
        return L.load().hgm_ctx_stream(self._h)

    def set_host_allreduce(self, rank, world, fn):
        """Route cross-rank sums through ``fn(np.ndarray) -> None`` (in place).
        Used for shard emulation (several processes on one device, gloo)."""
        def _cb(buf, count, _user):
            try:
                arr = np.ctypeslib.as_array(buf, shape=(count,))
                fn(arr)
                return 0
            except Exception:   # noqa: BLE001 - reported as a comm error by the library
                return -1
        cb = L.ALLREDUCE_FN(_cb)
        self._keep.append(cb)
        _check(L.load().hgm_ctx_set_host_allreduce(self._h, rank, world, cb, None), self)

    def kernel_timing(self, enable=True):
        _check(L.load().hgm_kernel_timing(self._h, int(enable)), self)

    def kernel_timing_pause(self, paused=True):
        _check(L.load().hgm_kernel_timing_pause(self._h, int(paused)), self)

    def kernel_timing_read(self, cls):
        ms, calls, by = C.c_double(), C.c_int64(), C.c_double()
        _check(L.load().hgm_kernel_timing_read(self._h, cls, C.byref(ms), C.byref(calls), C.byref(by)), self)
        return ms.value, calls.value, by.value

    def close(self):
        if self._h:
            L.load().hgm_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        if sys.is_finalizing():       # HIP runtime may already be torn down at exit
            return
        try:
            self.close()
        except Exception:   # noqa: BLE001
            pass


_default_ctx = None
_ctx_lock = threading.Lock()


def default_context() -> Context:
    global _default_ctx
    with _ctx_lock:
        if _default_ctx is None:
            dev = int(os.environ.get("HGM_DEVICE", os.environ.get("LOCAL_RANK", "0")))
            _default_ctx = Context(dev)
        return _default_ctx


def auto_pixel_order(N):
    """Stored pixel order for an N x N image: 4 x 4 tiles (one 128-B
    line of fp64 per tile) whenever 4 | N.  Super-blocks (a second tiling level) are
    supported but measured no better once the banded kernel runs 4 lanes per segment
    (profiles/r1_spmv_sweep_c4_order.jsonl).  Returns (tile, super_block)."""
    return (4 if N % 4 == 0 else 1), 0


def stored_pixel_index(N, tile, super_block=0):
    """Stored position of every reference pixel p = r + c*N of an N x N image in the tiled
    order (N, tile, super_block) (csrc/ops.hip pixel_index): super x super blocks column-major,
    tile x tile tiles inside in tile-column-major order, column-major inside a tile."""
    p = np.arange(N * N, dtype=np.int64)
    r, c = p % N, p // N

    def tiled(S, rr, cc):
        if tile <= 1:
            return rr + cc * S
        tr, tc = rr // tile, cc // tile
        return ((tc * (S // tile) + tr) * tile + (cc % tile)) * tile + (rr % tile)

    if super_block <= 1:
        return tiled(N, r, c)
    S = super_block
    return ((c // S) * (N // S) + (r // S)) * S * S + tiled(S, r % S, c % S)


class SparseOperator:
    """A CSR operator resident in HBM (``hgm_mat``)."""

    def __init__(self, ctx: Context, handle, shape, nnz, dtype):
        self.ctx = ctx
        self._h = handle
        self.shape = shape
        self.nnz = nnz
        self.dtype = dtype
        self._T = None

    @classmethod
    def from_scipy(cls, M, ctx: Context | None = None, dtype=L.HGM_F64):
        ctx = ctx or default_context()
        if not sp.issparse(M):
            M = sp.csr_matrix(np.asarray(M, dtype=np.float64))
        M = M.tocsr()
        rp = np.ascontiguousarray(M.indptr, dtype=np.int64)
        ci = np.ascontiguousarray(M.indices, dtype=np.int32)
        va = np.ascontiguousarray(M.data, dtype=np.float64)
        h = C.c_void_p()
        _check(L.load().hgm_mat_create_csr(ctx.handle, M.shape[0], M.shape[1], M.nnz,
                                           rp.ctypes.data_as(L.ip64), ci.ctypes.data_as(L.ip32),
                                           _dp(va), dtype, C.byref(h)), ctx)
        return cls(ctx, h, M.shape, int(M.nnz), dtype)

    @classmethod
    def from_csc(cls, M, ctx: Context | None = None, dtype=L.HGM_F64):
        """MATLAB sparse hand-over (CSC, 64-bit indices), transposed on device."""
        ctx = ctx or default_context()
        M = sp.csc_matrix(M)
        M.sort_indices()
        jc = np.ascontiguousarray(M.indptr, dtype=np.int64)
        ir = np.ascontiguousarray(M.indices, dtype=np.int64)
        pr = np.ascontiguousarray(M.data, dtype=np.float64)
        h = C.c_void_p()
        _check(L.load().hgm_mat_create_csc(ctx.handle, M.shape[0], M.shape[1], M.nnz,
                                           jc.ctypes.data_as(L.ip64), ir.ctypes.data_as(L.ip64),
                                           _dp(pr), dtype, C.byref(h)), ctx)
        return cls(ctx, h, M.shape, int(M.nnz), dtype)

    @classmethod
    def siddon(cls, N, n_angles, ctx: Context | None = None, dtype=L.HGM_F64, det_offset=None,
               order="auto"):
        """Parallel-beam projector generated on the device.

        ``order`` is the STORED pixel order (invisible at the boundary: products,
        downloads and solves use the reference column-major ``x(:)``): ``"reference"``,
        ``(tile, super_block)``, or ``"auto"`` = :func:`auto_pixel_order`."""
        from .problems import DETECTOR_OFFSET
        ctx = ctx or default_context()
        off = DETECTOR_OFFSET if det_offset is None else det_offset
        tile, sup = auto_pixel_order(N) if order == "auto" else ((1, 0) if order == "reference" else order)
        h = C.c_void_p()
        _check(L.load().hgm_mat_create_siddon_ordered(ctx.handle, N, n_angles, off, dtype, int(tile), int(sup),
                                                      C.byref(h)), ctx)
        return cls._wrap(ctx, h)

    @classmethod
    def fanbeam(cls, N, n_angles, ctx: Context | None = None, R=None, span=None, dtype=L.HGM_F64, det_offset=None,
                order="auto"):
        """Fan-beam (curved detector) projector generated on the device, bit-identical to
        :func:`hgmres.problems.fanbeam_projector` (the 'fancurved' geometry of
        run_2D_phantom.m:12-13).  ``span=None``: the fan covering the image's circumscribed
        circle; ``order`` as for :meth:`siddon`."""
        from .problems import DETECTOR_OFFSET, FAN_R
        ctx = ctx or default_context()
        off = DETECTOR_OFFSET if det_offset is None else det_offset
        tile, sup = auto_pixel_order(N) if order == "auto" else ((1, 0) if order == "reference" else order)
        h = C.c_void_p()
        _check(L.load().hgm_mat_create_fanbeam(ctx.handle, N, n_angles, float(FAN_R if R is None else R),
                                               float(0.0 if span is None else span), off, dtype, int(tile), int(sup),
                                               C.byref(h)), ctx)
        return cls._wrap(ctx, h)

    @classmethod
    def pixel_backprojector(cls, N, n_angles, ctx: Context | None = None, dtype=L.HGM_F64, det_offset=None,
                            order="auto"):
        """Unmatched pixel-driven back-projector B (n x m) generated on the device, bit-identical
        to :func:`hgmres.problems.pixel_driven_backprojector`.  ``order``: stored pixel (row)
        order, as for :meth:`siddon` (pair it with an A of the same order)."""
        from .problems import DETECTOR_OFFSET
        ctx = ctx or default_context()
        off = DETECTOR_OFFSET if det_offset is None else det_offset
        tile, sup = auto_pixel_order(N) if order == "auto" else ((1, 0) if order == "reference" else order)
        h = C.c_void_p()
        _check(L.load().hgm_mat_create_backprojector(ctx.handle, N, n_angles, off, dtype, int(tile), int(sup),
                                                     C.byref(h)), ctx)
        return cls._wrap(ctx, h)

    def pixel_order(self, which="cols"):
        """(N, tile, super_block) of the stored row/column index order; N = 0: reference order."""
        n_, t_, s_ = C.c_int(), C.c_int(), C.c_int()
        _check(L.load().hgm_mat_order(self._h, 0 if which == "rows" else 1, C.byref(n_), C.byref(t_),
                                      C.byref(s_)), self.ctx)
        return n_.value, t_.value, s_.value

    @classmethod
    def _wrap(cls, ctx, h):
        r, c_, nz, dt = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int()
        _check(L.load().hgm_mat_info(h, C.byref(r), C.byref(c_), C.byref(nz), C.byref(dt)), ctx)
        return cls(ctx, h, (r.value, c_.value), nz.value, dt.value)

    @property
    def T(self) -> "SparseOperator":
        """Device transpose (cached)."""
        if self._T is None:
            h = C.c_void_p()
            _check(L.load().hgm_mat_transpose(self.ctx.handle, self._h, C.byref(h)), self.ctx)
            self._T = SparseOperator._wrap(self.ctx, h)
            self._T._T = self
        return self._T

    def to_scipy(self) -> sp.csr_matrix:
        rows, cols = self.shape
        rp = np.empty(rows + 1, dtype=np.int64)
        ci = np.empty(max(self.nnz, 1), dtype=np.int32)
        va = np.empty(max(self.nnz, 1), dtype=np.float64)
        _check(L.load().hgm_mat_download(self.ctx.handle, self._h, rp.ctypes.data_as(L.ip64),
                                         ci.ctypes.data_as(L.ip32), _dp(va)), self.ctx)
        M = sp.csr_matrix((va[: self.nnz], ci[: self.nnz], rp), shape=self.shape)
        M.has_sorted_indices = False
        return M

    def row_ptr(self) -> np.ndarray:
        """The CSR row pointers only (rows + 1 int64; e.g. the nnz weights of a shard plan)."""
        rp = np.empty(self.shape[0] + 1, dtype=np.int64)
        _check(L.load().hgm_mat_download(self.ctx.handle, self._h, rp.ctypes.data_as(L.ip64), None, None),
               self.ctx)
        return rp

    def row_slice(self, lo: int, hi: int) -> "SparseOperator":
        """Rows [lo, hi) as a new device operator (pixel shard ``B(P_g,:)``)."""
        h = C.c_void_p()
        _check(L.load().hgm_mat_row_slice(self.ctx.handle, self._h, int(lo), int(hi), C.byref(h)), self.ctx)
        return SparseOperator._wrap(self.ctx, h)

    def tune(self, variant: int, group: int = 0):
        """Select the SpMV kernel variant (bits: 1 paired 16-B loads, 2 nontemporal,
        4 XCD-aware order) and lanes per row."""
        _check(L.load().hgm_mat_tune(self._h, int(variant), int(group)), self.ctx)

    def set_bands(self, band_width: int, group: int = 0):
        """Column banding of the x gather (0 = off, -1 = automatic)."""
        _check(L.load().hgm_mat_set_bands(self.ctx.handle, self._h, int(band_width), int(group)), self.ctx)

    def matvec_device(self, x_ptr: int, y_ptr: int):
        _check(L.load().hgm_spmv(self.ctx.handle, self._h, C.c_void_p(x_ptr), C.c_void_p(y_ptr)), self.ctx)

    def __matmul__(self, x):
        """Host convenience y = M @ x (copies through HBM)."""
        x = _f64(x, self.shape[1], "x")
        ctx = self.ctx
        lib = L.load()
        es = 8 if self.dtype == L.HGM_F64 else 4
        xd, yd = C.c_void_p(), C.c_void_p()
        _check(lib.hgm_dev_alloc(ctx.handle, es * max(1, self.shape[1]), C.byref(xd)), ctx)
        _check(lib.hgm_dev_alloc(ctx.handle, es * max(1, self.shape[0]), C.byref(yd)), ctx)
        try:
            xs = x if es == 8 else x.astype(np.float32)
            _check(lib.hgm_memcpy_h2d(ctx.handle, xd, xs.ctypes.data_as(C.c_void_p), es * self.shape[1]), ctx)
            _check(lib.hgm_spmv(ctx.handle, self._h, xd, yd), ctx)
            y = np.empty(self.shape[0], dtype=np.float64 if es == 8 else np.float32)
            _check(lib.hgm_memcpy_d2h(ctx.handle, y.ctypes.data_as(C.c_void_p), yd, es * self.shape[0]), ctx)
        finally:
            lib.hgm_dev_free(ctx.handle, xd)
            lib.hgm_dev_free(ctx.handle, yd)
        return y.astype(np.float64)

    def close(self):
        if self._T is not None and self._T is not self:
            T, self._T = self._T, None
            T._T = None
        if self._h:
            L.load().hgm_mat_destroy(self._h)
            self._h = None

    def __del__(self):
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:   # noqa: BLE001
            pass


def spmv_ab(A: "SparseOperator", B: "SparseOperator", q):
    """(B*q, A*(B*q)) through ``hgm_spmv_ab`` (host arrays in, host arrays out): the m-space
    operator of the AB solvers, one pass over B when B is A' value for value (fused.hip)."""
    ctx = A.ctx
    lib = L.load()
    m, n = A.shape
    es = 8 if A.dtype == L.HGM_F64 else 4
    dt = np.float64 if es == 8 else np.float32
    q = np.ascontiguousarray(np.asarray(q, dtype=dt).reshape(-1))
    if q.shape[0] != m:
        raise ValueError(f"q has length {q.shape[0]}, expected {m}")
    ptr = [C.c_void_p() for _ in range(3)]
    try:
        for p_, k in zip(ptr, (m, n, m)):
            _check(lib.hgm_dev_alloc(ctx.handle, es * max(1, k), C.byref(p_)), ctx)
        _check(lib.hgm_memcpy_h2d(ctx.handle, ptr[0], q.ctypes.data_as(C.c_void_p), es * m), ctx)
        _check(lib.hgm_spmv_ab(ctx.handle, A._h, B._h, ptr[0], ptr[1], ptr[2]), ctx)
        bq, abq = np.empty(n, dtype=dt), np.empty(m, dtype=dt)
        _check(lib.hgm_memcpy_d2h(ctx.handle, bq.ctypes.data_as(C.c_void_p), ptr[1], es * n), ctx)
        _check(lib.hgm_memcpy_d2h(ctx.handle, abq.ctypes.data_as(C.c_void_p), ptr[2], es * m), ctx)
    finally:
        for p_ in ptr:
            if p_.value:
                lib.hgm_dev_free(ctx.handle, p_)
    return bq.astype(np.float64), abq.astype(np.float64)


def fused_plan_info(A: "SparseOperator", B: "SparseOperator"):
    """The one-pass plan of (A, B) under the context's options (built if needed): dict with the
    build seconds, a checksum over every plan array, the partial slots and whether the device built
    the ray sets (``hgm_fused_plan_info``)."""
    ctx = A.ctx
    bs, ck, ns, dv = C.c_double(), C.c_uint64(), C.c_int64(), C.c_int()
    _check(L.load().hgm_fused_plan_info(ctx.handle, A._h, B._h, C.byref(bs), C.byref(ck), C.byref(ns), C.byref(dv)),
           ctx)
    return {"build_s": bs.value, "checksum": ck.value, "nslot": ns.value, "device_built": bool(dv.value)}


def as_operator(M, ctx=None, dtype=L.HGM_F64) -> SparseOperator:
    if isinstance(M, SparseOperator):
        return M
    return SparseOperator.from_scipy(M, ctx=ctx, dtype=dtype)


def _ops(A, B, ctx):
    ctx = ctx or (A.ctx if isinstance(A, SparseOperator) else default_context())
    Ao = as_operator(A, ctx)
    if B is None:
        Bo = Ao.T
    else:
        Bo = as_operator(B, ctx, Ao.dtype)
    if Bo.shape != (Ao.shape[1], Ao.shape[0]):
        raise ValueError(f"dimension mismatch: A is {Ao.shape}, B is {Bo.shape} (expected size(A'))")
    return ctx, Ao, Bo


def _opts(orth="mgs", H_out=None, device_ptrs=False, explicit_residual=False):
    o = L.hgm_opts()
    o.flags = (L.HGM_DEVICE_PTRS if device_ptrs else 0) | (L.HGM_EXPLICIT_RESIDUAL if explicit_residual else 0)
    o.orth = L.HGM_CGS2 if str(orth).lower() == "cgs2" else L.HGM_MGS
    o.H_out = _dp(H_out) if H_out is not None else None
    return o


def _gmres_call(fn_name, A, B, b, x_true, tol, maxit, lam, ctx, orth, return_H, extra=(), explicit_residual=False):
    ctx, Ao, Bo = _ops(A, B, ctx)
    m, n = Ao.shape
    maxit = int(maxit)
    b = _f64(b, m, "b")
    xt = _f64(x_true, n, "x_true")
    x = np.zeros(n)
    err = np.zeros(maxit)
    res = np.zeros(maxit)
    it = C.c_int(0)
    H = np.zeros((maxit + 1) * maxit) if return_H else None
    o = _opts(orth, H, explicit_residual=explicit_residual)
    fn = getattr(L.load(), fn_name)
    if fn_name == "hgm_gmres_bounds_ex":
        lam_, side, hyb = extra
        rc = fn(ctx.handle, C.byref(o), Ao._h, Bo._h, _dp(b), _dp(xt), float(tol), maxit, float(lam_), side, hyb,
                _dp(x), _dp(err), _dp(res), C.byref(it))
    else:
        rc = fn(ctx.handle, C.byref(o), Ao._h, Bo._h, _dp(b), _dp(xt), float(tol), maxit, float(lam),
                _dp(x), _dp(err), _dp(res), C.byref(it))
    _check(rc, ctx)
    k = it.value
    out = (x, err[:k].copy(), res[:k].copy(), k)
    if return_H:
        out = out + (H.reshape(maxit, maxit + 1).T.copy(),)
    return out


# ---------------------------------------------------------------------------
# Reference solver signatures
# ---------------------------------------------------------------------------
def hybrid_ab_gmres_rtp(A, B, b, x_true, tol, maxit, lambda_, *, ctx=None, orth="mgs", return_H=False,
                        explicit_residual=False):
    """``[x, error_norm, residual_norm, niters] = hybrid_ab_gmres_rtp(A,B,b,x_true,tol,maxit,lambda)``
    (hybrid_ab_gmres_rtp.m:1-45): n-space Arnoldi on ``B*A + lambda*I``, projected
    Tikhonov ``(AQk'AQk + lambda I) y = AQk' b``.  ``explicit_residual`` monitors
    ``norm(b - A*x)`` with an SpMV of x instead of ``b - (A*Q) y`` (HGM_EXPLICIT_RESIDUAL)."""
    return _gmres_call("hgm_hybrid_ab_gmres_rtp_ex", A, B, b, x_true, tol, maxit, lambda_, ctx, orth, return_H,
                       explicit_residual=explicit_residual)


def hybrid_ba_gmres_rtp(A, B, b, x_true, tol, maxit, lambda_, *, ctx=None, orth="mgs", return_H=False,
                        explicit_residual=False):
    """``hybrid_ba_gmres_rtp.m:1-42``: Arnoldi on ``B*A + lambda*I``, ``yk = Hk \\ beta e1``."""
    return _gmres_call("hgm_hybrid_ba_gmres_rtp_ex", A, B, b, x_true, tol, maxit, lambda_, ctx, orth, return_H,
                       explicit_residual=explicit_residual)


def _delta_ops(DeltaM, ctx):
    """DeltaM as one device operator, or as a factored product (L, R) = L*R applied to vectors."""
    if isinstance(DeltaM, (tuple, list)):
        L_, R_ = DeltaM
        return as_operator(_sparse(L_), ctx), as_operator(_sparse(R_), ctx)
    return as_operator(_sparse(DeltaM), ctx), None


def _sparse(M):
    if isinstance(M, SparseOperator) or sp.issparse(M):
        return M
    return sp.csr_matrix(np.asarray(M, dtype=np.float64))


def _bounds(A, B, b, x_true, tol, maxit, lam, side, hybrid, ctx, orth, return_H, explicit_residual=False,
            DeltaM=None, ritz_steps=0, return_ritz=False):
    if DeltaM is None:
        out = _gmres_call("hgm_gmres_bounds_ex", A, B, b, x_true, tol, maxit, lam, ctx, orth, return_H,
                          extra=(lam, side, hybrid), explicit_residual=explicit_residual)
        # outputs 5-8 need DeltaM (the reference's 8th / 7th argument)
        return out[:4] + (None, None, None, None) + out[4:]
    # outputs 5-8: filter factors phi and their first-order perturbation dphi (*_bounds.m:42-81)
    ctx, Ao, Bo = _ops(A, B, ctx)
    DL, DR = _delta_ops(DeltaM, ctx)
    m, n = Ao.shape
    maxit = int(maxit)
    b = _f64(b, m, "b")
    xt = _f64(x_true, n, "x_true")
    x, err, res, it = np.zeros(n), np.zeros(maxit), np.zeros(maxit), C.c_int(0)
    phi = np.zeros(maxit * maxit)
    dphi = np.zeros(maxit * maxit)
    mu = np.zeros(maxit)
    rres = np.zeros(maxit)
    H = np.zeros((maxit + 1) * maxit)          # also tells a breakdown at iteration k (below)
    o = _opts(orth, H, explicit_residual=explicit_residual)
    _check(L.load().hgm_gmres_bounds_filter(ctx.handle, C.byref(o), Ao._h, Bo._h, _dp(b), _dp(xt), float(tol),
                                            maxit, float(lam), side, hybrid, DL._h, DR._h if DR else None,
                                            int(ritz_steps), _dp(x), _dp(err), _dp(res), C.byref(it), _dp(phi),
                                            _dp(dphi), _dp(mu), _dp(rres)), ctx)
    k = it.value
    P_ = phi.reshape(maxit, maxit)
    D_ = dphi.reshape(maxit, maxit)
    phi_iter = [P_[j, : j + 1].copy() for j in range(k)]
    dphi_iter = [D_[j, : j + 1].copy() for j in range(k)]
    Hm = H.reshape(maxit, maxit + 1).T
    if k and Hm[k, k - 1] == 0.0:   # breakdown at iteration k (*_bounds.m:31 before :80): phi_iter{k} = []
        phi_iter[-1] = np.zeros(0)
        dphi_iter[-1] = np.zeros(0)
    out = (x, err[:k].copy(), res[:k].copy(), k, phi_iter[-1], dphi_iter[-1], phi_iter, dphi_iter)
    if return_H:
        out = out + (Hm.copy(),)
    if return_ritz:
        out = out + (mu[:k].copy(), rres[:k].copy())
    return out


def ABgmres_hybrid_bounds(A, B, b, x_true, tol, maxit, lambda_, DeltaM=None, *, ctx=None, orth="mgs", return_H=False,
                             explicit_residual=False, ritz_steps=0, return_ritz=False):
    """``ABgmres_hybrid_bounds.m``: m-space Arnoldi on ``A*B``, PTR Tikhonov, ``x = B*z``; outputs 5-8
    (filter factors) when ``DeltaM`` (a matrix, or a factored pair ``(L, R)`` = L*R) is given."""
    return _bounds(A, B, b, x_true, tol, maxit, lambda_, L.HGM_SIDE_AB, 1, ctx, orth, return_H,
                   explicit_residual=explicit_residual,
                   DeltaM=DeltaM, ritz_steps=ritz_steps, return_ritz=return_ritz)


def ABgmres_nonhybrid_bounds(A, B, b, x_true, tol, maxit, DeltaM=None, *, ctx=None, orth="mgs", return_H=False,
                             explicit_residual=False, ritz_steps=0, return_ritz=False):
    """``ABgmres_nonhybrid_bounds.m`` (outputs 5-8 with ``DeltaM``)."""
    return _bounds(A, B, b, x_true, tol, maxit, 0.0, L.HGM_SIDE_AB, 0, ctx, orth, return_H,
                   explicit_residual=explicit_residual,
                   DeltaM=DeltaM, ritz_steps=ritz_steps, return_ritz=return_ritz)


def BAgmres_hybrid_bounds(A, B, b, x_true, tol, maxit, lambda_, DeltaM=None, *, ctx=None, orth="mgs", return_H=False,
                             explicit_residual=False, ritz_steps=0, return_ritz=False):
    """``BAgmres_hybrid_bounds.m``: n-space Arnoldi on ``B*A``, PTR Tikhonov (outputs 5-8 with ``DeltaM``)."""
    return _bounds(A, B, b, x_true, tol, maxit, lambda_, L.HGM_SIDE_BA, 1, ctx, orth, return_H,
                   explicit_residual=explicit_residual,
                   DeltaM=DeltaM, ritz_steps=ritz_steps, return_ritz=return_ritz)


def BAgmres_nonhybrid_bounds(A, B, b, x_true, tol, maxit, DeltaM=None, *, ctx=None, orth="mgs", return_H=False,
                             explicit_residual=False, ritz_steps=0, return_ritz=False):
    """``BAgmres_nonhybrid_bounds.m`` (outputs 5-8 with ``DeltaM``).  The reference forms ``M = B*A``
    explicitly (``:4``); here the operator is applied as ``B*(A*q)``."""
    return _bounds(A, B, b, x_true, tol, maxit, 0.0, L.HGM_SIDE_BA, 0, ctx, orth, return_H,
                   explicit_residual=explicit_residual,
                   DeltaM=DeltaM, ritz_steps=ritz_steps, return_ritz=return_ritz)


def _gkb_ops(A, ctx, At=None, dtype=L.HGM_F64):
    ctx = ctx or (A.ctx if isinstance(A, SparseOperator) else default_context())
    Ao = as_operator(A, ctx, dtype)
    Ato = as_operator(At, ctx, Ao.dtype) if At is not None else Ao.T
    return ctx, Ao, Ato


def lsqr_solver(A, b, x_true, tol, maxit, *, ctx=None, At=None):
    """``[x, error_norm, residual_norm, niters] = lsqr_solver(A,b,x_true,tol,maxit)`` (lsqr_solver.m:1-54)."""
    ctx, Ao, Ato = _gkb_ops(A, ctx, At)
    m, n = Ao.shape
    maxit = int(maxit)
    b = _f64(b, m, "b")
    xt = _f64(x_true, n, "x_true")
    x, err, res, it = np.zeros(n), np.zeros(maxit), np.zeros(maxit), C.c_int(0)
    o = _opts()
    _check(L.load().hgm_lsqr_solver_ex(ctx.handle, C.byref(o), Ao._h, Ato._h, _dp(b), _dp(xt), float(tol), maxit,
                                       _dp(x), _dp(err), _dp(res), C.byref(it)), ctx)
    k = it.value
    return x, err[:k].copy(), res[:k].copy(), k


def lsmr_solver(A, b, x_true=None, tol=None, maxit=None, *, ctx=None, At=None, explicit_residual=False):
    """``[x, err_hist, res_hist, ar_hist, iters] = lsmr_solver(A,b,x_true,tol,maxit)``
    (lsmr_solver.m:1-83; ``tol`` defaults to 1e-6, ``maxit`` to ``min(m,n)``).  The monitors
    ``b - A*x`` and ``A'*r`` come from kept products unless ``explicit_residual``."""
    ctx, Ao, Ato = _gkb_ops(A, ctx, At)
    m, n = Ao.shape
    tol = 1e-6 if tol is None else float(tol)
    maxit = min(m, n) if maxit is None else int(maxit)
    b = _f64(b, m, "b")
    xt = None if x_true is None or np.size(x_true) == 0 else _f64(x_true, n, "x_true")
    x = np.zeros(n)
    eh, rh, ah, it = np.zeros(maxit), np.zeros(maxit), np.zeros(maxit), C.c_int(0)
    o = _opts(explicit_residual=explicit_residual)
    _check(L.load().hgm_lsmr_solver_ex(ctx.handle, C.byref(o), Ao._h, Ato._h, _dp(b), _dp(xt), tol, maxit,
                                       _dp(x), _dp(eh), _dp(rh), _dp(ah), C.byref(it)), ctx)
    k = it.value
    return x, eh[:k].copy(), rh[:k].copy(), ah[:k].copy(), k


def hybrid_lsqr_solver(A, b, x_true, tol, maxit, lambda_, *, ctx=None, At=None):
    """``hybrid_lsqr_solver.m:1-52`` (LSQR on ``[A; sqrt(lambda) I]``, augmentation implicit)."""
    ctx, Ao, Ato = _gkb_ops(A, ctx, At)
    m, n = Ao.shape
    maxit = int(maxit)
    b = _f64(b, m, "b")
    xt = _f64(x_true, n, "x_true")
    x, err, res, it = np.zeros(n), np.zeros(maxit), np.zeros(maxit), C.c_int(0)
    _check(L.load().hgm_hybrid_lsqr_solver(ctx.handle, Ao._h, Ato._h, _dp(b), _dp(xt), float(tol), maxit,
                                           float(lambda_), _dp(x), _dp(err), _dp(res), C.byref(it)), ctx)
    k = it.value
    return x, err[:k].copy(), res[:k].copy(), k


def hybrid_lsmr_solver(A, b, x_true, tol, maxit, lambda_, *, ctx=None, At=None):
    """``hybrid_lsmr_solver.m:1-57``."""
    ctx, Ao, Ato = _gkb_ops(A, ctx, At)
    m, n = Ao.shape
    maxit = int(maxit)
    b = _f64(b, m, "b")
    xt = _f64(x_true, n, "x_true")
    x, err, res, it = np.zeros(n), np.zeros(maxit), np.zeros(maxit), C.c_int(0)
    _check(L.load().hgm_hybrid_lsmr_solver(ctx.handle, Ao._h, Ato._h, _dp(b), _dp(xt), float(tol), maxit,
                                           float(lambda_), _dp(x), _dp(err), _dp(res), C.byref(it)), ctx)
    k = it.value
    return x, err[:k].copy(), res[:k].copy(), k


def arnoldi(A, B, b, k, gcv_type="ba", *, ctx=None, breakdown_tol=1e-12, orth="mgs"):
    """Arnoldi part of ``gcv_function.m:3-33``: returns (H, beta, kdone)."""
    ctx, Ao, Bo = _ops(A, B, ctx)
    side = L.HGM_SIDE_AB if gcv_type == "ab" else L.HGM_SIDE_BA
    b = _f64(b, Ao.shape[0], "b")
    H = np.zeros((k + 1) * k)
    beta, kd = C.c_double(), C.c_int()
    o = L.HGM_CGS2 if orth == "cgs2" else L.HGM_MGS
    _check(L.load().hgm_arnoldi(ctx.handle, Ao._h, Bo._h, _dp(b), int(k), side, float(breakdown_tol), o,
                                _dp(H), C.byref(beta), C.byref(kd)), ctx)
    return H.reshape(k, k + 1).T.copy(), beta.value, kd.value


def gcv_from_H(H, beta, lambda_, trace_m):
    """λ-dependent part of ``gcv_function.m:35-58`` on a cached H ((k+1) x k)."""
    H = np.asarray(H, dtype=np.float64)
    k = H.shape[1]
    Hf = np.ascontiguousarray(H.T).reshape(-1)
    g = C.c_double()
    rc = L.load().hgm_gcv_from_H(_dp(Hf), k, float(beta), float(lambda_), float(trace_m), C.byref(g))
    if rc != L.HGM_OK:
        raise ValueError("hgm_gcv_from_H: invalid arguments")
    return g.value


def gcv_function(lambda_, A, B, b, m, k_gcv, gcv_type, *, ctx=None):
    """``gcv_val = gcv_function(lambda,A,B,b,m,k_gcv,gcv_type)`` (gcv_function.m:1-59)."""
    ctx, Ao, Bo = _ops(A, B, ctx)
    side = L.HGM_SIDE_AB if gcv_type == "ab" else L.HGM_SIDE_BA
    b = _f64(b, Ao.shape[0], "b")
    g = C.c_double()
    _check(L.load().hgm_gcv_function(ctx.handle, float(lambda_), Ao._h, Bo._h, _dp(b), int(m), int(k_gcv), side,
                                     C.byref(g)), ctx)
    return g.value


def gcv_fminbnd(H, beta, trace_m, lo=1e-9, hi=1e-1, tolx=1e-8):
    """``fminbnd(@(l) gcv_function(l,...), lo, hi, optimset('TolX',tolx))`` on ONE cached
    Arnoldi (analyze_regularization.m:37-46): returns (lambda_opt, gcv_opt)."""
    H = np.asarray(H, dtype=np.float64)
    k = H.shape[1]
    Hf = np.ascontiguousarray(H.T).reshape(-1)
    lo_, g = C.c_double(), C.c_double()
    rc = L.load().hgm_gcv_fminbnd(_dp(Hf), k, float(beta), float(trace_m), float(lo), float(hi), float(tolx),
                                  C.byref(lo_), C.byref(g))
    if rc != L.HGM_OK:
        raise ValueError("hgm_gcv_fminbnd: invalid arguments")
    return lo_.value, g.value


# ---------------------------------------------------------------------------
# Host-only spectral helpers of the filter-factor bounds (spectral.cpp)
# ---------------------------------------------------------------------------
def eig(M):
    """MATLAB ``[V, D] = eig(M)`` of a real square matrix (host): (w, V), complex, unit 2-norm columns."""
    M = np.asarray(M, dtype=np.float64)
    n = M.shape[0]
    Mf = np.ascontiguousarray(M.T).reshape(-1)
    wr, wi, V = np.zeros(n), np.zeros(n), np.zeros(n * n)
    if L.load().hgm_eig(n, _dp(Mf), _dp(wr), _dp(wi), _dp(V)) != L.HGM_OK:
        raise HgmError("hgm_eig: QR iteration did not converge")
    V = V.reshape(n, n).T
    W = V.astype(np.complex128)
    j = 0
    while j < n:
        if wi[j] > 0 and j + 1 < n:
            W[:, j] = V[:, j] + 1j * V[:, j + 1]
            W[:, j + 1] = V[:, j] - 1j * V[:, j + 1]
            j += 2
        else:
            j += 1
    return wr + 1j * wi, W


def filter_factors(H, k, dK, mu, dmu, lambda_, side, hybrid):
    """phi / dphi of iteration k of the ``*_bounds.m`` files (``:42-78``) from H ((k+1) x k
    leading part), dK = Qk' DeltaM Qk, the k leading eigenvalues mu of M and dmu."""
    H = np.asarray(H, dtype=np.float64)
    Hf = np.ascontiguousarray(H.T).reshape(-1)
    dK = np.asarray(dK, dtype=np.float64)
    dKf = np.ascontiguousarray(dK.T).reshape(-1)
    mu = np.ascontiguousarray(mu, dtype=np.float64)
    dmu = np.ascontiguousarray(dmu, dtype=np.float64)
    phi, dphi = np.zeros(k), np.zeros(k)
    sd = L.HGM_SIDE_AB if side == "ab" else L.HGM_SIDE_BA
    rc = L.load().hgm_filter_factors(_dp(Hf), H.shape[0], int(k), _dp(dKf), dK.shape[0], _dp(mu), _dp(dmu),
                                     float(lambda_), sd, int(bool(hybrid)), _dp(phi), _dp(dphi))
    if rc != L.HGM_OK:
        raise ValueError("hgm_filter_factors: invalid arguments")
    return phi, dphi


def ritz(Hp, h_next, G, nev):
    """Leading Ritz pairs of a p-step Arnoldi: (mu, dmu, resid) (descending real part)."""
    Hp = np.asarray(Hp, dtype=np.float64)
    p = Hp.shape[1]
    Hf = np.ascontiguousarray(Hp.T).reshape(-1)
    G = np.asarray(G, dtype=np.float64)
    Gf = np.ascontiguousarray(G.T).reshape(-1)
    mu, dmu, rr = np.zeros(nev), np.zeros(nev), np.zeros(nev)
    rc = L.load().hgm_ritz(_dp(Hf), Hp.shape[0], p, float(h_next), _dp(Gf), G.shape[0], int(nev), _dp(mu),
                           _dp(dmu), _dp(rr))
    if rc != L.HGM_OK:
        raise ValueError("hgm_ritz: invalid arguments")
    return mu, dmu, rr
