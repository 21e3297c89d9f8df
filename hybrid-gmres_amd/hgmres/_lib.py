"""ctypes binding of libhgmres.so (include/hgmres.h).

The library is the product: there is no CPU fallback.  Loading fails loudly
when the HIP extension has not been built (``__graft_entry__.build()``)."""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HGM_LIB") or os.path.join(_HERE, "libhgmres.so")   # HGM_LIB: experiment builds

HGM_OK = 0
HGM_E_ARG = -1
HGM_E_HIP = -2
HGM_E_NOMEM = -3
HGM_E_COMM = -4
HGM_E_NOT_ASSIGNED = -5
HGM_E_UNSUPPORTED = -6

HGM_F64, HGM_F32 = 0, 1
# hgm_ctx_option
OPTIONS = {"parity": 1, "mgs_form": 2, "mgs_single": 3, "gram_err": 4, "gram_err_min": 5, "ring_poll": 6,
           "pend_norm": 7, "recon_serial": 8, "recon_serial_n": 9, "pipe_depth": 10, "sync_event_fence": 11,
           "mgs_ppl": 12, "mgs1_ppl": 13, "mgs_fused": 14, "lsqr_dev": 15, "paged16": 16,
           "band_dual": 17, "fused_ab": 18, "fused_region": 19, "fused_bs": 20, "fused_dbg": 21, "fused_pf": 22,
           "krylov_pad": 23, "fused_kind": 24, "fused_wregion": 25, "fused_waves": 26, "fused_group": 27,
           "fused_depth": 28, "fused_pairs": 29, "fused_acc32": 30, "fused_plan_dev": 31, "fused_reduce": 32,
           "host_spin_us": 33, "fused_rowpair": 34,
           "lsqr_res_img": 35, "lsmr_fuse_nmon": 36}
HGM_MGS, HGM_CGS2 = 0, 1
HGM_SIDE_AB, HGM_SIDE_BA = 0, 1
HGM_DEVICE_PTRS = 1
HGM_EXPLICIT_RESIDUAL = 2
HGM_UNIQUE_ID_BYTES = 128

c_int, c_int64, c_double, c_void_p = C.c_int, C.c_int64, C.c_double, C.c_void_p
P = C.POINTER
dp = P(c_double)
ip64 = P(c_int64)
ip32 = P(C.c_int32)

ALLREDUCE_FN = C.CFUNCTYPE(c_int, dp, c_int64, c_void_p)


class hgm_opts(C.Structure):
    _fields_ = [("flags", c_int), ("orth", c_int), ("H_out", dp)]


# name -> (restype, argtypes)
_SIGS = {
    "hgm_version": (c_int, []),
    "hgm_runtime_check": (c_int, [C.c_char_p, c_int]),
    "hgm_ctx_set_option": (c_int, [c_void_p, c_int, c_double]),
    "hgm_ctx_get_option": (c_int, [c_void_p, c_int, P(c_double)]),
    "hgm_device_count": (c_int, [P(c_int)]),
    "hgm_ctx_create": (c_int, [c_int, P(c_void_p)]),
    "hgm_comm_unique_id": (c_int, [c_void_p]),
    "hgm_ctx_create_dist": (c_int, [c_int, c_int, c_int, c_void_p, P(c_void_p)]),
    "hgm_ctx_set_host_allreduce": (c_int, [c_void_p, c_int, c_int, ALLREDUCE_FN, c_void_p]),
    "hgm_ctx_destroy": (None, [c_void_p]),
    "hgm_last_error": (C.c_char_p, [c_void_p]),
    "hgm_ctx_synchronize": (c_int, [c_void_p]),
    "hgm_ctx_stream": (c_void_p, [c_void_p]),
    "hgm_ctx_rank": (c_int, [c_void_p, P(c_int), P(c_int)]),
    "hgm_experiments": (c_int, []),
    "hgm_ctx_release_workspace": (c_int, [c_void_p, P(c_int64)]),
    "hgm_mem_info": (c_int, [c_void_p, P(c_int64), P(c_int64)]),
    "hgm_ctx_solve_path": (c_int, [c_void_p, c_int, P(c_int), c_int, P(c_int)]),
    "hgm_mat_create_csr": (c_int, [c_void_p, c_int64, c_int64, c_int64, ip64, ip32, dp, c_int, P(c_void_p)]),
    "hgm_mat_create_csc": (c_int, [c_void_p, c_int64, c_int64, c_int64, ip64, ip64, dp, c_int, P(c_void_p)]),
    "hgm_mat_transpose": (c_int, [c_void_p, c_void_p, P(c_void_p)]),
    "hgm_mat_create_siddon": (c_int, [c_void_p, c_int, c_int, c_double, c_int, P(c_void_p)]),
    "hgm_mat_create_siddon_ordered": (c_int, [c_void_p, c_int, c_int, c_double, c_int, c_int, c_int,
                                              P(c_void_p)]),
    "hgm_mat_create_fanbeam": (c_int, [c_void_p, c_int, c_int, c_double, c_double, c_double, c_int, c_int, c_int,
                                       P(c_void_p)]),
    "hgm_mat_order": (c_int, [c_void_p, c_int, P(c_int), P(c_int), P(c_int)]),
    "hgm_mat_create_backprojector": (c_int, [c_void_p, c_int, c_int, c_double, c_int, c_int, c_int, P(c_void_p)]),
    "hgm_mat_row_slice": (c_int, [c_void_p, c_void_p, c_int64, c_int64, P(c_void_p)]),
    "hgm_mat_info": (c_int, [c_void_p, ip64, ip64, ip64, P(c_int)]),
    "hgm_mat_tune": (c_int, [c_void_p, c_int, c_int]),
    "hgm_mat_set_bands": (c_int, [c_void_p, c_void_p, c_int64, c_int]),
    "hgm_mat_download": (c_int, [c_void_p, c_void_p, ip64, ip32, dp]),
    "hgm_mat_destroy": (None, [c_void_p]),
    "hgm_spmv": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "hgm_spmv_ab": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hgm_fused_plan_info": (c_int, [c_void_p, c_void_p, c_void_p, dp, P(C.c_uint64), ip64, P(c_int)]),
    "hgm_dev_alloc": (c_int, [c_void_p, c_int64, P(c_void_p)]),
    "hgm_dev_free": (c_int, [c_void_p, c_void_p]),
    "hgm_memcpy_h2d": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "hgm_memcpy_d2h": (c_int, [c_void_p, c_void_p, c_void_p, c_int64]),
    "hgm_hybrid_ab_gmres_rtp": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, dp, dp, dp, P(c_int)]),
    "hgm_hybrid_ba_gmres_rtp": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, dp, dp, dp, P(c_int)]),
    "hgm_gmres_bounds": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, c_int, c_int, dp, dp, dp, P(c_int)]),
    "hgm_lsqr_solver": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, dp, dp, dp, P(c_int)]),
    "hgm_lsmr_solver": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, dp, dp, dp, dp, P(c_int)]),
    "hgm_hybrid_lsqr_solver": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, dp, dp, dp, P(c_int)]),
    "hgm_hybrid_lsmr_solver": (c_int, [c_void_p, c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, dp, dp, dp, P(c_int)]),
    "hgm_hybrid_ab_gmres_rtp_ex": (c_int, [c_void_p, P(hgm_opts), c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, dp, dp, dp, P(c_int)]),
    "hgm_hybrid_ba_gmres_rtp_ex": (c_int, [c_void_p, P(hgm_opts), c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, dp, dp, dp, P(c_int)]),
    "hgm_gmres_bounds_ex": (c_int, [c_void_p, P(hgm_opts), c_void_p, c_void_p, dp, dp, c_double, c_int, c_double, c_int, c_int, dp, dp, dp, P(c_int)]),
    "hgm_lsqr_solver_ex": (c_int, [c_void_p, P(hgm_opts), c_void_p, c_void_p, dp, dp, c_double, c_int, dp, dp, dp, P(c_int)]),
    "hgm_lsmr_solver_ex": (c_int, [c_void_p, P(hgm_opts), c_void_p, c_void_p, dp, dp, c_double, c_int, dp, dp, dp, dp, P(c_int)]),
    "hgm_arnoldi": (c_int, [c_void_p, c_void_p, c_void_p, dp, c_int, c_int, c_double, c_int, dp, dp, P(c_int)]),
    "hgm_gcv_from_H": (c_int, [dp, c_int, c_double, c_double, c_double, dp]),
    "hgm_gcv_function": (c_int, [c_void_p, c_double, c_void_p, c_void_p, dp, c_int64, c_int, c_int, dp]),
    "hgm_gcv_fminbnd": (c_int, [dp, c_int, c_double, c_double, c_double, c_double, c_double, dp, dp]),
    "hgm_gmres_bounds_filter": (c_int, [c_void_p, P(hgm_opts), c_void_p, c_void_p, dp, dp, c_double, c_int, c_double,
                                        c_int, c_int, c_void_p, c_void_p, c_int, dp, dp, dp, P(c_int), dp, dp, dp, dp]),
    "hgm_filter_factors": (c_int, [dp, c_int, c_int, dp, c_int, dp, dp, c_double, c_int, c_int, dp, dp]),
    "hgm_ritz": (c_int, [dp, c_int, c_int, c_double, dp, c_int, c_int, dp, dp, dp]),
    "hgm_eig": (c_int, [c_int, dp, dp, dp, dp]),
    "hgm_kernel_timing": (c_int, [c_void_p, c_int]),
    "hgm_kernel_timing_read": (c_int, [c_void_p, c_int, dp, ip64, dp]),
    "hgm_kernel_timing_pause": (c_int, [c_void_p, c_int]),
}

_lib = None


def load() -> C.CDLL:
    """Load libhgmres.so (once).  Raises ImportError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libhgmres.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950).  There is no CPU fallback."
        )
    # PyTorch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64.so.1 (same sonames as
    # /opt/rocm's).  Whichever is loaded first serves the process; loading ours first and
    # torch later leaves two HIP runtimes' state in the process and aborts at exit (double
    # free).  So bind to torch's runtime when torch is present.
    try:
        import torch  # noqa: F401
    except ImportError:   # pragma: no cover - torch is plumbing, not required
        pass
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    n, paths = runtime_check(lib)
    if n > 1:
        raise ImportError(f"two HIP runtimes are mapped in this process ({paths}): load PyTorch before "
                          "libhgmres (import hgmres / hgmres.load_library() does), or not at all")
    _lib = lib
    return lib


def runtime_check(lib=None):
    """(number of distinct HIP runtime files mapped, their paths) — hgm_runtime_check."""
    lib = lib or load()
    buf = C.create_string_buffer(4096)
    n = lib.hgm_runtime_check(buf, len(buf))
    return n, buf.value.decode(errors="replace")


def declared_symbols():
    return list(_SIGS)
