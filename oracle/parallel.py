"""ORACLE — all-core operator wrapper for the bench's cpu_baseline leg (test infrastructure).

:class:`ParallelCSR` wraps a CSR matrix so that ``M @ v`` runs ``oracle/spmv_omp.c``
(rows split over OpenMP threads, each row summed sequentially in stored order, no
FMA): bitwise the same product as scipy's single-threaded ``csr_matvec`` that
``oracle/restatement.py`` uses, on every host core.  The restatement's solvers take it
unchanged (they only use ``@``, ``.T``, ``.shape`` and ``fro_norm``).

Build: ``__graft_entry__.build()`` compiles ``oracle/_build/liboracle_spmv.so``
(``gcc -O3 -fopenmp -ffp-contract=off``).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle_spmv.so")
_lib = None


def build(force=False):
    """Compile the OpenMP SpMV (CPU only; no ROCm involved)."""
    if os.path.exists(LIB) and not force and os.path.getmtime(LIB) >= os.path.getmtime(
            os.path.join(HERE, "spmv_omp.c")):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["gcc", "-O3", "-fopenmp", "-ffp-contract=off", "-shared", "-fPIC",
                    os.path.join(HERE, "spmv_omp.c"), "-o", LIB], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
        lib = C.CDLL(LIB)
        P = C.POINTER
        lib.oracle_csr_matvec.argtypes = [C.c_int64, P(C.c_int64), P(C.c_int32), P(C.c_double), P(C.c_double),
                                          P(C.c_double)]
        lib.oracle_csr_matvec.restype = None
        lib.oracle_csr_matvec_f32.argtypes = [C.c_int64, P(C.c_int64), P(C.c_int32), P(C.c_float), P(C.c_float),
                                              P(C.c_float)]
        lib.oracle_csr_matvec_f32.restype = None
        lib.oracle_csr_matvec_f32_order.argtypes = [C.c_int64, P(C.c_int64), P(C.c_int32), P(C.c_float),
                                                    P(C.c_float), P(C.c_float), C.c_int, C.c_int]
        lib.oracle_csr_matvec_f32_order.restype = None
        lib.oracle_num_threads.restype = C.c_int
        _lib = lib
    return _lib


def num_threads() -> int:
    return int(load().oracle_num_threads())


class ParallelCSR:
    """CSR operator for the oracle whose products run on all host cores.  ``T`` may be
    given (an explicit transpose, e.g. the device's ``A'``); otherwise it is formed once
    with scipy (``M.T.tocsr()``, whose rows keep increasing column order: the order in
    which scipy's ``csc_matvec`` accumulates ``M.T @ u``).  A float32 M keeps float32 values
    and computes in single precision (scipy's ``csr_matvec<float>``), for the fp32 oracle."""

    def __init__(self, M, T=None):
        M = sp.csr_matrix(M)
        self.M = M
        self.shape = M.shape
        self.dtype = np.float32 if M.dtype == np.float32 else np.float64
        self.rp = np.ascontiguousarray(M.indptr, dtype=np.int64)
        self.ci = np.ascontiguousarray(M.indices, dtype=np.int32)
        self.val = np.ascontiguousarray(M.data, dtype=self.dtype)
        self._T = T
        load()

    @property
    def T(self):
        if self._T is None:
            self._T = ParallelCSR(self.M.T.tocsr())
            self._T._T = self
        return self._T

    def _mv(self, v):
        if self.dtype == np.float32:
            if np.asarray(v).dtype != np.float32:
                raise TypeError("fp32 operator: the vector must be float32")
            v = np.ascontiguousarray(v, dtype=np.float32)
            y = np.empty(self.shape[0], dtype=np.float32)
            fp = C.POINTER(C.c_float)
            load().oracle_csr_matvec_f32(self.shape[0], self.rp.ctypes.data_as(C.POINTER(C.c_int64)),
                                         self.ci.ctypes.data_as(C.POINTER(C.c_int32)), self.val.ctypes.data_as(fp),
                                         v.ctypes.data_as(fp), y.ctypes.data_as(fp))
            return y
        v = np.ascontiguousarray(v, dtype=np.float64)
        y = np.empty(self.shape[0])
        dp = C.POINTER(C.c_double)
        load().oracle_csr_matvec(self.shape[0], self.rp.ctypes.data_as(C.POINTER(C.c_int64)),
                                 self.ci.ctypes.data_as(C.POINTER(C.c_int32)), self.val.ctypes.data_as(dp),
                                 v.ctypes.data_as(dp), y.ctypes.data_as(dp))
        return y

    def matvec_f32_order(self, v, ways, rev):
        """fp32 product in another summation order (spmv_omp.c oracle_csr_matvec_f32_order)."""
        assert self.dtype == np.float32
        v = np.ascontiguousarray(v, dtype=np.float32)
        y = np.empty(self.shape[0], dtype=np.float32)
        fp = C.POINTER(C.c_float)
        load().oracle_csr_matvec_f32_order(self.shape[0], self.rp.ctypes.data_as(C.POINTER(C.c_int64)),
                                           self.ci.ctypes.data_as(C.POINTER(C.c_int32)),
                                           self.val.ctypes.data_as(fp), v.ctypes.data_as(fp),
                                           y.ctypes.data_as(fp), int(ways), int(rev))
        return y

    def __matmul__(self, v):
        v = np.asarray(v)
        if v.ndim == 1:
            return self._mv(v)
        return np.stack([self._mv(v[:, j]) for j in range(v.shape[1])], axis=1)

    def fro_norm(self):
        return float(np.linalg.norm(self.val.astype(np.float64)))
