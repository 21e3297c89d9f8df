import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hybrid-gmres_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def golden_problem(name):
    """(A, B, b, x_true, fixture) from a golden npz with raw operators."""
    import scipy.sparse as sp
    g = load_golden(name)
    shape = tuple(int(v) for v in g["shape"])
    A = sp.csr_matrix((g["A_data"], g["A_indices"], g["A_indptr"]), shape=shape)
    B = sp.csr_matrix((g["B_data"], g["B_indices"], g["B_indptr"]), shape=(shape[1], shape[0]))
    return A, B, g["b"], g["x_true"], g


@pytest.fixture(scope="session")
def gpu_ctx():
    import hgmres
    n = _device_count()
    if n < 1:
        pytest.fail("no HIP device visible for a -m gpu test")
    return hgmres.default_context()


def _device_count():
    import ctypes
    import hgmres
    lib = hgmres.load_library()
    c = ctypes.c_int(0)
    lib.hgm_device_count(ctypes.byref(c))
    return c.value
