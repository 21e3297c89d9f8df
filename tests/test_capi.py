"""CPU-side checks of the C-ABI library (no GPU needed): it loads, exports every
symbol include/hgmres.h declares, and its host-only dense code (projected
solves / GCV / fminbnd) agrees with the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.optimize as so

from conftest import ROOT
import hgmres
from hgmres import _lib as L
from hgmres.problems import tomo_problem
from oracle import restatement as R


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "hgmres.h")).read()
    return sorted(set(re.findall(r"HGM_API\s+[\w\s\*]+?\b(hgm_\w+)\s*\(", txt)))


def test_library_loads_and_exports_header_symbols():
    lib = hgmres.load_library()
    syms = header_symbols()
    assert len(syms) >= 40
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(L.declared_symbols())     # the ctypes binding covers the whole ABI
    assert lib.hgm_version() == 100


def test_exported_symbol_table_is_exactly_the_header():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(l.split()[-1] for l in out.splitlines() if " T " in l)
    assert exported == header_symbols()


def test_bad_arguments_without_gpu():
    lib = hgmres.load_library()
    assert lib.hgm_ctx_create(0, None) == L.HGM_E_ARG
    assert lib.hgm_mat_create_csr(None, 1, 1, 0, None, None, None, 0, None) == L.HGM_E_ARG
    assert lib.hgm_gcv_from_H(None, 3, 1.0, 1.0, 10.0, None) == L.HGM_E_ARG


@pytest.fixture(scope="module")
def H_case():
    P = tomo_problem(24, 12, noise=1e-2, seed=0, backprojector="pixel")
    H, beta = R.arnoldi(P.A, P.B, P.b, 10, "ba")
    return P, H, beta


def test_gcv_from_H_host_code_matches_oracle(H_case):
    P, H, beta = H_case
    for lam in (1e-8, 1e-5, 1e-3, 1e-1):
        g = hgmres.gcv_from_H(H, beta, lam, P.A.shape[1])
        gr = R.gcv_from_H(H, beta, lam, P.A.shape[1])
        assert abs(g - gr) <= 1e-10 * abs(gr)


def test_gcv_fallback_value(H_case):
    # singular projected system -> NaN -> 1e20 (gcv_function.m:56-57), as the oracle
    P, H, beta = H_case
    Hz = np.zeros_like(H)
    assert R.gcv_from_H(Hz, 0.0, 0.0, 0.0) == 1e20
    assert hgmres.gcv_from_H(Hz, 0.0, 0.0, 0.0) == 1e20


def test_gcv_fminbnd_host_code(H_case):
    P, H, beta = H_case
    f = lambda l: R.gcv_from_H(H, beta, l, P.A.shape[1])   # noqa: E731
    lam, gv = hgmres.gcv_fminbnd(H, beta, P.A.shape[1], 1e-9, 1e-1, 1e-8)
    ls = so.fminbound(f, 1e-9, 1e-1, xtol=1e-8)
    assert 1e-9 <= lam <= 1e-1
    assert f(lam) <= f(ls) * (1 + 1e-8) + 1e-300


def test_no_cpu_fallback_without_device():
    """The product path fails loudly instead of falling back to the CPU."""
    n = ctypes.c_int(0)
    hgmres.load_library().hgm_device_count(ctypes.byref(n))
    if n.value > 0:
        pytest.skip("a device is visible")
    with pytest.raises(hgmres.HgmError):
        hgmres.Context(0)


def test_hip_runtime_order_guard(tmp_path):
    """One HIP runtime per process.  hgmres loads PyTorch's runtime
    before libhgmres, so importing torch afterwards maps no second copy and the process
    exits 0; loading libhgmres by hand BEFORE torch maps two runtimes, which
    hgm_runtime_check reports and hgm_ctx_create refuses (that process still aborts in the
    runtimes' exit handlers, hence only its output is checked)."""
    import subprocess
    import sys
    pkg = os.path.join(ROOT, "hybrid-gmres_amd")
    good = subprocess.run([sys.executable, "-c",
                           f"import sys; sys.path.insert(0, {pkg!r})\n"
                           "import hgmres; from hgmres import _lib as L\n"
                           "hgmres.load_library(); import torch\n"
                           "print(L.runtime_check()[0])"], capture_output=True, text=True, timeout=300,
                          cwd=str(tmp_path))
    assert good.returncode == 0, good.stderr[-2000:]
    assert good.stdout.strip().splitlines()[-1] == "1"
    bad = subprocess.run([sys.executable, "-c",
                          "import ctypes\n"
                          f"lib = ctypes.CDLL({L.LIB_PATH!r}, mode=ctypes.RTLD_GLOBAL)\n"
                          "import torch\n"
                          "buf = ctypes.create_string_buffer(4096)\n"
                          "h = ctypes.c_void_p()\n"
                          "print(lib.hgm_runtime_check(buf, 4096), lib.hgm_ctx_create(0, ctypes.byref(h)), flush=True)\n"],
                         capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert bad.stdout.split()[:2] == ["2", str(L.HGM_E_HIP)], (bad.stdout, bad.stderr[-2000:])


def test_ctx_option_api_without_gpu():
    lib = hgmres.load_library()
    v = ctypes.c_double()
    assert lib.hgm_ctx_set_option(None, 1, 1.0) == L.HGM_E_ARG
    assert lib.hgm_ctx_get_option(None, 1, ctypes.byref(v)) == L.HGM_E_ARG
    assert set(L.OPTIONS.values()) == set(range(1, 37))
    txt = open(os.path.join(ROOT, "include", "hgmres.h")).read()
    for name, val in L.OPTIONS.items():   # the Python names mirror the header's enum
        assert re.search(rf"HGM_OPT_{name.upper()}\s*=\s*{val}\b", txt), name


def test_default_build_is_not_the_experiments_build():
    """the default library carries the production one-pass kernels only; the
    measured variants live in an experiments build (hgm_experiments() == 1, make
    EXTRA=-DHGM_EXPERIMENTS=1).  The header marks their option values [experiments]."""
    lib = hgmres.load_library()
    if os.environ.get("HGM_LIB"):
        pytest.skip("HGM_LIB selects another build")
    assert lib.hgm_experiments() == 0
    txt = open(os.path.join(ROOT, "include", "hgmres.h")).read()
    for opt in ("HGM_OPT_FUSED_DBG", "HGM_OPT_FUSED_KIND", "HGM_OPT_FUSED_WAVES", "HGM_OPT_FUSED_ACC32"):
        line = [l for l in txt.splitlines() if opt + " =" in l][0]
        assert "[experiments]" in line, opt


def test_new_ctx_calls_reject_null_without_gpu():
    """hgm_ctx_solve_path / hgm_ctx_release_workspace / hgm_mem_info on a NULL context: HGM_E_ARG."""
    lib = hgmres.load_library()
    n = ctypes.c_int()
    assert lib.hgm_ctx_solve_path(None, 0, None, 0, ctypes.byref(n)) == L.HGM_E_ARG
    assert lib.hgm_ctx_release_workspace(None, None) == L.HGM_E_ARG
    assert lib.hgm_mem_info(None, None, None) == L.HGM_E_ARG
