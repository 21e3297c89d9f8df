"""hgmres — MI355X-native Arnoldi/GMRES + Golub–Kahan inner loop behind the
reference's MATLAB solver signatures (luisayang-malaxiangguo/Hybrid-GMRES).

The compute path is ``libhgmres.so`` (hand-written HIP for gfx950, C ABI in
``include/hgmres.h``); this package is the thin host mirror of the reference
interface plus the synthetic 2-D tomography problem generator.
"""
from .core import spmv_ab, fused_plan_info  # noqa: F401
from .core import (  # noqa: F401
    ABgmres_hybrid_bounds,
    ABgmres_nonhybrid_bounds,
    BAgmres_hybrid_bounds,
    BAgmres_nonhybrid_bounds,
    Context,
    HgmError,
    OutputNotAssigned,
    SparseOperator,
    arnoldi,
    as_operator,
    default_context,
    eig,
    filter_factors,
    ritz,
    gcv_fminbnd,
    gcv_from_H,
    gcv_function,
    hybrid_ab_gmres_rtp,
    hybrid_ba_gmres_rtp,
    hybrid_lsmr_solver,
    hybrid_lsqr_solver,
    lsmr_solver,
    lsqr_solver,
)
from . import problems  # noqa: F401
from . import regtools  # noqa: F401
from . import analysis  # noqa: F401
from ._lib import LIB_PATH, load as load_library  # noqa: F401

__all__ = [
    "hybrid_ab_gmres_rtp", "hybrid_ba_gmres_rtp", "lsqr_solver", "lsmr_solver",
    "hybrid_lsqr_solver", "hybrid_lsmr_solver", "gcv_function", "arnoldi", "gcv_from_H",
    "gcv_fminbnd", "ABgmres_hybrid_bounds", "ABgmres_nonhybrid_bounds",
    "BAgmres_hybrid_bounds", "BAgmres_nonhybrid_bounds", "Context", "SparseOperator",
    "as_operator", "default_context", "HgmError", "OutputNotAssigned", "problems", "regtools", "analysis",
    "eig", "filter_factors", "ritz",
]
