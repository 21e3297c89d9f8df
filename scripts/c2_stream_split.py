"""Attribution of the C2 ray-major A SpMV's HBM traffic (VERDICT r4 "Next" #6): the same CSR
streamed with its real column indices and with every column index set to 0 (the x gathers then hit
one line, so the counters see the val/col stream alone).  The difference is the x-gather traffic.
Run under rocprofv3 --pmc (one counter group per run), once per mode:
    python scripts/c2_stream_split.py real|zero|tiled [reps]
real / zero: the reference-order operator uploaded from the host (identical kernel and launch),
tiled: the bench's device-generated 4 x 4-tiled operator.  The kernel is launched `reps` times
(default 50) after one warm-up."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-gmres_amd"), ROOT]
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import torch  # noqa: E402,F401
import hgmres  # noqa: E402
from hgmres import _lib as L  # noqa: E402

mode = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ctx = hgmres.Context(0)
At = hgmres.SparseOperator.siddon(512, 30, ctx=ctx)
if mode == "tiled":
    A = At
else:
    S = At.to_scipy()
    if mode == "zero":
        S = sp.csr_matrix((S.data, np.zeros_like(S.indices), S.indptr), shape=S.shape)
    A = hgmres.SparseOperator.from_scipy(S, ctx)
m, n = A.shape
dev = torch.device("cuda", 0)
x = torch.from_numpy(np.random.default_rng(0).standard_normal(n)).to(dev)
y = torch.empty(m, dtype=torch.float64, device=dev)
lib = L.load()
P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
# the stored-order product (no permutation kernels around it): hgm_spmv takes reference-order
# vectors, so for the tiled operator the two pix_permute launches show up beside it in the trace
for _ in range(reps + 1):
    assert lib.hgm_spmv(ctx.handle, A._h, P(x), P(y)) == 0
ctx.synchronize()
print({"mode": mode, "m": m, "n": n, "nnz": A.nnz, "reps": reps,
       "algorithmic_bytes": 12.0 * A.nnz + 8.0 * (m + 1) + 8.0 * n + 8.0 * m})
