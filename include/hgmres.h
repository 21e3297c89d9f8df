/*
 * hgmres.h — C ABI of the MI355X-native Arnoldi/GMRES + Golub–Kahan inner loop.
 *
 * This is the drop-in boundary for the reference's solver functions
 * (luisayang-malaxiangguo/Hybrid-GMRES, pure MATLAB).  The reference has no
 * FFI of its own; each entry point below replaces one MATLAB function with the
 * same positional arguments and output meaning, and is what a MATLAB mex
 * gateway or a ctypes binding calls:
 *
 *   hgm_hybrid_ab_gmres_rtp  <- hybrid_ab_gmres_rtp.m:1   [x,error_norm,residual_norm,niters]
 *   hgm_hybrid_ba_gmres_rtp  <- hybrid_ba_gmres_rtp.m:1   [x,error_norm,residual_norm,niters]
 *   hgm_gmres_bounds         <- ABgmres_hybrid_bounds.m:1-2, ABgmres_nonhybrid_bounds.m:1-2,
 *                               BAgmres_hybrid_bounds.m:1-2, BAgmres_nonhybrid_bounds.m:1-2
 *                               (outputs 1-4; outputs 5-8: hgm_gmres_bounds_filter below)
 *   hgm_lsqr_solver          <- lsqr_solver.m:1           [x,error_norm,residual_norm,niters]
 *   hgm_lsmr_solver          <- lsmr_solver.m:1           [x,err_hist,res_hist,ar_hist,iters]
 *   hgm_hybrid_lsqr_solver   <- hybrid_lsqr_solver.m:1
 *   hgm_hybrid_lsmr_solver   <- hybrid_lsmr_solver.m:1
 *   hgm_gcv_function         <- gcv_function.m:1          gcv_val
 *   hgm_arnoldi / hgm_gcv_from_H  <- gcv_function.m:18-33 / :35-58 split (Arnoldi once, lambda on H;
 *                               pattern of plot_gcv_surface.m:58-122)
 *   hgm_gmres_bounds_filter  <- outputs 5-8 of the four *_bounds.m (phi/dphi filter-factor bounds,
 *                               eig(M) of :4-9 replaced by device Ritz pairs)
 *   hgm_mat_create_csc       <- MATLAB sparse (CSC, jc/ir/pr) operand hand-over
 *   hgm_spmv                 <- the `A*v` / `B*u` / `A'*u` mtimes inside every solver
 *
 * Conventions:
 *   - int status: 0 ok, < 0 error (hgm_last_error(ctx) has the message).  A Krylov
 *     breakdown (H(k+1,k) == 0) is NOT an error: the solver stops with niters = k,
 *     exactly like the reference's `break`.  HGM_E_NOT_ASSIGNED mirrors MATLAB's
 *     'Output argument "x" not assigned' (breakdown at k = 1 where the reference never
 *     assigns x: hybrid_ab_gmres_rtp.m:4,33 and *_bounds.m:37-38,86).
 *   - Caller-owned host buffers: x has size n, histories have size maxit; the
 *     library writes *niters entries (the MATLAB wrapper truncates to 1:niters).
 *   - Matrices are library-owned device objects behind opaque handles.
 *   - One context = one HIP device + one HIP stream; not thread-safe per context.
 *   - Multi-GPU: one process per GPU (hgm_ctx_create_dist over RCCL).  Operators are
 *     pixel-sharded: rank g holds A_g = A(:,P_g) (ray-major CSR, local columns) and
 *     B_g = B(P_g,:); n-vectors (x, x_true) are passed as the rank's shard, m-vectors
 *     (b) replicated on every rank.
 */
#ifndef HGMRES_H
#define HGMRES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HGM_API __attribute__((visibility("default")))

#define HGM_VERSION 100
#define HGM_UNIQUE_ID_BYTES 128

typedef struct hgm_ctx hgm_ctx;
typedef struct hgm_mat hgm_mat;

enum hgm_status {
    HGM_OK = 0,
    HGM_E_ARG = -1,          /* bad argument / dimension mismatch (MATLAB: error()) */
    HGM_E_HIP = -2,          /* HIP runtime error */
    HGM_E_NOMEM = -3,        /* device allocation failed */
    HGM_E_COMM = -4,         /* RCCL / host all-reduce failure */
    HGM_E_NOT_ASSIGNED = -5, /* MATLAB 'Output argument "x" not assigned during call' */
    HGM_E_UNSUPPORTED = -6
};

enum hgm_dtype { HGM_F64 = 0, HGM_F32 = 1 };
enum hgm_orth { HGM_MGS = 0, HGM_CGS2 = 1 };
enum hgm_side { HGM_SIDE_AB = 0, HGM_SIDE_BA = 1 };

/* Flags for the *_ex entry points. */
enum hgm_flags {
    HGM_DEVICE_PTRS = 1,       /* b, x_true, x are device pointers (inputs resident in HBM) */
    HGM_EXPLICIT_RESIDUAL = 2  /* BA-side GMRES: monitor norm(b - A*x) with an explicit SpMV of x
                                  instead of b - (A*Q) y from the kept operator products */
};

typedef struct hgm_opts {
    int flags;        /* hgm_flags */
    int orth;         /* hgm_orth: Arnoldi orthogonalisation (reference: MGS) */
    double* H_out;    /* optional host buffer, (maxit+1) x maxit column-major Hessenberg */
} hgm_opts;

/* Per-context numerics and scheduling options (hgm_ctx_set_option).  Each changes only the
 * context it is set on; nothing is read from the process environment.  Values are passed
 * as doubles (integral options take integral values).  Defaults in brackets. */
enum hgm_ctx_option {
    /* Fixed-order parity mode [0]: every SpMV row is summed sequentially in
     * stored order (scipy's csr_matvec), every dot product / norm in the documented fixed
     * order of oracle/restatement.py's fixed_order() (64-element sequential chunks, twice,
     * then sequential), MGS runs one dot + axpy pass per column exactly as
     * hybrid_ba_gmres_rtp.m:20-26, x = Q*y sums sequentially over the columns, and the
     * monitors are formed explicitly (b - A*x).  Single rank, reference pixel order.  fp64, and
     * fp32 operators for the Golub-Kahan solvers (lsqr_solver / lsmr_solver: float32 vectors and
     * sums in the same order, scalars in double; oracle/restatement.py lsqr_solver_f32).
     * For parity checks only: a fraction of the production kernels' throughput. */
    HGM_OPT_PARITY = 1,
    HGM_OPT_MGS_FORM = 2,          /* MGS for long vectors: 1 one-reduction form [1], 0 one launch per pass */
    HGM_OPT_MGS_SINGLE = 3,        /* one-workgroup MGS sweep for short bases [1] */
    HGM_OPT_GRAM_ERR = 4,          /* Gram error monitor of the n-space GMRES solvers, and of the
                                      AB *_bounds solvers when B is the device transpose of A [1] */
    HGM_OPT_GRAM_ERR_MIN = 5,      /* ... used while ||x-x_true||^2/||x_true||^2 >= this [0.01] */
    HGM_OPT_RING_POLL = 6,         /* single GPU: host polls the pinned ring instead of events [1] */
    HGM_OPT_PEND_NORM = 7,         /* pending normalisation of the Krylov vector: 0 off, 1 n-space [1],
                                      2 n-space and m-space (the one pass over B divides) */
    HGM_OPT_RECON_SERIAL = 8,      /* GMRES reconstruction: -1 automatic [-1], 0 aux stream, 1 main stream */
    HGM_OPT_RECON_SERIAL_N = 9,    /* automatic: serialise from this n on [4194304] */
    HGM_OPT_PIPE_DEPTH = 10,       /* speculative Arnoldi steps in flight, 1..6 [2] */
    HGM_OPT_SYNC_EVENT_FENCE = 11, /* system-scope release on the pipeline events [0] */
    HGM_OPT_MGS_PPL = 12,          /* row pairs per lane of the MGS update / pass kernels [1] */
    HGM_OPT_MGS1_PPL = 13,         /* element pairs per lane of the one-reduction MGS sweep's tiles (one
                                      workgroup per tile): 1, 2, 4, or 0 by vector length [0] */
    HGM_OPT_MGS_FUSED = 14,        /* one-reduction MGS (single rank): the partial-row reduction and the
                                      triangular solve run in the update kernel's prologue, redundantly per
                                      block (2 launches per sweep), instead of a one-block solve kernel [1] */
    HGM_OPT_LSQR_DEV = 15,         /* lsqr_solver / lsmr_solver: beta, alpha, the rotations and the stop test
                                      stay on the device (no host round trip per iteration) [1] */
    HGM_OPT_PAGED16 = 16,          /* streaming SpMV: LDS-paged x gathers also for operators with <= 65,536
                                      columns (instead of their 16-bit column indices) [1] */
    HGM_OPT_BAND_DUAL = 17,        /* banded ray-major operators over a whole tiled N x N grid: rows steeper
                                      than 45 deg are cut into 64-pixel-row strips instead of 64-column strips,
                                      so every ray crosses its strips [1]; read when an operator is banded
                                      (creation, hgm_mat_set_bands) */
    HGM_OPT_FUSED_AB = 18,         /* the m-space operator A*(B*q) of the AB solvers in ONE pass over B's
                                      pixel-major entries when B is A' value for value (a device transpose
                                      pair over a tiled pixel grid, or a pixel shard of whole tile columns
                                      of one: on a communicator every rank runs it on its shard, followed by
                                      the m-vector all-reduce) [1]: the kept B*q and A*(B*q) come out of one
                                      kernel (plan built on first use) */
    /* [experiments] options 19-22, 24, 26-30 and the marked values of 32 and 34 select measured
     * variants of the one-pass kernel (DESIGN.md §3.5 records each measurement): only an experiments
     * build (hgm_experiments() == 1) has their kernels; the default library accepts only the
     * production value in brackets. */
    HGM_OPT_FUSED_REGION = 19,     /* [experiments] kind-0 pass: pixel square per workgroup [64] */
    HGM_OPT_FUSED_BS = 20,         /* [experiments] kind-0 pass: 512 or 1024 threads [1024] */
    HGM_OPT_FUSED_DBG = 21,        /* [experiments] timing only: bits skip the pass's phases, results WRONG;
                                      hgm_spmv_ab only, every solver refuses it [0] */
    HGM_OPT_FUSED_PF = 22,         /* [experiments] kind-0 pass: sub-chunk batches in registers 1..4 [2] */
    HGM_OPT_KRYLOV_PAD = 23        /* elements added to the Krylov basis' leading dimension when it
                                      is a multiple of 4096 (a power-of-two column stride sends
                                      every column's element i to the same HBM channel) [-1 = auto] */,
    HGM_OPT_FUSED_KIND = 24,       /* [experiments] kernel of the one-pass A*(B*q): 0 the sub-chunk pass
                                      (options 19-22), 1 the row-wave pass [1] */
    HGM_OPT_FUSED_WREGION = 25,    /* ... row-wave pass: pixel square (side) per workgroup [32] */
    HGM_OPT_FUSED_WAVES = 26,      /* [experiments] row-wave pass: waves per workgroup, 1, 2 or 4 [4] */
    HGM_OPT_FUSED_GROUP = 27,      /* [experiments] row-wave pass: pixel rows per load batch, 4 or 8 [8] */
    HGM_OPT_FUSED_DEPTH = 28,      /* [experiments] row-wave pass: batches in its load ring, 2..4 [2] */
    HGM_OPT_FUSED_PAIRS = 29,      /* [experiments] row-wave pass: two entries per lane [1] */
    HGM_OPT_FUSED_ACC32 = 30       /* [experiments] fp32 pass (lsqr_solver / lsmr_solver of configs[4]): how a
                                      region's rays accumulate: 0 ds_add_f32, 1 fp32 read-add-write,
                                      2 fp64 accumulators and partials [1] */,
    HGM_OPT_FUSED_PLAN_DEV = 31,   /* ... the row-wave plan's region ray sets and slots built on the device
                                      (an LDS bitmap per region) [1]; 0 the host build (same bytes) */
    HGM_OPT_FUSED_REDUCE = 32,     /* ... the row-wave pass's partial reduction: 1 by bands of 64 rays over
                                      runs of consecutive slots, 0 per ray through its slot list [0] (the
                                      same sums: bitwise equal); [experiments] 2, 3, 4: per ray with 1, 2
                                      or 4 lanes per ray instead of 8 (another fixed order) */
    HGM_OPT_HOST_SPIN_US = 33      /* host waits (stream / event / ring polls): microseconds of pure spinning
                                      before each further poll yields the core (sched_yield) [200; -1 when
                                      the process's CPU affinity holds fewer than 4 cores]; < 0: the
                                      blocking hipStreamSynchronize / hipEventSynchronize.  PROCESS-WIDE: the
                                      last value set on any context applies to every context */,
    HGM_OPT_FUSED_ROWPAIR = 34     /* ... row-wave pass: two consecutive pixel rows per 128-entry chunk [4]:
                                      0 one row per chunk; 4 the second row right after the first, one
                                      accumulator array per wave, the two rows' q reads and adds by two
                                      instructions each (other lanes on their dummy slot); [experiments]
                                      1 (a private array per row parity), 2 (the second row from the lane
                                      after the first row's last pair), 3 (the row split by selects of the
                                      products): the 2048-slot shape only */,
    HGM_OPT_LSQR_RES_IMG = 35      /* one-pass lsqr_solver: the exact final residual norm(b - A*x) of
                                      lsqr_solver.m:52 from A*x kept in double alongside x (A*v_k is the
                                      pass's A*v_hat / alpha) instead of one more SpMV [1] */,
    HGM_OPT_LSMR_FUSE_NMON = 36    /* one-pass lsmr_solver with x_true: the n-space step (:40, :61-67, :72)
                                      and the n-space monitor (:71's A'r image) in one launch [1] (the
                                      same bits as two) */
};

/* Host all-reduce hook (sum, in place, host memory) used instead of RCCL for
 * shard emulation / testing on one device. */
typedef int (*hgm_allreduce_fn)(double* buf, int64_t count, void* user);

/* ---- context ---------------------------------------------------------- */
HGM_API int hgm_version(void);
/* 1 for an experiments build (make EXTRA=-DHGM_EXPERIMENTS=1), which also carries the measured
 * variants of the one-pass kernel that the options marked [experiments] below select; the default
 * library (0) has the production kernels only and refuses those values with HGM_E_ARG. */
HGM_API int hgm_experiments(void);
/* Number of distinct HIP runtime files (libamdhip64*) mapped into the process, their paths
 * ';'-separated in msg.  More than one (e.g. PyTorch's bundled copy loaded AFTER this library
 * pulled /opt/rocm's) is refused: hgm_ctx_create then fails with HGM_E_HIP.  Load PyTorch
 * before this library, or not at all. */
HGM_API int hgm_runtime_check(char* msg, int len);
HGM_API int hgm_device_count(int* count);
HGM_API int hgm_ctx_create(int device, hgm_ctx** ctx);
HGM_API int hgm_comm_unique_id(void* id_out /* HGM_UNIQUE_ID_BYTES */);
/* RCCL context: rank `rank` of `world` on `device`, the id from hgm_comm_unique_id on rank 0.
 * world == 1 with an all-zero id is a plain context; world == 1 with a real id makes a one-rank
 * communicator, so the solvers take the sharded code path with real RCCL all-reduces (the whole
 * operator is the one shard) — rehearses the transport on a single GPU. */
HGM_API int hgm_ctx_create_dist(int device, int rank, int world, const void* unique_id, hgm_ctx** ctx);
HGM_API int hgm_ctx_set_host_allreduce(hgm_ctx* ctx, int rank, int world, hgm_allreduce_fn fn, void* user);
HGM_API void hgm_ctx_destroy(hgm_ctx* ctx);
HGM_API const char* hgm_last_error(const hgm_ctx* ctx);
HGM_API int hgm_ctx_synchronize(hgm_ctx* ctx);
HGM_API void* hgm_ctx_stream(hgm_ctx* ctx);
HGM_API int hgm_ctx_rank(const hgm_ctx* ctx, int* rank, int* world);
/* Free the context's device workspace (the scratch and Krylov buffers its solves grow and keep for
 * reuse; operators are untouched), after the context's streams are idle; *bytes_freed (optional).
 * The next solve allocates again.  For long-lived contexts that share one GPU with other work. */
HGM_API int hgm_ctx_release_workspace(hgm_ctx* ctx, int64_t* bytes_freed);
/* Free and total device memory of the context's GPU (hipMemGetInfo: device-wide, all processes). */
HGM_API int hgm_mem_info(hgm_ctx* ctx, int64_t* free_bytes, int64_t* total_bytes);
/* Path decisions of the context's last solve (test hook: on a communicator every rank must issue
 * the same collective sequence, so these must agree across the ranks).  what = 0: one entry per
 * iteration of the last GMRES-family solve, 1 when that iteration's error monitor came from the
 * Gram form (no x formed, no collective) and 0 when x was formed (an all-reduced error sum);
 * what = 1: one entry, 1 when the last lsqr_solver / lsmr_solver took the one-pass path (agreed
 * over the ranks).  *n = entries available, at most cap written. */
HGM_API int hgm_ctx_solve_path(const hgm_ctx* ctx, int what, int* out, int cap, int* n);
/* Set / read one hgm_ctx_option (HGM_E_ARG for an unknown option or a value out of range). */
HGM_API int hgm_ctx_set_option(hgm_ctx* ctx, int option, double value);
HGM_API int hgm_ctx_get_option(const hgm_ctx* ctx, int option, double* value);

/* ---- sparse operators --------------------------------------------------- */
/* CSR from host arrays (row_ptr: rows+1 int64, col_idx: nnz int32, val: nnz
 * doubles; dtype selects the device storage precision). */
HGM_API int hgm_mat_create_csr(hgm_ctx* ctx, int64_t rows, int64_t cols, int64_t nnz,
                               const int64_t* row_ptr, const int32_t* col_idx,
                               const double* val, int dtype, hgm_mat** out);
/* MATLAB sparse hand-over: CSC of an rows x cols matrix (jc: cols+1, ir: nnz,
 * pr: nnz, 64-bit mwIndex).  The device CSR (row-major) is built by a
 * deterministic device transpose. */
HGM_API int hgm_mat_create_csc(hgm_ctx* ctx, int64_t rows, int64_t cols, int64_t nnz,
                               const int64_t* jc, const int64_t* ir, const double* pr,
                               int dtype, hgm_mat** out);
/* Deterministic device transpose (stable: entries of each output row keep
 * increasing column order). */
HGM_API int hgm_mat_transpose(hgm_ctx* ctx, const hgm_mat* in, hgm_mat** out);
/* Rows [lo, hi) of `in` as a new device operator with the same columns (the pixel
 * shard B_g = B(P_g,:) of SURVEY.md §8(e); A_g = A(:,P_g) is then hgm_mat_transpose of
 * it).  When `in`'s rows are stored tiled (hgm_mat_create_siddon_ordered), [lo, hi) are
 * STORED positions and the slice keeps their stored order as its own (reference) row order:
 * a shard of whole tile columns keeps the tiled gather locality (hgmres.core.stored_pixel_index
 * maps reference pixels to stored positions). */
HGM_API int hgm_mat_row_slice(hgm_ctx* ctx, const hgm_mat* in, int64_t lo, int64_t hi, hgm_mat** out);
/* Parallel-beam Siddon projector generated on the device (ray-major CSR,
 * bit-compatible geometry with hgmres.problems.siddon_projector). */
HGM_API int hgm_mat_create_siddon(hgm_ctx* ctx, int N, int n_angles, double det_offset,
                                  int dtype, hgm_mat** out);
/* The same operator with its N x N pixel (column) space STORED in a tiled order: tile x tile
 * tiles (4 x 4 fp64 = one 128-B line) inside super x super blocks (0 = none).  This is
 * invisible at the boundary: hgm_spmv, hgm_mat_download and every solver take and return
 * vectors and indices in the reference's column-major x(:) order; the permutation is
 * applied once per vector on the way in and out.  Transposes inherit it (rows of A').
 * tile must divide N (and super); super must divide N. */
HGM_API int hgm_mat_create_siddon_ordered(hgm_ctx* ctx, int N, int n_angles, double det_offset,
                                          int dtype, int tile, int super_block, hgm_mat** out);
/* Fan-beam projector with a curved (equiangular) detector generated on the device, standing in
 * for the CTtype 'fancurved' of run_2D_phantom.m:12-13.  PRtomo_mismatched is not vendored by the
 * reference, so the geometry is this library's own choice (hgmres.problems.fan_geometry lists its
 * departures from AIR Tools II fanbeamtomo; parity with either is unpinned), bit-identical to
 * hgmres.problems.fanbeam_projector: n_angles source positions over a full turn
 * at distance R*N from the centre (R > 1/sqrt(2)), p = ceil(sqrt(2) N) rays per source at
 * equiangular fan angles ((d - (p-1)/2) + det_offset) * span / p; span <= 0 selects the fan that
 * covers the image's circumscribed circle, 2 asin(1 / (sqrt(2) R)).  Rows a*p + d; tile /
 * super_block: stored pixel (column) order as for hgm_mat_create_siddon_ordered. */
HGM_API int hgm_mat_create_fanbeam(hgm_ctx* ctx, int N, int n_angles, double R, double span, double det_offset,
                                   int dtype, int tile, int super_block, hgm_mat** out);
/* Unmatched pixel-driven back-projector B (n x m, pixel-major) generated on the device:
 * for every pixel centre and angle, linear interpolation between the two nearest detector
 * bins (bit-identical to hgmres.problems.pixel_driven_backprojector; the role of
 * PRtomo_mismatched in run_2D_phantom.m:13-14).  tile/super_block: stored row (pixel) order,
 * as for hgm_mat_create_siddon_ordered, so B pairs with an operator of the same order. */
HGM_API int hgm_mat_create_backprojector(hgm_ctx* ctx, int N, int n_angles, double det_offset, int dtype,
                                         int tile, int super_block, hgm_mat** out);
/* Stored order of the row (which = 0) or column (which = 1) index space: N = 0 means the
 * reference order. */
HGM_API int hgm_mat_order(const hgm_mat* mat, int which, int* N, int* tile, int* super_block);
HGM_API int hgm_mat_info(const hgm_mat* mat, int64_t* rows, int64_t* cols, int64_t* nnz, int* dtype);
/* SpMV kernel selection for this operator (tuning/benchmark hook): variant bits
 * 1 = 16-byte paired loads, 2 = nontemporal val/col loads, 4 = XCD-aware row-block
 * order, 8 = nnz-balanced streaming kernel (4096-entry chunks, LDS-staged products),
 * 16 = with the streaming kernel, gather x through LDS-staged 128-B pages (the operator's page
 * index; streaming operators are created with it);
 * group = lanes per row, or per segment reduction with bit 8 (4, 8, 16, 32 or 64;
 * 0 keeps the current choice). */
HGM_API int hgm_mat_tune(hgm_mat* mat, int variant, int group);
/* Column banding of the SpMV x-gather (cache blocking): band_width pixels per band
 * (0 = off, -1 = automatic: on for long-row operators whose x exceeds one XCD's L2),
 * group = lanes per (band,row) segment (0 = automatic).  Operators are created with
 * the automatic choice. */
HGM_API int hgm_mat_set_bands(hgm_ctx* ctx, hgm_mat* mat, int64_t band_width, int group);
HGM_API int hgm_mat_download(hgm_ctx* ctx, const hgm_mat* mat, int64_t* row_ptr, int32_t* col_idx, double* val);
HGM_API void hgm_mat_destroy(hgm_mat* mat);

/* y = A*x on device pointers (elements of the matrix dtype), on the context stream. */
HGM_API int hgm_spmv(hgm_ctx* ctx, const hgm_mat* A, const void* x_dev, void* y_dev);

/* The m-space operator of the AB solvers (ABgmres_*_bounds.m:25, gcv_function.m:20):
 * Bq = B*q (n) and ABq = A*(B*q) (m), device pointers, on the context stream.  When B is A' value
 * for value (hgm_mat_transpose) over a tiled pixel grid, fp64, one rank, both come out of ONE pass
 * over B's entries (HGM_OPT_FUSED_AB; the plan is built on first use); otherwise two SpMVs.  Bq is
 * in the reference pixel order, as hgm_spmv's. */
HGM_API int hgm_spmv_ab(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* B, const void* q_dev, void* Bq_dev,
                        void* ABq_dev);
/* The one-pass plan of the pair (A, B) under the context's current options, built if it is not
 * yet: the seconds its build took, a 64-bit FNV-1a checksum over every plan array (so two builds
 * can be compared byte for byte), the partial slots, and whether the device built the ray sets
 * (HGM_OPT_FUSED_PLAN_DEV).  HGM_E_ARG when the pair has no plan (two-pass path). */
HGM_API int hgm_fused_plan_info(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* B, double* build_s,
                                uint64_t* checksum, int64_t* nslot, int* device_built);

/* ---- device memory helpers (for callers without their own allocator) ---- */
HGM_API int hgm_dev_alloc(hgm_ctx* ctx, int64_t bytes, void** ptr);
HGM_API int hgm_dev_free(hgm_ctx* ctx, void* ptr);
HGM_API int hgm_memcpy_h2d(hgm_ctx* ctx, void* dst, const void* src, int64_t bytes);
HGM_API int hgm_memcpy_d2h(hgm_ctx* ctx, void* dst, const void* src, int64_t bytes);

/* ---- solvers (MATLAB signatures; host buffers) --------------------------- */
HGM_API int hgm_hybrid_ab_gmres_rtp(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* B,
                                    const double* b, const double* x_true, double tol, int maxit,
                                    double lambda, double* x, double* error_norm,
                                    double* residual_norm, int* niters);
HGM_API int hgm_hybrid_ba_gmres_rtp(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* B,
                                    const double* b, const double* x_true, double tol, int maxit,
                                    double lambda, double* x, double* error_norm,
                                    double* residual_norm, int* niters);
/* side = HGM_SIDE_AB (m-space Arnoldi on A*B) or HGM_SIDE_BA (n-space on B*A);
 * hybrid = 1: PTR Tikhonov (HkᵀHk+λI)\(Hkᵀ t), 0: GMRES Hk\βe1. */
HGM_API int hgm_gmres_bounds(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* B, const double* b,
                             const double* x_true, double tol, int maxit, double lambda, int side,
                             int hybrid, double* x, double* error_norm, double* residual_norm,
                             int* niters);
HGM_API int hgm_lsqr_solver(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* At, const double* b,
                            const double* x_true, double tol, int maxit, double* x,
                            double* error_norm, double* residual_norm, int* niters);
/* x_true may be NULL (err_hist stays NaN, lsmr_solver.m:28,72). */
HGM_API int hgm_lsmr_solver(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* At, const double* b,
                            const double* x_true, double tol, int maxit, double* x,
                            double* err_hist, double* res_hist, double* ar_hist, int* iters);
HGM_API int hgm_hybrid_lsqr_solver(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* At,
                                   const double* b, const double* x_true, double tol, int maxit,
                                   double lambda, double* x, double* error_norm,
                                   double* residual_norm, int* niters);
HGM_API int hgm_hybrid_lsmr_solver(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* At,
                                   const double* b, const double* x_true, double tol, int maxit,
                                   double lambda, double* x, double* error_norm,
                                   double* residual_norm, int* niters);

/* Extended forms: options (device pointers, orthogonalisation, Hessenberg out). */
HGM_API int hgm_hybrid_ab_gmres_rtp_ex(hgm_ctx* ctx, const hgm_opts* opts, const hgm_mat* A,
                                       const hgm_mat* B, const double* b, const double* x_true,
                                       double tol, int maxit, double lambda, double* x,
                                       double* error_norm, double* residual_norm, int* niters);
HGM_API int hgm_hybrid_ba_gmres_rtp_ex(hgm_ctx* ctx, const hgm_opts* opts, const hgm_mat* A,
                                       const hgm_mat* B, const double* b, const double* x_true,
                                       double tol, int maxit, double lambda, double* x,
                                       double* error_norm, double* residual_norm, int* niters);
HGM_API int hgm_gmres_bounds_ex(hgm_ctx* ctx, const hgm_opts* opts, const hgm_mat* A,
                                const hgm_mat* B, const double* b, const double* x_true, double tol,
                                int maxit, double lambda, int side, int hybrid, double* x,
                                double* error_norm, double* residual_norm, int* niters);
HGM_API int hgm_lsqr_solver_ex(hgm_ctx* ctx, const hgm_opts* opts, const hgm_mat* A,
                               const hgm_mat* At, const double* b, const double* x_true, double tol,
                               int maxit, double* x, double* error_norm, double* residual_norm,
                               int* niters);
HGM_API int hgm_lsmr_solver_ex(hgm_ctx* ctx, const hgm_opts* opts, const hgm_mat* A,
                               const hgm_mat* At, const double* b, const double* x_true, double tol,
                               int maxit, double* x, double* err_hist, double* res_hist,
                               double* ar_hist, int* iters);

/* ---- GCV (gcv_function.m) ------------------------------------------------ */
/* Arnoldi only: H is (k+1) x k column-major (zero columns kept after a break,
 * gcv_function.m:33); *kdone = steps completed before the < breakdown_tol break. */
HGM_API int hgm_arnoldi(hgm_ctx* ctx, const hgm_mat* A, const hgm_mat* B, const double* b,
                        int k, int side, double breakdown_tol, int orth, double* H,
                        double* beta, int* kdone);
/* λ-dependent part of gcv_function.m:35-58 on a cached H (host only). */
HGM_API int hgm_gcv_from_H(const double* H, int k, double beta, double lambda, double trace_m,
                           double* gcv_val);
HGM_API int hgm_gcv_function(hgm_ctx* ctx, double lambda, const hgm_mat* A, const hgm_mat* B,
                             const double* b, int64_t m, int k_gcv, int side, double* gcv_val);
/* fminbnd (Brent) over λ ∈ [lo, hi] of GCV on one cached Arnoldi (analyze_regularization.m:37-46). */
HGM_API int hgm_gcv_fminbnd(const double* H, int k, double beta, double trace_m, double lo,
                            double hi, double tolx, double* lambda_opt, double* gcv_opt);

/* ---- filter-factor / perturbation bounds (outputs 5-8 of *_bounds.m) ---------
 * ABgmres_hybrid_bounds.m:1-2, ABgmres_nonhybrid_bounds.m:1-2, BAgmres_hybrid_bounds.m:1-2,
 * BAgmres_nonhybrid_bounds.m:1-2: [x, err, res, niters, phi_final, dphi_final, phi_iter, dphi_iter].
 * The dense eig(M) of *_bounds.m:4-9 is replaced by the Ritz pairs of a ritz_steps-step Arnoldi
 * on M = A*B (AB) / B*A (BA) with CGS2 (ritz_steps = dim reproduces eig(M); 0 = automatic,
 * max(2 niters + 10, 20) capped at dim).  DeltaM = dM_left (dim x dim), or dM_left * dM_right
 * when dM_right != NULL (e.g. A*E / E*A of analyze_regularization.m:14-15, never formed).
 * phi_iter / dphi_iter: maxit x maxit column-major, column k-1 holds iteration k's k values
 * (phi_final = column niters-1).  mu (optional, niters): the Ritz values used (mu_full(1:k));
 * ritz_resid (optional, niters): ||M u_i - mu_i u_i||.  Complex Ritz pairs: the real parts, as
 * the reference's real(diag(D)); their dMu is the phase-invariant Re(y^H G y).  Single rank. */
HGM_API int hgm_gmres_bounds_filter(hgm_ctx* ctx, const hgm_opts* opts, const hgm_mat* A, const hgm_mat* B,
                                    const double* b, const double* x_true, double tol, int maxit, double lambda,
                                    int side, int hybrid, const hgm_mat* dM_left, const hgm_mat* dM_right,
                                    int ritz_steps, double* x, double* error_norm, double* residual_norm,
                                    int* niters, double* phi_iter, double* dphi_iter, double* mu,
                                    double* ritz_resid);
/* Host only: phi / dphi of iteration k (*_bounds.m:42-78) from H ((k+1) x k leading part of a
 * column-major array with leading dimension ldh), dK = Qk' DeltaM Qk (k x k, lddk), the k
 * leading eigenvalues mu of M (descending) and dmu_i = u_i' DeltaM u_i. */
HGM_API int hgm_filter_factors(const double* H, int ldh, int k, const double* dK, int lddk, const double* mu,
                               const double* dmu, double lambda, int side, int hybrid, double* phi, double* dphi);
/* Host only: the nev leading Ritz pairs (descending real part) of a p-step Arnoldi (Hp: p x p,
 * ldh; h_next = H(p+1,p)) with dmu_i = y_i' G y_i (G = Qp' DeltaM Qp, p x p, ldg) and
 * resid_i = |h_next| |e_p' y_i| (optional). */
HGM_API int hgm_ritz(const double* Hp, int ldh, int p, double h_next, const double* G, int ldg, int nev, double* mu,
                     double* dmu, double* resid);
/* Host only: MATLAB eig of a real n x n column-major matrix: eigenvalues wr + i wi, unit 2-norm
 * eigenvectors in V (optional, LAPACK dgeev layout: a complex pair j, j+1 with wi[j] > 0 has
 * V(:,j) +- i V(:,j+1)).  HGM_E_ARG when the QR iteration does not converge. */
HGM_API int hgm_eig(int n, const double* A, double* wr, double* wi, double* V);

/* ---- timing hooks used by bench.py ---------------------------------------- */
/* Average device time (ms) of the named kernel class over the calls since the
 * last reset, measured with HIP events on the context stream.  classes:
 * 0 = SpMV on A (ray-major), 1 = SpMV on B/Aᵀ (pixel-major), 2 = MGS pass.
 * enable: 0 = off, 1 = every class, HGM_TIMING_CLASSES(mask) = only the classes whose
 * bit is set (each timed launch carries events, so time only what is read). */
#define HGM_TIMING_CLASSES(mask) (0x100 | (mask))
HGM_API int hgm_kernel_timing(hgm_ctx* ctx, int enable);
HGM_API int hgm_kernel_timing_read(hgm_ctx* ctx, int cls, double* total_ms, int64_t* calls,
                                   double* bytes);
/* Pause (1) / resume (0) the armed timing without a sync or a reset: launches enqueued
 * while paused carry no events (bench.py times a sample of the solves in its timed region). */
HGM_API int hgm_kernel_timing_pause(hgm_ctx* ctx, int paused);

#ifdef __cplusplus
}
#endif
#endif /* HGMRES_H */
