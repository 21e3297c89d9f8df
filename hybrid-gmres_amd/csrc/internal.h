// Internal declarations of libhgmres (MI355X / gfx950).  Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "hgmres.h"

// Measured variants of the one-pass kernel (the kind-0 sub-chunk pass, row-pair modes 1-3, other
// wave / batch / depth / pairing shapes, other fp32 accumulations and reductions, the phase-skipping
// timing bits) are compiled only into an experiments build (make EXTRA=-DHGM_EXPERIMENTS=1, used by
// scripts/fused_micro.py); the default library carries the production kernels alone and refuses
// those option values (hgm_ctx_set_option, hgm_experiments()).
#ifndef HGM_EXPERIMENTS
#define HGM_EXPERIMENTS 0
#endif

namespace hgm {

struct Error {
    int code;
    std::string msg;
};

#define HGM_HIP(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            throw ::hgm::Error{HGM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)}; \
    } while (0)

#define HGM_REQUIRE(cond, msg)                                \
    do {                                                      \
        if (!(cond)) throw ::hgm::Error{HGM_E_ARG, (msg)};    \
    } while (0)

constexpr int BS = 256;              // threads per block (4 waves of 64)
constexpr int MAX_PARTS = 1024;      // max blocks of a partial-sum reduction
constexpr int NSCAL = 512;           // device scalar slots per context

// Device allocation that grows on demand and is reused across solves.
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t b);
    void release();
    ~DevBuf() { release(); }
};

// Kernel classes timed by hgm_kernel_timing (bench roofline).
enum KClass { KC_SPMV_A = 0, KC_SPMV_B = 1, KC_MGS = 2, KC_FUSED = 3, KC_N = 4 };

struct Timing {
    bool on = false;
    bool paused = false;   // hgm_kernel_timing_pause: armed but not recording
    unsigned mask = 0xffu;   // timed classes
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[KC_N];
    double bytes[KC_N] = {0, 0, 0, 0};
    std::vector<hipEvent_t> pool;
    hipEvent_t get();
    void clear();
};

// Per-context numerics / scheduling options (hgm_ctx_set_option; defaults = production).
struct Numerics {
    bool parity = false;            // HGM_OPT_PARITY: fixed-order parity mode
    int mgs_form = 1;               // 1 one-reduction MGS, 0 one launch per pass
    bool mgs_single = true;         // one-workgroup sweep for short bases
    bool gram_err = true;           // Gram error monitor
    double gram_err_min = 0.01;
    bool ring_poll = true;
    int pend_norm = 1;              // 1: n-space (SpMV epilogues); 2: also m-space (the one pass)
    int recon_serial = -1;          // -1 automatic, 0 aux stream, 1 main stream
    int64_t recon_serial_n = int64_t(4) << 20;
    int pipe_depth = 2;
    bool sync_event_fence = false;
    int mgs_ppl = 1;
    int mgs1_ppl = 0;               // one-reduction sweep: element pairs per lane of a tile (0: by length)
    bool mgs_fused = true;          // one-reduction MGS: solve folded into the update kernel
    bool lsqr_dev = true;           // LSQR / LSMR: device-resident beta/alpha/rotations (no host round trip)
    bool paged16 = true;            // streaming SpMV: paged gathers also for 16-bit-index operators
    bool band_dual = true;          // banded tiled ray-major operators: steep rows in row strips
    bool fused_ab = true;           // m-space operator A*(B*q) in one pass over B (fused.hip)
    int fused_region = 64;          // ... pixel square per workgroup (its rays accumulate in LDS)
    int fused_bs = 1024;            // ... threads per workgroup (512, 1024)
    int fused_pf = 2;               // ... sub-chunk batches in registers (pipeline depth 1..4)
    int fused_kind = 1;             // ... 0 sub-chunk pass, 1 row-wave pass
    int fused_wregion = 32;         // ... row-wave pass: pixel square per workgroup
    int fused_waves = 4;            // ... row-wave pass: waves per workgroup (1, 2, 4)
    int fused_group = 8;            // ... row-wave pass: rows per load batch (4, 8)
    int fused_depth = 2;            // ... row-wave pass: batches in the load ring (2..4)
    bool fused_pairs = true;        // ... row-wave pass: two entries per lane
    int fused_acc32 = 1;            // ... fp32 row-wave pass: 0 ds_add_f32, 1 read-add-write, 2 fp64 accumulators
    bool fused_plan_dev = true;     // ... row-wave plan's ray sets built on the device (false: the host build)
    int fused_rowpair = 4;          // ... row-wave pass: units of two consecutive rows per chunk (k_fused_rw RP 1-4)
    int fused_reduce = 0;           // ... row-wave partial reduction: 0 by ray (rs_slot), 1 by ray band (runs;
                                    //     bitwise equal, measured 2-4% slower pass at C4, profiles/r4_c4_reduce_band_ab.jsonl)
    bool lsqr_res_img = true;       // one-pass LSQR: final residual from the A*x image (no SpMV)
    bool lsmr_fuse_nmon = true;     // one-pass fp32 LSMR: the n-space step and monitor in one launch
    int krylov_pad = -1;            // Krylov basis column padding (elements; -1 auto, kernels.hip krylov_ld)
    int fused_dbg = 0;              // ... timing experiments: skip phases (wrong results)
};
struct FusedPlan;

}  // namespace hgm

struct hgm_ctx {
    hgm::Numerics num;
    int device = 0;
    hipStream_t stream = nullptr;
    int rank = 0, world = 1;
    ncclComm_t nccl = nullptr;
    hgm_allreduce_fn host_ar = nullptr;
    void* host_ar_user = nullptr;
    std::string err;
    std::map<std::string, hgm::DevBuf> ws;   // named workspace buffers
    double* dscal = nullptr;                  // device scalar slots
    double* hscal = nullptr;                  // pinned host mirror
    double* hstage = nullptr;                 // pinned host staging (allreduce / small copies)
    size_t hstage_bytes = 0;
    double* hup = nullptr;                    // pinned upload buffer (projected-solve y)
    size_t hup_bytes = 0;
    // pinned, device-mapped host memory the pipelined GMRES loop exchanges its per-iteration
    // scalars through (kernels write H/Gram columns and monitors into it, read y from it)
    double* hring = nullptr;
    double* hring_dev = nullptr;
    size_t hring_bytes = 0;
    hipEvent_t ev_pipe = nullptr;
    // second stream: GMRES reconstruction/monitors overlap the next Arnoldi step (single GPU)
    hipStream_t aux = nullptr;
    hipEvent_t ev_step[8] = {};
    unsigned ev_flags[9] = {};   // creation flags of ev_step[0..7], ev_pipe (capi.cpp sync_event)
    // prefix of workspace names while launching on `aux` (its scratch must not alias the
    // main stream's scratch: the two run concurrently)
    std::string ws_tag;
    // host-side diagnostics (HGM_HOST_STATS=1): time the host spends blocked in pipe_wait
    bool host_stats = false;
    double wait_s = 0.0;
    long waits = 0;
    // kernel-timing events armed for the next launch(es): recorded inside the dispatch
    // packets (hipExtLaunchKernelGGL), so they bracket kernel execution only
    hipEvent_t arm_start = nullptr, arm_stop = nullptr, cur_stop = nullptr;
    hgm::Timing timing;
    // path decisions of the last solve (hgm_ctx_solve_path): per GMRES iteration, whether the error
    // monitor came from the Gram form (1) or x was formed (0); whether the last Golub-Kahan solve
    // took the one-pass path.  On a communicator both decide the collective sequence.
    std::vector<int> path_mon;
    int path_onepass = -1;

    template <typename T>
    T* buf(const std::string& name, size_t count) {
        auto& b = ws_tag.empty() ? ws[name] : ws[ws_tag + name];
        b.ensure(count * sizeof(T) + 256);
        return reinterpret_cast<T*>(b.p);
    }
};

namespace hgm {
// Storage order of an N x N pixel index space.  Trivial (N == 0): the
// reference's column-major x(:).  Otherwise pixel (r, c) is stored at
// pixel_index(N, tile, super, r, c): super x super blocks (column-major over blocks, each
// contiguous; super == 0: one block), tile x tile tiles inside (tile-column-major), and
// column-major inside a tile.  A 4 x 4 tile of doubles is one 128-B cache line, so the x
// gathers of a ray share lines; a super-block is the x-slice a column band keeps in L2.
struct PixOrder {
    int N = 0, tile = 1, super = 0;
    bool trivial() const { return N == 0; }
    bool operator==(const PixOrder& o) const {
        return trivial() ? o.trivial() : (N == o.N && tile == o.tile && super == o.super);
    }
    bool operator!=(const PixOrder& o) const { return !(*this == o); }
};
}  // namespace hgm

struct hgm_mat {
    hgm_ctx* ctx = nullptr;
    int64_t rows = 0, cols = 0, nnz = 0;
    // index-space orders of the rows / columns (pixel spaces may be stored tiled)
    hgm::PixOrder row_order, col_order;
    // grid of a trivially-ordered index space that is a window of whole tile columns of a tiled
    // N x N grid (a pixel shard: hgm_mat_row_slice / transpose); only the band geometry reads it
    hgm::PixOrder row_grid, col_grid;
    int dtype = HGM_F64;
    int64_t* rp = nullptr;   // rows+1
    int32_t* ci = nullptr;   // nnz
    uint16_t* ci16 = nullptr;  // narrow copy of ci when cols <= 65536 (row-kernel SpMV reads it)
    void* val = nullptr;     // nnz (double or float)
    int group = 64;          // lanes per row in the SpMV kernel
    int variant = 0;         // SpmvVariant bits
    double fro = -1.0;       // cached ||M||_F (lsmr_solver.m:71 is loop-invariant)
    // identity (operators are immutable once built): transpose_of = the uid of the operator
    // this one is the device transpose of, value for value (hgm_mat_transpose)
    uint64_t uid = 0, transpose_of = 0;
    // Column-banded copy (cache blocking of the x gather): the columns are
    // cut into nbands contiguous bands of band_w pixels; segment (b, r) of row r that lies
    // in band b is [brp[b*rows + r], brp[b*rows + r + 1]) of bci/bval (band-major order).
    // band_dual: rows whose pixel-row span exceeds their pixel-column span (steeper than 45
    // deg) are cut into strips of band_w / N pixel ROWS instead (same band count, tiled N x N
    // grid), so both kinds of ray cross their strips in short chords.
    int64_t band_w = 0;
    int nbands = 0;
    bool band_dual = false;
    int bgroup = 16;         // lanes per segment in the banded kernel
    int64_t* brp = nullptr;
    int32_t* bci = nullptr;
    void* bval = nullptr;
    // chunk -> first segment starting in it, for the nnz-balanced streaming kernel
    int32_t* cfo = nullptr;      // rows as segments (nchunks+1)
    int32_t* bcfo = nullptr;     // (band,row) segments
    int sgroup = 8, bsgroup = 16;  // lanes per segment in the streaming reduction
    // x-page index of the paged streaming kernel, built over the stream the
    // SpMV reads (the banded copy when there is one): chunk k's entries gather from the distinct
    // 128-B pages of x pg_ids[pg_ptr[k] .. pg_ptr[k+1]) (staged in LDS), and entry e from
    // page-local position pg_lidx[e] = slot * (128 / sizeof value) + col % (128 / sizeof value).
    // pg_ptr[k+1] == pg_ptr[k]: the chunk touches more pages than fit; it gathers through the
    // 32-bit column indices instead.
    int32_t* pg_ptr = nullptr;
    int32_t* pg_ids = nullptr;
    uint16_t* pg_lidx = nullptr;
    // one-pass A*(B*q) plan over this pixel-major operator (fused.hip), built on first use
    hgm::FusedPlan* fused = nullptr;
    int64_t fused_key = -1;          // the option tuple the plan was built for (fused.hip fused_key)
    int64_t fused_failed_key = -1;   // the last tuple whose plan was refused (-1: none)
};

namespace hgm {
// SpMV kernel variants (bit flags): 16-byte paired loads, nontemporal val/col loads,
// XCD-aware row-block order, nnz-balanced streaming (chunked) kernel.
enum SpmvVariant { SPMV_VEC = 1, SPMV_NT = 2, SPMV_XCD = 4, SPMV_STREAM = 8, SPMV_PAGED = 16 };

// entries per streaming chunk (256 threads x 16): C4 sweep, 2048 -> 4096 took A from
// 2.90 to 2.48 ms and B from 2.78 to 2.47 ms (profiles/r1_spmv_sweep_c4_sch.jsonl)
#ifndef HGM_SCH
#define HGM_SCH 4096
#endif
constexpr int SCH = HGM_SCH;
// x pages per streaming chunk that the paged kernel stages in LDS (one 128-B line each).  The
// chunk's product buffer (SCH values) is reused for them, extended to HGM_PG_MAX64 pages in fp64
// (C4 A chunks touch 235 pages on average, up to 272: scripts/page_stats.py); fp32: 128 pages.
// With the dual strips the fp64 chunks over 256 pages are the axis-aligned angles' (256-269):
// 272 pages (34 KB of LDS) took C4 A from 2.07-2.10 to 2.05-2.06 ms, C3 A equal within noise
// (alternating builds, profiles/r2_pgmax272_ab.jsonl); 320 / 384 were slower (r2_pgmax_sweep.txt).
#ifndef HGM_PG_MAX64
#define HGM_PG_MAX64 272
#endif
#ifndef HGM_PG_MAX32
#define HGM_PG_MAX32 (SCH * 4 / 128)
#endif
constexpr int PG_BYTES = 128;
// LDS rounds of page staging per chunk.  fp32: two (128 pages each; 27.8 % of C4 A's chunks touch
// more than 128 pages, 2.0 % more than 256: scripts/page_stats_angles.py; C5 A 1.43 -> 1.32 ms).
// fp64: one (a second round cost every chunk more than it saved the 18.8 % above 256 pages:
// C4 A 2.32 -> 2.42 ms, C3 A 0.25 -> 0.27 ms; profiles/r2_tworound_fp64_ab.jsonl).
#ifndef HGM_PG_ROUNDS32
#define HGM_PG_ROUNDS32 2
#endif
template <typename T> constexpr int pg_rounds() { return sizeof(T) == 4 ? HGM_PG_ROUNDS32 : 1; }
template <typename T> constexpr int pg_max() { return sizeof(T) == 8 ? HGM_PG_MAX64 : HGM_PG_MAX32; }
template <typename T> constexpr int stream_lds_bytes(bool paged) {
    return paged && pg_max<T>() * PG_BYTES > SCH * (int)sizeof(T) ? pg_max<T>() * PG_BYTES : SCH * (int)sizeof(T);
}

struct SegIndex {
    int64_t nnz, nseg, nchunks;
    const int64_t* sp;       // nseg+1 segment pointers
    const int32_t* fo;       // nchunks+1
};
inline int64_t stream_chunks(int64_t nnz) { return (nnz + SCH - 1) / SCH; }
}

namespace hgm {

// ---------------- kernels (kernels.hip) ----------------
enum Epi { EPI_NONE = 0, EPI_ADD = 1, EPI_SUB = 2, EPI_RSUB = 3, EPI_DIVH = 4, EPI_ADDQ = 5 };

// Pending normalisation of the Krylov vector (gmres_family): Q(:,k) holds
// v_k before its division by h = H(k,k-1) = sqrt(sum parts), and the step's two SpMVs apply
// it in their epilogues instead of a separate scale pass:
//   EPI_DIVH (A): y = (A v) / h; every block sums `parts` in the fixed order of
//                 k_mgs_normalize, block 0 stores h to hdev and to the host ring (hring);
//   EPI_ADDQ (B): y = t + a (v_r / h), h from hdev (q written back over v when q != nullptr;
//                 the GMRES step leaves that to the MGS dots kernel).
template <typename T>
struct PendNorm {
    const T* parts = nullptr;
    int np = 0;
    T* hdev = nullptr;
    T* hring = nullptr;
    T* q = nullptr;
    // device-resident epilogue coefficient (EPI_ADD / EPI_SUB): a = (T)sqrt((double)*asq), the
    // bits the host computes from the same sum of squares (device-side Golub-Kahan scalars)
    const T* asq = nullptr;
};

int pick_group(int64_t rows, int64_t nnz);
// y = epi(M x): EPI_ADD: t + a*z ; EPI_SUB: t - a*z ; EPI_RSUB: z - t  (two roundings, no FMA)
// sumsq_out (optional, device): also *sumsq_out = sum_r y_r^2 (fused into the row kernel)
template <typename T>
void spmv(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z, int kclass,
          T* sumsq_out = nullptr, const PendNorm<T>* pn = nullptr);
// whether spmv() can apply EPI_DIVH / EPI_ADDQ for this operator's kernel choice
bool spmv_pn_ok(const hgm_mat* M, int epi);
template <typename T>
void epilogue(hgm_ctx* c, int64_t n, T* y, int epi, T a, const T* z);

int parts_for(int64_t n);
// local reductions: write result to *out_dev (device)
template <typename T> void dot(hgm_ctx* c, int64_t n, const T* a, const T* b, T* out_dev);
template <typename T> void sumsq(hgm_ctx* c, int64_t n, const T* a, T* out_dev);
template <typename T> void sumsq_diff(hgm_ctx* c, int64_t n, const T* a, const T* b, T* out_dev);
// out[j] = Q(:,j)' * w, j < ncols (local)
template <typename T>
void multidot(hgm_ctx* c, int64_t n, int ncols, const T* Q, int64_t ldq, const T* w, T* out_dev,
              const T* extra = nullptr);   // out[ncols] = extra' * w when extra != nullptr
// A multidot (out[j] = Q(:,j)' w, j < ncols, and out[ncols] = e' w) that mgs() may run
// as extra workgroups of its first two passes instead of two launches of its own
// (same partial layout and summation order as multidot(), so the same bits).
template <typename T>
struct MdotJob {
    int64_t n = 0;
    int ncols = 0;
    const T* Q = nullptr;
    int64_t ldq = 0;
    const T* w = nullptr;
    const T* e = nullptr;
    T* out = nullptr;
};
// x = Q(:,0:k) y fused with *err_out = ||x - xt||^2 (local)
template <typename T>
void gemv_err(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, const T* xt, T* err_out);
// one-launch GMRES reconstruction: x = Q y, *err_out = ||x - xt||^2 (local) and
// *res_out = ||b - AQ y||^2 over the m rows (AQ = A*Q(:,0:k), replicated)
template <typename T>
void recon(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y, T* x, const T* xt, T* err_out,
           int64_t m, const T* AQ, int64_t ldaq, const T* b, T* res_out);

// MGS sweep of v = Q(:,kk+1) against Q(:,0..kk); writes Hcol[0..kk+1] (device) and
// normalises Q(:,kk+1) unless H(kk+1,kk) == 0.  dist: n-vectors sharded (scalar all-reduce
// per pass).  kclass timing under KC_MGS.
// Leading dimension of a Krylov basis of vectors of length dim.  Short single-GPU bases
// get ldq = 4096 k (zero-padded past dim) so one workgroup runs the whole MGS sweep with
// no bounds checks (kernels.hip, k_mgs_single); the caller zeroes a padded basis.
int64_t krylov_ld(const hgm_ctx* c, int64_t dim, bool dist);
bool krylov_padded(const hgm_ctx* c, int64_t ldq);
// src (optional): the vector to orthogonalise when it is not already Q(:,kk+1); the result
// is written to Q(:,kk+1) either way.
// side (optional): a multidot enqueued with the sweep (see MdotJob).
template <typename T>
void mgs(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, bool dist, const T* src = nullptr,
         const MdotJob<T>* side = nullptr, PendNorm<T>* defer = nullptr, const T* pend_h = nullptr,
         const T* xe = nullptr, T* qg = nullptr, const double* cp_src = nullptr, double* cp_dst = nullptr);
// (cp_src / cp_dst: one value copied into the host ring with a system-scope store by the sweep's
// first workgroup, instead of a copy_sys launch of its own; a communicator's side dot)
// Gram error monitor (one-reduction form only, mgs_gram_ok): with xe = x_true the sweep of
// step kk also writes qg[0..kk+1] = [q_kk'q_0 .. q_kk'q_{kk-1}, q_kk'q_kk, q_kk'x_true] (host
// ring, system-scope stores), so ||Q y - x_true||^2 = xt'xt - 2 y'(Q'xt) + y'(Q'Q)y needs no
// pass over the basis.
bool mgs_gram_ok(const hgm_ctx* c, int64_t ldq, int maxit, bool dist);
// defer (single GPU, one-reduction form only): leave v = Q(:,kk+1) unnormalised and return
// its norm partials in *defer (np > 0) for the next step's SpMV epilogues (EPI_DIVH / EPI_ADDQ);
// np == 0 on return means the sweep normalised v itself.  pend_h (device h): Q(:,kk) still
// holds v_kk from the previous step's deferral; the dots kernel divides it and writes q_kk.
template <typename T>
void cgs2(hgm_ctx* c, int64_t n, T* Q, int64_t ldq, int kk, T* Hcol, bool dist);

// x = Q(:,0:k) * y  (mode 0) ; x = x - Q*y (mode 1)
template <typename T>
void gemv(hgm_ctx* c, int64_t n, int k, const T* Q, int64_t ldq, const T* y_dev, T* x, int mode);
template <typename T> void div_scalar(hgm_ctx* c, int64_t n, const T* in, T* out, T s);
// v = v / norm(v) on the device, *nrm_out = norm(v) (system-scope store, e.g. the host ring)
template <typename T> void normalize_to(hgm_ctx* c, int64_t n, T* v, T* nrm_out);
template <typename T> void lsqr_update(hgm_ctx* c, int64_t n, T* x, T* w, const T* v, T a, T b);
// Device-resident LSQR scalars (kernels.hip): the Givens rotation from the sums of squares *ssb
// (beta^2) and *ssa (alpha^2) in one thread (st = [rho_bar, phi_bar, stop]); the step
// v /= alpha, x += coef0 w, w = v - coef1 w (skipped after the stop), with ||x - x_true||^2 fused
// into err_out when xt != NULL; out = in / sqrt(*ss).
// Scalars that rode an m-vector all-reduce (multi-GPU Golub-Kahan solves: the previous iteration's
// ||x - x_true||^2 and ||A'r||^2 partials summed as trailing elements of [A*v_hat | alpha^2]),
// copied to their history slots by the rotation kernel that runs right after that all-reduce.
template <typename T>
struct ScalarCopy {
    const T* src = nullptr;
    T* dst = nullptr;
    const double* dsrc = nullptr;
    double* ddst = nullptr;
};
template <typename T>
void lsqr_rot(hgm_ctx* c, const T* ssb, const T* ssa, double* st, T* coef, double* phib_hist, int k, double nb,
              double tol, const ScalarCopy<T>& cp = ScalarCopy<T>{});
// the copies of cp alone (one thread), on the context stream
template <typename T>
void copy_scalars(hgm_ctx* c, const ScalarCopy<T>& cp);
template <typename T>
void lsqr_step(hgm_ctx* c, int64_t n, T* x, T* w, T* v, const T* ssa, const T* coef, const double* st, int k,
               const T* xt, T* err_out);
template <typename T> void div_sqrt(hgm_ctx* c, int64_t n, const T* in, T* out, const T* ss);
// m-space half of a Golub-Kahan step after the one-pass w = A*v_hat (fused_pass): av = w / alpha
// (optional: the kept A*v_k), t = av - alpha*u, *ss_out = ||t||^2 (alpha = sqrt(*ssa), device)
template <typename T>
void gkb_mstep(hgm_ctx* c, int64_t n, const T* w, const T* ssa, const T* u, T* t, T* av, T* ss_out);
// gkb_mstep, then u = t / sqrt(||t||^2) (nz: a zero norm leaves t, as div_sqrt_nz), the norm's
// partials re-formed by every block of the division (no k_finalize launch; the same bits)
template <typename T>
void gkb_mstep_div(hgm_ctx* c, int64_t n, const T* w, const T* ssa, T* u, T* t, T* av, T* ss_out, bool nz);
// (one-pass LSQR) A*x and A*w images in double (kernels.hip k_lsqr_img)
template <typename T>
void lsqr_img(hgm_ctx* c, int64_t m, const T* wm, const T* ssa, const T* coef, const double* st, int k, double* ax,
              double* aw, bool init);
template <typename T>
void lsmr_update(hgm_ctx* c, int64_t n, T* x, T* h, T* hbar, const T* v, T c_hbar, T c_x, T c_h,
                 bool first);
// LSMR kept-product monitor step (kernels.hip: k_lsmr_mon): image of v_k = c1*p1 + c0*p0 (or
// p1 if p0 == nullptr), then the h / hbar / x image recurrences; *out = ||rhs - image(x)||^2
// (cf != NULL: [c1, c0, f, e, cx] read on the device, from lsmr_rot)
template <typename T>
void lsmr_monitor(hgm_ctx* c, int64_t n, const T* p1, const T* p0, double c1, double c0, double* Ih, double* Ihb,
                  double* Ix, const T* rhs, double f, double e, double cx, bool first, double* out,
                  const double* cf = nullptr);
// The n-space monitor in carried-residual form with T images (the fp32 solves; kernels.hip
// k_lsmr_mon_r): Ir starts as A'b; *out = ||Ir_k||^2; coefficients from lsmr_rot's cf.
template <typename T>
void lsmr_monitor_r(hgm_ctx* c, int64_t n, const T* p1, const T* p0, T* Ih, T* Ihb, T* Ir, bool first, double* out,
                    const double* cf);
// Device-resident LSMR scalars (kernels.hip): the rotations :42-67 in one thread from *ssb = beta^2 and
// *ssa = alpha^2 (st = [alpha, alphabar, rho, rhobar, cbar, sbar, zetabar, theta/rho, stop]); the
// n-space step v /= alpha, hbar / x / h updates (skipped after the stop) with ||x - x_true||^2 fused
// into err_out when xt != NULL; the stop test :76 on the m-space monitor; out = in / sqrt(*ss)
// unless the sum is zero.
template <typename T>
void lsmr_rot(hgm_ctx* c, const T* ssb, const T* ssa, double* st, T* coef, double* cfm, double* cfn,
              const ScalarCopy<T>& cp = ScalarCopy<T>{});
template <typename T>
void lsmr_step(hgm_ctx* c, int64_t n, T* x, T* h, T* hbar, T* v, const T* ssa, const T* coef, const double* st,
               int k, const T* xt, T* err_out);
// lsmr_step + lsmr_monitor_r in one launch (same bits; HGM_OPT_LSMR_FUSE_NMON); false when it does
// not apply (no x_true, a small n, unaligned vectors): the caller runs the two
template <typename T>
bool lsmr_step_mon(hgm_ctx* c, int64_t n, T* x, T* h, T* hbar, T* v, const T* ssa, const T* coef, const double* st,
                   int k, const T* xt, T* err_out, const T* p1, const T* p0, T* Ih, T* Ihb, T* Ir, bool first,
                   double* mon_out, const double* cf);
void lsmr_stop(hgm_ctx* c, const double* rr, double nb, double tol, double* st, int k);
template <typename T> void div_sqrt_nz(hgm_ctx* c, int64_t n, const T* in, T* out, const T* ss);
// out[i] = epi(in[i], a, z[i]) (out may alias z): the epilogue of an SpMV applied to its raw product
template <typename T> void epilogue_to(hgm_ctx* c, int64_t n, const T* in, T* out, int epi, T a, const T* z);
template <typename T> void fill(hgm_ctx* c, int64_t n, T* x, T v);
template <typename T> void scale(hgm_ctx* c, int64_t n, const T* in, T* out, T a);   // out = a * in
// x_i = deterministic pseudo-random value in (-1, 1) (splitmix64 of seed + i)
template <typename T> void fill_hash(hgm_ctx* c, int64_t n, T* x, uint64_t seed);
template <typename T> void convert(hgm_ctx* c, int64_t n, const double* in, T* out);
template <typename T> void convert_back(hgm_ctx* c, int64_t n, const T* in, double* out);
template <typename T> void fro2(hgm_ctx* c, const hgm_mat* M, double* out_dev);

// ---------------- fixed-order parity mode (kernels.hip; ctx->num.parity) ----------------
// The documented fixed summation order of a length-n sum of terms t_i (oracle/restatement.py
// fixed_order()): level 1 sums 64-term chunks sequentially, level 2 sums 64-value
// chunks of those sequentially, and the level-2 values are summed sequentially.  Terms:
// OP 0 a_i b_i, OP 1 a_i a_i, OP 2 (a_i - b_i)^2.  The index space may be the concatenation
// of two segments [a1 (n1) | a2 (n2)] (the augmented vectors of hybrid_lsqr_solver.m:6).
// *out is written with a system-scope store.
template <typename T>
void fixed_reduce(hgm_ctx* c, int op, int64_t n1, const T* a1, const T* b1, int64_t n2, const T* a2, const T* b2,
                  T* out);

// ---------------- operators (ops.hip) ----------------
hgm_mat* mat_alloc(hgm_ctx* c, int64_t rows, int64_t cols, int64_t nnz, int dtype);
void mat_free(hgm_mat* M);
hgm_mat* transpose(hgm_ctx* c, const hgm_mat* M);
// rows [lo, hi) as a new operator (pixel shard B(P_g,:)); rows must be in the reference order
hgm_mat* row_slice(hgm_ctx* c, const hgm_mat* M, int64_t lo, int64_t hi);
// build / drop the column-banded copy (band_w <= 0 or >= cols drops it)
void set_bands(hgm_ctx* c, hgm_mat* M, int64_t band_w);
// chunk index of the nnz-balanced streaming kernel over the rows
void build_stream_index(hgm_ctx* c, hgm_mat* M);
// x-page index of the paged streaming kernel (over the banded copy when M has bands)
void build_page_index(hgm_ctx* c, hgm_mat* M);
void free_page_index(hgm_mat* M);
// everything a freshly created operator gets: automatic bands + streaming index
void finalize_operator(hgm_ctx* c, hgm_mat* M);
int64_t auto_band_width(const hgm_mat* M);
hgm_mat* siddon(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, int tile = 1, int super = 0);
hgm_mat* fanbeam(hgm_ctx* c, int N, int n_angles, double R, double span, double det_offset, int dtype, int tile = 1,
                 int super = 0);
hgm_mat* backprojector(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, int tile = 1, int super = 0);
// n-vector between the reference order and a pixel order o: dir 0: out[stored(p)] = in[p]
// (reference -> stored), dir 1: out[p] = in[stored(p)] (stored -> reference)
template <typename T>
void pix_permute(hgm_ctx* c, const PixOrder& o, const T* in, T* out, int dir);
// stored pixel index -> reference (column-major) index, in place on n indices
void pix_unmap_indices(hgm_ctx* c, const PixOrder& o, int32_t* idx, int64_t n);
// reference index of every stored position (host vector, for host-side row reordering)
std::vector<int64_t> pix_reference_of_stored(const PixOrder& o);

// ---------------- one-pass m-space operator (fused.hip) ----------------
// w = A*(B*q) and the kept B*q in one pass over B's pixel-major entries when B is A' value for
// value.  fused_ab_plan: B's plan (built on first use), or nullptr when the
// pair / context does not qualify (the two-pass path then runs).
bool fused_ab_eligible(const hgm_ctx* c, const hgm_mat* A, const hgm_mat* B);
const FusedPlan* fused_ab_plan(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B);
// With xt and zx_out (the row-wave kernel only; returns whether it did): also *zx_out =
// x_true'(B*q), the m-space Gram error monitor's side dot, from the row sums as they form.
// With pn (pn->np > 0, fused_pend_ok): q still holds the unnormalised v of the previous MGS sweep,
// and the pass applies q = v / h itself (FusedArgs::pn).
bool fused_ab(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P, const double* q, double* Bq, double* ABq,
              const double* xt = nullptr, double* zx_out = nullptr, const PendNorm<double>* pn = nullptr);
// whether the pass takes the pending normalisation of q for this plan (the row-wave kernel)
bool fused_pend_ok(const hgm_ctx* c, const FusedPlan* P);
// The general pass (T = double or float; fp32 and every epilogue: the row-wave kernel).  Over B's
// rows j (pixels) and columns i (rays):
//   z_j = B(j,:) q ; zs_j = z_j - a ev_j with a = (T)sqrt((double)*easq) (no ev: zs = z) ;
//   zraw = z, zout = zs (either optional; zout may alias ev) ; w_i = sum_j B(j,i) zs_j ;
//   side_out (optional) = sum_j zs_j x_true_j, or sum_j zs_j^2 with side_sq.
// The Golub-Kahan step of lsqr_solver.m:26-27 / lsmr_solver.m:38-39 is q = u_{k+1}, ev = v_k,
// easq = beta^2: zout = v_hat, side_out = alpha^2 and w = A*v_hat, so A*v_{k+1} = w / alpha needs
// no second pass over the operator.  Returns whether the side sum was formed.
template <typename T>
struct FusedArgs {
    const T* q = nullptr;
    T* zraw = nullptr;
    T* w = nullptr;
    const T* xt = nullptr;
    const T* ev = nullptr;
    const T* easq = nullptr;
    T* zout = nullptr;
    bool side_sq = false;
    T* side_out = nullptr;
    // pending normalisation of q (pn.np > 0: the row-wave pass, fused_pend_ok): q = v / h
    // with h = sqrt(sum of pn.parts), published to pn.hdev and pn.hring (fused.hip k_fused_rw)
    PendNorm<T> pn;
};
template <typename T>
bool fused_pass(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P, const FusedArgs<T>& fa);
// whether the Golub-Kahan form (row epilogue / side sum of squares, or fp32) runs for this plan
bool fused_gk_ok(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P);
// *dst = *src (one scalar, device to the host-visible ring, system scope), on the context stream
void copy_sys(hgm_ctx* c, const double* src, double* dst);
void fused_plan_free(FusedPlan* P);
uint64_t fused_plan_checksum(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P);
double fused_plan_build_seconds(const FusedPlan* P);
int64_t fused_plan_slots(const FusedPlan* P);
bool fused_plan_device_built(const FusedPlan* P);

// Solver entry check: HGM_OPT_FUSED_DBG skips phases of the one-pass kernel (timing experiments of
// hgm_spmv_ab only, scripts/fused_micro.py): a solve would return wrong results, so it is refused.
inline void solver_guard(const hgm_ctx* c) {
    HGM_REQUIRE(c->num.fused_dbg == 0, "fused_dbg is a timing experiment (hgm_spmv_ab only): set it to 0 to solve");
}

// ---------------- comm / scalars (capi.cpp) ----------------
void allreduce(hgm_ctx* c, double* dev, int64_t count);
void allreduce(hgm_ctx* c, float* dev, int64_t count);
// batched small device->host reads behind one stream synchronisation
struct Reader {
    hgm_ctx* c;
    struct Item { void* host; const void* dev; size_t bytes; };
    std::vector<Item> items;
    explicit Reader(hgm_ctx* cc) : c(cc) {}
    void add(void* host, const void* dev, size_t bytes) { items.push_back({host, dev, bytes}); }
    void go();
};
void h2d(hgm_ctx* c, void* dev, const void* host, size_t bytes);
// small upload through a pinned buffer (truly asynchronous); the caller must not issue
// another h2d_pinned before the stream has passed the previous one (one per iteration)
void h2d_pinned(hgm_ctx* c, void* dev, const void* host, size_t bytes);
void read_scalars(hgm_ctx* c, int first, int count);   // dscal -> hscal (sync)
// wait for stream s by spinning on hipStreamQuery (no sleeping wake-up after long waits); the spin
// yields the core after HGM_OPT_HOST_SPIN_US (process-wide: g_host_spin_us; < 0 = blocking waits)
void stream_sync(hipStream_t s);
extern std::atomic<int> g_host_spin_us;
// the back-off of a host spin loop: call once per poll
struct HostPause {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    int polls = 0;
    bool yielding = false;
    void operator()();
};
// zero-initialised pinned host ring of >= bytes (c->hring / c->hring_dev), after a
// stream synchronisation (no kernel may still be writing the previous one)
void pinned_ring(hgm_ctx* c, size_t bytes);
// record c->ev_pipe on the stream / wait for it on the host
void pipe_record(hgm_ctx* c);
void pipe_wait(hgm_ctx* c);
// the auxiliary stream (created on first use) and the per-step events on the main stream
hipStream_t aux_stream(hgm_ctx* c);
void step_record(hgm_ctx* c, int k);
void step_wait(hgm_ctx* c, int k);

// Launch subsequent work on stream s with workspace prefix tag (restored on scope exit).
struct StreamScope {
    hgm_ctx* c;
    hipStream_t saved;
    std::string saved_tag;
    StreamScope(hgm_ctx* cc, hipStream_t s, const char* tag) : c(cc), saved(cc->stream), saved_tag(cc->ws_tag) {
        if (s != saved) {
            c->stream = s;
            c->ws_tag = tag;
        }
    }
    ~StreamScope() {
        c->stream = saved;
        c->ws_tag = saved_tag;
    }
};
void sync(hgm_ctx* c);
void timing_begin(hgm_ctx* c, int cls, hipEvent_t* start);
void timing_end(hgm_ctx* c, int cls, hipEvent_t start, double bytes);

// ---------------- dense host LA (dense.cpp) ----------------
namespace dense {
// MATLAB mldivide for square M (col-major n x n): symmetric + positive diagonal ->
// Cholesky (LU fallback if not PD); otherwise LU with partial pivoting.
void mldivide_square(int n, const double* M, const double* b, double* x);
// MATLAB mldivide for rectangular m x n (m > n): Householder QR with column pivoting.
void qr_ls(int m, int n, const double* M, const double* b, double* x);
// singular values of a square n x n matrix (one-sided Jacobi), descending.
void svd_values(int n, const double* M, double* s);
double gcv_from_H(const double* H, int ldh, int k, double beta, double lambda, double trace_m);
// MATLAB fminbnd (Brent / Forsythe-Malcolm-Moler fmin) of gcv_from_H over [lo, hi].
double gcv_fminbnd(const double* H, int k, double beta, double trace_m, double lo, double hi,
                   double tolx, double* gopt);
// spectral.cpp: MATLAB eig of a real n x n (col-major) matrix: eigenvalues wr + i wi, unit 2-norm
// eigenvectors in the LAPACK dgeev layout (V may be NULL).  false: no convergence.
bool eig_general(int n, const double* A, double* wr, double* wi, double* V);
// phi / dphi of iteration k of the *_bounds.m files (H: (k+1) x k leading part, ldh; dK = Qk' DeltaM Qk;
// mu / dmu: the k leading eigenvalues of M (descending) and u_i' DeltaM u_i)
void filter_factors(const double* H, int ldh, int k, const double* dK, int lddk, const double* mu,
                    const double* dmu, double lambda, int side, int hybrid, double* phi, double* dphi);
// Ritz values of a p-step Arnoldi (Hp p x p, h_next = H(p+1,p)), descending by real part, with
// y_i' G y_i (G = Qp' DeltaM Qp) and the residual norms |h_next| |e_p' y_i| of the first nev
void ritz(const double* Hp, int ldh, int p, double h_next, const double* G, int ldg, int nev, double* mu,
          double* dmu, double* resid);
}  // namespace dense

}  // namespace hgm
