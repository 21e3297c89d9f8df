// Solver loops of the reference, driven from the host over the HIP kernels.
//
// Each function follows one reference .m file; the per-line correspondence is
// cited inline.  Vectors live in HBM for the whole solve; per iteration the host
// only receives the new Hessenberg column (k+2 doubles) and a few scalars, and
// sends back the k-vector y of the projected solve.
//
// Multi-GPU (ctx->world > 1): the pixel dimension n is sharded
// (A_g = A(:,P_g), B_g = B(P_g,:)); every `A*v` is followed by an all-reduce of the
// m-vector, every inner product of n-vectors by a scalar all-reduce; m-vectors
// (b, u, the AB-side Krylov basis, A*Q columns) are replicated.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <type_traits>
#include <vector>

#include "internal.h"

namespace hgm {

namespace {

constexpr double EPSD = std::numeric_limits<double>::epsilon();

inline int64_t round_up(int64_t x, int64_t a) { return (x + a - 1) / a * a; }

// Scalar slots in ctx->dscal.
enum Slot { S_NB = 0, S_NXT = 1, S_BETA = 2, S_RES = 3, S_ERR = 4, S_ALPHA = 5, S_AR = 6, S_FRO = 7,
            S_AUX = 8, S_AUX2 = 9 };

template <typename T>
T* dslot(hgm_ctx* c, int i) {
    return reinterpret_cast<T*>(c->dscal) + i;
}

// sharded code path: world > 1, or a one-rank RCCL communicator (hgm_ctx_create_dist)
inline bool dist_n(hgm_ctx* c) { return c->world > 1 || c->nccl != nullptr; }

// y = A x (+epilogue) where the output is an m-vector assembled across ranks.
template <typename T>
void apply_A(hgm_ctx* c, const hgm_mat* A, const T* x, T* y, int epi, T a, const T* z) {
    if (!dist_n(c)) {
        spmv<T>(c, A, x, y, epi, a, z, KC_SPMV_A);
    } else if (epi == EPI_NONE) {
        spmv<T>(c, A, x, y, EPI_NONE, T(0), nullptr, KC_SPMV_A);
        allreduce(c, y, A->rows);
    } else {
        // z may alias y (u = A*v - alpha*u): assemble in scratch, then apply the epilogue
        T* tmp = c->buf<T>("ar_tmp", A->rows + 1);
        spmv<T>(c, A, x, tmp, EPI_NONE, T(0), nullptr, KC_SPMV_A);
        allreduce(c, tmp, A->rows);
        epilogue<T>(c, A->rows, tmp, epi, a, z);
        HGM_HIP(hipMemcpyAsync(y, tmp, sizeof(T) * A->rows, hipMemcpyDeviceToDevice, c->stream));
    }
}

// y = B u (+epilogue): B's rows are this rank's pixels, no exchange.
template <typename T>
void apply_B(hgm_ctx* c, const hgm_mat* B, const T* u, T* y, int epi, T a, const T* z) {
    spmv<T>(c, B, u, y, epi, a, z, KC_SPMV_B);
}

// local sum of squares of an n-vector (+ all-reduce) into slot
template <typename T>
void nsumsq(hgm_ctx* c, int64_t n, const T* v, T* slot) {
    sumsq<T>(c, n, v, slot);
    if (dist_n(c)) allreduce(c, slot, 1);
}
template <typename T>
void nsumsq_diff(hgm_ctx* c, int64_t n, const T* a, const T* b, T* slot) {
    sumsq_diff<T>(c, n, a, b, slot);
    if (dist_n(c)) allreduce(c, slot, 1);
}

template <typename T>
T read1(hgm_ctx* c, const T* dev) {
    T v;
    Reader r(c);
    r.add(&v, dev, sizeof(T));
    r.go();
    return v;
}

// The Golub-Kahan solvers' one-pass plan, agreed over the ranks.  The one-pass path all-reduces
// [A*v_hat | alpha^2] (m + 1 values) per iteration and the two-pass path A*v (m) plus n-space
// norms, so on a communicator every rank must take the same one: each rank plans its own shard
// (a plan can be refused on some shards only, e.g. the centre tile columns of a fan-beam cut),
// the refusals are summed over the ranks, and the pass runs only if no rank refused.
template <typename T>
const FusedPlan* agreed_gk_plan(hgm_ctx* c, const hgm_mat* A, const hgm_mat* At, bool allowed) {
    const FusedPlan* fp = allowed ? fused_ab_plan(c, A, At) : nullptr;
    if (fp && !fused_gk_ok(c, At, fp)) fp = nullptr;
    if (dist_n(c)) {
        double* f = reinterpret_cast<double*>(c->dscal) + 96;
        const double refused = fp ? 0.0 : 1.0;
        h2d(c, f, &refused, sizeof(double));
        allreduce(c, f, 1);
        if (read1<double>(c, f) != 0.0) fp = nullptr;
    }
    c->path_onepass = fp ? 1 : 0;
    return fp;
}

// Input vector hand-over: device pointer (HGM_DEVICE_PTRS) or host buffer.
template <typename T>
const T* stage_in(hgm_ctx* c, const char* name, const double* p, int64_t n, bool dev) {
    if (p == nullptr) return nullptr;
    if (dev && std::is_same<T, double>::value) return reinterpret_cast<const T*>(p);
    T* d = c->buf<T>(name, n > 0 ? n : 1);
    if (std::is_same<T, double>::value) {
        h2d(c, d, p, sizeof(double) * n);
    } else {
        const double* src = p;
        if (!dev) {
            double* tmp = c->buf<double>(std::string(name) + "_f64", n > 0 ? n : 1);
            h2d(c, tmp, p, sizeof(double) * n);
            src = tmp;
        }
        convert<T>(c, n, src, d);
    }
    return d;
}

template <typename T>
void stage_out(hgm_ctx* c, double* out, const T* d, int64_t n, bool dev) {
    if (out == nullptr || n == 0) return;
    if (std::is_same<T, double>::value) {
        if (dev) {
            HGM_HIP(hipMemcpyAsync(out, d, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
            stream_sync(c->stream);
        } else {
            HGM_HIP(hipMemcpyAsync(out, d, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
            stream_sync(c->stream);
        }
    } else {
        double* tmp = dev ? out : c->buf<double>("out_f64", n);
        convert_back<T>(c, n, d, tmp);
        if (!dev) HGM_HIP(hipMemcpyAsync(out, tmp, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
        stream_sync(c->stream);
    }
}

// The stored order of the pixel (n) space shared by A's columns and B's (or A''s) rows;
// the ray (m) space is always in the reference order.
PixOrder n_order(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B) {
    HGM_REQUIRE(A->row_order.trivial() && (!B || B->col_order.trivial()),
                "the ray (m) space must be stored in the reference order");
    if (B) HGM_REQUIRE(B->row_order == A->col_order, "A's columns and B's rows must share one pixel order");
    HGM_REQUIRE(A->col_order.trivial() || !dist_n(c), "pixel-sharded solves need the reference pixel order");
    return A->col_order;
}

// n-vector hand-over in the reference order, permuted into / out of the stored order
template <typename T>
const T* stage_in_n(hgm_ctx* c, const char* name, const double* p, int64_t n, bool dev, const PixOrder& o) {
    const T* d = stage_in<T>(c, name, p, n, dev);
    if (d == nullptr || o.trivial()) return d;
    T* q = c->buf<T>(std::string(name) + "_pix", n);
    pix_permute<T>(c, o, d, q, 0);
    return q;
}

template <typename T>
void stage_out_n(hgm_ctx* c, double* out, const T* d, int64_t n, bool dev, const PixOrder& o) {
    if (out == nullptr || n == 0) return;
    if (o.trivial()) {
        stage_out<T>(c, out, d, n, dev);
        return;
    }
    if (dev && std::is_same<T, double>::value) {   // straight into the caller's device buffer
        pix_permute<T>(c, o, d, reinterpret_cast<T*>(out), 1);
        stream_sync(c->stream);
        return;
    }
    T* q = c->buf<T>("out_pix", n);
    pix_permute<T>(c, o, d, q, 1);
    stage_out<T>(c, out, q, n, dev);
}

void check_dims(const hgm_mat* A, const hgm_mat* B) {
    HGM_REQUIRE(A != nullptr, "A is NULL");
    if (B) {
        HGM_REQUIRE(B->rows == A->cols && B->cols == A->rows,
                    "dimension mismatch: B must be size(A') (n x m)");
        HGM_REQUIRE(B->dtype == A->dtype, "A and B must have the same dtype");
    }
}

}  // namespace

// ============================================================================
// GMRES family (Arnoldi + projected solve)
// ============================================================================
enum Proj { PROJ_LS = 0, PROJ_PTR = 1, PROJ_ABRTP = 2 };

struct GmresSpec {
    int side;             // HGM_SIDE_BA: n-space Krylov of B*A (+λI) ; HGM_SIDE_AB: m-space of A*B
    int proj;             // Proj
    bool lambda_in_op;    // RTP: operator B*(A*v) + lambda*v
    bool x_preassigned;   // hybrid_ba_gmres_rtp.m:4 initialises x = zeros
};

// Ring polling (single GPU): the host waits for step k by watching the entries of ring
// slot k turn from a NaN sentinel into values instead of an event recorded after the step.
// A recorded event (a marker packet, or a completion signal on the step's last dispatch)
// makes the next kernel wait for an end-of-kernel release: ~4.5 us per step on the main
// stream (rocprofv3 trace).  Every ring entry is written exactly once per
// solve by a system-scope store (st_sys), so a non-sentinel value is final.
constexpr uint64_t RING_SENTINEL = 0x7FF4DEADBEEF0001ull;   // a NaN no kernel produces
// Spin until ring[i] for i in idx are all non-sentinel.  Checks the streams that write them
// (main and, when it is a different one, aux) for errors, and for all going idle with an entry
// never written (a bug), every RING_CHECK_MS so a fault cannot hang.  Not more often: a
// hipStreamQuery on a stream with work queued puts a marker packet behind that work, and the
// kernel queued after the marker then starts ~5.7 us late (round 6: at the 1 ms interval every
// Arnoldi step from the fourth on waited so at C4, profiles/r6_hip_api_trace_gaps.txt).
constexpr int RING_CHECK_MS = 200;
static void ring_wait(hgm_ctx* c, const double* ring, const std::vector<size_t>& idx, hipStream_t aux = nullptr) {
    const volatile uint64_t* r = reinterpret_cast<const volatile uint64_t*>(ring);
    const auto t0 = std::chrono::steady_clock::now();
    auto last = t0;
    bool idle_seen = false;
    HostPause pause;
    for (;;) {
        bool all = true;
        for (size_t i : idx)
            if (r[i] == RING_SENTINEL) {
                all = false;
                break;
            }
        if (all) break;
        pause();
        const auto now = std::chrono::steady_clock::now();
        if (now - last > std::chrono::milliseconds(RING_CHECK_MS)) {
            last = now;
            hipError_t q = hipStreamQuery(c->stream);
            if (q != hipSuccess && q != hipErrorNotReady) HGM_HIP(q);
            if (aux && aux != c->stream && q == hipSuccess) {   // idle only when both streams are
                q = hipStreamQuery(aux);
                if (q != hipSuccess && q != hipErrorNotReady) HGM_HIP(q);
            }
            if (q == hipSuccess) {
                if (idle_seen) throw Error{HGM_E_HIP, "ring poll: stream idle with a ring entry never written"};
                idle_seen = true;   // one more round: the last stores may still be in flight
            }
        }
    }
    if (c->host_stats) {
        c->wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
}

int gmres_family(hgm_ctx* c, const GmresSpec& sp, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B,
                 const double* b_in, const double* xt_in, double tol, int maxit, double lambda, double* x_out,
                 double* err_out, double* res_out, int* niters) {
    check_dims(A, B);
    solver_guard(c);
    HGM_REQUIRE(B != nullptr, "B is NULL");
    const PixOrder po = n_order(c, A, B);
    HGM_REQUIRE(b_in != nullptr && xt_in != nullptr, "b and x_true are required");
    HGM_REQUIRE(A->dtype == HGM_F64, "GMRES family is fp64 (the reference's precision)");
    const auto t_start = std::chrono::steady_clock::now();
    const double wait0 = c->wait_s;
    const long waits0 = c->waits;
    HGM_REQUIRE(maxit >= 1, "maxit must be >= 1");
    c->path_mon.clear();
    using T = double;
    const bool dev = o && (o->flags & HGM_DEVICE_PTRS);
    const int orth = o ? o->orth : HGM_MGS;
    const int64_t m = A->rows, n = A->cols;
    const bool nspace = sp.side == HGM_SIDE_BA;
    const int64_t dim = nspace ? n : m;
    const bool dist = nspace && dist_n(c);
    // parity mode (HGM_OPT_PARITY): the reference's own sequence of operations in
    // fixed summation orders; every fused or reformulated monitor below is switched off
    const bool parity = c->num.parity;
    HGM_REQUIRE(!parity || (!dist_n(c) && po.trivial()), "parity mode: single rank, reference pixel order");
    const int64_t ldq = krylov_ld(c, dim, dist);
    hipStream_t st = c->stream;

    T* Q = c->buf<T>("Q", (size_t)ldq * (maxit + 1));
    if (krylov_padded(c, ldq)) HGM_HIP(hipMemsetAsync(Q, 0, sizeof(T) * ldq * (maxit + 1), st));
    T* x = c->buf<T>("x", n > 0 ? n : 1);
    T* t = c->buf<T>("t_m", m > 0 ? m : 1);        // m-vector scratch (A*q, residual)
    T* tn = c->buf<T>("t_n", n > 0 ? n : 1);       // n-vector scratch (AB side: B*q)
    T* z = c->buf<T>("z_m", m > 0 ? m : 1);        // AB side: z = Q*y
    T* tr = c->buf<T>("t_res", m > 0 ? m : 1);     // m-vector of the residual monitor (aux stream)
    const int64_t ldaq = round_up(m > 0 ? m : 1, 64);
    // n-space side: keep the operator's products A*Q(:,j) (the RTP Gram matrix needs them,
    // and the residual monitor b - A*x = b - (A*Q) y reuses them instead of another SpMV)
    const bool reuse = !(o && (o->flags & HGM_EXPLICIT_RESIDUAL)) && !parity;
    const bool aq_res = nspace && reuse;
    T* AQ = (sp.proj == PROJ_ABRTP || aq_res) ? c->buf<T>("AQ", (size_t)ldaq * maxit) : nullptr;
    // m-space side: keep B*Q(:,j) and A*(B*Q(:,j)) (the latter is the new Arnoldi vector
    // before orthogonalisation), so x = B*(Q y) = (B*Q) y and b - A*x = b - (A*B*Q) y are
    // GEMVs over k kept columns instead of two SpMVs per iteration (*_bounds.m:37-40)
    const bool bq_res = !nspace && reuse;
    const int64_t ldbq = round_up(n > 0 ? n : 1, 64);
    T* BQ = bq_res ? c->buf<T>("BQ", (size_t)ldbq * maxit) : nullptr;
    T* ABQ = bq_res ? c->buf<T>("ABQ", (size_t)ldaq * maxit) : nullptr;
    // Per-iteration exchange ring in pinned host memory: slot k holds
    // [H(:,k) | Gram column k, AQk'b] (LH doubles), the monitors [res^2, err^2] of
    // iteration k, and the projected solution y_k.  Single GPU: the kernels write the
    // slots in place and read y from it (zero-copy, no copy kernels).  Multi-GPU m-space side
    // (the sharded AB-GMRES of configs[3]): the same, since the m-space sweep is replicated and
    // every ring entry is written after its all-reduce (a sum that is all-reduced is formed in a
    // device slot, all-reduced there and copied into the ring by copy_sys).  Multi-GPU n-space
    // side: the all-reduced sweep scalars live in a device mirror and each slot is copied out once.
    const size_t LH = 2 * (size_t)(maxit + 2);
    const size_t offM = (size_t)maxit * LH, offY = offM + 2 * (size_t)maxit;
    const size_t offS = offY + (size_t)maxit * maxit;   // [beta, ||b||^2, ||x_true||^2] (polling)
    const bool zc = !dist_n(c) || !nspace;
    // Gram error monitor: step k's MGS sweep appends [Q(:,k)'Q(:,0:k-1),
    // Q(:,k)'Q(:,k), Q(:,k)'x_true] to the ring (LQ doubles) and the host evaluates
    // ||Q y_k - x_true||^2 from them, so an iteration's reconstruction reads only the kept A*Q.
    const bool gem_ok = zc && c->num.ring_poll && orth == HGM_MGS && mgs_gram_ok(c, ldq, maxit, dist) &&
                        c->num.gram_err;
    const bool gem_n = aq_res && gem_ok;
    // m-space side (AB-GMRES, x = (B*Q) y = Z y): when B is A' value for value (a device
    // transpose), Z'Z = Q'(A*B*Q) are the sweep's own dots Q'w_k = (I + L) H(0:k,k) (one-reduction
    // form, L the strictly lower Q'Q), and Z'x_true = x_true'(B*q_k) is one dot per step riding on
    // the sweep as a side job, so an iteration's reconstruction reads no n-vector: the kept B*Q
    // columns are combined once, at the end (C4: the 0.3 ms GEMV per iteration)
    const bool pair_t = B && (B->transpose_of == A->uid || A->transpose_of == B->uid);
    // (multi-GPU too: the m-space sweep is replicated, the side dot is all-reduced and the
    // Gram row published with the H column; a shard pair A_g = B_g' qualifies)
    const bool gem_ab = bq_res && orth == HGM_MGS && mgs_gram_ok(c, ldq, maxit, dist) && c->num.gram_err &&
                        (zc ? c->num.ring_poll : true) && sp.proj != PROJ_ABRTP && pair_t;
    const bool gem = gem_n || gem_ab;
    const double gem_min = c->num.gram_err_min;
    const size_t LQ = (size_t)maxit + 2, offQG = offS + 4;
    const size_t ring_n = offQG + (gem ? (size_t)maxit * LQ : 0);
    // single GPU: reconstructions run on the auxiliary stream, concurrently with the
    // Arnoldi steps (multi-GPU keeps one stream: the communicator's collectives must be
    // issued in one order).  For large n the concurrent GEMV over the kept columns evicts
    // the SpMVs' L2-resident x-slices and costs the SpMVs more than it hides, so it is
    // serialised behind the steps (HGM_RECON_SERIAL=0/1 overrides).
    // (with the Gram error monitor the per-iteration reconstruction reads only the kept A*Q,
    // so it stays on the aux stream at any n: C3 1,376 vs 1,368 iters/s serialised)
    bool recon_serial = !gem && (int64_t)n >= c->num.recon_serial_n;
    if (c->num.recon_serial >= 0) recon_serial = c->num.recon_serial != 0;
    // (a communicator's solve keeps one stream whatever the ring)
    // On a communicator the m-space solve's residual-only reconstructions (gem_ab: the kept A*B*Q
    // columns and b are replicated, so no collective runs in them) go to the auxiliary stream as
    // well; a reconstruction that forms x all-reduces its error and stays on the step stream, so
    // the communicator's collectives keep one stream and one order on every rank.
    // Scratch invariant: reconstructions on the auxiliary stream and the x-forming ones
    // on the step stream share the recon_parts / recon_noerr scratch buffers.  That is safe only
    // because the host waits for reconstruction k's ring slots (ring_wait on both streams) before
    // it enqueues reconstruction k+1 on either stream, so two reconstructions never run at once.
    const bool rs_aux_dist = dist_n(c) && gem_ab && !recon_serial && zc;
    hipStream_t rs_stream = (zc && !recon_serial && (!dist_n(c) || rs_aux_dist)) ? aux_stream(c) : st;
    if (rs_stream != st) stream_sync(rs_stream);
    pinned_ring(c, sizeof(double) * ring_n);
    const double* hr = c->hring;
    const bool poll = zc && c->num.ring_poll && !parity;
    // the reconstruction's pipeline event: not needed when the host polls the ring and the
    // reconstruction runs on the step stream (an event there is a bubble between two kernels)
    const bool pipe_ev = !(poll && rs_stream == st);
    if (zc) {
        // the kernels store into the mapped ring with system-scope stores, and the pipeline
        // events carry no system-scope release, so a store may land after its kernel's event
        // has completed: the host spins on a sentinel for every entry it reads, with or without
        // polling (an event wait then only saves the spinning)
        uint64_t* r = reinterpret_cast<uint64_t*>(c->hring);
        for (size_t i = 0; i < (size_t)maxit * LH; ++i) r[i] = RING_SENTINEL;
        for (size_t i = offM; i < offM + 2 * (size_t)maxit; ++i) r[i] = RING_SENTINEL;
        if (poll)
            for (size_t i = offS; i < offS + 3; ++i) r[i] = RING_SENTINEL;
        for (size_t i = offQG; i < ring_n; ++i) r[i] = RING_SENTINEL;
    }
    T* dr = zc ? c->hring_dev : c->buf<T>("ring_dev", ring_n);
    auto publish = [&](size_t off, size_t cnt) {
        if (!zc)
            HGM_HIP(hipMemcpyAsync(c->hring + off, dr + off, sizeof(T) * cnt, hipMemcpyDeviceToHost, c->stream));
    };
    // inputs staged after the ring reset (its stream sync then finds the GPU idle)
    const T* b = stage_in<T>(c, "in_b", b_in, m, dev);
    const T* xt = stage_in_n<T>(c, "in_xt", xt_in, n, dev, po);
    fill<T>(c, n, x, T(0));

    std::vector<double> H((size_t)(maxit + 1) * maxit, 0.0);
    std::vector<double> err(maxit, 0.0), res(maxit, 0.0);
    auto Hh = [&](int i, int j) -> double& { return H[(size_t)j * (maxit + 1) + i]; };

    // ||b|| (m, replicated) and ||x_true|| (n, sharded) — MATLAB recomputes them every
    // iteration (hybrid_*_rtp.m:32-33); the values are loop-invariant.
    double nb = 0, nxt = 0, beta = 0, xt2 = 0;
    T* q0 = Q;
    // (a communicator all-reduces the x_true norm over the pixel shards: the second branch, whatever
    // stream the reconstructions use)
    if (poll && dev && rs_stream != st && !dist_n(c)) {
        // no host round trip before the first step: the norms land in the ring (read at
        // iteration 0) and r0 is divided on the device.  With device inputs the two norms
        // run on the aux stream, beside B*b (x_true in the caller's order: same norm).
        StreamScope scope(c, rs_stream, "aux:");
        sumsq<T>(c, m, b, dr + offS + 1);
        sumsq<T>(c, n, reinterpret_cast<const T*>(xt_in), dr + offS + 2);   // ||x_true - 0||^2
    } else if (poll && dist_n(c)) {
        sumsq<T>(c, m, b, dr + offS + 1);                    // (m: replicated)
        sumsq<T>(c, n, xt, dslot<T>(c, S_NXT));              // ||x_true - 0||^2 over the pixel shards
        allreduce(c, dslot<T>(c, S_NXT), 1);
        copy_sys(c, dslot<T>(c, S_NXT), dr + offS + 2);
    } else if (poll) {
        sumsq<T>(c, m, b, dr + offS + 1);
        sumsq<T>(c, n, xt, dr + offS + 2);                   // ||x_true - 0||^2
    } else {
        sumsq<T>(c, m, b, dslot<T>(c, S_NB));
        nsumsq_diff<T>(c, n, xt, x, dslot<T>(c, S_NXT));   // ||x_true - 0||^2
    }
    // r0
    if (nspace) {
        apply_B<T>(c, B, b, q0, EPI_NONE, T(0), nullptr);   // d = B*b   (hybrid_*_rtp.m:7,9; *_bounds r0 = B*(b - A*0))
    } else {
        HGM_HIP(hipMemcpyAsync(q0, b, sizeof(T) * m, hipMemcpyDeviceToDevice, st));   // r0 = b - A*(B*0) = b
    }
    if (poll) {
        normalize_to<T>(c, dim, q0, dr + offS);           // :10,:13  beta = norm(r0); Q(:,1) = r0 / beta
    } else {
        if (nspace) nsumsq<T>(c, dim, q0, dslot<T>(c, S_BETA));
        else sumsq<T>(c, dim, q0, dslot<T>(c, S_BETA));
        read_scalars(c, 0, 3);
        nb = std::sqrt(c->hscal[S_NB]);
        nxt = std::sqrt(c->hscal[S_NXT]);
        xt2 = c->hscal[S_NXT];
        beta = std::sqrt(c->hscal[S_BETA]);               // :10  beta = norm(r0)
        div_scalar<T>(c, dim, q0, q0, (T)beta);           // :13  Q(:,1) = r0 / beta
    }

    bool x_assigned = sp.x_preassigned;
    int k = 0;
    std::vector<double> y, rhs, M;
    std::vector<double> G((size_t)maxit * maxit, 0.0), cvec(maxit, 0.0);
    // Gram error monitor: Q'Q, Q'x_true and the errors it produced (-1: formed explicitly)
    // (m-space: the Gram of Z = B*Q, from H and the strictly lower Q'Q in SQ)
    std::vector<double> GQ(gem ? (size_t)maxit * maxit : 0), cq(maxit, 0.0), gerr(maxit, -1.0);
    std::vector<double> SQ(gem_ab ? (size_t)maxit * maxit : 0);
    // Pending normalisation (one-reduction MGS): step k leaves v_{k+1} = Q(:,k+1)
    // undivided and step k+1 applies q = v / H(k+1,k) where it reads it — n-space (single GPU):
    // A: (A*v)/h, which also publishes h = H(k+1,k); B: B*(A*q) + lambda*q; m-space: the one pass
    // over B stages q = v/h and publishes h; the MGS dots kernel writes q back over v — so the
    // sweep needs no scale pass.  Step k's event is then
    // recorded at the end of step k+1.  HGM_OPT_PEND_NORM = 0 keeps the scale pass.
    // m-space side with B = A' value for value: B*q and A*(B*q) in one pass over B (fused.hip)
    const FusedPlan* fplan = nspace ? nullptr : fused_ab_plan(c, A, B);
    // (m-space, round 6: the one pass over B applies q = v / h as it stages q, so the m-space sweep
    // needs no scale pass either; the m-vectors are replicated, so this holds on a communicator too,
    // every rank forming the same h from the same replicated partials)
    // (m-space only with HGM_OPT_PEND_NORM = 2: the pass's staging then waits for the division, which
    // measured ~1.4 % slower at C4 than the scale pass it replaces)
    const bool pn_ok = !dist && orth == HGM_MGS && c->num.pend_norm >= 1 && !parity &&
                       (nspace ? spmv_pn_ok(A, EPI_DIVH) && spmv_pn_ok(B, EPI_ADDQ)
                               : c->num.pend_norm == 2 && std::is_same_v<T, double> && fplan != nullptr &&
                                     fused_pend_ok(c, fplan) && !krylov_padded(c, ldq));
    PendNorm<T> pend;                                  // np > 0: Q(:,next step) awaits its division
    T* pn_h = c->buf<T>("pn_h", 2);
    // Enqueue Arnoldi step kq: operator application + orthogonalisation (+ Gram column).
    auto enqueue_step = [&](int kq) {
        bool zx_fused = false;                            // x_true'(B*q_k) formed by the fused pass
        bool zx_rode = false;                             // ... and summed over the ranks with A*(B*q_k)
        T* qk = Q + (int64_t)kq * ldq;
        T* v = Q + (int64_t)(kq + 1) * ldq;
        const bool pending_in = pend.np > 0;
        // ---- operator (hybrid_*_rtp.m:19 ; *_bounds.m:25) ----
        if (nspace && pending_in) {
            T* Aq = AQ ? AQ + (int64_t)kq * ldaq : t;
            PendNorm<T> pa = pend;
            pa.hdev = pn_h;
            pa.hring = dr + (size_t)(kq - 1) * LH + kq;    // H(kq, kq-1) of step kq-1
            spmv<T>(c, A, qk, Aq, EPI_DIVH, T(0), nullptr, KC_SPMV_A, nullptr, &pa);   // A*q = (A*v)/h
            PendNorm<T> pb;
            pb.hdev = pn_h;
            // B*(A*q) + lambda*q with q = v/h (lambda = 0: B*(A*q) + 0*q); the MGS dots kernel
            // writes q back over v
            spmv<T>(c, B, Aq, v, EPI_ADDQ, T(sp.lambda_in_op ? lambda : 0.0), qk, KC_SPMV_B, nullptr, &pb);
        } else if (nspace) {
            T* Aq = AQ ? AQ + (int64_t)kq * ldaq : t;
            apply_A<T>(c, A, qk, Aq, EPI_NONE, T(0), nullptr);
            if (sp.lambda_in_op) apply_B<T>(c, B, Aq, v, EPI_ADD, T(lambda), qk);   // B*(A*v) + lambda*v
            else apply_B<T>(c, B, Aq, v, EPI_NONE, T(0), nullptr);                  // B*(A*v)
        } else {
            T* Bq = BQ ? BQ + (int64_t)kq * ldbq : tn;
            // A*(B*Q(:,k)) lands in its kept column (MGS reads it from there and writes the
            // orthogonalised vector to Q(:,k+1), no copy), or in Q(:,k+1) for CGS2
            T* w = (ABQ && orth != HGM_CGS2) ? ABQ + (int64_t)kq * ldaq : v;
            if (fplan) {
                // both in one pass over B; with the m-space Gram error monitor the pass also forms
                // the side dot x_true'(B*Q(:,k)) (else the MGS sweep's extra workgroups do)
#ifndef HGM_FUSED_ZX
#define HGM_FUSED_ZX 1
#endif
                const bool zxf = HGM_FUSED_ZX && gem_ab;
                // (on a communicator the rank-local dot goes to a device slot, all-reduced below)
                T* zx_dst = zxf ? (dist_n(c) ? dslot<T>(c, S_AUX2) : dr + offQG + (size_t)kq * LQ + kq + 2) : nullptr;
                // on a communicator the side dot rides the m-vector all-reduce as its element m
                // (when the column's stride leaves room past m): one collective per step, not two
                const int64_t wld = (ABQ && orth != HGM_CGS2) ? ldaq : ldq;
                const bool ride = zxf && dist_n(c) && wld > m;
                PendNorm<T> pq;                                // q_k = v_k / H(k,k-1) as the pass stages it
                if (pending_in) {
                    pq = pend;
                    pq.hdev = pn_h;
                    pq.hring = dr + (size_t)(kq - 1) * LH + kq;  // H(kq, kq-1) of step kq-1
                }
                if constexpr (std::is_same_v<T, double>)
                    zx_fused = fused_ab(c, B, fplan, qk, Bq, w, zxf ? xt : nullptr, ride ? w + m : zx_dst,
                                        pending_in ? &pq : nullptr);
                zx_rode = ride && zx_fused;
                if (dist_n(c)) allreduce(c, w, zx_rode ? m + 1 : m);             // (as apply_A)
                // (the all-reduced side dot goes into the ring with the MGS sweep below)
            } else {
                apply_B<T>(c, B, qk, Bq, EPI_NONE, T(0), nullptr);                  // B*Q(:,k)
                apply_A<T>(c, A, Bq, w, EPI_NONE, T(0), nullptr);                   // A*(B*Q(:,k))
            }
            if (ABQ && orth == HGM_CGS2)
                HGM_HIP(hipMemcpyAsync(ABQ + (int64_t)kq * ldaq, v, sizeof(T) * m, hipMemcpyDeviceToDevice,
                                       c->stream));
        }
        // ---- orthogonalisation (hybrid_*_rtp.m:20-26) ----
        T* Hcol = dr + (size_t)kq * LH;                  // -> host H(:,k)
        // column k of AQk'*AQk and AQk'*b (hybrid_ab_gmres_rtp.m:31-32); A*Q(:,j) was
        // computed inside M_reg_op(Q(:,j)) at :19 — the same deterministic SpMV.  With MGS
        // it runs as extra workgroups of the sweep's first two passes.
        MdotJob<T> gram;
        if (sp.proj == PROJ_ABRTP) {
            gram.n = m;
            gram.ncols = kq + 1;
            gram.Q = AQ;
            gram.ldq = ldaq;
            gram.w = AQ + (int64_t)kq * ldaq;
            gram.e = b;                                   // + b'*AQ(:,k)
            gram.out = Hcol + (maxit + 2);
        }
        const MdotJob<T>* side = sp.proj == PROJ_ABRTP ? &gram : nullptr;
        if (orth == HGM_CGS2) {
            cgs2<T>(c, dim, Q, ldq, kq, Hcol, dist);
            if (side) multidot<T>(c, m, gram.ncols, AQ, ldaq, gram.w, gram.out, b);
        } else {
            PendNorm<T>* defer = (pn_ok && kq + 1 < maxit) ? &pend : nullptr;
            if (!defer) pend.np = 0;
            MdotJob<T> zx;                                // gem_ab: x_true'(B*q_k) -> row entry k+2
            T* zx_ring = dr + offQG + (size_t)kq * LQ + kq + 2;
            if (gem_ab) {
                zx.n = n;
                zx.w = BQ + (int64_t)kq * ldbq;
                zx.e = xt;
                zx.out = dist_n(c) ? dslot<T>(c, S_AUX2) : zx_ring;   // (the fused pass's zx_dst too)
            }
            // the Gram row's extra dot: x_true (n-space) or b (m-space, unused: the row is for L)
            const double* cps = nullptr;
            double* cpd = nullptr;
            if constexpr (std::is_same_v<T, double>)
                if (zx_rode) {
                    cps = reinterpret_cast<const double*>(ABQ ? ABQ + (int64_t)kq * ldaq + m : v + m);
                    cpd = dr + offQG + (size_t)kq * LQ + kq + 2;
                }
            mgs<T>(c, dim, Q, ldq, kq, Hcol, dist, (!nspace && ABQ) ? ABQ + (int64_t)kq * ldaq : nullptr,
                   gem_ab ? (zx_fused ? nullptr : &zx) : side, defer, pending_in ? (const T*)pn_h : nullptr,
                   gem ? (gem_n ? xt : b) : nullptr, gem ? dr + offQG + (size_t)kq * LQ : nullptr, cps, cpd);
            if (gem_ab && dist_n(c) && !zx_rode) {        // x_true'(B*q_k) over the pixel shards
                allreduce(c, zx.out, 1);
                if constexpr (std::is_same_v<T, double>) copy_sys(c, zx.out, zx_ring);
            }
        }
        // Step kq-1's column is complete (H(kq,kq-1) came from this step's A product).  The
        // event goes at the end of the step: a marker between two kernels costs a bubble.
        if (poll) return;                                 // the host polls the ring instead
        if (pending_in) {
            publish((size_t)(kq - 1) * LH, LH);
            if (gem_ab) publish(offQG + (size_t)(kq - 1) * LQ, (size_t)kq + 2);   // its Gram row
            step_record(c, kq - 1);
        }
        if (pend.np == 0) {                               // else: recorded at the end of step kq+1
            publish((size_t)kq * LH, LH);
            if (gem_ab) publish(offQG + (size_t)kq * LQ, (size_t)kq + 3);   // the Gram row (m-space)
            step_record(c, kq);
        }
    };
    // Reconstruction + monitors of iteration kq from y_kq (in the ring) on the auxiliary
    // stream, then the event the host waits on.  Everything it reads (Q(:,0..kq), y_kq)
    // is complete when it is enqueued (the host has seen step kq finish), so it needs no
    // stream dependency; it writes only x, its own scratch and ring slot kq.
    int x_pending = -1;   // the last reconstruction, when it left x unformed (Gram error monitor)
    auto enqueue_recon = [&](int kq, bool want_x) {
        StreamScope scope(c, (rs_aux_dist && want_x) ? st : rs_stream, (rs_aux_dist && want_x) ? "" : "aux:");
        const int kk = kq + 1;
        const T* yk = c->hring_dev + offY + (size_t)kq * maxit;
        T* rslot = dr + offM + 2 * (size_t)kq;
        T* eslot = rslot + 1;
        // an error sum over the pixel shards is all-reduced in a device slot, then copied into the
        // (host-mapped) ring
        T* eloc = (dist_n(c) && zc) ? dslot<T>(c, S_ERR) : eslot;
        auto err_done = [&](bool reduce) {
            if (reduce && dist_n(c)) allreduce(c, eloc, 1);
            if constexpr (std::is_same_v<T, double>)
                if (eloc != eslot) copy_sys(c, eloc, eslot);
        };
        // ---- reconstruction (hybrid_*_rtp.m:30/33 ; *_bounds.m:37-38) ----
        if (aq_res) {
            // x = Q(:,1:k)*yk with ||x - x_true||^2 (:33/:36) and ||b - A*x||^2 (:32/:35)
            // evaluated as ||b - (A*Q(:,1:k))*yk||^2, all in one launch (+ finalize)
            // (want_x false: the Gram error monitor has the error, x is formed at the end)
            recon<T>(c, n, kk, Q, ldq, yk, want_x ? x : nullptr, xt, eslot, m, AQ, ldaq, b, rslot);
            x_pending = want_x ? -1 : kq;
            if (dist_n(c)) allreduce(c, eslot, 1);
            publish(offM + 2 * (size_t)kq, 2);
            if (pipe_ev) pipe_record(c);
            return;
        }
        if (bq_res) {
            // xk = B*(Q(:,1:k)*yk) = (B*Q(:,1:k))*yk with ||xk - x_true||^2, and
            // ||b - A*xk||^2 = ||b - (A*B*Q(:,1:k))*yk||^2 (*_bounds.m:37-40), one launch
            // (want_x false: the m-space Gram error monitor has the error, x is formed at the end)
            recon<T>(c, n, kk, BQ, ldbq, yk, want_x ? x : nullptr, xt, eloc, m, ABQ, ldaq, b, rslot);
            x_pending = want_x ? -1 : kq;
            if (want_x) err_done(true);
            publish(offM + 2 * (size_t)kq, 2);
            if (pipe_ev) pipe_record(c);
            return;
        }
        if (nspace) {
            // x = Q(:,1:k)*yk, fused with the error monitor ||x - x_true||^2 (:33 / :36)
            gemv_err<T>(c, n, kk, Q, ldq, yk, x, xt, eslot);
            if (dist_n(c)) allreduce(c, eslot, 1);
        } else {
            gemv<T>(c, m, kk, Q, ldq, yk, z, 0);                 // zk = Q(:,1:k)*yk
            apply_B<T>(c, B, z, x, EPI_NONE, T(0), nullptr);     // xk = B*zk
            sumsq_diff<T>(c, n, x, xt, eloc);
            err_done(true);
        }
        // ---- monitors (hybrid_*_rtp.m:32-33 / :35-36): norm(b - A*x) ----
        if (!dist_n(c)) {
            spmv<T>(c, A, x, tr, EPI_RSUB, T(0), b, KC_SPMV_A, rslot);   // sum of squares fused
        } else {
            apply_A<T>(c, A, x, tr, EPI_RSUB, T(0), b);
            sumsq<T>(c, m, tr, rslot);
        }
        publish(offM + 2 * (size_t)kq, 2);
        if (pipe_ev) pipe_record(c);
    };
    // Software pipeline over two streams, L = HGM_OPT_PIPE_DEPTH:
    //     main: S0 S1 S2 S3 ...          (S_k: Arnoldi step k -> H(:,k), Q(:,k+1))
    //     aux :       R0 R1 R2 ...       (R_k: x = Q y_k, monitors of iteration k)
    // At iteration k the host waits for S_k and R_{k-1}, solves for y_k, enqueues R_k
    // and then S_{k+L+1}; the GPU meanwhile runs S_{k+1..k+L} and overlaps R_k with
    // them, so it never waits for the host.  When `residual_norm(k) <= tol` stops the loop the
    // speculative steps are discarded: they write only Q(:,>k+1), AQ(:,>k), their own
    // ring slots and scratch — never x or a history — so every output equals the
    // reference's.  (Multi-GPU: both sequences share one stream, same semantics.)
    const int L = c->num.pipe_depth;                     // speculative steps in flight
    for (int j = 0; j <= L && j < maxit; ++j) enqueue_step(j);
    // the mapped-ring entries of step kq (H column, Gram column, Gram error row)
    auto wait_step = [&](int kq) {
        std::vector<size_t> idx;
        for (int i = 0; i < kq + 2; ++i) idx.push_back((size_t)kq * LH + i);
        if (sp.proj == PROJ_ABRTP)
            for (int i = 0; i < kq + 2; ++i) idx.push_back((size_t)kq * LH + (maxit + 2) + i);
        if (gem)
            for (int i = 0; i < kq + 2; ++i) idx.push_back(offQG + (size_t)kq * LQ + i);
        if (gem_ab) idx.push_back(offQG + (size_t)kq * LQ + kq + 2);
        ring_wait(c, hr, idx);
    };
    // the monitors of reconstruction R_kq (the error slot is not written when the Gram error
    // monitor supplied the error)
    auto wait_mon = [&](int kq) {
        if (!zc) return;
        std::vector<size_t> idx{offM + 2 * (size_t)kq};
        if (gerr[kq] < 0) idx.push_back(offM + 2 * (size_t)kq + 1);
        ring_wait(c, hr, idx, rs_stream);
    };
    bool done = false;
    for (k = 0; k < maxit; ++k) {
        if (k >= 1) {                                    // R_{k-1}
            if (pipe_ev) pipe_wait(c);
            wait_mon(k - 1);
        }
        if (poll) {
            // S_k: H(0:k+1,k) (+ Gram column k).  H(k+1,k) is written by a kernel that starts
            // after every kernel of step k has finished (the scale pass of step k, or with the
            // pending normalisation the A product of step k+1), so once it is visible Q(:,0:k)
            // and the kept products of step k, which R_k reads, are complete.
            wait_step(k);
            if (k == 0) {                                // the setup norms (written before step 0;
                                                         // with device inputs partly on the aux stream)
                ring_wait(c, hr, {offS, offS + 1, offS + 2}, rs_stream);
                beta = hr[offS];
                nb = std::sqrt(hr[offS + 1]);
                nxt = std::sqrt(hr[offS + 2]);
                xt2 = hr[offS + 2];
            }
        } else {
            step_wait(c, k);                             // S_k: H(:,k) (+ Gram column k)
            if (zc) wait_step(k);
        }
        if (k >= 1) {
            const double* mk = hr + offM + 2 * (size_t)(k - 1);
            res[k - 1] = std::sqrt(mk[0]) / nb;
            err[k - 1] = gerr[k - 1] >= 0 ? gerr[k - 1] : std::sqrt(mk[1]) / nxt;
            if (res[k - 1] <= tol) {                     // :35 / :38 / *_bounds :79-83
                k = k - 1;
                done = true;
                break;
            }
        }
        const double* hk = hr + (size_t)k * LH;
        for (int i = 0; i < k + 2; ++i) Hh(i, k) = hk[i];
        if (sp.proj == PROJ_ABRTP) {
            for (int i = 0; i <= k; ++i) G[(size_t)k * maxit + i] = hk[(maxit + 2) + i];
            cvec[k] = hk[(maxit + 2) + k + 1];
        }
        if (gem_n) {
            const double* gk = hr + offQG + (size_t)k * LQ;
            for (int i = 0; i < k; ++i) GQ[(size_t)k * maxit + i] = GQ[(size_t)i * maxit + k] = gk[i];
            GQ[(size_t)k * maxit + k] = gk[k];
            cq[k] = gk[k + 1];
        } else if (gem_ab) {
            // z_j'z_k = q_j'(A*B*q_k) = H(j,k) + sum_{i<j} (q_j'q_i) H(i,k): the sweep solved
            // (I + L) h = Q'w_k for h = H(0:k,k), so this is its right-hand side again
            const double* gk = hr + offQG + (size_t)k * LQ;
            for (int i = 0; i < k; ++i) SQ[(size_t)k * maxit + i] = gk[i];
            for (int j = 0; j <= k; ++j) {
                long double g = Hh(j, k);
                for (int i = 0; i < j; ++i) g += (long double)SQ[(size_t)j * maxit + i] * Hh(i, k);
                GQ[(size_t)k * maxit + j] = GQ[(size_t)j * maxit + k] = (double)g;
            }
            cq[k] = gk[k + 2];
        }
        if (Hh(k + 1, k) == 0) {                         // :25  if H(k+1,k) == 0, break
            done = true;
            break;
        }
        const int kk = k + 1;                            // MATLAB k
        y.assign(kk, 0.0);
        if (sp.proj == PROJ_LS) {
            // yk = H(1:k+1,1:k) \ [beta; zeros(k,1)]   (hybrid_ba_gmres_rtp.m:28-29)
            M.assign((size_t)(kk + 1) * kk, 0.0);
            for (int j = 0; j < kk; ++j)
                for (int i = 0; i <= kk; ++i) M[(size_t)j * (kk + 1) + i] = Hh(i, j);
            rhs.assign(kk + 1, 0.0);
            rhs[0] = beta;
            dense::qr_ls(kk + 1, kk, M.data(), rhs.data(), y.data());
        } else if (sp.proj == PROJ_PTR) {
            // yk = (Hk'*Hk + lambda*eye(k)) \ (Hk'*tk)   (*_hybrid_bounds.m:34-36)
            M.assign((size_t)kk * kk, 0.0);
            for (int i = 0; i < kk; ++i)
                for (int j = 0; j < kk; ++j) {
                    double s = 0;
                    for (int r = 0; r <= kk; ++r) s += Hh(r, i) * Hh(r, j);
                    M[(size_t)j * kk + i] = s + (i == j ? lambda : 0.0);
                }
            rhs.assign(kk, 0.0);
            for (int i = 0; i < kk; ++i) rhs[i] = Hh(0, i) * beta;
            dense::mldivide_square(kk, M.data(), rhs.data(), y.data());
        } else {
            // yk = (AQk'*AQk + lambda*eye(k)) \ (AQk'*b)   (hybrid_ab_gmres_rtp.m:32)
            M.assign((size_t)kk * kk, 0.0);
            for (int j = 0; j < kk; ++j)
                for (int i = 0; i <= j; ++i) {
                    const double g = G[(size_t)j * maxit + i];
                    M[(size_t)j * kk + i] = g;
                    M[(size_t)i * kk + j] = g;
                }
            for (int i = 0; i < kk; ++i) M[(size_t)i * kk + i] += lambda;
            dense::mldivide_square(kk, M.data(), cvec.data(), y.data());
        }
        std::memcpy(c->hring + offY + (size_t)k * maxit, y.data(), sizeof(double) * kk);
        bool want_x = true;
        // (the last iteration's reconstruction forms x anyway: there the GEMV carries the error)
        if (gem && k + 1 < maxit) {
            // ||Q y - x_true||^2 = x_true'x_true - 2 y'(Q'x_true) + y'(Q'Q) y (hybrid_*_rtp.m:33/:36
            // with x = Q y), used when it is at least gem_min ||x_true||^2 (the cancellation then
            // costs at most a factor 1/gem_min of the terms' rounding)
            long double e2 = xt2;
            for (int i = 0; i < kk; ++i) {
                long double gy = 0;
                for (int j = 0; j < kk; ++j) gy += (long double)GQ[(size_t)i * maxit + j] * y[j];
                e2 += (long double)y[i] * (gy - 2.0L * cq[i]);
            }
            if (xt2 > 0 && e2 >= (long double)gem_min * xt2) {
                gerr[k] = std::sqrt((double)e2) / nxt;
                want_x = false;
            }
        }
        c->path_mon.push_back(want_x ? 0 : 1);
        enqueue_recon(k, want_x);
        x_assigned = true;
        if (k + L + 1 < maxit) enqueue_step(k + L + 1);  // speculative, see above
    }
    if (x_pending >= 0) {
        // the last reconstruction left x unformed (Gram error monitor): x = Q(:,0:k) y_k
        // behind it, on the same stream
        StreamScope scope(c, rs_stream, "aux:");
        const T* yk = c->hring_dev + offY + (size_t)x_pending * maxit;
        if (nspace) gemv<T>(c, n, x_pending + 1, Q, ldq, yk, x, 0);
        else gemv<T>(c, n, x_pending + 1, BQ, ldbq, yk, x, 0);          // x = (B*Q) y
        x_pending = -1;
    }
    bool staged = false;
    if (!done) {
        // all maxit iterations ran: the last monitors are still outstanding.  With the
        // reconstruction on the aux stream, x is staged out behind it there (one sync, no
        // host wake-up in between).
        // (x_out == NULL: nothing to stage, so wait for the last monitors explicitly)
        // (a communicator's last reconstruction formed x on the step stream: staged out there below)
        if (rs_stream != st && !rs_aux_dist && x_assigned && x_out != nullptr) {
            StreamScope scope(c, rs_stream, "aux:");
            stage_out_n<T>(c, x_out, x, n, dev, po);     // ends with a sync of the aux stream
            staged = true;
        } else if (pipe_ev) {
            pipe_wait(c);
        }
        k = maxit - 1;
        wait_mon(k);
        const double* mk = hr + offM + 2 * (size_t)k;
        res[k] = std::sqrt(mk[0]) / nb;
        err[k] = gerr[k] >= 0 ? gerr[k] : std::sqrt(mk[1]) / nxt;
    }
    if (k == maxit) k = maxit - 1;
    const int nit = k + 1;                               // niters = k
    if (rs_stream != st) stream_sync(rs_stream);
    if (!x_assigned) throw Error{HGM_E_NOT_ASSIGNED, "Output argument \"x\" not assigned during call (breakdown at k = 1)"};
    if (!staged) stage_out_n<T>(c, x_out, x, n, dev, po);
    if (c->host_stats) {
        const double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
        std::fprintf(stderr, "hgm gmres: %d iters, %.1f us total, %.1f us blocked in %ld waits\n", nit, tot * 1e6,
                     (c->wait_s - wait0) * 1e6, c->waits - waits0);
    }
    if (err_out) std::memcpy(err_out, err.data(), sizeof(double) * nit);
    if (res_out) std::memcpy(res_out, res.data(), sizeof(double) * nit);
    if (niters) *niters = nit;
    if (o && o->H_out) std::memcpy(o->H_out, H.data(), sizeof(double) * H.size());
    return HGM_OK;
}

// ============================================================================
// LSQR (lsqr_solver.m) and hybrid LSQR on [A; sqrt(lambda) I] (hybrid_lsqr_solver.m)
// ============================================================================
template <typename T>
int lsqr_t(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* At, const double* b_in,
           const double* xt_in, double tol, int maxit, bool hybrid, double lambda, double* x_out,
           double* err_out, double* res_out, int* niters) {
    check_dims(A, At);
    solver_guard(c);
    HGM_REQUIRE(At != nullptr, "At is NULL");
    const PixOrder po = n_order(c, A, At);
    HGM_REQUIRE(b_in != nullptr && xt_in != nullptr, "b and x_true are required");
    HGM_REQUIRE(maxit >= 1, "maxit must be >= 1");
    const bool parity = c->num.parity;   // fixed summation orders
    HGM_REQUIRE(!parity || (!dist_n(c) && po.trivial()), "parity mode: single rank, reference pixel order");
    const bool dev = o && (o->flags & HGM_DEVICE_PTRS);
    const int64_t m = A->rows, n = A->cols;
    const T* b = stage_in<T>(c, "in_b", b_in, m, dev);
    const T* xt = stage_in_n<T>(c, "in_xt", xt_in, n, dev, po);
    T* x = c->buf<T>("x", n + 1);
    T* w = c->buf<T>("w", n + 1);
    T* v = c->buf<T>("v", n + 1);
    T* u = c->buf<T>("u", m + 1);
    T* un = hybrid ? c->buf<T>("u_n", n + 1) : nullptr;    // lower block of u_aug
    T* t = c->buf<T>("t_m", m + 1);
    T* sl = reinterpret_cast<T*>(c->dscal);
    const T sq = (T)std::sqrt(lambda);
    fill<T>(c, n, x, T(0));
    std::vector<double> err(maxit, 0.0), res(maxit, 0.0);

    sumsq<T>(c, m, b, sl + S_NB);
    nsumsq_diff<T>(c, n, xt, x, sl + S_NXT);
    std::vector<T> hs(4);
    Reader r0(c);
    r0.add(&hs[0], sl + S_NB, sizeof(T));
    r0.add(&hs[1], sl + S_NXT, sizeof(T));
    r0.go();
    const double nb = std::sqrt((double)hs[0]);
    const double nxt = std::sqrt((double)hs[1]);
    // One pass over the operator per iteration: with At = A' value for value on a
    // tiled pixel grid, the step v_hat = A'*u - beta*v (:26) and A*v_hat come out of one pass over
    // At (fused.hip, row epilogue), alpha^2 = ||v_hat||^2 as its side sum, and the next step's
    // A*v_{k+1} (:22) is (A*v_hat) / alpha: an m-vector operation instead of a second pass.
    // wm = [A*v_hat | alpha^2] (m + 1: alpha^2 rides the m-vector all-reduce on a communicator).
    const FusedPlan* fp = agreed_gk_plan<T>(c, A, At, !hybrid && !parity);
    T* wm = fp ? c->buf<T>("gkb_wm", m + 3) : nullptr;        // (+ the partials riding the all-reduce)
    // beta = norm(b) (lsqr_solver.m:7; hybrid: norm([b;0]) = norm(b), hybrid_lsqr_solver.m:9)
    double beta = nb;
    div_scalar<T>(c, m, b, u, (T)beta);                                        // :8  u = b / beta
    if (hybrid) fill<T>(c, n, un, T(0));                                       // u_aug = [b;0]/beta
    if (hybrid) {
        apply_B<T>(c, At, u, v, EPI_ADD, sq, un);                              // A_aug'*u_aug
    } else if (fp) {
        FusedArgs<T> fa;                                                       // :10 v_hat = A'*u, A*v_hat
        fa.q = u;
        fa.zraw = v;
        fa.w = wm;
        fa.side_sq = true;
        fa.side_out = wm + m;                                                  // ||v_hat||^2
        fused_pass<T>(c, At, fp, fa);
        if (dist_n(c)) allreduce(c, wm, m + 1);
    } else {
        apply_B<T>(c, At, u, v, EPI_NONE, T(0), nullptr);                      // :10 v_hat = A'*u
    }
    if (!fp) nsumsq<T>(c, n, v, sl + S_ALPHA);
    double alpha = std::sqrt((double)read1<T>(c, fp ? wm + m : sl + S_ALPHA));   // :11
    div_scalar<T>(c, n, v, v, (T)alpha);                                       // :12
    HGM_HIP(hipMemcpyAsync(w, v, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));   // :14 w = v
    double phi_bar = beta, rho_bar = alpha;                                    // :15-16
    // non-hybrid: the stop test uses phi_bar (host), so the error history (:43) stays on the
    // device and is read once after the loop instead of once per iteration
    T* errh = hybrid ? nullptr : c->buf<T>("lsqr_errh", maxit);
    double *img_ax = nullptr, *img_aw = nullptr;   // (one-pass) A*x, A*w images for :52
    int k = 0;
    // Device-resident scalars (single rank, production kernels): beta and alpha stay on the
    // device as sums of squares, the SpMV epilogues read them there (PendNorm::asq), and the
    // Givens rotation (:31-38) and the stop test (:44-46) run in a one-thread kernel, in the same
    // double arithmetic as the host loop below -- the same bits, with no host round trip per
    // iteration.  The host reads the stop flag once per batch of iterations (none when tol <= 0
    // cannot stop early); an iteration enqueued past the stop leaves x and w untouched.
    const bool dev_scalars = !fp && !hybrid && !parity && !dist_n(c) && c->num.lsqr_dev;
    if (fp) {
        // one pass per iteration, device-resident scalars (as below; on a communicator too: alpha^2
        // rides the m-vector all-reduce, beta^2 is a sum over the replicated m-vector)
        double* st = c->buf<double>("lsqr_st", 4);
        double* phib = c->buf<double>("lsqr_phib", maxit);
        T* coef = c->buf<T>("lsqr_coef", 2);
        const double st0[4] = {rho_bar, phi_bar, 0.0, 0.0};
        h2d(c, st, st0, sizeof(st0));
        FusedArgs<T> fa;
        fa.q = u;
        fa.ev = v;                                 // v_k (divided by the previous lsqr_step)
        fa.easq = sl + S_BETA;
        fa.zout = v;                               // v_hat_{k+1} in place
        fa.w = wm;
        fa.side_sq = true;
        fa.side_out = wm + m;
        // HGM_OPT_LSQR_DEV = 0: the same pass with host scalars -- beta^2 and alpha^2 read back per
        // iteration, the rotation and the stop test on the host in the same double arithmetic as
        // k_lsqr_rot (the coefficients uploaded for lsqr_step), so the iterates keep their bits
        const bool host_sc = !c->num.lsqr_dev;
        const int batch = tol > 0 && !host_sc ? 8 : maxit;
        int stop = 0;
        // On a communicator the error partial ||x - x_true||^2 (:43, summed over the pixel shards)
        // rides the NEXT iteration's m-vector all-reduce as element m+1, and the rotation kernel after
        // that all-reduce copies the sum into the history: one collective per iteration instead of
        // two (the stop test uses phi_bar, replicated).  The last iteration's partial is summed after
        // the loop.
        const bool ride = dist_n(c) && !host_sc;
        T* ride_e = ride ? wm + m + 1 : nullptr;
        if (ride) HGM_HIP(hipMemsetAsync(ride_e, 0, sizeof(T), c->stream));
        int last = -1;
        // the final residual (:52) from A*x kept alongside x (A*v_k is the pass's A*v_hat / alpha):
        // no SpMV after the loop (HGM_OPT_LSQR_RES_IMG)
        if (c->num.lsqr_res_img) {
            img_ax = c->buf<double>("lsqr_ax", m + 1);
            img_aw = c->buf<double>("lsqr_aw", m + 1);
            lsqr_img<T>(c, m, wm, wm + m, coef, st, 0, img_ax, img_aw, true);
        }
        for (k = 0; k < maxit && stop == 0;) {
            const int kend = std::min(maxit, k + batch);
            for (; k < kend; ++k) {
                gkb_mstep_div<T>(c, m, wm, wm + m, u, t, nullptr, sl + S_BETA, false);   // :22-24
                fused_pass<T>(c, At, fp, fa);                                        // :26-27 (+ A*v_hat)
                if (dist_n(c)) allreduce(c, wm, (ride && k > 0) ? m + 2 : m + 1);
                if (host_sc) {
                    T ss[2] = {T(0), T(0)};
                    Reader rr(c);
                    rr.add(&ss[0], sl + S_BETA, sizeof(T));
                    rr.add(&ss[1], wm + m, sizeof(T));
                    rr.go();
                    beta = std::sqrt((double)ss[0]);                                 // :23
                    alpha = std::sqrt((double)ss[1]);                                // :27
                    const double rho = std::sqrt(rho_bar * rho_bar + beta * beta);   // :31-38
                    const double cs = rho_bar / rho, sn = beta / rho;
                    const double theta = sn * alpha;
                    rho_bar = -cs * alpha;
                    const double phi = cs * phi_bar;
                    phi_bar = sn * phi_bar;
                    const T cf[2] = {(T)(phi / rho), (T)(theta / rho)};
                    h2d_pinned(c, coef, cf, sizeof(cf));    // the next Reader syncs past its use
                    res[k] = std::fabs(phi_bar) / nb;                                // :44
                    if (res[k] <= tol) stop = k + 1;                                 // :46 (<=)
                } else {
                    ScalarCopy<T> cp;
                    if (ride && k > 0) {
                        cp.src = ride_e;
                        cp.dst = errh + k - 1;
                    }
                    lsqr_rot<T>(c, sl + S_BETA, wm + m, st, coef, phib, k, nb, tol, cp);   // :31-38, :44-46
                }
                lsqr_step<T>(c, n, x, w, v, wm + m, coef, st, k, xt, ride ? ride_e : errh + k);   // :28, :40-41, :43
                last = k;
                if (img_ax) lsqr_img<T>(c, m, wm, wm + m, coef, st, k, img_ax, img_aw, false);
                if (dist_n(c) && !ride) allreduce(c, errh + k, 1);
                if (stop) {
                    ++k;
                    break;
                }
            }
            if (host_sc) continue;
            double sv = 0;
            Reader rs(c);
            rs.add(&sv, st + 2, sizeof(double));
            rs.go();
            stop = (int)sv;
        }
        if (ride && last >= 0) {                       // the last iteration's error partial
            allreduce(c, ride_e, 1);
            ScalarCopy<T> cp;
            cp.src = ride_e;
            cp.dst = errh + last;
            copy_scalars<T>(c, cp);
        }
        k = stop > 0 ? stop - 1 : maxit;
        if (!host_sc) {
            std::vector<double> pbh(maxit);
            Reader rh(c);
            rh.add(pbh.data(), phib, sizeof(double) * maxit);
            rh.go();
            for (int i = 0; i < maxit && i <= k; ++i) res[i] = std::fabs(pbh[i]) / nb;   // :44
        }
    }
    if (dev_scalars) {
        double* st = c->buf<double>("lsqr_st", 4);
        double* phib = c->buf<double>("lsqr_phib", maxit);
        T* coef = c->buf<T>("lsqr_coef", 2);
        const double st0[4] = {rho_bar, phi_bar, 0.0, 0.0};
        h2d(c, st, st0, sizeof(st0));
        PendNorm<T> pa, pb;
        pa.asq = sl + S_ALPHA;                     // A*v - alpha*u
        pb.asq = sl + S_BETA;                      // A'*u - beta*v
        const int batch = tol > 0 ? 8 : maxit;
        int stop = 0;
        for (k = 0; k < maxit && stop == 0;) {
            const int kend = std::min(maxit, k + batch);
            for (; k < kend; ++k) {
                spmv<T>(c, A, v, t, EPI_SUB, T(0), u, KC_SPMV_A, nullptr, &pa);     // :22
                sumsq<T>(c, m, t, sl + S_BETA);                                      // :23
                div_sqrt<T>(c, m, t, u, sl + S_BETA);                                // :24
                spmv<T>(c, At, u, v, EPI_SUB, T(0), v, KC_SPMV_B, nullptr, &pb);     // :26
                sumsq<T>(c, n, v, sl + S_ALPHA);                                     // :27
                lsqr_rot<T>(c, sl + S_BETA, sl + S_ALPHA, st, coef, phib, k, nb, tol);   // :31-38, :44-46
                lsqr_step<T>(c, n, x, w, v, sl + S_ALPHA, coef, st, k, xt, errh + k);     // :28, :40-41, :43
            }
            double sv = 0;
            Reader rs(c);
            rs.add(&sv, st + 2, sizeof(double));
            rs.go();
            stop = (int)sv;
        }
        k = stop > 0 ? stop - 1 : maxit;
        std::vector<double> pbh(maxit);
        Reader rh(c);
        rh.add(pbh.data(), phib, sizeof(double) * maxit);
        rh.go();
        for (int i = 0; i < maxit && i <= k; ++i) res[i] = std::fabs(pbh[i]) / nb;   // :44
    }
    for (; !dev_scalars && !fp && k < maxit; ++k) {
        // :22-24  u_hat = A*v - alpha*u ; beta = norm(u_hat) ; u = u_hat / beta
        apply_A<T>(c, A, v, t, EPI_SUB, (T)alpha, u);
        sumsq<T>(c, m, t, sl + S_BETA);
        if (hybrid) {
            // lower block of u_hat: (sqrt(lambda)*v) - (alpha*u_n), same norm as the upper block
            T* tl = c->buf<T>("t_n", n + 1);
            fill<T>(c, n, tl, T(0));
            epilogue<T>(c, n, tl, EPI_ADD, sq, v);                     // tl = 0 + sq*v (exact: sq*v)
            epilogue<T>(c, n, tl, EPI_SUB, (T)alpha, un);              // tl = tl - alpha*u_n
            if (parity) {
                // norm of the augmented [u_m; u_n] (:23) in one fixed order over the concatenation
                fixed_reduce<T>(c, 1, m, t, t, n, tl, tl, sl + S_BETA);
                HGM_HIP(hipMemsetAsync(sl + S_AUX, 0, sizeof(T), c->stream));
            } else {
                nsumsq<T>(c, n, tl, sl + S_AUX);
            }
            Reader rr(c);
            rr.add(&hs[0], sl + S_BETA, sizeof(T));
            rr.add(&hs[1], sl + S_AUX, sizeof(T));
            rr.go();
            beta = std::sqrt((double)(hs[0] + hs[1]));
            div_scalar<T>(c, m, t, u, (T)beta);
            div_scalar<T>(c, n, tl, un, (T)beta);
            // :26 v_hat = A_aug'*u_aug - beta*v = (A'*u + sq*un) - beta*v
            T* vh = c->buf<T>("t_n2", n + 1);   // A_aug'*u_aug reads v in the epilogue: not in place
            apply_B<T>(c, At, u, vh, EPI_ADD, sq, un);
            epilogue<T>(c, n, vh, EPI_SUB, (T)beta, v);
            HGM_HIP(hipMemcpyAsync(v, vh, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));
        } else {
            beta = std::sqrt((double)read1<T>(c, sl + S_BETA));
            div_scalar<T>(c, m, t, u, (T)beta);
            // :26 v_hat = A'*u - beta*v   (in place is safe: row i reads v(i) only in its epilogue)
            apply_B<T>(c, At, u, v, EPI_SUB, (T)beta, v);
        }
        nsumsq<T>(c, n, v, sl + S_ALPHA);
        alpha = std::sqrt((double)read1<T>(c, sl + S_ALPHA));                 // :27
        div_scalar<T>(c, n, v, v, (T)alpha);                                   // :28
        // :31-38 Givens rotation (host scalars)
        const double rho = std::sqrt(rho_bar * rho_bar + beta * beta);
        const double cs = rho_bar / rho;
        const double sn = beta / rho;
        const double theta = sn * alpha;
        rho_bar = -cs * alpha;
        const double phi = cs * phi_bar;
        phi_bar = sn * phi_bar;
        lsqr_update<T>(c, n, x, w, v, (T)(phi / rho), (T)(theta / rho));     // :40-41
        nsumsq_diff<T>(c, n, x, xt, hybrid ? sl + S_ERR : errh + k);
        if (hybrid) {
            apply_A<T>(c, A, x, t, EPI_RSUB, T(0), b);                        // hybrid :43  b - A*x
            sumsq<T>(c, m, t, sl + S_RES);
            Reader rr(c);
            rr.add(&hs[0], sl + S_ERR, sizeof(T));
            rr.add(&hs[1], sl + S_RES, sizeof(T));
            rr.go();
            err[k] = std::sqrt((double)hs[0]) / nxt;
            res[k] = std::sqrt((double)hs[1]) / nb;
            if (res[k] < tol) break;                                           // hybrid :45 (<)
        } else {
            res[k] = std::fabs(phi_bar) / nb;                                  // :44 (:43 below)
            if (res[k] <= tol) break;                                          // :46 (<=)
        }
    }
    if (k == maxit) k = maxit - 1;
    const int nit = k + 1;
    if (!hybrid) {
        std::vector<T> eh(nit);
        Reader re(c);
        re.add(eh.data(), errh, sizeof(T) * nit);
        re.go();
        for (int i = 0; i < nit; ++i) err[i] = std::sqrt((double)eh[i]) / nxt;   // :43
        if (img_ax) {
            // :52 norm(b - A*x) from the kept image (replicated m-vector: no collective)
            double* b64 = c->buf<double>("lsqr_b64", m + 1);
            if constexpr (std::is_same_v<T, double>) {
                HGM_HIP(hipMemcpyAsync(b64, b, sizeof(double) * m, hipMemcpyDeviceToDevice, c->stream));
            } else {
                convert_back<T>(c, m, b, b64);
            }
            double* rs = c->buf<double>("lsqr_rs", 1);
            sumsq_diff<double>(c, m, b64, img_ax, rs);
            double hv = 0;
            Reader rr(c);
            rr.add(&hv, rs, sizeof(double));
            rr.go();
            res[nit - 1] = std::sqrt(hv) / nb;
        } else {
            apply_A<T>(c, A, x, t, EPI_RSUB, T(0), b);                        // :52 exact final residual
            sumsq<T>(c, m, t, sl + S_RES);
            res[nit - 1] = std::sqrt((double)read1<T>(c, sl + S_RES)) / nb;
        }
    }
    stage_out_n<T>(c, x_out, x, n, dev, po);
    if (err_out) std::memcpy(err_out, err.data(), sizeof(double) * nit);
    if (res_out) std::memcpy(res_out, res.data(), sizeof(double) * nit);
    if (niters) *niters = nit;
    return HGM_OK;
}

// ============================================================================
// LSMR (lsmr_solver.m)
// ============================================================================
template <typename T>
int lsmr_t(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* At, const double* b_in,
           const double* xt_in, double tol, int maxit, double* x_out, double* err_out, double* res_out,
           double* ar_out, int* iters) {
    check_dims(A, At);
    solver_guard(c);
    HGM_REQUIRE(At != nullptr, "At is NULL");
    const PixOrder po = n_order(c, A, At);
    HGM_REQUIRE(b_in != nullptr, "b is required");
    const bool parity = c->num.parity;   // fixed summation orders
    HGM_REQUIRE(!parity || (!dist_n(c) && po.trivial()), "parity mode: single rank, reference pixel order");
    const bool dev = o && (o->flags & HGM_DEVICE_PTRS);
    const int64_t m = A->rows, n = A->cols;
    if (maxit <= 0) maxit = (int)std::min<int64_t>(m, n);                    // :5 default min(m,n)
    HGM_REQUIRE(maxit >= 1, "maxit must be >= 1");
    const T* b = stage_in<T>(c, "in_b", b_in, m, dev);
    const T* xt = stage_in_n<T>(c, "in_xt", xt_in, n, dev, po);
    T* x = c->buf<T>("x", n + 1);
    T* v = c->buf<T>("v", n + 1);
    T* h = c->buf<T>("h", n + 1);
    T* hbar = c->buf<T>("hbar", n + 1);
    T* u = c->buf<T>("u", m + 1);
    T* r = c->buf<T>("t_m", m + 1);
    T* atr = c->buf<T>("t_n", n + 1);
    T* sl = reinterpret_cast<T*>(c->dscal);
    fill<T>(c, n, x, T(0));                                                    // :7
    fill<T>(c, n, hbar, T(0));                                                 // :26
    std::vector<double> err(maxit, std::numeric_limits<double>::quiet_NaN());  // :28
    std::vector<double> res(maxit, 0.0), ar(maxit, 0.0);
    std::vector<T> hs(4);

    sumsq<T>(c, m, b, sl + S_NB);
    if (xt) nsumsq_diff<T>(c, n, xt, x, sl + S_NXT);
    // ||A||_F (lsmr_solver.m:71, loop-invariant): cached per matrix (parity mode: recomputed in
    // the fixed order, not cached)
    double normA = A->fro;
    if (A->fro < 0 || parity) {
        double* f = reinterpret_cast<double*>(c->dscal) + 64;
        if (A->dtype == HGM_F32) fro2<float>(c, A, f); else fro2<double>(c, A, f);
        if (dist_n(c)) allreduce(c, f, 1);
        double fv;
        Reader rf(c);
        rf.add(&fv, f, sizeof(double));
        rf.go();
        normA = std::sqrt(fv);
        if (!parity) const_cast<hgm_mat*>(A)->fro = normA;
    }
    Reader r0(c);
    r0.add(&hs[0], sl + S_NB, sizeof(T));
    if (xt) r0.add(&hs[1], sl + S_NXT, sizeof(T));
    r0.go();
    const double nb = std::sqrt((double)hs[0]);
    const double nxt = xt ? std::sqrt((double)hs[1]) : 0.0;
    // Monitors from kept products (default; HGM_EXPLICIT_RESIDUAL applies the two extra SpMVs
    // of :69 and :71 instead): the raw products A*v_k and A'*u_{k+1} of the bidiagonalisation
    // are kept, and the images A*x, A'A*x follow the x/h/hbar recurrences (lsmr_monitor).  The
    // iterates u, v, x, h, hbar are the same bits either way (the epilogues below are the
    // fused ones, applied as a separate pass).
    const bool kept = !(o && (o->flags & HGM_EXPLICIT_RESIDUAL)) && !parity;
    T *Av = nullptr, *Atu0 = nullptr, *Atu1 = nullptr, *Atb = nullptr;
    double *Ihm = nullptr, *Ihbm = nullptr, *Ixm = nullptr, *Ihn = nullptr, *Ihbn = nullptr, *Ixn = nullptr;
    double* dmon = reinterpret_cast<double*>(c->dscal) + 72;   // [||r||^2, ||A'r||^2]
    if (kept) {
        Av = c->buf<T>("lsmr_Av", m + 1);
        Atu0 = c->buf<T>("lsmr_Atu0", n + 1);
        Atu1 = c->buf<T>("lsmr_Atu1", n + 1);
        Atb = c->buf<T>("lsmr_Atb", n + 1);
        Ihm = c->buf<double>("lsmr_Ihm", m + 1);
        Ihbm = c->buf<double>("lsmr_Ihbm", m + 1);
        Ixm = c->buf<double>("lsmr_Ixm", m + 1);
        Ihn = c->buf<double>("lsmr_Ihn", n + 1);
        Ihbn = c->buf<double>("lsmr_Ihbn", n + 1);
        Ixn = c->buf<double>("lsmr_Ixn", n + 1);
        fill<double>(c, m, Ixm, 0.0);                                          // A*x_0 = 0
        fill<double>(c, n, Ixn, 0.0);                                          // A'A*x_0 = 0
    }
    // One pass over the operator per iteration (as lsqr_t): the step :38-39 and
    // A*v_hat in one pass over At, A*v_{k+1} (:34, the kept A*v) = (A*v_hat) / alpha.
    const FusedPlan* fp = agreed_gk_plan<T>(c, A, At, !parity);
    T* wm = fp ? c->buf<T>("gkb_wm", m + 3) : nullptr;                         // [A*v_hat | alpha^2 | ridden]
    HGM_HIP(hipMemcpyAsync(u, b, sizeof(T) * m, hipMemcpyDeviceToDevice, c->stream));   // :10
    double beta = nb;                                                          // :11
    if (beta > 0) div_scalar<T>(c, m, u, u, (T)beta);                          // :12
    T* v0 = kept ? Atu0 : v;                                                   // raw A'*u_0 kept
    if (fp) {
        FusedArgs<T> fa;                                                       // :14 (+ A*v_hat, ||v_hat||^2)
        fa.q = u;
        fa.zraw = v0;
        fa.w = wm;
        fa.side_sq = true;
        fa.side_out = wm + m;
        fused_pass<T>(c, At, fp, fa);
        if (dist_n(c)) allreduce(c, wm, m + 1);
    } else {
        apply_B<T>(c, At, u, v0, EPI_NONE, T(0), nullptr);                     // :14
        nsumsq<T>(c, n, v0, sl + S_ALPHA);
    }
    double alpha = std::sqrt((double)read1<T>(c, fp ? wm + m : sl + S_ALPHA));   // :15
    // A'*b for the monitors' A'r = A'b - A'A*x: beta * A'*u_0 (u_0 = b / beta, :12-14), the product
    // just formed, instead of one more pass over the operator per solve (equal up to rounding)
    if (kept) scale<T>(c, n, Atu0, Atb, (T)beta);
    if (alpha > 0) div_scalar<T>(c, n, v0, v, (T)alpha);                       // :16
    else if (kept) HGM_HIP(hipMemcpyAsync(v, v0, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));
    double zetabar = alpha * beta, alphabar = alpha, rho = 1, rhobar = 1, cbar = 1, sbar = 0;   // :19-23
    HGM_HIP(hipMemcpyAsync(h, v, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));   // :25
    double prev_ch = 0.0;                                                      // (theta/rho) of the previous :67
    // tol <= 0: `res < tol` (:76) can never hold, so the monitors stay on the device and are
    // read once after the loop instead of once per iteration
    // (and with the device-resident scalars below at any tol)
    const bool defer_mon = kept && (!(tol > 0) || (fp && c->num.lsqr_dev));
    double* dmonh = defer_mon ? c->buf<double>("lsmr_monh", 2 * (size_t)maxit) : nullptr;
    T* errh = defer_mon ? c->buf<T>("lsmr_errh", maxit) : nullptr;
    auto monitors = [&](int kk, double m0, double m1, double e2) {
        const double nr = std::sqrt(m0);
        res[kk] = nr / (nb + EPSD);                                            // :70
        ar[kk] = std::sqrt(m1) / (normA * std::max(nr, EPSD));                 // :71
        if (xt) err[kk] = std::sqrt(e2) / nxt;                                 // :72-73
    };
    int k = 0;
    // Device-resident scalars (the one-pass path with kept monitors): beta and alpha
    // stay on the device as sums of squares, the rotations :42-67 run in one thread (lsmr_rot, the
    // loop's double arithmetic below), the n-space step divides v by alpha and carries the error sum,
    // and the stop test :76 runs on the device after the monitors -- no host round trip per
    // iteration.  The host reads the stop flag once per batch of 8 iterations (none with tol <= 0);
    // an iteration enqueued past the stop leaves x untouched, and its histories are dropped.
    const bool dev_scalars = fp && kept && c->num.lsqr_dev;
    if (dev_scalars) {
        // fp32 solves: the n-space monitor carries A'r in T (lsmr_monitor_r; Ir_0 = A'b)
        constexpr bool img_t = std::is_same_v<T, float>;
        T *Ihn_t = nullptr, *Ihbn_t = nullptr, *Irn_t = nullptr;
        if constexpr (img_t) {
            Ihn_t = c->buf<T>("lsmr_Ihn_t", n + 4);
            Ihbn_t = c->buf<T>("lsmr_Ihbn_t", n + 4);
            Irn_t = c->buf<T>("lsmr_Irn_t", n + 4);
            HGM_HIP(hipMemcpyAsync(Irn_t, Atb, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));
        }
        double* st = c->buf<double>("lsmr_st", 9);
        double* cfm = c->buf<double>("lsmr_cf", 10);
        double* cfn = cfm + 5;
        T* coef = c->buf<T>("lsmr_coef", 3);
        const double st0[9] = {alpha, alphabar, rho, rhobar, cbar, sbar, zetabar, 0.0, 0.0};
        h2d(c, st, st0, sizeof(st0));
        FusedArgs<T> fa;
        fa.q = u;
        fa.ev = v;
        fa.easq = sl + S_BETA;
        fa.zout = v;
        fa.w = wm;
        fa.side_sq = true;
        fa.side_out = wm + m;
        const int batch = tol > 0 ? 8 : maxit;
        int stop = 0;
        // On a communicator the n-space partials of iteration k -- ||x - x_true||^2 (:72) and, in
        // fp64, ||A'r||^2 (:71) -- ride iteration k+1's m-vector all-reduce as elements m+1, m+2, and
        // the rotation kernel copies the sums into the histories: one collective per iteration
        // instead of three (fp32: two; its ||A'r||^2 is a double sum that a float element cannot
        // carry).  The stop test (:76) reads only the replicated m-space residual.  The last
        // iteration's partials are summed after the loop.
        constexpr bool ride_d_ok = std::is_same_v<T, double>;
        const bool ride = dist_n(c);
        T* ride_e = (ride && xt) ? wm + m + 1 : nullptr;
        double* ride_d = nullptr;
        if constexpr (ride_d_ok)
            if (ride) ride_d = reinterpret_cast<double*>(wm + m + 2);
        const int64_t ride_n = ride_d ? 2 : 1;       // trailing elements past alpha^2
        if (ride) HGM_HIP(hipMemsetAsync(wm + m + 1, 0, sizeof(T) * ride_n, c->stream));
        int last = -1;
        for (k = 0; k < maxit && stop == 0;) {
            const int kend = std::min(maxit, k + batch);
            for (; k < kend; ++k) {
                gkb_mstep_div<T>(c, m, wm, wm + m, u, r, Av, sl + S_BETA, true);  // :34-36 (+ kept A*v_k)
                fa.zraw = Atu1;                                                   // A'*u_{k+1} (kept)
                fused_pass<T>(c, At, fp, fa);                                     // :38-39 (+ A*v_hat)
                if (dist_n(c)) allreduce(c, wm, (ride && k > 0) ? m + 1 + ride_n : m + 1);
                ScalarCopy<T> cp;
                if (ride && k > 0) {
                    if (ride_e) {
                        cp.src = ride_e;
                        cp.dst = errh + k - 1;
                    }
                    if (ride_d) {
                        cp.dsrc = ride_d;
                        cp.ddst = dmonh + 2 * (size_t)(k - 1) + 1;
                    }
                }
                lsmr_rot<T>(c, sl + S_BETA, wm + m, st, coef, cfm, cfn, cp);      // :42-67 scalars
                double* dm = dmonh + 2 * (size_t)k;
                T* e_out = xt ? (ride_e ? ride_e : errh + k) : nullptr;
                double* d_out = ride_d ? ride_d : dm + 1;
                // (fp32: the n-space step and the n-space monitor in one launch when it applies)
                const bool nmon = img_t && lsmr_step_mon<T>(c, n, x, h, hbar, v, wm + m, coef, st, k, xt, e_out,
                                                            Atu1, Atu0, Ihn_t, Ihbn_t, Irn_t, k == 0, d_out, cfn);
                if (!nmon) lsmr_step<T>(c, n, x, h, hbar, v, wm + m, coef, st, k, xt, e_out);   // :40, :61-67, :72
                last = k;
                if (xt && dist_n(c) && !ride_e) allreduce(c, errh + k, 1);
                lsmr_monitor<T>(c, m, Av, nullptr, 0, 0, Ihm, Ihbm, Ixm, b, 0, 0, 0, k == 0, dm, cfm);
                if (!nmon && img_t) lsmr_monitor_r<T>(c, n, Atu1, Atu0, Ihn_t, Ihbn_t, Irn_t, k == 0, d_out, cfn);
                else if (!nmon) lsmr_monitor<T>(c, n, Atu1, Atu0, 0, 0, Ihn, Ihbn, Ixn, Atb, 0, 0, 0, k == 0, d_out, cfn);
                if (dist_n(c) && !ride_d) allreduce(c, dm + 1, 1);
                std::swap(Atu0, Atu1);
                if (tol > 0) lsmr_stop(c, dm, nb, tol, st, k);                   // :76
            }
            if (tol > 0) {
                double sv = 0;
                Reader rs(c);
                rs.add(&sv, st + 8, sizeof(double));
                rs.go();
                stop = (int)sv;
            }
        }
        if (ride && last >= 0) {                       // the last iteration's ridden partials
            allreduce(c, wm + m + 1, ride_n);
            ScalarCopy<T> cp;
            if (ride_e) {
                cp.src = ride_e;
                cp.dst = errh + last;
            }
            if (ride_d) {
                cp.dsrc = ride_d;
                cp.ddst = dmonh + 2 * (size_t)last + 1;
            }
            copy_scalars<T>(c, cp);
        }
        k = stop > 0 ? stop - 1 : maxit;
    }
    for (k = dev_scalars ? k : 0; !dev_scalars && k < maxit; ++k) {
        const double alpha_k = alpha;
        if (fp) {
            // :34 A*v_k = (A*v_hat)/alpha_k (kept), u = A*v - alpha*u, ||u||^2
            gkb_mstep<T>(c, m, wm, wm + m, u, r, kept ? Av : nullptr, sl + S_BETA);
            beta = std::sqrt((double)read1<T>(c, sl + S_BETA));               // :35
            if (beta > 0) div_scalar<T>(c, m, r, u, (T)beta);                  // :36
            else HGM_HIP(hipMemcpyAsync(u, r, sizeof(T) * m, hipMemcpyDeviceToDevice, c->stream));
            FusedArgs<T> fa;                                                   // :38 v = A.'*u - beta*v, one pass
            fa.q = u;
            fa.zraw = kept ? Atu1 : nullptr;                                   // A'*u_{k+1} (kept)
            fa.ev = v;
            fa.easq = sl + S_BETA;
            fa.zout = v;
            fa.w = wm;
            fa.side_sq = true;
            fa.side_out = wm + m;                                              // ||v||^2 (:39)
            fused_pass<T>(c, At, fp, fa);
            if (dist_n(c)) allreduce(c, wm, m + 1);
            alpha = std::sqrt((double)read1<T>(c, wm + m));                    // :39
        } else {
            if (kept) {
                apply_A<T>(c, A, v, Av, EPI_NONE, T(0), nullptr);              // A*v_k (kept)
                epilogue_to<T>(c, m, Av, u, EPI_SUB, (T)alpha, u);             // :34 u = A*v - alpha*u
            } else {
                apply_A<T>(c, A, v, u, EPI_SUB, (T)alpha, u);                  // :34 u = A*v - alpha*u
            }
            sumsq<T>(c, m, u, sl + S_BETA);
            beta = std::sqrt((double)read1<T>(c, sl + S_BETA));               // :35
            if (beta > 0) div_scalar<T>(c, m, u, u, (T)beta);                  // :36
            if (kept) {
                apply_B<T>(c, At, u, Atu1, EPI_NONE, T(0), nullptr);           // A'*u_{k+1} (kept)
                epilogue_to<T>(c, n, Atu1, v, EPI_SUB, (T)beta, v);            // :38 v = A.'*u - beta*v
            } else {
                apply_B<T>(c, At, u, v, EPI_SUB, (T)beta, v);                  // :38 v = A.'*u - beta*v
            }
            nsumsq<T>(c, n, v, sl + S_ALPHA);
            alpha = std::sqrt((double)read1<T>(c, sl + S_ALPHA));             // :39
        }
        if (alpha > 0) div_scalar<T>(c, n, v, v, (T)alpha);                    // :40
        const double alphahat = alphabar;                                      // :42
        const double rhoold = rho;                                             // :43
        rho = std::hypot(alphahat, beta);                                      // :44
        const double cc = alphahat / rho, ss = beta / rho;                     // :45-46
        const double thetanew = ss * alpha;                                    // :48
        alphabar = cc * alpha;                                                 // :49
        const double rhobarold = rhobar;                                       // :51
        const double thetabar = sbar * rho;                                    // :52
        rhobar = std::hypot(cbar * rho, thetanew);                             // :53
        cbar = (cbar * rho) / rhobar;                                          // :54
        sbar = thetanew / rhobar;                                              // :55
        const double zeta = cbar * zetabar;                                    // :58
        zetabar = -sbar * zetabar;                                             // :59
        const double c_hbar = (thetabar * rho) / (rhoold * rhobarold);         // :64
        const double c_x = zeta / (rho * rhobar);                              // :66
        const double c_h = thetanew / rho;                                     // :67
        lsmr_update<T>(c, n, x, h, hbar, v, (T)c_hbar, (T)c_x, (T)c_h, k == 0);
        double mon[2] = {0.0, 0.0};
        Reader rr(c);
        if (kept) {
            // :69 ||b - A*x||^2 and :71 ||A'b - A'A*x||^2 from the kept images
            double* dm = defer_mon ? dmonh + 2 * (size_t)k : dmon;
            lsmr_monitor<T>(c, m, Av, nullptr, 1.0, 0.0, Ihm, Ihbm, Ixm, b, prev_ch, c_hbar, c_x, k == 0, dm);
            lsmr_monitor<T>(c, n, Atu1, Atu0, beta, alpha_k, Ihn, Ihbn, Ixn, Atb, prev_ch, c_hbar, c_x, k == 0,
                            dm + 1);
            if (dist_n(c)) allreduce(c, dm + 1, 1);
            std::swap(Atu0, Atu1);
            if (!defer_mon) rr.add(mon, dmon, sizeof(double) * 2);
        } else {
            apply_A<T>(c, A, x, r, EPI_RSUB, T(0), b);                         // :69 r = b - A*x
            sumsq<T>(c, m, r, sl + S_RES);
            apply_B<T>(c, At, r, atr, EPI_NONE, T(0), nullptr);                // :71 A.'*r
            nsumsq<T>(c, n, atr, sl + S_AR);
            rr.add(&hs[0], sl + S_RES, sizeof(T));
            rr.add(&hs[1], sl + S_AR, sizeof(T));
        }
        prev_ch = c_h;
        if (xt) nsumsq_diff<T>(c, n, x, xt, defer_mon ? errh + k : sl + S_ERR);
        if (defer_mon) continue;
        if (xt) rr.add(&hs[2], sl + S_ERR, sizeof(T));
        rr.go();
        if (!kept) {
            mon[0] = (double)hs[0];
            mon[1] = (double)hs[1];
        }
        monitors(k, mon[0], mon[1], xt ? (double)hs[2] : 0.0);
        if (res[k] < tol) break;                                               // :76 (<)
    }
    if (k == maxit) k = maxit - 1;
    const int nit = k + 1;
    if (defer_mon) {
        std::vector<double> mh(2 * (size_t)nit);
        std::vector<T> eh(nit, T(0));
        Reader re(c);
        re.add(mh.data(), dmonh, sizeof(double) * mh.size());
        if (xt) re.add(eh.data(), errh, sizeof(T) * nit);
        re.go();
        for (int i = 0; i < nit; ++i) monitors(i, mh[2 * i], mh[2 * i + 1], (double)eh[i]);
    }
    stage_out_n<T>(c, x_out, x, n, dev, po);
    if (err_out) std::memcpy(err_out, err.data(), sizeof(double) * nit);
    if (res_out) std::memcpy(res_out, res.data(), sizeof(double) * nit);
    if (ar_out) std::memcpy(ar_out, ar.data(), sizeof(double) * nit);
    if (iters) *iters = nit;
    return HGM_OK;
}

// ============================================================================
// hybrid LSMR (hybrid_lsmr_solver.m)
// ============================================================================
int hybrid_lsmr(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* At, const double* b_in,
                const double* xt_in, double tol, int maxit, double lambda, double* x_out, double* err_out,
                double* res_out, int* niters) {
    check_dims(A, At);
    solver_guard(c);
    HGM_REQUIRE(At != nullptr, "At is NULL");
    const PixOrder po = n_order(c, A, At);
    HGM_REQUIRE(A->dtype == HGM_F64, "hybrid LSMR is fp64");
    HGM_REQUIRE(!c->num.parity || (!dist_n(c) && po.trivial()), "parity mode: single rank, reference pixel order");
    HGM_REQUIRE(b_in != nullptr && xt_in != nullptr, "b and x_true are required");
    HGM_REQUIRE(maxit >= 1, "maxit must be >= 1");
    using T = double;
    const bool dev = o && (o->flags & HGM_DEVICE_PTRS);
    const int64_t m = A->rows, n = A->cols;
    const int64_t ldv = round_up(n > 0 ? n : 1, 64);
    const T* b = stage_in<T>(c, "in_b", b_in, m, dev);
    const T* xt = stage_in_n<T>(c, "in_xt", xt_in, n, dev, po);
    T* V = c->buf<T>("Q", (size_t)ldv * maxit);
    T* x = c->buf<T>("x", n + 1);
    T* u = c->buf<T>("u", m + 1);
    T* t = c->buf<T>("t_m", m + 1);
    T* yd = c->buf<T>("y", maxit + 8);
    T* sl = reinterpret_cast<T*>(c->dscal);
    fill<T>(c, n, x, T(0));
    std::vector<double> err(maxit, 0.0), res(maxit, 0.0);
    std::vector<double> Bk((size_t)(maxit + 1) * maxit, 0.0);                  // :11
    auto BK = [&](int i, int j) -> double& { return Bk[(size_t)j * (maxit + 1) + i]; };

    sumsq<T>(c, m, b, sl + S_NB);
    nsumsq_diff<T>(c, n, xt, x, sl + S_NXT);
    read_scalars(c, 0, 2);
    const double nb = std::sqrt(c->hscal[S_NB]);
    const double nxt = std::sqrt(c->hscal[S_NXT]);
    const double beta1 = nb;                                                   // :7
    div_scalar<T>(c, m, b, u, beta1);                                          // :8
    T* v0 = V;
    apply_B<T>(c, At, u, v0, EPI_NONE, 0.0, nullptr);                          // :13
    nsumsq<T>(c, n, v0, sl + S_ALPHA);
    double alpha1 = std::sqrt(read1<T>(c, sl + S_ALPHA));                      // :14
    div_scalar<T>(c, n, v0, v0, alpha1);                                       // :15-16
    int k = 0;
    std::vector<double> Gm, G2, LHS, RHS, y;
    for (k = 0; k < maxit; ++k) {
        T* vk = V + (int64_t)k * ldv;
        BK(k, k) = alpha1;                                                     // :23
        apply_A<T>(c, A, vk, t, EPI_SUB, alpha1, u);                           // :24
        sumsq<T>(c, m, t, sl + S_BETA);
        const double beta_k = std::sqrt(read1<T>(c, sl + S_BETA));            // :25
        div_scalar<T>(c, m, t, u, beta_k);                                     // :26
        BK(k + 1, k) = beta_k;                                                 // :27
        if (k < maxit - 1) {                                                   // :29
            T* vn = V + (int64_t)(k + 1) * ldv;
            apply_B<T>(c, At, u, vn, EPI_SUB, beta_k, vk);                     // :30
            nsumsq<T>(c, n, vn, sl + S_ALPHA);
            const double a1 = std::sqrt(read1<T>(c, sl + S_ALPHA));            // :31
            div_scalar<T>(c, n, vn, vn, a1);                                   // :32-33
            alpha1 = a1;                                                       // :34
        }
        const int kk = k + 1;
        // :37-44  LHS = (Bk'*Bk)^2 + (alpha_k1*beta_k1)^2 e1 e1' + lambda I ; RHS = B_k(1,1) beta1 (Bk'*Bk) e1
        Gm.assign((size_t)kk * kk, 0.0);
        for (int i = 0; i < kk; ++i)
            for (int j = 0; j < kk; ++j) {
                double s = 0;
                for (int r = 0; r <= kk; ++r) s += BK(r, i) * BK(r, j);
                Gm[(size_t)j * kk + i] = s;
            }
        G2.assign((size_t)kk * kk, 0.0);
        for (int i = 0; i < kk; ++i)
            for (int j = 0; j < kk; ++j) {
                double s = 0;
                for (int l = 0; l < kk; ++l) s += Gm[(size_t)l * kk + i] * Gm[(size_t)j * kk + l];
                G2[(size_t)j * kk + i] = s;
            }
        const double ab = alpha1 * beta_k;
        LHS = G2;
        LHS[0] += ab * ab;
        for (int i = 0; i < kk; ++i) LHS[(size_t)i * kk + i] += lambda;
        RHS.assign(kk, 0.0);
        const double sc = BK(0, 0) * beta1;
        for (int i = 0; i < kk; ++i) RHS[i] = sc * Gm[i];
        y.assign(kk, 0.0);
        dense::mldivide_square(kk, LHS.data(), RHS.data(), y.data());          // :44
        h2d_pinned(c, yd, y.data(), sizeof(double) * kk);
        gemv<T>(c, n, kk, V, ldv, yd, x, 0);                                   // :45
        nsumsq_diff<T>(c, n, x, xt, sl + S_ERR);                               // :47
        apply_A<T>(c, A, x, t, EPI_RSUB, 0.0, b);                              // :48
        sumsq<T>(c, m, t, sl + S_RES);
        read_scalars(c, S_RES, 2);
        res[k] = std::sqrt(c->hscal[S_RES]) / nb;
        err[k] = std::sqrt(c->hscal[S_ERR]) / nxt;
        if (res[k] <= tol) break;                                              // :50
    }
    if (k == maxit) k = maxit - 1;
    const int nit = k + 1;
    stage_out_n<T>(c, x_out, x, n, dev, po);
    if (err_out) std::memcpy(err_out, err.data(), sizeof(double) * nit);
    if (res_out) std::memcpy(res_out, res.data(), sizeof(double) * nit);
    if (niters) *niters = nit;
    return HGM_OK;
}

// ============================================================================
// Arnoldi for GCV (gcv_function.m:3-33)
// ============================================================================
int arnoldi(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const double* b_in, int kg, int side,
            double btol, int orth, double* H_out, double* beta_out, int* kdone) {
    check_dims(A, B);
    solver_guard(c);
    HGM_REQUIRE(B != nullptr, "B is NULL");
    (void)n_order(c, A, B);   // H does not depend on the stored pixel order (up to rounding)
    HGM_REQUIRE(A->dtype == HGM_F64, "Arnoldi is fp64");
    HGM_REQUIRE(kg >= 1, "k must be >= 1");
    using T = double;
    const int64_t m = A->rows, n = A->cols;
    const bool nspace = side == HGM_SIDE_BA;
    const int64_t dim = nspace ? n : m;
    const bool dist = nspace && dist_n(c);
    const int64_t ldq = krylov_ld(c, dim, dist);
    HGM_REQUIRE(!c->num.parity || !dist_n(c), "parity mode: single rank");
    const T* b = stage_in<T>(c, "in_b", b_in, m, false);
    T* Q = c->buf<T>("Q", (size_t)ldq * (kg + 1));
    if (krylov_padded(c, ldq)) HGM_HIP(hipMemsetAsync(Q, 0, sizeof(T) * ldq * (kg + 1), c->stream));
    T* Hd = c->buf<T>("H", (size_t)(kg + 1) * kg);
    T* t = c->buf<T>("t_m", m + 1);
    T* tn = c->buf<T>("t_n", n + 1);
    HGM_HIP(hipMemsetAsync(Hd, 0, sizeof(T) * (kg + 1) * kg, c->stream));
    if (nspace) apply_B<T>(c, B, b, Q, EPI_NONE, 0.0, nullptr);                // :8  r0 = B*b
    else HGM_HIP(hipMemcpyAsync(Q, b, sizeof(T) * m, hipMemcpyDeviceToDevice, c->stream));   // :5
    if (nspace) nsumsq<T>(c, dim, Q, dslot<T>(c, S_BETA));
    else sumsq<T>(c, dim, Q, dslot<T>(c, S_BETA));
    const double beta = std::sqrt(read1<T>(c, dslot<T>(c, S_BETA)));           // :12
    div_scalar<T>(c, dim, Q, Q, beta);                                         // :15
    std::vector<double> H((size_t)(kg + 1) * kg, 0.0);
    int done = 0;
    const FusedPlan* fplan = nullptr;                                          // A*(B*q) in one pass
    if constexpr (std::is_same_v<T, double>) if (!nspace) fplan = fused_ab_plan(c, A, B);
    // The steps are enqueued back to back, with no host round trip per step: the breakdown
    // test H(k+1,k) < btol runs on the host afterwards, and the steps past a breakdown (which
    // wrote only Q(:,>k+1) and H(:,>k) on the device) are discarded.
    for (int k = 0; k < kg; ++k) {
        T* qk = Q + (int64_t)k * ldq;
        T* v = Q + (int64_t)(k + 1) * ldq;
        if (nspace) {
            apply_A<T>(c, A, qk, t, EPI_NONE, 0.0, nullptr);
            apply_B<T>(c, B, t, v, EPI_NONE, 0.0, nullptr);                    // :22 B*(A*Q(:,k))
        } else if (fplan) {
            if constexpr (std::is_same_v<T, double>) {
                fused_ab(c, B, fplan, qk, tn, v);                                 // :20
                if (dist_n(c)) allreduce(c, v, A->rows);
            }
        } else {
            apply_B<T>(c, B, qk, tn, EPI_NONE, 0.0, nullptr);
            apply_A<T>(c, A, tn, v, EPI_NONE, 0.0, nullptr);                   // :20 A*(B*Q(:,k))
        }
        T* Hcol = Hd + (int64_t)k * (kg + 1);
        if (orth == HGM_CGS2) cgs2<T>(c, dim, Q, ldq, k, Hcol, dist);
        else mgs<T>(c, dim, Q, ldq, k, Hcol, dist);                            // :25-31
    }
    std::vector<double> Hall((size_t)(kg + 1) * kg);
    Reader rd(c);
    rd.add(Hall.data(), Hd, sizeof(T) * Hall.size());
    rd.go();
    for (int k = 0; k < kg; ++k) {
        std::memcpy(&H[(size_t)k * (kg + 1)], &Hall[(size_t)k * (kg + 1)], sizeof(double) * (k + 2));
        done = k + 1;
        if (H[(size_t)k * (kg + 1) + k + 1] < btol) {                          // :30  H(k+1,k) < 1e-12 -> break
            // the reference breaks before Q(:,k+1) = v/H(k+1,k); H(k+1,k) keeps its value
            break;
        }
    }
    if (H_out) std::memcpy(H_out, H.data(), sizeof(double) * H.size());
    if (beta_out) *beta_out = beta;
    if (kdone) *kdone = done;
    return HGM_OK;
}

// explicit instantiations used by capi.cpp
template int lsqr_t<double>(hgm_ctx*, const hgm_opts*, const hgm_mat*, const hgm_mat*, const double*, const double*,
                            double, int, bool, double, double*, double*, double*, int*);
template int lsqr_t<float>(hgm_ctx*, const hgm_opts*, const hgm_mat*, const hgm_mat*, const double*, const double*,
                           double, int, bool, double, double*, double*, double*, int*);
template int lsmr_t<double>(hgm_ctx*, const hgm_opts*, const hgm_mat*, const hgm_mat*, const double*, const double*,
                            double, int, double*, double*, double*, double*, int*);
template int lsmr_t<float>(hgm_ctx*, const hgm_opts*, const hgm_mat*, const hgm_mat*, const double*, const double*,
                           double, int, double*, double*, double*, double*, int*);

}  // namespace hgm
