// extern "C" boundary of libhgmres (include/hgmres.h): context / communicator /
// operator management and the solver entry points that replace the reference's
// MATLAB functions.  Every entry point converts C++ exceptions into a status code
// and keeps the message for hgm_last_error().
#include <limits.h>
#include <link.h>
#include <sched.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <set>
#include <vector>

#include "internal.h"

namespace hgm {

// solvers.cpp
struct GmresSpec {
    int side;
    int proj;
    bool lambda_in_op;
    bool x_preassigned;
};
int gmres_family(hgm_ctx* c, const GmresSpec& sp, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B,
                 const double* b_in, const double* xt_in, double tol, int maxit, double lambda, double* x_out,
                 double* err_out, double* res_out, int* niters);
template <typename T>
int lsqr_t(hgm_ctx*, const hgm_opts*, const hgm_mat*, const hgm_mat*, const double*, const double*, double, int,
           bool, double, double*, double*, double*, int*);
template <typename T>
int lsmr_t(hgm_ctx*, const hgm_opts*, const hgm_mat*, const hgm_mat*, const double*, const double*, double, int,
           double*, double*, double*, double*, int*);
int hybrid_lsmr(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* At, const double* b_in,
                const double* xt_in, double tol, int maxit, double lambda, double* x_out, double* err_out,
                double* res_out, int* niters);
int arnoldi(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const double* b_in, int kg, int side, double btol,
            int orth, double* H_out, double* beta_out, int* kdone);
// bounds.cpp
int gmres_bounds_filter(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B, const double* b,
                        const double* xt, double tol, int maxit, double lambda, int side, int hybrid,
                        const hgm_mat* dML, const hgm_mat* dMR, int ritz_steps, double* x_out, double* err_out,
                        double* res_out, int* niters, double* phi, double* dphi, double* mu_out, double* ritz_res);

enum { PROJ_LS = 0, PROJ_PTR = 1, PROJ_ABRTP = 2 };

void DevBuf::ensure(size_t b) {
    if (b <= bytes) return;
    release();
    if (hipMalloc(&p, b) != hipSuccess) {
        p = nullptr;
        bytes = 0;
        throw Error{HGM_E_NOMEM, "hipMalloc failed for workspace (" + std::to_string(b) + " bytes)"};
    }
    bytes = b;
}
void DevBuf::release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
}

hipEvent_t Timing::get() {
    if (!pool.empty()) {
        hipEvent_t e = pool.back();
        pool.pop_back();
        return e;
    }
    // timing-only events: no system-scope fence on record (no L2 writeback/invalidate
    // around the timed kernels, which would slow them and the work after them)
    hipEvent_t e;
    HGM_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    return e;
}
void Timing::clear() {
    for (int k = 0; k < KC_N; ++k) {
        for (auto& pr : ev[k]) {
            pool.push_back(pr.first);
            pool.push_back(pr.second);
        }
        ev[k].clear();
        bytes[k] = 0;
    }
}

// SpMV classes and the one pass arm events that the kernel launches carry in their dispatch packets
// (first launch: start, last launch: stop); other classes use stream markers.
void timing_begin(hgm_ctx* c, int cls, hipEvent_t* start) {
    *start = nullptr;
    if (!c->timing.on || c->timing.paused || cls < 0 || cls >= KC_N || !((c->timing.mask >> cls) & 1u)) return;
    *start = c->timing.get();
    // (round 6: the one pass too -- its marker events had put a ~4 us bubble before the pass and
    // after its reduction in every timed step; the pass's first launch carries the start event and
    // its reduction, launched `last`, the stop event)
    if (cls == KC_SPMV_A || cls == KC_SPMV_B || cls == KC_FUSED) {
        c->arm_start = *start;
        c->arm_stop = c->cur_stop = c->timing.get();
    } else {
        HGM_HIP(hipEventRecord(*start, c->stream));
    }
}
void timing_end(hgm_ctx* c, int cls, hipEvent_t start, double bytes) {
    if (!start) return;
    hipEvent_t stop;
    if (cls == KC_SPMV_A || cls == KC_SPMV_B || cls == KC_FUSED) {
        stop = c->cur_stop;
        // events not consumed by a launch (nothing launched) are recorded as markers
        if (c->arm_start) HGM_HIP(hipEventRecord(c->arm_start, c->stream));
        if (c->arm_stop) HGM_HIP(hipEventRecord(c->arm_stop, c->stream));
        c->arm_start = c->arm_stop = c->cur_stop = nullptr;
    } else {
        stop = c->timing.get();
        HGM_HIP(hipEventRecord(stop, c->stream));
    }
    c->timing.ev[cls].push_back({start, stop});
    c->timing.bytes[cls] += bytes;
}

static void ensure_stage(hgm_ctx* c, size_t bytes) {
    if (bytes <= c->hstage_bytes) return;
    if (c->hstage) (void)hipHostFree(c->hstage);
    c->hstage = nullptr;
    size_t nb = bytes < 4096 ? 4096 : bytes;
    HGM_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->hstage), nb, hipHostMallocDefault));
    c->hstage_bytes = nb;
}

// Host waits of the solvers spin on the stream / event instead of a blocking synchronise, which may
// sleep and then adds its wake-up to every host round trip (the GPU idles meanwhile).  The spin is
// bounded: after HGM_OPT_HOST_SPIN_US of pure spinning every further poll yields the
// core (sched_yield), so a long wait (a plan build, the stage-out, a rank waiting on its peers)
// hands the core to RCCL's proxy and other runnable threads; with nothing else runnable the yield
// returns at once, so the wake-up latency stays that of the spin.  A negative value waits with the
// blocking hipStreamSynchronize / hipEventSynchronize instead.
// Default: 200 us, or the blocking waits when the process may run on fewer than 4 cores (ranks
// pinned together: 2 ranks on 2 cores ran the 2-rank C3 solve 10-17 % faster blocking,
// profiles/r5_pinned_2rank.jsonl).
static int host_spin_default() {
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0 && CPU_COUNT(&cs) < 4) return -1;
    return 200;
}
std::atomic<int> g_host_spin_us{host_spin_default()};

void HostPause::operator()() {
    if (++polls < 64) return;
    polls = 0;
    const auto now = std::chrono::steady_clock::now();
    if (!yielding &&
        std::chrono::duration_cast<std::chrono::microseconds>(now - t0).count() >= g_host_spin_us.load())
        yielding = true;
    if (yielding) sched_yield();
}

void stream_sync(hipStream_t s) {
    if (g_host_spin_us.load() < 0) {
        HGM_HIP(hipStreamSynchronize(s));
        return;
    }
    HostPause pause;
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) HGM_HIP(q);
        pause();
    }
}
static void event_sync(hipEvent_t e) {
    if (g_host_spin_us.load() < 0) {
        HGM_HIP(hipEventSynchronize(e));
        return;
    }
    HostPause pause;
    for (;;) {
        const hipError_t q = hipEventQuery(e);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) HGM_HIP(q);
        pause();
    }
}

void Reader::go() {
    size_t tot = 0;
    for (auto& it : items) tot += (it.bytes + 15) / 16 * 16;
    ensure_stage(c, tot);
    char* h = reinterpret_cast<char*>(c->hstage);
    size_t off = 0;
    for (auto& it : items) {
        if (it.bytes) HGM_HIP(hipMemcpyAsync(h + off, it.dev, it.bytes, hipMemcpyDeviceToHost, c->stream));
        off += (it.bytes + 15) / 16 * 16;
    }
    stream_sync(c->stream);
    off = 0;
    for (auto& it : items) {
        if (it.bytes) std::memcpy(it.host, h + off, it.bytes);
        off += (it.bytes + 15) / 16 * 16;
    }
    items.clear();
}

void h2d(hgm_ctx* c, void* dev, const void* host, size_t bytes) {
    if (bytes == 0) return;
    // pageable source: hipMemcpyAsync stages it before returning, so the host buffer may be reused
    HGM_HIP(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, c->stream));
}

void h2d_pinned(hgm_ctx* c, void* dev, const void* host, size_t bytes) {
    if (bytes == 0) return;
    if (bytes > c->hup_bytes) {
        if (c->hup) (void)hipHostFree(c->hup);
        c->hup = nullptr;
        const size_t nb = bytes < 4096 ? 4096 : bytes;
        HGM_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->hup), nb, hipHostMallocDefault));
        c->hup_bytes = nb;
    }
    std::memcpy(c->hup, host, bytes);
    HGM_HIP(hipMemcpyAsync(dev, c->hup, bytes, hipMemcpyHostToDevice, c->stream));
}

void read_scalars(hgm_ctx* c, int first, int count) {
    HGM_HIP(hipMemcpyAsync(c->hscal + first, c->dscal + first, sizeof(double) * count, hipMemcpyDeviceToHost,
                           c->stream));
    stream_sync(c->stream);
}

void sync(hgm_ctx* c) {
    stream_sync(c->stream);
    if (c->aux && c->aux != c->stream) stream_sync(c->aux);
}

void pinned_ring(hgm_ctx* c, size_t bytes) {
    stream_sync(c->stream);
    if (bytes > c->hring_bytes) {
        if (c->hring) (void)hipHostFree(c->hring);
        c->hring = nullptr;
        c->hring_dev = nullptr;
        c->hring_bytes = 0;
        const size_t nb = bytes < 65536 ? 65536 : bytes;
        HGM_HIP(hipHostMalloc(reinterpret_cast<void**>(&c->hring), nb, hipHostMallocMapped | hipHostMallocCoherent));
        void* d = nullptr;
        HGM_HIP(hipHostGetDevicePointer(&d, c->hring, 0));
        c->hring_dev = reinterpret_cast<double*>(d);
        c->hring_bytes = nb;
    }
    std::memset(c->hring, 0, bytes);
}

// Events the host waits on before reading the pinned ring.  Every scalar the kernels put
// in the ring is a system-scope store (st_sys, device_common.h), so the event needs no
// system-scope release of its own (an L2 writeback + invalidate per record, ~4% of the
// C2 step).  HGM_OPT_SYNC_EVENT_FENCE = 1 restores the fenced events.
// With ranks the ring is a device buffer copied out by hipMemcpyAsync, so those events
// keep the fence.
static void sync_event(hgm_ctx* c, hipEvent_t& e, unsigned& have) {
    const bool fence = c->num.sync_event_fence;
    const unsigned want = hipEventDisableTiming | ((fence || c->world > 1) ? 0u : hipEventDisableSystemFence);
    if (e && have != want) {
        HGM_HIP(hipEventDestroy(e));
        e = nullptr;
    }
    if (!e) {
        HGM_HIP(hipEventCreateWithFlags(&e, want));
        have = want;
    }
}

void pipe_record(hgm_ctx* c) {
    sync_event(c, c->ev_pipe, c->ev_flags[8]);
    HGM_HIP(hipEventRecord(c->ev_pipe, c->stream));
}

hipStream_t aux_stream(hgm_ctx* c) {
    if (!c->aux) HGM_HIP(hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking));
    return c->aux;
}

void step_record(hgm_ctx* c, int k) {
    hipEvent_t& e = c->ev_step[k & 7];
    sync_event(c, e, c->ev_flags[k & 7]);
    HGM_HIP(hipEventRecord(e, c->stream));
}

void step_wait(hgm_ctx* c, int k) {
    if (!c->host_stats) {
        event_sync(c->ev_step[k & 7]);
        return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    event_sync(c->ev_step[k & 7]);
    c->wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void pipe_wait(hgm_ctx* c) {
    if (!c->host_stats) {
        event_sync(c->ev_pipe);
        return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    event_sync(c->ev_pipe);
    c->wait_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    c->waits += 1;
}

template <typename T>
static void allreduce_t(hgm_ctx* c, T* dev, int64_t count, ncclDataType_t dt) {
    if (count <= 0) return;
    if (c->nccl) {              // includes a one-rank communicator (hgm_ctx_create_dist)
        if (ncclAllReduce(dev, dev, (size_t)count, dt, ncclSum, c->nccl, c->stream) != ncclSuccess)
            throw Error{HGM_E_COMM, "ncclAllReduce failed"};
        return;
    }
    if (c->world <= 1) return;
    if (!c->host_ar) throw Error{HGM_E_COMM, "world > 1 but no communicator"};
    // host all-reduce hook (shard emulation / tests): always exchanged as doubles
    ensure_stage(c, sizeof(double) * count + sizeof(T) * count);
    double* h = c->hstage;
    if (sizeof(T) == sizeof(double)) {
        HGM_HIP(hipMemcpyAsync(h, dev, sizeof(double) * count, hipMemcpyDeviceToHost, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
        if (c->host_ar(h, count, c->host_ar_user) != 0) throw Error{HGM_E_COMM, "host all-reduce failed"};
        HGM_HIP(hipMemcpyAsync(dev, h, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
    } else {
        std::vector<T> tmp(count);
        HGM_HIP(hipMemcpyAsync(tmp.data(), dev, sizeof(T) * count, hipMemcpyDeviceToHost, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
        for (int64_t i = 0; i < count; ++i) h[i] = (double)tmp[i];
        if (c->host_ar(h, count, c->host_ar_user) != 0) throw Error{HGM_E_COMM, "host all-reduce failed"};
        for (int64_t i = 0; i < count; ++i) tmp[i] = (T)h[i];
        HGM_HIP(hipMemcpyAsync(dev, tmp.data(), sizeof(T) * count, hipMemcpyHostToDevice, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
    }
}
void allreduce(hgm_ctx* c, double* dev, int64_t count) { allreduce_t<double>(c, dev, count, ncclDouble); }
void allreduce(hgm_ctx* c, float* dev, int64_t count) { allreduce_t<float>(c, dev, count, ncclFloat); }

}  // namespace hgm

using namespace hgm;

#define HGM_TRY(ctx, body)                                      \
    try {                                                       \
        body;                                                   \
    } catch (const hgm::Error& e) {                             \
        if (ctx) (ctx)->err = e.msg;                            \
        return e.code;                                          \
    } catch (const std::exception& e) {                         \
        if (ctx) (ctx)->err = e.what();                         \
        return HGM_E_HIP;                                       \
    }

// y = A x with x and y in the reference index order (the operator may store a pixel space
// in a tiled order: permute on the way in / out)
template <typename T>
static void spmv_ref(hgm_ctx* c, const hgm_mat* A, const T* x, T* y) {
    const T* xs = x;
    if (!A->col_order.trivial()) {
        T* t = c->buf<T>("spmv_x_pix", A->cols);
        pix_permute<T>(c, A->col_order, x, t, 0);
        xs = t;
    }
    if (A->row_order.trivial()) {
        spmv<T>(c, A, xs, y, EPI_NONE, T(0), nullptr, KC_SPMV_A);
        return;
    }
    T* t = c->buf<T>("spmv_y_pix", A->rows);
    spmv<T>(c, A, xs, t, EPI_NONE, T(0), nullptr, KC_SPMV_A);
    pix_permute<T>(c, A->row_order, t, y, 1);
}

// Distinct HIP runtime files (libamdhip64*) mapped into this process.  PyTorch-ROCm ships its
// own copy (torch/lib/libamdhip64.so, requested under that name) next to /opt/rocm's
// (libamdhip64.so.7, which this library needs): if this library is loaded first and torch
// after it, both get mapped and the process aborts at exit (double free in the runtimes'
// static destructors).  Python loads torch first (hgmres/_lib.py); this check turns any
// other order into a clear error instead of silent undefined behaviour.
static int hip_runtime_cb(struct dl_phdr_info* info, size_t, void* data) {
    auto* names = static_cast<std::set<std::string>*>(data);
    const char* nm = info->dlpi_name;
    if (nm && std::strstr(nm, "libamdhip64")) {
        char real[PATH_MAX];
        names->insert(realpath(nm, real) ? std::string(real) : std::string(nm));
    }
    return 0;
}
static std::set<std::string> hip_runtimes() {
    std::set<std::string> names;
    dl_iterate_phdr(hip_runtime_cb, &names);
    return names;
}

static int ctx_init(hgm_ctx* c, int device) {
    c->device = device;
    if (hip_runtimes().size() > 1) return HGM_E_HIP;   // see hgm_runtime_check
    const char* hs = std::getenv("HGM_HOST_STATS");
    c->host_stats = hs && hs[0] == '1';
    if (hipSetDevice(device) != hipSuccess) return HGM_E_HIP;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return HGM_E_HIP;
    if (hipMalloc(reinterpret_cast<void**>(&c->dscal), sizeof(double) * NSCAL) != hipSuccess) return HGM_E_NOMEM;
    if (hipMemset(c->dscal, 0, sizeof(double) * NSCAL) != hipSuccess) return HGM_E_HIP;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->hscal), sizeof(double) * NSCAL, hipHostMallocDefault) !=
        hipSuccess)
        return HGM_E_NOMEM;
    return HGM_OK;
}

extern "C" {

HGM_API int hgm_version(void) { return HGM_VERSION; }

HGM_API int hgm_experiments(void) { return HGM_EXPERIMENTS; }

HGM_API int hgm_runtime_check(char* msg, int len) {
    const std::set<std::string> names = hip_runtimes();
    if (msg && len > 0) {
        std::string m;
        for (const auto& s : names) m += (m.empty() ? "" : ";") + s;
        std::snprintf(msg, (size_t)len, "%s", m.c_str());
    }
    return (int)names.size();
}

HGM_API int hgm_device_count(int* count) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (count) *count = n;
    return HGM_OK;
}

HGM_API int hgm_ctx_create(int device, hgm_ctx** out) {
    if (!out) return HGM_E_ARG;
    *out = nullptr;
    hgm_ctx* c = new hgm_ctx();
    int st = ctx_init(c, device);
    if (st != HGM_OK) {
        hgm_ctx_destroy(c);
        return st;
    }
    *out = c;
    return HGM_OK;
}

HGM_API int hgm_comm_unique_id(void* id_out) {
    if (!id_out) return HGM_E_ARG;
    static_assert(sizeof(ncclUniqueId) <= HGM_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return HGM_E_COMM;
    std::memset(id_out, 0, HGM_UNIQUE_ID_BYTES);
    std::memcpy(id_out, &id, sizeof(id));
    return HGM_OK;
}

HGM_API int hgm_ctx_create_dist(int device, int rank, int world, const void* unique_id, hgm_ctx** out) {
    if (!out || !unique_id || world < 1 || rank < 0 || rank >= world) return HGM_E_ARG;
    int st = hgm_ctx_create(device, out);
    if (st != HGM_OK) return st;
    hgm_ctx* c = *out;
    c->rank = rank;
    c->world = world;
    // world 1 with a non-zero id: a one-rank communicator, so the solve takes the sharded code
    // path with real RCCL all-reduces (rehearses the transport on one GPU)
    const unsigned char* u = static_cast<const unsigned char*>(unique_id);
    const bool one_rank = world == 1 && std::any_of(u, u + sizeof(ncclUniqueId), [](unsigned char x) { return x != 0; });
    if (world > 1 || one_rank) {
        ncclUniqueId id;
        std::memcpy(&id, unique_id, sizeof(id));
        if (ncclCommInitRank(&c->nccl, world, id, rank) != ncclSuccess) {
            c->nccl = nullptr;
            hgm_ctx_destroy(c);
            *out = nullptr;
            return HGM_E_COMM;
        }
    }
    return HGM_OK;
}

HGM_API int hgm_ctx_set_host_allreduce(hgm_ctx* c, int rank, int world, hgm_allreduce_fn fn, void* user) {
    if (!c || world < 1 || rank < 0 || rank >= world || (world > 1 && !fn)) return HGM_E_ARG;
    c->rank = rank;
    c->world = world;
    c->host_ar = fn;
    c->host_ar_user = user;
    return HGM_OK;
}

HGM_API void hgm_ctx_destroy(hgm_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->host_stats)
        std::fprintf(stderr, "hgm host stats: %ld pipeline waits, %.3f ms blocked (%.2f us/wait)\n", c->waits,
                     c->wait_s * 1e3, c->waits ? c->wait_s * 1e6 / c->waits : 0.0);
    if (c->nccl) ncclCommDestroy(c->nccl);
    c->timing.clear();
    for (auto e : c->timing.pool) (void)hipEventDestroy(e);
    c->ws.clear();
    if (c->dscal) (void)hipFree(c->dscal);
    if (c->hscal) (void)hipHostFree(c->hscal);
    if (c->hstage) (void)hipHostFree(c->hstage);
    if (c->hup) (void)hipHostFree(c->hup);
    if (c->hring) (void)hipHostFree(c->hring);
    if (c->ev_pipe) (void)hipEventDestroy(c->ev_pipe);
    for (auto e : c->ev_step)
        if (e) (void)hipEventDestroy(e);
    if (c->aux) {
        (void)hipStreamSynchronize(c->aux);
        (void)hipStreamDestroy(c->aux);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

HGM_API const char* hgm_last_error(const hgm_ctx* c) { return c ? c->err.c_str() : "null context"; }

HGM_API int hgm_ctx_set_option(hgm_ctx* c, int option, double v) {
    if (!c) return HGM_E_ARG;
    hgm::Numerics& n = c->num;
    const bool b01 = v == 0.0 || v == 1.0;
    auto bad = [&](const char* what) {
        c->err = std::string("hgm_ctx_set_option: ") + what;
        return HGM_E_ARG;
    };
    if (!HGM_EXPERIMENTS) {
        // measured variants of the one-pass kernel: compiled into the experiments build only
        bool variant = false;
        switch (option) {
            case HGM_OPT_FUSED_REGION: variant = v != 64; break;
            case HGM_OPT_FUSED_BS: variant = v != 1024; break;
            case HGM_OPT_FUSED_DBG: variant = v != 0; break;
            case HGM_OPT_FUSED_PF: variant = v != 2; break;
            case HGM_OPT_FUSED_KIND: variant = v != 1; break;
            case HGM_OPT_FUSED_WAVES: variant = v != 4; break;
            case HGM_OPT_FUSED_GROUP: variant = v != 8; break;
            case HGM_OPT_FUSED_DEPTH: variant = v != 2; break;
            case HGM_OPT_FUSED_PAIRS: variant = v != 1; break;
            case HGM_OPT_FUSED_ACC32: variant = v != 1; break;
            case HGM_OPT_FUSED_REDUCE: variant = !(v == 0 || v == 1); break;
            case HGM_OPT_FUSED_ROWPAIR: variant = !(v == 0 || v == 4); break;
            default: break;
        }
        if (variant) return bad("a measured variant of the one-pass kernel: experiments build only (HGM_EXPERIMENTS=1)");
    }
    switch (option) {
        case HGM_OPT_PARITY: if (!b01) return bad("parity is 0 or 1"); n.parity = v != 0; break;
        case HGM_OPT_MGS_FORM: if (!b01) return bad("mgs form is 0 or 1"); n.mgs_form = (int)v; break;
        case HGM_OPT_MGS_SINGLE: if (!b01) return bad("mgs single is 0 or 1"); n.mgs_single = v != 0; break;
        case HGM_OPT_GRAM_ERR: if (!b01) return bad("gram err is 0 or 1"); n.gram_err = v != 0; break;
        case HGM_OPT_GRAM_ERR_MIN: if (!(v >= 0.0)) return bad("gram err min >= 0"); n.gram_err_min = v; break;
        case HGM_OPT_RING_POLL: if (!b01) return bad("ring poll is 0 or 1"); n.ring_poll = v != 0; break;
        case HGM_OPT_PEND_NORM:
            if (!(v == 0.0 || v == 1.0 || v == 2.0)) return bad("pend norm is 0, 1 or 2");
            n.pend_norm = (int)v;
            break;
        case HGM_OPT_RECON_SERIAL:
            if (v != -1.0 && !b01) return bad("recon serial is -1, 0 or 1");
            n.recon_serial = (int)v;
            break;
        case HGM_OPT_RECON_SERIAL_N: if (!(v >= 0.0)) return bad("recon serial n >= 0"); n.recon_serial_n = (int64_t)v; break;
        case HGM_OPT_PIPE_DEPTH:
            if (!(v >= 1.0 && v <= 6.0) || v != (double)(int)v) return bad("pipe depth is 1..6");
            n.pipe_depth = (int)v;
            break;
        case HGM_OPT_SYNC_EVENT_FENCE: if (!b01) return bad("sync event fence is 0 or 1"); n.sync_event_fence = v != 0; break;
        case HGM_OPT_MGS_PPL:
            if (!(v >= 1.0 && v <= 8.0) || v != (double)(int)v) return bad("mgs ppl is 1..8");
            n.mgs_ppl = (int)v;
            break;
        case HGM_OPT_MGS1_PPL:
            if (!(v == 0.0 || v == 1.0 || v == 2.0 || v == 4.0)) return bad("mgs1 ppl is 0, 1, 2 or 4");
            n.mgs1_ppl = (int)v;
            break;
        case HGM_OPT_MGS_FUSED: n.mgs_fused = v != 0.0; break;
        case HGM_OPT_LSQR_DEV: n.lsqr_dev = v != 0.0; break;
        case HGM_OPT_PAGED16: n.paged16 = v != 0.0; break;
        case HGM_OPT_BAND_DUAL: n.band_dual = v != 0.0; break;
        case HGM_OPT_FUSED_AB: if (!b01) return bad("fused_ab is 0 or 1"); n.fused_ab = v != 0; break;
        case HGM_OPT_FUSED_REGION:
            if (!(v >= 8 && v <= 1024 && v == std::floor(v))) return bad("fused_region is an integer in [8, 1024]");
            n.fused_region = (int)v;
            break;
        case HGM_OPT_FUSED_BS:
            if (!(v == 512 || v == 1024)) return bad("fused_bs is 512 or 1024");
            n.fused_bs = (int)v;
            break;
        case HGM_OPT_FUSED_PF: if (v < 0 || v > 4) return bad("fused_pf is 0..4"); n.fused_pf = v < 1 ? 1 : (int)v; break;
        case HGM_OPT_KRYLOV_PAD: if (v < -1 || v > 65536 || v != (double)(int64_t)v || (v > 0 && (int64_t)v % 64)) return bad("krylov_pad is -1 or a multiple of 64 in 0..65536"); n.krylov_pad = (int)v; break;
        case HGM_OPT_FUSED_DBG:
            if (!(v >= 0 && v <= 15 && v == std::floor(v))) return bad("fused_dbg is 0..15");
            n.fused_dbg = (int)v;
            break;
        case HGM_OPT_FUSED_KIND: if (!b01) return bad("fused_kind is 0 or 1"); n.fused_kind = (int)v; break;
        case HGM_OPT_FUSED_WREGION:
            if (!(v >= 4 && v <= 256 && v == std::floor(v))) return bad("fused_wregion is an integer in [4, 256]");
            n.fused_wregion = (int)v;
            break;
        case HGM_OPT_FUSED_WAVES:
            if (!(v == 1 || v == 2 || v == 4)) return bad("fused_waves is 1, 2 or 4");
            n.fused_waves = (int)v;
            break;
        case HGM_OPT_FUSED_GROUP:
            if (!(v == 4 || v == 8)) return bad("fused_group is 4 or 8");
            n.fused_group = (int)v;
            break;
        case HGM_OPT_FUSED_DEPTH:
            if (!(v == 2 || v == 3 || v == 4)) return bad("fused_depth is 2, 3 or 4");
            n.fused_depth = (int)v;
            break;
        case HGM_OPT_FUSED_PAIRS: if (!b01) return bad("fused_pairs is 0 or 1"); n.fused_pairs = v != 0; break;
        case HGM_OPT_FUSED_ACC32:
            if (!(v == 0 || v == 1 || v == 2)) return bad("fused_acc32 is 0, 1 or 2");
            n.fused_acc32 = (int)v;
            break;
        case HGM_OPT_FUSED_PLAN_DEV: if (!b01) return bad("fused_plan_dev is 0 or 1"); n.fused_plan_dev = v != 0; break;
        case HGM_OPT_FUSED_REDUCE:
            if (!(v == 0 || v == 1 || v == 2 || v == 3 || v == 4)) return bad("fused_reduce is 0 to 4");
            n.fused_reduce = (int)v;
            break;
        case HGM_OPT_FUSED_ROWPAIR:
            if (!(v == 0 || v == 1 || v == 2 || v == 3 || v == 4)) return bad("fused_rowpair is 0 to 4");
            n.fused_rowpair = (int)v;
            break;
        case HGM_OPT_LSQR_RES_IMG: if (!b01) return bad("lsqr_res_img is 0 or 1"); n.lsqr_res_img = v != 0; break;
        case HGM_OPT_LSMR_FUSE_NMON: if (!b01) return bad("lsmr_fuse_nmon is 0 or 1"); n.lsmr_fuse_nmon = v != 0; break;
        case HGM_OPT_HOST_SPIN_US:
            if (!(v == std::floor(v) && std::fabs(v) <= 1e9)) return bad("host_spin_us is an integer");
            g_host_spin_us.store((int)v);
            break;
        default: return bad("unknown option");
    }
    return HGM_OK;
}

HGM_API int hgm_ctx_get_option(const hgm_ctx* c, int option, double* v) {
    if (!c || !v) return HGM_E_ARG;
    const hgm::Numerics& n = c->num;
    switch (option) {
        case HGM_OPT_PARITY: *v = n.parity; break;
        case HGM_OPT_MGS_FORM: *v = n.mgs_form; break;
        case HGM_OPT_MGS_SINGLE: *v = n.mgs_single; break;
        case HGM_OPT_GRAM_ERR: *v = n.gram_err; break;
        case HGM_OPT_GRAM_ERR_MIN: *v = n.gram_err_min; break;
        case HGM_OPT_RING_POLL: *v = n.ring_poll; break;
        case HGM_OPT_PEND_NORM: *v = n.pend_norm; break;
        case HGM_OPT_RECON_SERIAL: *v = n.recon_serial; break;
        case HGM_OPT_RECON_SERIAL_N: *v = (double)n.recon_serial_n; break;
        case HGM_OPT_PIPE_DEPTH: *v = n.pipe_depth; break;
        case HGM_OPT_SYNC_EVENT_FENCE: *v = n.sync_event_fence; break;
        case HGM_OPT_MGS_PPL: *v = n.mgs_ppl; break;
        case HGM_OPT_MGS1_PPL: *v = n.mgs1_ppl; break;
        case HGM_OPT_MGS_FUSED: *v = n.mgs_fused; break;
        case HGM_OPT_LSQR_DEV: *v = n.lsqr_dev; break;
        case HGM_OPT_PAGED16: *v = n.paged16; break;
        case HGM_OPT_BAND_DUAL: *v = n.band_dual; break;
        case HGM_OPT_FUSED_AB: *v = n.fused_ab; break;
        case HGM_OPT_FUSED_REGION: *v = n.fused_region; break;
        case HGM_OPT_FUSED_BS: *v = n.fused_bs; break;
        case HGM_OPT_FUSED_DBG: *v = n.fused_dbg; break;
        case HGM_OPT_FUSED_PF: *v = n.fused_pf; break;
        case HGM_OPT_KRYLOV_PAD: *v = n.krylov_pad; break;
        case HGM_OPT_FUSED_KIND: *v = n.fused_kind; break;
        case HGM_OPT_FUSED_WREGION: *v = n.fused_wregion; break;
        case HGM_OPT_FUSED_WAVES: *v = n.fused_waves; break;
        case HGM_OPT_FUSED_GROUP: *v = n.fused_group; break;
        case HGM_OPT_FUSED_DEPTH: *v = n.fused_depth; break;
        case HGM_OPT_FUSED_PAIRS: *v = n.fused_pairs; break;
        case HGM_OPT_FUSED_ACC32: *v = n.fused_acc32; break;
        case HGM_OPT_FUSED_PLAN_DEV: *v = n.fused_plan_dev; break;
        case HGM_OPT_FUSED_REDUCE: *v = n.fused_reduce; break;
        case HGM_OPT_FUSED_ROWPAIR: *v = n.fused_rowpair; break;
        case HGM_OPT_LSQR_RES_IMG: *v = n.lsqr_res_img; break;
        case HGM_OPT_LSMR_FUSE_NMON: *v = n.lsmr_fuse_nmon; break;
        case HGM_OPT_HOST_SPIN_US: *v = g_host_spin_us.load(); break;
        default: return HGM_E_ARG;
    }
    return HGM_OK;
}

HGM_API int hgm_ctx_synchronize(hgm_ctx* c) {
    if (!c) return HGM_E_ARG;
    HGM_TRY(c, sync(c));
    return HGM_OK;
}

HGM_API void* hgm_ctx_stream(hgm_ctx* c) { return c ? (void*)c->stream : nullptr; }

HGM_API int hgm_ctx_rank(const hgm_ctx* c, int* rank, int* world) {
    if (!c) return HGM_E_ARG;
    if (rank) *rank = c->rank;
    if (world) *world = c->world;
    return HGM_OK;
}

HGM_API int hgm_ctx_release_workspace(hgm_ctx* c, int64_t* bytes_freed) {
    if (!c) return HGM_E_ARG;
    HGM_TRY(c, {
        HGM_HIP(hipSetDevice(c->device));
        HGM_HIP(hipStreamSynchronize(c->stream));
        if (c->aux) HGM_HIP(hipStreamSynchronize(c->aux));
        int64_t b = 0;
        for (auto& kv : c->ws) b += (int64_t)kv.second.bytes;
        c->ws.clear();   // DevBuf destructors free the device memory
        if (bytes_freed) *bytes_freed = b;
    });
    return HGM_OK;
}

HGM_API int hgm_mem_info(hgm_ctx* c, int64_t* free_bytes, int64_t* total_bytes) {
    if (!c) return HGM_E_ARG;
    size_t f = 0, t = 0;
    if (hipSetDevice(c->device) != hipSuccess || hipMemGetInfo(&f, &t) != hipSuccess) return HGM_E_HIP;
    if (free_bytes) *free_bytes = (int64_t)f;
    if (total_bytes) *total_bytes = (int64_t)t;
    return HGM_OK;
}

HGM_API int hgm_ctx_solve_path(const hgm_ctx* c, int what, int* out, int cap, int* n) {
    if (!c || (what != 0 && what != 1) || cap < 0 || (cap > 0 && !out)) return HGM_E_ARG;
    std::vector<int> v;
    if (what == 0) v = c->path_mon;
    else if (c->path_onepass >= 0) v.push_back(c->path_onepass);
    for (int i = 0; i < cap && i < (int)v.size(); ++i) out[i] = v[i];
    if (n) *n = (int)v.size();
    return HGM_OK;
}

// ---- matrices ----------------------------------------------------------------
HGM_API int hgm_mat_create_csr(hgm_ctx* c, int64_t rows, int64_t cols, int64_t nnz, const int64_t* row_ptr,
                               const int32_t* col_idx, const double* val, int dtype, hgm_mat** out) {
    if (!c || !out || rows < 0 || cols < 0 || nnz < 0 || !row_ptr || (nnz > 0 && (!col_idx || !val)))
        return HGM_E_ARG;
    if (dtype != HGM_F64 && dtype != HGM_F32) return HGM_E_ARG;
    if (row_ptr[0] != 0 || row_ptr[rows] != nnz) {
        c->err = "row_ptr must start at 0 and end at nnz";
        return HGM_E_ARG;
    }
    *out = nullptr;
    hgm_mat* M = nullptr;
    HGM_TRY(c, {
        HGM_HIP(hipSetDevice(c->device));
        M = mat_alloc(c, rows, cols, nnz, dtype);
        HGM_HIP(hipMemcpyAsync(M->rp, row_ptr, sizeof(int64_t) * (rows + 1), hipMemcpyHostToDevice, c->stream));
        if (nnz > 0) {
            HGM_HIP(hipMemcpyAsync(M->ci, col_idx, sizeof(int32_t) * nnz, hipMemcpyHostToDevice, c->stream));
            if (dtype == HGM_F64) {
                HGM_HIP(hipMemcpyAsync(M->val, val, sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
            } else {
                double* tmp = c->buf<double>("mat_f64", nnz);
                HGM_HIP(hipMemcpyAsync(tmp, val, sizeof(double) * nnz, hipMemcpyHostToDevice, c->stream));
                convert<float>(c, nnz, tmp, reinterpret_cast<float*>(M->val));
            }
        }
        HGM_HIP(hipStreamSynchronize(c->stream));
        finalize_operator(c, M);
    });
    *out = M;
    return HGM_OK;
}

HGM_API int hgm_mat_create_csc(hgm_ctx* c, int64_t rows, int64_t cols, int64_t nnz, const int64_t* jc,
                               const int64_t* ir, const double* pr, int dtype, hgm_mat** out) {
    if (!c || !out || !jc || (nnz > 0 && (!ir || !pr))) return HGM_E_ARG;
    // CSC of M (rows x cols) == CSR of M^T (cols x rows); build M by a device transpose
    std::vector<int32_t> ci(nnz > 0 ? nnz : 1);
    for (int64_t i = 0; i < nnz; ++i) {
        if (ir[i] < 0 || ir[i] >= rows) {
            c->err = "ir index out of range";
            return HGM_E_ARG;
        }
        ci[i] = (int32_t)ir[i];
    }
    hgm_mat* Mt = nullptr;
    int st = hgm_mat_create_csr(c, cols, rows, nnz, jc, ci.data(), pr, dtype, &Mt);
    if (st != HGM_OK) return st;
    st = hgm_mat_transpose(c, Mt, out);
    hgm_mat_destroy(Mt);
    return st;
}

HGM_API int hgm_mat_transpose(hgm_ctx* c, const hgm_mat* in, hgm_mat** out) {
    if (!c || !in || !out) return HGM_E_ARG;
    *out = nullptr;
    HGM_TRY(c, {
        *out = transpose(c, in);
        finalize_operator(c, *out);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_create_siddon(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, hgm_mat** out) {
    if (!c || !out) return HGM_E_ARG;
    *out = nullptr;
    HGM_TRY(c, {
        *out = siddon(c, N, n_angles, det_offset, dtype);
        finalize_operator(c, *out);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_row_slice(hgm_ctx* c, const hgm_mat* in, int64_t lo, int64_t hi, hgm_mat** out) {
    if (!c || !in || !out) return HGM_E_ARG;
    *out = nullptr;
    HGM_TRY(c, {
        HGM_HIP(hipSetDevice(c->device));
        *out = row_slice(c, in, lo, hi);
        finalize_operator(c, *out);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_create_siddon_ordered(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, int tile,
                                          int super_block, hgm_mat** out) {
    if (!c || !out) return HGM_E_ARG;
    *out = nullptr;
    HGM_TRY(c, {
        *out = siddon(c, N, n_angles, det_offset, dtype, tile, super_block);
        finalize_operator(c, *out);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_create_fanbeam(hgm_ctx* c, int N, int n_angles, double R, double span, double det_offset,
                                   int dtype, int tile, int super_block, hgm_mat** out) {
    if (!c || !out) return HGM_E_ARG;
    *out = nullptr;
    HGM_TRY(c, {
        HGM_HIP(hipSetDevice(c->device));
        *out = fanbeam(c, N, n_angles, R, span, det_offset, dtype, tile, super_block);
        finalize_operator(c, *out);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_create_backprojector(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, int tile,
                                         int super_block, hgm_mat** out) {
    if (!c || !out) return HGM_E_ARG;
    *out = nullptr;
    HGM_TRY(c, {
        HGM_HIP(hipSetDevice(c->device));
        *out = backprojector(c, N, n_angles, det_offset, dtype, tile, super_block);
        finalize_operator(c, *out);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_order(const hgm_mat* M, int which, int* N, int* tile, int* super_block) {
    if (!M || (which != 0 && which != 1)) return HGM_E_ARG;
    const PixOrder& o = which == 0 ? M->row_order : M->col_order;
    if (N) *N = o.N;
    if (tile) *tile = o.trivial() ? 1 : o.tile;
    if (super_block) *super_block = o.trivial() ? 0 : o.super;
    return HGM_OK;
}

HGM_API int hgm_mat_info(const hgm_mat* M, int64_t* rows, int64_t* cols, int64_t* nnz, int* dtype) {
    if (!M) return HGM_E_ARG;
    if (rows) *rows = M->rows;
    if (cols) *cols = M->cols;
    if (nnz) *nnz = M->nnz;
    if (dtype) *dtype = M->dtype;
    return HGM_OK;
}

HGM_API int hgm_mat_set_bands(hgm_ctx* c, hgm_mat* M, int64_t band_width, int group) {
    if (!c || !M || band_width < -1) return HGM_E_ARG;
    if (group != 0 && group != 4 && group != 8 && group != 16 && group != 32 && group != 64) return HGM_E_ARG;
    HGM_TRY(c, {
        HGM_HIP(hipSetDevice(c->device));
        set_bands(c, M, band_width == -1 ? auto_band_width(M) : band_width);
        if (group && M->nbands > 1) M->bgroup = group;
        if (M->variant & SPMV_STREAM) build_page_index(c, M);
    });
    return HGM_OK;
}

HGM_API int hgm_mat_tune(hgm_mat* M, int variant, int group) {
    if (!M || variant < 0 || variant > 31) return HGM_E_ARG;
    if (group != 0 && group != 2 && group != 4 && group != 8 && group != 16 && group != 32 && group != 64) return HGM_E_ARG;
    if (group == 2 && !(variant & SPMV_STREAM)) return HGM_E_ARG;   // (2 lanes: streaming reduction only)
    if ((variant & SPMV_PAGED) && !M->pg_ptr) {   // page index on demand (over the current stream)
        HGM_TRY(M->ctx, {
            HGM_HIP(hipSetDevice(M->ctx->device));
            build_page_index(M->ctx, M);
        });
    }
    M->variant = variant;
    if (group && (variant & SPMV_STREAM)) M->sgroup = M->bsgroup = group;   // lanes per segment reduction
    else if (group) M->group = group;
    return HGM_OK;
}

}  // extern "C"

namespace hgm {
// CSR in the reference index orders (see hgm_mat_create_siddon_ordered)
static void mat_download_impl(hgm_ctx* c, const hgm_mat* M, int64_t* row_ptr, int32_t* col_idx, double* val) {
    {
        HGM_HIP(hipSetDevice(c->device));
        // stored arrays (column indices mapped back to the reference order on the device)
        std::vector<int64_t> rp((size_t)M->rows + 1);
        HGM_HIP(hipMemcpy(rp.data(), M->rp, sizeof(int64_t) * (M->rows + 1), hipMemcpyDeviceToHost));
        if (!col_idx && !val && M->row_order.trivial()) {   // row pointers only (e.g. a shard plan)
            if (row_ptr) std::memcpy(row_ptr, rp.data(), sizeof(int64_t) * (M->rows + 1));
            return;
        }
        std::vector<int32_t> ci((size_t)M->nnz);
        std::vector<double> vv((size_t)M->nnz);
        if (M->nnz) {
            const int32_t* src = M->ci;
            if (!M->col_order.trivial()) {
                int32_t* t = c->buf<int32_t>("mat_ci_ref", M->nnz);
                HGM_HIP(hipMemcpyAsync(t, M->ci, sizeof(int32_t) * M->nnz, hipMemcpyDeviceToDevice, c->stream));
                pix_unmap_indices(c, M->col_order, t, M->nnz);
                HGM_HIP(hipStreamSynchronize(c->stream));
                src = t;
            }
            HGM_HIP(hipMemcpy(ci.data(), src, sizeof(int32_t) * M->nnz, hipMemcpyDeviceToHost));
            if (M->dtype == HGM_F64) {
                HGM_HIP(hipMemcpy(vv.data(), M->val, sizeof(double) * M->nnz, hipMemcpyDeviceToHost));
            } else {
                double* tmp = c->buf<double>("mat_f64", M->nnz);
                convert_back<float>(c, M->nnz, reinterpret_cast<const float*>(M->val), tmp);
                HGM_HIP(hipStreamSynchronize(c->stream));
                HGM_HIP(hipMemcpy(vv.data(), tmp, sizeof(double) * M->nnz, hipMemcpyDeviceToHost));
            }
        }
        if (M->row_order.trivial()) {
            if (row_ptr) std::memcpy(row_ptr, rp.data(), sizeof(int64_t) * (M->rows + 1));
            if (col_idx && M->nnz) std::memcpy(col_idx, ci.data(), sizeof(int32_t) * M->nnz);
            if (val && M->nnz) std::memcpy(val, vv.data(), sizeof(double) * M->nnz);
        } else {
            // rows stored in a pixel order: emit them in the reference order
            HGM_REQUIRE((int64_t)M->row_order.N * M->row_order.N == M->rows, "download: row order size");
            const std::vector<int64_t> ref = pix_reference_of_stored(M->row_order);
            std::vector<int64_t> stored_of(ref.size());
            for (size_t s = 0; s < ref.size(); ++s) stored_of[(size_t)ref[s]] = (int64_t)s;
            int64_t off = 0;
            for (int64_t p = 0; p < M->rows; ++p) {
                const int64_t s = stored_of[(size_t)p];
                const int64_t b = rp[(size_t)s], e = rp[(size_t)s + 1];
                if (row_ptr) row_ptr[p] = off;
                if (col_idx) std::memcpy(col_idx + off, ci.data() + b, sizeof(int32_t) * (e - b));
                if (val) std::memcpy(val + off, vv.data() + b, sizeof(double) * (e - b));
                off += e - b;
            }
            if (row_ptr) row_ptr[M->rows] = off;
        }
    }
}
}  // namespace hgm

extern "C" {

HGM_API int hgm_mat_download(hgm_ctx* c, const hgm_mat* M, int64_t* row_ptr, int32_t* col_idx, double* val) {
    if (!c || !M) return HGM_E_ARG;
    HGM_TRY(c, hgm::mat_download_impl(c, M, row_ptr, col_idx, val));
    return HGM_OK;
}

HGM_API void hgm_mat_destroy(hgm_mat* M) {
    if (!M) return;
    (void)hipDeviceSynchronize();   // hipFree below is device-synchronous anyway; never touch M->ctx here
    mat_free(M);
}

HGM_API int hgm_spmv(hgm_ctx* c, const hgm_mat* A, const void* x, void* y) {
    if (!c || !A || !x || !y) return HGM_E_ARG;
    HGM_TRY(c, {
        if (A->dtype == HGM_F64) spmv_ref<double>(c, A, (const double*)x, (double*)y);
        else spmv_ref<float>(c, A, (const float*)x, (float*)y);
    });
    return HGM_OK;
}

HGM_API int hgm_spmv_ab(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const void* q, void* Bq, void* ABq) {
    if (!c || !A || !B || !q || !Bq || !ABq) return HGM_E_ARG;
    HGM_TRY(c, {
        HGM_REQUIRE(A->rows == B->cols && A->cols == B->rows, "spmv_ab: B must be size(A')");
        HGM_REQUIRE(A->dtype == B->dtype, "spmv_ab: A and B share the dtype");
        HGM_REQUIRE(A->col_order == B->row_order && A->row_order.trivial() && B->col_order.trivial(),
                    "spmv_ab: A's columns and B's rows share the pixel order");
        // one rank: on a communicator (a pixel shard) the product would be this rank's partial
        // A_g*(B_g*q) before the all-reduce, which this single-operator call does not perform
        HGM_REQUIRE(c->world == 1 && c->nccl == nullptr, "spmv_ab: a single-rank context (no communicator)");
        auto run = [&](auto tag) {
            using T = decltype(tag);
            T* bq = B->row_order.trivial() ? (T*)Bq : c->buf<T>("spmv_ab_bq", B->rows);
            const FusedPlan* P = fused_ab_plan(c, A, B);
            if (P && !fused_gk_ok(c, B, P) && sizeof(T) == 4) P = nullptr;
            if (P) {
                FusedArgs<T> fa;
                fa.q = (const T*)q;
                fa.zraw = bq;
                fa.w = (T*)ABq;
                fused_pass<T>(c, B, P, fa);
            } else {
                spmv<T>(c, B, (const T*)q, bq, EPI_NONE, T(0), nullptr, KC_SPMV_B);
                spmv<T>(c, A, bq, (T*)ABq, EPI_NONE, T(0), nullptr, KC_SPMV_A);
            }
            if (!B->row_order.trivial()) pix_permute<T>(c, B->row_order, bq, (T*)Bq, 1);
        };
        if (A->dtype == HGM_F64) run(double(0));
        else run(float(0));
    });
    return HGM_OK;
}

HGM_API int hgm_fused_plan_info(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, double* build_s, uint64_t* checksum,
                                int64_t* nslot, int* device_built) {
    if (!c || !A || !B) return HGM_E_ARG;
    HGM_TRY(c, {
        const FusedPlan* P = fused_ab_plan(c, A, B);
        HGM_REQUIRE(P != nullptr, "fused plan: this pair has none (two-pass path)");
        if (build_s) *build_s = fused_plan_build_seconds(P);
        if (checksum) *checksum = fused_plan_checksum(c, B, P);
        if (nslot) *nslot = fused_plan_slots(P);
        if (device_built) *device_built = fused_plan_device_built(P) ? 1 : 0;
    });
    return HGM_OK;
}

HGM_API int hgm_dev_alloc(hgm_ctx* c, int64_t bytes, void** ptr) {
    if (!c || !ptr || bytes < 0) return HGM_E_ARG;
    if (hipSetDevice(c->device) != hipSuccess) return HGM_E_HIP;
    if (hipMalloc(ptr, bytes > 0 ? bytes : 1) != hipSuccess) {
        c->err = "hipMalloc failed";
        return HGM_E_NOMEM;
    }
    return HGM_OK;
}
HGM_API int hgm_dev_free(hgm_ctx* c, void* ptr) {
    if (!c) return HGM_E_ARG;
    if (ptr) (void)hipFree(ptr);
    return HGM_OK;
}
HGM_API int hgm_memcpy_h2d(hgm_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c) return HGM_E_ARG;
    HGM_TRY(c, {
        HGM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
    });
    return HGM_OK;
}
HGM_API int hgm_memcpy_d2h(hgm_ctx* c, void* dst, const void* src, int64_t bytes) {
    if (!c) return HGM_E_ARG;
    HGM_TRY(c, {
        HGM_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
    });
    return HGM_OK;
}

// ---- solvers ------------------------------------------------------------------
#define HGM_SOLVE(ctx, expr)                               \
    do {                                                   \
        if (!(ctx)) return HGM_E_ARG;                      \
        int rc_ = HGM_OK;                                  \
        HGM_TRY(ctx, {                                     \
            HGM_HIP(hipSetDevice((ctx)->device));          \
            rc_ = (expr);                                  \
        });                                                \
        return rc_;                                        \
    } while (0)

HGM_API int hgm_hybrid_ab_gmres_rtp_ex(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B,
                                       const double* b, const double* xt, double tol, int maxit, double lambda,
                                       double* x, double* err, double* res, int* niters) {
    // n-space Arnoldi on B*A + lambda*I with the AQk Gram projected solve (hybrid_ab_gmres_rtp.m)
    HGM_SOLVE(c, gmres_family(c, GmresSpec{HGM_SIDE_BA, PROJ_ABRTP, true, false}, o, A, B, b, xt, tol, maxit,
                              lambda, x, err, res, niters));
}
HGM_API int hgm_hybrid_ba_gmres_rtp_ex(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B,
                                       const double* b, const double* xt, double tol, int maxit, double lambda,
                                       double* x, double* err, double* res, int* niters) {
    HGM_SOLVE(c, gmres_family(c, GmresSpec{HGM_SIDE_BA, PROJ_LS, true, true}, o, A, B, b, xt, tol, maxit,
                              lambda, x, err, res, niters));
}
HGM_API int hgm_gmres_bounds_ex(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B, const double* b,
                                const double* xt, double tol, int maxit, double lambda, int side, int hybrid,
                                double* x, double* err, double* res, int* niters) {
    if (side != HGM_SIDE_AB && side != HGM_SIDE_BA) return HGM_E_ARG;
    HGM_SOLVE(c, gmres_family(c, GmresSpec{side, hybrid ? PROJ_PTR : PROJ_LS, false, false}, o, A, B, b, xt, tol,
                              maxit, hybrid ? lambda : 0.0, x, err, res, niters));
}
HGM_API int hgm_lsqr_solver_ex(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* At, const double* b,
                               const double* xt, double tol, int maxit, double* x, double* err, double* res,
                               int* niters) {
    if (A && A->dtype == HGM_F32)
        HGM_SOLVE(c, lsqr_t<float>(c, o, A, At, b, xt, tol, maxit, false, 0.0, x, err, res, niters));
    HGM_SOLVE(c, lsqr_t<double>(c, o, A, At, b, xt, tol, maxit, false, 0.0, x, err, res, niters));
}
HGM_API int hgm_lsmr_solver_ex(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* At, const double* b,
                               const double* xt, double tol, int maxit, double* x, double* eh, double* rh, double* ah,
                               int* iters) {
    if (A && A->dtype == HGM_F32)
        HGM_SOLVE(c, lsmr_t<float>(c, o, A, At, b, xt, tol, maxit, x, eh, rh, ah, iters));
    HGM_SOLVE(c, lsmr_t<double>(c, o, A, At, b, xt, tol, maxit, x, eh, rh, ah, iters));
}

HGM_API int hgm_hybrid_ab_gmres_rtp(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const double* b,
                                    const double* xt, double tol, int maxit, double lambda, double* x, double* err,
                                    double* res, int* niters) {
    return hgm_hybrid_ab_gmres_rtp_ex(c, nullptr, A, B, b, xt, tol, maxit, lambda, x, err, res, niters);
}
HGM_API int hgm_hybrid_ba_gmres_rtp(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const double* b,
                                    const double* xt, double tol, int maxit, double lambda, double* x, double* err,
                                    double* res, int* niters) {
    return hgm_hybrid_ba_gmres_rtp_ex(c, nullptr, A, B, b, xt, tol, maxit, lambda, x, err, res, niters);
}
HGM_API int hgm_gmres_bounds(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const double* b, const double* xt,
                             double tol, int maxit, double lambda, int side, int hybrid, double* x, double* err,
                             double* res, int* niters) {
    return hgm_gmres_bounds_ex(c, nullptr, A, B, b, xt, tol, maxit, lambda, side, hybrid, x, err, res, niters);
}
HGM_API int hgm_lsqr_solver(hgm_ctx* c, const hgm_mat* A, const hgm_mat* At, const double* b, const double* xt,
                            double tol, int maxit, double* x, double* err, double* res, int* niters) {
    return hgm_lsqr_solver_ex(c, nullptr, A, At, b, xt, tol, maxit, x, err, res, niters);
}
HGM_API int hgm_lsmr_solver(hgm_ctx* c, const hgm_mat* A, const hgm_mat* At, const double* b, const double* xt,
                            double tol, int maxit, double* x, double* eh, double* rh, double* ah, int* iters) {
    return hgm_lsmr_solver_ex(c, nullptr, A, At, b, xt, tol, maxit, x, eh, rh, ah, iters);
}
HGM_API int hgm_hybrid_lsqr_solver(hgm_ctx* c, const hgm_mat* A, const hgm_mat* At, const double* b,
                                   const double* xt, double tol, int maxit, double lambda, double* x, double* err,
                                   double* res, int* niters) {
    if (A && A->dtype == HGM_F32)
        HGM_SOLVE(c, lsqr_t<float>(c, nullptr, A, At, b, xt, tol, maxit, true, lambda, x, err, res, niters));
    HGM_SOLVE(c, lsqr_t<double>(c, nullptr, A, At, b, xt, tol, maxit, true, lambda, x, err, res, niters));
}
HGM_API int hgm_hybrid_lsmr_solver(hgm_ctx* c, const hgm_mat* A, const hgm_mat* At, const double* b,
                                   const double* xt, double tol, int maxit, double lambda, double* x, double* err,
                                   double* res, int* niters) {
    HGM_SOLVE(c, hybrid_lsmr(c, nullptr, A, At, b, xt, tol, maxit, lambda, x, err, res, niters));
}

HGM_API int hgm_arnoldi(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B, const double* b, int k, int side,
                        double breakdown_tol, int orth, double* H, double* beta, int* kdone) {
    if (side != HGM_SIDE_AB && side != HGM_SIDE_BA) return HGM_E_ARG;
    HGM_SOLVE(c, arnoldi(c, A, B, b, k, side, breakdown_tol, orth, H, beta, kdone));
}

HGM_API int hgm_gcv_from_H(const double* H, int k, double beta, double lambda, double trace_m, double* gcv) {
    if (!H || !gcv || k < 1) return HGM_E_ARG;
    *gcv = dense::gcv_from_H(H, k + 1, k, beta, lambda, trace_m);
    return HGM_OK;
}

HGM_API int hgm_gcv_function(hgm_ctx* c, double lambda, const hgm_mat* A, const hgm_mat* B, const double* b,
                             int64_t m, int k_gcv, int side, double* gcv) {
    if (!c || !gcv || !A || k_gcv < 1) return HGM_E_ARG;
    std::vector<double> H((size_t)(k_gcv + 1) * k_gcv);
    double beta = 0;
    int kd = 0;
    int st = hgm_arnoldi(c, A, B, b, k_gcv, side, 1e-12, HGM_MGS, H.data(), &beta, &kd);
    if (st != HGM_OK) return st;
    // gcv_function.m:33 k = size(H,2) = k_gcv; trace term m ('ab') or n ('ba') (:46-50)
    const double trace_m = side == HGM_SIDE_AB ? (double)m : (double)A->cols * 1.0;
    double tm = trace_m;
    if (side == HGM_SIDE_BA && (c->world > 1 || c->nccl)) {
        double nloc = (double)A->cols;
        std::vector<double> v{nloc};
        HGM_TRY(c, {
            double* d = reinterpret_cast<double*>(c->dscal) + 100;
            HGM_HIP(hipMemcpyAsync(d, v.data(), sizeof(double), hipMemcpyHostToDevice, c->stream));
            allreduce(c, d, 1);
            HGM_HIP(hipMemcpyAsync(v.data(), d, sizeof(double), hipMemcpyDeviceToHost, c->stream));
            HGM_HIP(hipStreamSynchronize(c->stream));
        });
        tm = v[0];
    }
    *gcv = dense::gcv_from_H(H.data(), k_gcv + 1, k_gcv, beta, lambda, tm);
    return HGM_OK;
}

HGM_API int hgm_gcv_fminbnd(const double* H, int k, double beta, double trace_m, double lo, double hi, double tolx,
                            double* lambda_opt, double* gcv_opt) {
    if (!H || k < 1 || !lambda_opt || !(hi > lo)) return HGM_E_ARG;
    *lambda_opt = dense::gcv_fminbnd(H, k, beta, trace_m, lo, hi, tolx, gcv_opt);
    return HGM_OK;
}

HGM_API int hgm_gmres_bounds_filter(hgm_ctx* c, const hgm_opts* o, const hgm_mat* A, const hgm_mat* B,
                                    const double* b, const double* xt, double tol, int maxit, double lambda,
                                    int side, int hybrid, const hgm_mat* dM_left, const hgm_mat* dM_right,
                                    int ritz_steps, double* x, double* err, double* res, int* niters,
                                    double* phi_iter, double* dphi_iter, double* mu, double* ritz_resid) {
    if (side != HGM_SIDE_AB && side != HGM_SIDE_BA) return HGM_E_ARG;
    HGM_SOLVE(c, gmres_bounds_filter(c, o, A, B, b, xt, tol, maxit, lambda, side, hybrid, dM_left, dM_right,
                                     ritz_steps, x, err, res, niters, phi_iter, dphi_iter, mu, ritz_resid));
}

HGM_API int hgm_filter_factors(const double* H, int ldh, int k, const double* dK, int lddk, const double* mu,
                               const double* dmu, double lambda, int side, int hybrid, double* phi, double* dphi) {
    if (!H || !dK || !mu || !dmu || !phi || !dphi || k < 1 || ldh < k + 1 || lddk < k) return HGM_E_ARG;
    if (side != HGM_SIDE_AB && side != HGM_SIDE_BA) return HGM_E_ARG;
    try {
        dense::filter_factors(H, ldh, k, dK, lddk, mu, dmu, lambda, side, hybrid, phi, dphi);
    } catch (const Error& e) {
        return e.code;
    }
    return HGM_OK;
}

HGM_API int hgm_ritz(const double* Hp, int ldh, int p, double h_next, const double* G, int ldg, int nev, double* mu,
                     double* dmu, double* resid) {
    if (!Hp || !G || !mu || !dmu || p < 1 || nev < 1 || nev > p || ldh < p || ldg < p) return HGM_E_ARG;
    try {
        dense::ritz(Hp, ldh, p, h_next, G, ldg, nev, mu, dmu, resid);
    } catch (const Error& e) {
        return e.code;
    }
    return HGM_OK;
}

HGM_API int hgm_eig(int n, const double* A, double* wr, double* wi, double* V) {
    if (n < 1 || !A || !wr || !wi) return HGM_E_ARG;
    return dense::eig_general(n, A, wr, wi, V) ? HGM_OK : HGM_E_ARG;
}

HGM_API int hgm_kernel_timing(hgm_ctx* c, int enable) {
    if (!c) return HGM_E_ARG;
    HGM_TRY(c, {
        sync(c);
        c->timing.clear();
        c->timing.on = enable != 0;
        c->timing.paused = false;
        c->timing.mask = (enable & 0x100) ? (unsigned)(enable & 0xff) : 0xffu;
    });
    return HGM_OK;
}

HGM_API int hgm_kernel_timing_pause(hgm_ctx* c, int paused) {
    if (!c) return HGM_E_ARG;
    c->timing.paused = paused != 0;
    return HGM_OK;
}

HGM_API int hgm_kernel_timing_read(hgm_ctx* c, int cls, double* total_ms, int64_t* calls, double* bytes) {
    if (!c || cls < 0 || cls >= KC_N) return HGM_E_ARG;
    HGM_TRY(c, {
        sync(c);
        double tot = 0;
        for (auto& pr : c->timing.ev[cls]) {
            float ms = 0;
            HGM_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
            tot += ms;
        }
        if (total_ms) *total_ms = tot;
        if (calls) *calls = (int64_t)c->timing.ev[cls].size();
        if (bytes) *bytes = c->timing.bytes[cls];
    });
    return HGM_OK;
}

}  // extern "C"
