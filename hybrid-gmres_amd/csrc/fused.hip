// One pass over B for the m-space Arnoldi operator w = A*(B*q) (ABgmres_*_bounds.m:25,
// gcv_function.m:20) when B is A' value for value (a device transpose pair) -- DESIGN.md §3.5.
//
// The two-pass form streams the same values twice (B*q pixel-major, then A*z ray-major: 24.5 GB
// of algorithmic traffic per step at C4).  Here B's pixel-major entries are read ONCE:
//   z_j = sum_i B(j,i) q_i                  (row sums: the kept column B*q, written out)
//   w_i = sum_j A(i,j) z_j = sum_j B(j,i) z_j
// The second sum scatters from pixel rows into rays.  To keep it deterministic (no atomics) and
// its partials few, the pixels are grouped into REGIONS (R x R pixel squares of the image): one
// workgroup owns one region and accumulates the region's rays in LDS (a 64 x 64 square is
// crossed by ~3,900 of the 272,271 C4 rays), so one partial per (region, ray) leaves the kernel;
// a ray-major pass then sums each ray's partials in region order.
//
// Inside a region the entries are processed in SUB-CHUNKS of <= FCH entries (whole pixel rows of
// one region).  Per sub-chunk the plan holds a local CSC: the distinct rays of the sub-chunk
// (`lr_*`: global ray id, first position, region-ray index) and perm[e] = the sub-chunk position
// of the k-th entry in ray order.  The kernel
//   1. loads the values (registers) and scatters q_ray to every entry of the ray (LDS, via perm),
//   2. forms the products and the row sums z_j (FG lanes per row, fixed tree), writes z,
//   3. forms u_e = B(j,i) z_j (LDS) and sums each local ray's u_e in position order,
//   4. adds that to the region accumulator (one owner thread per ray per sub-chunk, sub-chunks
//      in a fixed order): every sum has a fixed order, so products are bitwise reproducible.
// Per entry the pass reads the value (8 B) and perm (2 B); the local-ray records add ~1.4 B.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <numeric>
#include <thread>

#include "device_common.h"

namespace hgm {

namespace {
constexpr int FCH = 4096;      // entries per sub-chunk
constexpr int FRMAX = 3968;    // rays per region (LDS accumulators; 64 x 64 pixels at 47 angles: ~3,900)
constexpr int FLRMAX = 768;    // distinct rays per sub-chunk (C4: <= ~700)
constexpr int FROWS = 128;     // pixel rows per sub-chunk
}  // namespace
#ifndef HGM_FUSED_FGR
#define HGM_FUSED_FGR 16       // lanes per pixel-row sum (fixes the summation order)
#endif

// A sub-chunk's entries sit at LDS positions ("coordinates") e - (e0 & ~1): the values are loaded
// in 16-byte pairs aligned in memory, so with an odd e0 coordinate 0 is the previous sub-chunk's
// last entry, loaded and never used.
struct FusedSub {
    int64_t e0;        // first entry (B's CSR order)
    int64_t lr0;       // first local-ray record
    int32_t r0;        // first row
    uint32_t p0q;      // perm of this sub-chunk at perm[4 * p0q] (padded to 4 entries: 8-byte loads)
    uint16_t len;      // entries
    uint16_t nrow;     // rows
    uint16_t nlr;      // local rays
    uint16_t pad;
};
static_assert(sizeof(FusedSub) == 32, "FusedSub layout");

struct FusedPlan {
    int kind = 0;                 // 0 sub-chunk pass (k_fused_ab), 1 row-wave pass (k_fused_rw)
    int elem = 8;                 // value size (kind 1: fp64 or fp32; the slots are byte offsets)
    int region = 0, waves = 0, maxr = 0, group = 0, depth = 0;
    bool pairs = false;
    int rowpair = 0;              // kind 1: units of two consecutive rows (k_fused_rw RP 1 / 2; runs
                                  // split so every unit spans one chunk)
    int64_t nreg = 0, nsub = 0, nlr = 0, nslot = 0, m = 0, maxlen = 0;
    // kind 1: per (region, wave) a range of row runs; the region's rays; every entry's index
    // among its region's rays
    int32_t* wrun = nullptr;      // nreg * waves + 1
    int2* runs = nullptr;         // (first row, rows)
    int32_t* ray_tab = nullptr;   // nslot: global ray of each region-local ray
    uint16_t* lidx = nullptr;     // nnz (+ padding): the slot as an LDS byte offset (index * elem)
    int32_t* reg_sub = nullptr;   // nreg+1
    int64_t* reg_base = nullptr;  // nreg+1
    FusedSub* subs = nullptr;     // nsub
    uint16_t* perm = nullptr;     // per sub-chunk: coordinate of its k-th entry in ray order
    int32_t* lr_ray = nullptr;    // nlr
    uint32_t* lr_pk = nullptr;    // nlr: first position | entries << 12 | region ray index << 20
    int64_t* rs_ptr = nullptr;    // m+1
    int32_t* rs_slot = nullptr;   // nslot
    // kind 1: the partials by ray band (k_fused_reduce_band): band b = rays [64 b, 64 b + 64); its
    // runs (first slot, first ray - 64 b, rays) of consecutive rays in consecutive slots of one
    // region, regions in increasing order
    int64_t nband = 0, nrun = 0;
    int32_t* band_ptr = nullptr;  // nband + 1
    int4* band_run = nullptr;     // nrun
    double* part = nullptr;       // nslot (fp32 plans use it as float)
    double* zx_part = nullptr;    // kind 1: nreg (the regions' side sums; fp32 plans: float)
    double build_s = 0;
    bool dev_built = false;       // kind 1: ray sets built on the device (HGM_OPT_FUSED_PLAN_DEV)
};

void fused_plan_free(FusedPlan* P) {
    if (!P) return;
    for (void* p : {(void*)P->reg_sub, (void*)P->reg_base, (void*)P->subs, (void*)P->perm, (void*)P->lr_ray,
                    (void*)P->lr_pk, (void*)P->rs_ptr, (void*)P->rs_slot, (void*)P->part, (void*)P->wrun,
                    (void*)P->runs, (void*)P->ray_tab, (void*)P->lidx, (void*)P->zx_part, (void*)P->band_ptr,
                    (void*)P->band_run})
        if (p) (void)hipFree(p);
    delete P;
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
// Workgroup barrier for LDS hand-offs only: this wave's LDS accesses retire (lgkmcnt), then
// s_barrier; the empty asm statements keep the compiler from moving memory accesses across it.
// __syncthreads() is a release/acquire fence as well, and with the kernel's global stores (z) in
// flight its fence drains vmcnt -- every global load still in flight, the next sub-chunk's batch
// included -- at every barrier.
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// FBS threads per workgroup; LDS 77 KB (two workgroups per CU), so FBS sets the waves in flight.
// Every global read of a sub-chunk is issued as a batch (values and perm, entry j on thread
// j mod FBS: every load instruction coalesced; the local-ray records and row pointers; then the q
// gathers of its rays) and the loops over entries run from LDS.  The local rays come longest first
// (plan order), so the lanes of a wave walk rays of about the same length.  FGR lanes per row sum.
// Measured variants (C4, one box): consecutive entries per thread for 16-byte LDS accesses made
// every value load strided (4.71 vs 3.73 ms); software pipelining of the next sub-chunk's loads
// cost the registers two workgroups per CU need (4.39 ms, spilling at 1024 threads).
// dbg (HGM_OPT_FUSED_DBG, timing experiments only; the results are then wrong): bit 1 skips the
// q scatter, 2 the row sums, 4 the per-ray sums, 8 the two elementwise passes.
// D: sub-chunk batches in registers (1: no prefetch; D > 1: D - 1 batches in flight while one is
// processed).  Two 1024-thread workgroups per CU leave 64 VGPRs a lane (D = 2); deeper pipelines
// run one 1024- or two 512-thread workgroups per CU (128 VGPRs).
template <int FBS, int FGR, int D>
__global__ __launch_bounds__(FBS) __attribute__((amdgpu_waves_per_eu(D <= 2 ? FBS / 128 : 4, 8))) void k_fused_ab(
    const FusedSub* __restrict__ subs, const int32_t* __restrict__ reg_sub, const int64_t* __restrict__ reg_base,
    const uint16_t* __restrict__ perm, const int32_t* __restrict__ lr_ray, const uint32_t* __restrict__ lr_pk,
    const int64_t* __restrict__ rp, const double* __restrict__ val, const double* __restrict__ q,
    double* __restrict__ z, double* __restrict__ part, int dbg) {
    constexpr int VP = FCH / 2 / FBS;                   // value pairs per thread
    constexpr int PQ = FCH / 4 / FBS;                   // perm quads per thread
    constexpr int RPT = (FLRMAX + FBS - 1) / FBS;       // local rays per thread
    static_assert(FBS > FROWS, "one row pointer per thread");
    __shared__ __attribute__((aligned(16))) double prod[FCH];
    __shared__ double acc[FRMAX];
    __shared__ __attribute__((aligned(16))) uint16_t sperm[FCH];
    __shared__ int32_t srp[FROWS + 1];
    __shared__ double zrow[FROWS];
    __shared__ __attribute__((aligned(16))) uint8_t rowid[FCH];
    const int g = blockIdx.x;
    const int64_t pb = reg_base[g];
    const int nr = (int)(reg_base[g + 1] - pb);
    for (int r = threadIdx.x; r < nr; r += FBS) acc[r] = 0.0;
    const int s0 = reg_sub[g], s1 = reg_sub[g + 1];
    const int gid = threadIdx.x / FGR, gl = threadIdx.x % FGR;
    // one sub-chunk's operands, loaded branch-free through buffer resources sized to it (a load
    // past the end returns 0): conditional loads made hipcc wait for every earlier load at each
    // branch, so a batch went out one round trip at a time.  The ray ids go first, so the q
    // gathers that depend on them wait for those alone (vmcnt retires in issue order).
    struct Batch {
        FusedSub sc;
        int32_t ray[RPT];
        uint32_t pk[RPT];
        uint32_t rpv;       // low word of the row pointer (rp - first coordinate fits 32 bits)
        double2 v[VP];
        uint2 pq[PQ];
        double qv[RPT];
    };
    // issue(s, bt, live): with !live an empty batch (the same loads against empty ranges: no
    // memory traffic), so every iteration issues the same memory operations and the compiler's
    // in-order vmcnt bookkeeping stays exact -- a conditional batch made it wait for everything.
    auto issue = [&](int s, Batch& bt, bool live) {
        s = live ? s : s0;
        const int4 w0 = reinterpret_cast<const int4*>(subs + s)[0];   // uniform: scalar loads
        const int4 w1 = reinterpret_cast<const int4*>(subs + s)[1];
        bt.sc.e0 = (int64_t)(uint32_t)w0.x | ((int64_t)w0.y << 32);
        bt.sc.lr0 = (int64_t)(uint32_t)w0.z | ((int64_t)w0.w << 32);
        bt.sc.r0 = w1.x;
        bt.sc.p0q = (uint32_t)w1.y;
        bt.sc.len = live ? (uint16_t)(w1.z & 0xffff) : 0;
        bt.sc.nrow = live ? (uint16_t)((uint32_t)w1.z >> 16) : 0;
        bt.sc.nlr = live ? (uint16_t)(w1.w & 0xffff) : 0;
        const int64_t ea = bt.sc.e0 & ~int64_t(1);
        const int span = bt.sc.len + (int)(bt.sc.e0 & 1);   // coordinates in use
        // (values: whole pairs, the last one may end one entry past nnz: the allocation is padded)
        const __amdgpu_buffer_rsrc_t rv = buf_rsrc(val + ea, ((span + 1) & ~1) * 8);
        const __amdgpu_buffer_rsrc_t rpm = buf_rsrc(perm + 4 * (int64_t)bt.sc.p0q, ((bt.sc.len + 3) & ~3) * 2);
        const __amdgpu_buffer_rsrc_t rk = buf_rsrc(lr_pk + bt.sc.lr0, bt.sc.nlr * 4);
        const __amdgpu_buffer_rsrc_t ry = buf_rsrc(lr_ray + bt.sc.lr0, bt.sc.nlr * 4);
        const __amdgpu_buffer_rsrc_t rr = buf_rsrc(rp + bt.sc.r0, (bt.sc.nrow + 1) * 8);
#pragma unroll
        for (int i = 0; i < RPT; ++i)
            bt.ray[i] = (int32_t)__builtin_amdgcn_raw_buffer_load_b32(ry, (threadIdx.x + i * FBS) * 4, 0, 0);
        asm volatile("" ::: "memory");                     // (issued before the rest of the batch)
#pragma unroll
        for (int i = 0; i < RPT; ++i)
            bt.pk[i] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rk, (threadIdx.x + i * FBS) * 4, 0, 0);
        bt.rpv = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rr, threadIdx.x * 8, 0, 0);
#pragma unroll
        for (int i = 0; i < VP; ++i)
            bt.v[i] = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rv, (threadIdx.x + i * FBS) * 16, 0, 2));
#pragma unroll
        for (int i = 0; i < PQ; ++i)
            bt.pq[i] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rpm, (threadIdx.x + i * FBS) * 8, 0, 2));
    };
    auto gather_q = [&](Batch& bt) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) bt.qv[i] = q[bt.ray[i]];     // (ray 0 past nlr: a harmless read)
    };
    // process(cur, nx, more): sub-chunk `cur`; with `more`, the q gathers of `nx` (whose batch is
    // in flight) go out halfway through.  Two batches alternate roles (the loop is unrolled by
    // two), so no register copy of an in-flight load forces a wait.
    auto process = [&](Batch& cur, Batch& nx, bool more) {
        const FusedSub sc = cur.sc;
        const int span = sc.len + (int)(sc.e0 & 1), nrow = sc.nrow;
        const double2* v = cur.v;
        const uint2* pq = cur.pq;
        const uint32_t* pk = cur.pk;
        const double* qv = cur.qv;
        const int rpv = (int)(cur.rpv - (uint32_t)(sc.e0 & ~int64_t(1)));
        lds_sync();                                   // the previous sub-chunk is done with the LDS
#pragma unroll
        for (int i = 0; i < PQ; ++i) reinterpret_cast<uint2*>(sperm)[threadIdx.x + i * FBS] = pq[i];
        if (threadIdx.x <= nrow) srp[threadIdx.x] = rpv;
        lds_sync();
        if (more) gather_q(nx);                           // s+1's ray ids are in by now
        // q of every local ray to each of its entries (pk: first position | length << 12 | rr << 20)
        if (!(dbg & 1)) {
#pragma unroll
            for (int i = 0; i < RPT; ++i) {
                const int k0 = (int)(pk[i] & 0xfffu), k1 = k0 + (int)((pk[i] >> 12) & 0xffu);
                int k = k0;
                for (; k + 4 <= k1; k += 4) {              // (4 index reads in flight, then 4 stores)
                    const int a0 = sperm[k], a1 = sperm[k + 1], a2 = sperm[k + 2], a3 = sperm[k + 3];
                    prod[a0] = qv[i];
                    prod[a1] = qv[i];
                    prod[a2] = qv[i];
                    prod[a3] = qv[i];
                }
                for (; k < k1; ++k) prod[sperm[k]] = qv[i];
            }
        }
        lds_sync();
        if (!(dbg & 8)) {
#pragma unroll
            for (int i = 0; i < VP; ++i) {
                const int jp = threadIdx.x + i * FBS;
                if (2 * jp < span) {
                    double2 t = reinterpret_cast<double2*>(prod)[jp];
                    t.x = v[i].x * t.x;
                    t.y = v[i].y * t.y;
                    reinterpret_cast<double2*>(prod)[jp] = t;
                }
            }
        }
        lds_sync();
        // z_j = B(j,:) q: FGR lanes per row, strided partials, fixed tree
        if (!(dbg & 2)) {
            for (int ri = gid; ri < nrow; ri += FBS / FGR) {
                const int a = srp[ri], b = srp[ri + 1];
                double t = 0.0;
                for (int j = a + gl; j < b; j += FGR) {
                    t += prod[j];
                    rowid[j] = (uint8_t)ri;
                }
                t = group_sum<double, FGR>(t);
                if (gl == 0) zrow[ri] = t;
            }
        }
        lds_sync();
        {   // z out: one store per thread, the rows past nrow fall outside the range and are dropped
            const __amdgpu_buffer_rsrc_t rz = buf_rsrc(z + sc.r0, nrow * 8);
            buf_store(zrow[threadIdx.x & (FROWS - 1)], rz, threadIdx.x * 8);
        }
        if (!(dbg & 8)) {
#pragma unroll
            for (int i = 0; i < VP; ++i) {
                const int jp = threadIdx.x + i * FBS;
                if (2 * jp < span) {   // (the row ids of unused coordinates are stale: masked)
                    const uint32_t rid = reinterpret_cast<const uint16_t*>(rowid)[jp];
                    double2 t;
                    t.x = v[i].x * zrow[rid & (FROWS - 1)];
                    t.y = v[i].y * zrow[(rid >> 8) & (FROWS - 1)];
                    reinterpret_cast<double2*>(prod)[jp] = t;
                }
            }
        }
        lds_sync();
        // each local ray's share, in position order, into the region accumulator
        if (!(dbg & 4)) {
#pragma unroll
            for (int i = 0; i < RPT; ++i) {
                const int k0 = (int)(pk[i] & 0xfffu), k1 = k0 + (int)((pk[i] >> 12) & 0xffu);
                if (k1 > k0) {
                    double t = 0.0;
                    int k = k0;
                    for (; k + 4 <= k1; k += 4) {          // (loads batched, sums in position order)
                        const int a0 = sperm[k], a1 = sperm[k + 1], a2 = sperm[k + 2], a3 = sperm[k + 3];
                        const double p0 = prod[a0], p1 = prod[a1], p2 = prod[a2], p3 = prod[a3];
                        t += p0;
                        t += p1;
                        t += p2;
                        t += p3;
                    }
                    for (; k < k1; ++k) t += prod[sperm[k]];
                    acc[pk[i] >> 20] += t;
                }
            }
        }
    };
    Batch b[D > 1 ? D : 2];
    if constexpr (D > 1) {
        // b[u] is processed while b[u+1 .. u+D-1] are in flight; the loop is unrolled by D so every
        // batch index is static (registers) and no register copy of an in-flight load forces a wait
#pragma unroll
        for (int i = 0; i < D - 1; ++i) issue(s0 + i, b[i], s0 + i < s1);
        gather_q(b[0]);
        for (int s = s0; s < s1; s += D) {
#pragma unroll
            for (int u = 0; u < D; ++u) {
                if (u > 0 && s + u >= s1) break;
                issue(s + u + D - 1, b[(u + D - 1) % D], s + u + D - 1 < s1);
                process(b[u], b[(u + 1) % D], true);
            }
        }
    } else {
        issue(s0, b[0], s0 < s1);
        gather_q(b[0]);
        for (int s = s0; s < s1; ++s) {
            if (s > s0) {
                issue(s, b[0], true);
                gather_q(b[0]);
            }
            process(b[0], b[1], false);
        }
    }
    lds_sync();
    for (int r = threadIdx.x; r < nr; r += FBS) part[pb + r] = acc[r];
}

// w_i = sum of ray i's region partials.  RG lanes per ray: lane l takes the ray's partials l, l+RG,
// ... in region order (loads batched 4 at a time), then the RG lane sums are added by a fixed
// tree: the slot indices of a ray are read contiguously across its lanes.
#ifndef HGM_FUSED_RG
#define HGM_FUSED_RG 8
#endif
// With zx_out, block 0 first adds the nzx regional shares of the side dot x_true'(B*q) (fixed
// order) into *zx_out.
#ifndef HGM_FUSED_RB
#define HGM_FUSED_RB 16
#endif
template <int RG, typename T, typename TP = T, int RB = HGM_FUSED_RB>
__global__ __launch_bounds__(BS) void k_fused_reduce(int64_t m, const int64_t* __restrict__ rs_ptr,
                                                     const int32_t* __restrict__ rs_slot,
                                                     const TP* __restrict__ part, T* __restrict__ w,
                                                     const T* __restrict__ zx_part, int nzx, T* zx_out) {
    if (zx_out && blockIdx.x == 0) {
        __shared__ T sh[4];
        const T t = reduce_parts<T, false>(zx_part, nzx, sh);
        if (threadIdx.x == 0) st_sys(zx_out, t);           // (the host ring: system scope, device_common.h)
    }
    const int gl = threadIdx.x % RG;
    for (int64_t i = ((int64_t)blockIdx.x * BS + threadIdx.x) / RG; i < m; i += (int64_t)gridDim.x * (BS / RG)) {
        TP s = TP(0);
        const int64_t k0 = rs_ptr[i], k1 = rs_ptr[i + 1];
        int64_t k = k0 + gl;
        if constexpr (RB >= 2) {
            // a ray's partials in batches of RB per lane with the batch's tail clamped to the ray's
            // last slot (read again, not added): every slot read, then every partial read in flight
            // (C4: ~14 partials per lane, one batch instead of three batches and a serial tail).  The
            // lane adds its partials in slot order whatever RB is, so every RB gives the same bits;
            // the host sizes RB to the partials per lane (fused_reduce_rb: a pixel shard's rays
            // cross few of its regions)
            for (; k < k1; k += RB * RG) {
                int32_t sl[RB];
                TP p[RB];
#pragma unroll
                for (int u = 0; u < RB; ++u) sl[u] = rs_slot[std::min<int64_t>(k + u * RG, k1 - 1)];
#pragma unroll
                for (int u = 0; u < RB; ++u) p[u] = part[sl[u]];
#pragma unroll
                for (int u = 0; u < RB; ++u)
                    if (k + u * RG < k1) s += p[u];
            }
        }
        for (; RB < 8 && k + (RB - 1) * RG < k1; k += RB * RG) {   // RB slot reads, then RB partial reads in flight
            int32_t sl[RB];
            TP p[RB];
#pragma unroll
            for (int u = 0; u < RB; ++u) sl[u] = rs_slot[k + u * RG];
#pragma unroll
            for (int u = 0; u < RB; ++u) p[u] = part[sl[u]];
#pragma unroll
            for (int u = 0; u < RB; ++u) s += p[u];
        }
        for (; k < k1; k += RG) s += part[rs_slot[k]];
        if constexpr (RG > 1) s = group_sum<TP, RG>(s);
        if (gl == 0) w[i] = (T)s;
    }
}

// The same sums by ray band (HGM_OPT_FUSED_REDUCE = 1; measured 2-4 % slower, off by default): one wave per
// band of 64 consecutive rays, lane l owning ray 64 b + l.  The band's runs come in region order;
// a lane adds each partial of its ray to accumulator (j mod 8), j = the partial's index in the
// ray's region-ordered list -- the exact sums lane j mod 8 of k_fused_reduce<8> forms -- and the 8
// accumulators of a ray then go through the same group_sum<8>: the bits of k_fused_reduce<8>.  The
// partials are read in runs of consecutive slots (coalesced) instead of through the 4-B rs_slot
// gather (C4: 126 MB less per pass).  RUNB runs' loads are issued before their adds.
constexpr int RUNB = 16;
template <typename T, typename TP = T>
__global__ __launch_bounds__(BS) void k_fused_reduce_band(int64_t m, int64_t nband, const int32_t* __restrict__ band_ptr,
                                                          const int4* __restrict__ band_run,
                                                          const TP* __restrict__ part, T* __restrict__ w,
                                                          const T* __restrict__ zx_part, int nzx, T* zx_out) {
    __shared__ TP tr[BS / 64][64][9];             // per wave: the lanes' 8 sums (+1: bank spread)
    if (zx_out && blockIdx.x == 0) {
        __shared__ T sh[4];
        const T t = reduce_parts<T, false>(zx_part, nzx, sh);
        if (threadIdx.x == 0) st_sys(zx_out, t);
    }
    const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int64_t band = (int64_t)blockIdx.x * (BS / 64) + wv;
    if (band >= nband) return;                    // (a whole wave: no barrier follows)
    TP a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
    int jc = 0;
    const int r0 = band_ptr[band], r1 = band_ptr[band + 1];
    for (int rc = r0; rc < r1; rc += 64) {
        const int nr = min(64, r1 - rc);
        const int4 d = ln < nr ? band_run[rc + ln] : make_int4(0, 0, 0, 0);
        for (int rb = 0; rb < nr; rb += RUNB) {
            TP p[RUNB];
            bool in[RUNB];
#pragma unroll
            for (int u = 0; u < RUNB; ++u) {      // the loads of RUNB runs first (runs past nr: empty)
                const int r = min(rb + u, 63);
                const int slo = __builtin_amdgcn_readlane(d.x, r), rlo = __builtin_amdgcn_readlane(d.y, r);
                const int cnt = rb + u < nr ? __builtin_amdgcn_readlane(d.z, r) : 0;
                in[u] = (unsigned)(ln - rlo) < (unsigned)cnt;
                p[u] = part[in[u] ? slo + (ln - rlo) : slo];
            }
#pragma unroll
            for (int u = 0; u < RUNB; ++u) {      // then the adds, in run (= region) order
                const int g = jc & 7;
                a0 = (in[u] && g == 0) ? a0 + p[u] : a0;
                a1 = (in[u] && g == 1) ? a1 + p[u] : a1;
                a2 = (in[u] && g == 2) ? a2 + p[u] : a2;
                a3 = (in[u] && g == 3) ? a3 + p[u] : a3;
                a4 = (in[u] && g == 4) ? a4 + p[u] : a4;
                a5 = (in[u] && g == 5) ? a5 + p[u] : a5;
                a6 = (in[u] && g == 6) ? a6 + p[u] : a6;
                a7 = (in[u] && g == 7) ? a7 + p[u] : a7;
                jc += in[u] ? 1 : 0;
            }
        }
    }
    TP* t = tr[wv][ln];
    t[0] = a0; t[1] = a1; t[2] = a2; t[3] = a3; t[4] = a4; t[5] = a5; t[6] = a6; t[7] = a7;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (one wave: its LDS accesses run in order)
    const int64_t ray0 = band * 64;
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {              // 8 rays at a time: lanes 8i..8i+7 = ray 8 s8 + i
        const int rr = s8 * 8 + (ln >> 3);
        TP v = tr[wv][rr][ln & 7];
        v = group_sum<TP, 8>(v);
        if ((ln & 7) == 0 && ray0 + rr < m) w[ray0 + rr] = (T)v;
    }
}

// ------------------------------------------------------------------------------------------
// Row-wave pass (kind 1).  One workgroup of W waves per region; the region's rays get LDS
// slots: q of each ray (shared) and one accumulator per wave (private).  A wave walks its share
// of the region's pixel rows one row at a time, the row's entries across its 64 lanes (NCH
// chunks of 64): p = v * q[slot] in registers, z_j = the wave sum of p (fixed tree), then
// acc[slot] += v * z_j.  A pixel row meets each ray at most once, so the lanes of one row hit
// distinct slots: no conflicts, no atomics, no barriers; the wave's rows go in a fixed order and
// the W accumulators are added in wave order at the end, so every sum has a fixed order.
// Per entry the pass reads the value (8 B) and its slot (2 B) once, and touches the LDS three
// times (q read, accumulator read and write).
//
// Loads are software-pipelined in batches of G rows (never crossing a run of consecutive rows):
// the row pointers of batch b+2 and the entries of batch b+1 are in flight while batch b is
// processed.  Every load goes through a buffer resource sized to its row (past the end: 0), so
// each batch issues the same instructions and the compiler's in-order vmcnt waits stay exact.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Lane exchanges of gfx950 for a transposed reduction (fp64 as two dwords): swap32 swaps lanes
// 32-63 of a with lanes 0-31 of b, swap16 the odd 16-lane rows of a with the even rows of b.
__device__ __forceinline__ void swap32(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16(double& a, double& b) {
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
    a = __hiloint2double((int)hi[0], (int)lo[0]);
    b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// The 64-lane sums of G values at once (G = 4 or 8), by a butterfly that halves the values per
// lane while it halves the lanes per sum: lane l ends with the sum of P[l / (64 / G)], the same
// bits in each lane of its group.  Fixed order.  Per row this is ~6 exchanges and adds instead of
// a full wave reduction each (DPP tree + 8 readlanes).
template <int G, typename T>
__device__ __forceinline__ T rows_sum_t(T (&P)[G]) {
    static_assert(G == 4 || G == 8, "rows per batch");
#pragma unroll
    for (int i = 0; i < G / 2; ++i) {          // lane bit 5
        swap32(P[i], P[i + G / 2]);
        P[i] = P[i] + P[i + G / 2];
    }
#pragma unroll
    for (int i = 0; i < G / 4; ++i) {          // lane bit 4
        swap16(P[i], P[i + G / 4]);
        P[i] = P[i] + P[i + G / 4];
    }
    if constexpr (G == 8) {                    // lane bit 3: row_ror 8 within 16-lane rows
        const bool hi = (threadIdx.x & 8) != 0;
        T s = hi ? P[1] : P[0];
        const T t = hi ? P[0] : P[1];
        s = s + dpp_mov<0x128>(t);
        s += dpp_mov<0xB1>(s);                 // lane ^ 1
        s += dpp_mov<0x4E>(s);                 // lane ^ 2
        s += dpp_mov<0x141>(s);                // other quad of the 8-lane half
        return s;
    } else {
        return row16_sum(P[0]);
    }
}

// acc += t in the LDS unit (ds_add_f64 / ds_add_f32, no return value): the update needs no round
// trip.  DETERMINISM INVARIANT: the order of the adds into one accumulator is
// fixed because (1) the accumulator array is private to the wave (acc[wv]), (2) the LDS executes
// one wave's DS instructions in issue order, and (3) within one instruction the 64 lanes address
// distinct slots (a pixel row meets a ray at most once; out-of-row lanes use their own dummy slot).
// So no atomicity is involved -- only an in-place read-modify-write in program order -- and the
// sums are bitwise reproducible (test_gpu_fused.py repeats every product and solve bit for bit).
// Breaking any of (1)-(3) (shared accumulators, a second wave, duplicate slots per row) would
// make the order depend on timing.
// cache policy of the row-wave pass's entry stream (values, slots): the default (0); nt (2) measured
// 1.7-2.2 % slower (a unit's chunk shares its boundary lines with the next unit's)
#ifndef HGM_RW_AUX
#define HGM_RW_AUX 0
#endif
// the regions' partials are written once and read once, by the reduction: non-temporal stores
// (fp64 pass + reduction 2.244 vs 2.252 ms, fp32 equal; profiles/r5_micro_part_nt_ab.txt)
#ifndef HGM_PART_NT
#define HGM_PART_NT 1
#endif
// Row-pair mode 4's products and fp32 accumulator updates as fused multiply-adds (one rounding per
// term instead of two; the library otherwise builds with -ffp-contract=off for MATLAB's epilogues).
#ifndef HGM_FUSED_FMA
#define HGM_FUSED_FMA 1
#endif
__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }

template <typename T>
__device__ __forceinline__ void lds_add(T* p, T t) {
    (void)__hip_atomic_fetch_add(p, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

// DBG (timing experiments only, HGM_OPT_FUSED_DBG with the row-wave pass; results WRONG): bit 1
// skips the q reads, 2 the accumulator updates, 4 the row-sum butterfly.
// D: batches in the ring (D - 1 in flight while one is processed).  PR: two entries per lane (a
// 16-byte value pair (8-byte in fp32) and a 4-byte slot pair per lane from the row's pair-aligned
// start, chunks of 128 entries): half the load instructions of one entry per lane (chunks of 64).
//
// T: double (the GMRES family) or float (BASELINE configs[4], the Golub-Kahan path in fp32): the
// values, q, the row sums, the LDS slots and the partials are T; slots are LDS byte offsets
// (slot * sizeof(T), the plan's element size).
//
// Row epilogue (the Golub-Kahan step v_hat = A'*u - beta*v of lsqr_solver.m:26 / lsmr_solver.m:38
// with q = u): zs_j = z_j - a * ev[j] with a = (T)sqrt((double)*easq), two roundings (no FMA, as
// the two-pass EPI_SUB epilogue); the scatter then forms A*zs, i.e. A*v_hat, so the next step's
// A*v_{k+1} = (A*v_hat)/alpha needs no second pass over the operator.  Without ev: zs = z - 0*0,
// the same bits as z.  Outputs (either may be null): zraw[j] = z_j, zout[j] = zs_j (zout may be ev:
// a row is read and written by the same lanes of one wave, read first).
// Side sum (one value per region, in zx_part): side_sq == 0: sum_j zs_j * xt[j] (the m-space Gram
// error monitor's x_true'(B*q)); side_sq == 1: sum_j zs_j^2 (alpha^2 of the Golub-Kahan step).
// GK: the row epilogue / zout / side_sq code exists (false: the GMRES family's instruction stream).
// pn (pending normalisation of q, the m-space AB-GMRES step; internal.h PendNorm, pn.np > 0): q still
// holds the previous MGS sweep's unnormalised v; every wave re-reduces the sweep's norm partials
// exactly as k_mgs_normalize does (stride BS, then block_sum_all: the same bits), h = sqrt(sum), and
// stages q = v / h (v when h = 0, as k_mgs_normalize leaves it) into its LDS slots; workgroup 0
// publishes h to pn.hdev and H(k+1,k) of the host ring (the MGS sweep that follows writes q back).
// AM: how the accumulators are updated (AccT: their type; the partials are AccT too):
//   0  ds_add of T: fp64 ds_add_f64 (the fp64 production form); fp32 ds_add_f32 measured 11.3 ms
//      at C5 -- the no-return fp32 LDS add runs at a fraction of ds_add_f64's rate on gfx950
//      (9.5 ms of it; scripts/fused_micro.py, profiles/r4_micro_f32.jsonl) -- so fp32 does not use it;
//   1  fp32 read-add-write (ds_read_b32, v_add_f32, ds_write_b32; a wave's rows in order): the fp32
//      production form, 2.00 ms at C5 against 2.44 ms for the two fp32 SpMVs;
//   2  fp64 accumulators for an fp32 pass: products formed in double and added by ds_add_f64,
//      partials and their reduction in double, w rounded to float once: 2.16 ms (half the
//      workgroups per CU: 72 KB of LDS).
template <typename T, int AM> struct AccT { using t = T; };
template <> struct AccT<float, 2> { using t = double; };
//
// RP (row pairs, round 5): the G rows of a batch go as G/2 units of two consecutive rows, whose
// entries are contiguous in B's CSR: one chunk of CH entries from the unit's first pair carries
// both rows (the first row from lane 0, the second right after it), so a row of ~60 entries no
// longer leaves half the lanes idle.  The products are split by row into P[2u] / P[2u+1] (the
// butterfly then sums rows exactly as without RP), and each wave has TWO private accumulator
// arrays, one per row parity of a unit: both rows of a unit add in one LDS instruction, and since
// the first row's lanes address array 0 and the second row's array 1, the addresses of one
// instruction stay distinct (two consecutive pixel rows share most of their rays).  The
// determinism invariant of lds_add holds per array; the arrays are added in a fixed order at the
// end.  The plan keeps every unit's span within one chunk (fused_plan_build_rw splits runs).
// RP = 3 is RP 1 with ONE accumulator array per wave (no extra LDS: the occupancy of the plain
// pass) and each unit's two rows added by two instructions, every lane of the other row on its
// dummy slot.
// RP = 2 places the second row at its own pair-aligned start on the lane after the first row's last
// pair (row membership per lane, not per entry: fewer instructions per unit); a unit then fits when
// the two rows' pair counts add up to <= 64 lanes.
template <typename T, bool GK, int AM, int W, int MAXR, int G, int NCH, int D, bool PR, int DBG = 0, int RP = 0>
__global__ __launch_bounds__(64 * W) void k_fused_rw(const int64_t* __restrict__ reg_base, const int32_t* __restrict__ ray_tab,
                                                     const int32_t* __restrict__ wrun, const int2* __restrict__ runs,
                                                     const int64_t* __restrict__ rp, const T* __restrict__ val,
                                                     const uint16_t* __restrict__ lidx, const T* __restrict__ q,
                                                     T* __restrict__ zraw, typename AccT<T, AM>::t* __restrict__ part,
                                                     const T* __restrict__ xt, T* __restrict__ zx_part,
                                                     const T* ev, const T* __restrict__ easq, T* zout, int side_sq,
                                                     PendNorm<T> pn) {
    static_assert(D >= 2 && D <= 4, "ring depth");
    static_assert(!RP || (PR && NCH == 1 && DBG == 0 && G % 2 == 0), "row pairs: pairs, one chunk");
    constexpr int NA = (RP == 1 || RP == 2) ? 2 : 1;   // private accumulator arrays per wave
    using TA = typename AccT<T, AM>::t;
    constexpr int EPL = PR ? 2 : 1;              // entries per lane per chunk
    constexpr int CH = 64 * EPL;                 // entries per chunk
    constexpr int ES = (int)sizeof(T);
    constexpr int AS = (int)(sizeof(TA) / sizeof(T));   // accumulator offset = slot offset * AS
    __shared__ T qloc[MAXR];                     // (the last 64: the lanes' dummy slots)
    __shared__ TA acc[W][NA][MAXR];
    const int g = blockIdx.x;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int ln = threadIdx.x & 63;
    const int64_t pb = reg_base[g];
    const int nr = (int)(reg_base[g + 1] - pb);
    // Staging: q at the region's rays into LDS, the accumulators zeroed.  All ray_tab loads, then all
    // q gathers, are issued before any is used (NQ per thread), so the pending-normalisation sum
    // below overlaps them.
    // Pending normalisation (pn.np > 0): h = sqrt(sum of pn.parts) in reduce_parts' order for a
    // BS-thread block (thread t sums parts t, t + BS, ...; wave sums; (s0 + s1) + (s2 + s3)), which
    // every wave forms by itself for the BS / 64 virtual waves: the bits of k_mgs_normalize's h with
    // no barrier and no LDS.
    // the wave's runs (<= 64, the plan checks) in lanes: readlane in the loop, no loads there (a
    // conditional load makes the compiler wait for every load in flight after it, and scalar loads'
    // lgkmcnt waits would also wait on the LDS); a range-checked buffer load (zeros past the wave's
    // runs) issued before the staging, so it is in flight with it (round 6)
    int ua = wrun[g * W + wv];
    const int ub = wrun[g * W + wv + 1];
    const int2 runv = __builtin_bit_cast(
        int2, __builtin_amdgcn_raw_buffer_load_b64(buf_rsrc(runs + ua, (ub - ua) * 8), ln * 8, 0, 0));
    static_assert(BS == 256 && MAX_PARTS <= 4 * BS, "pending-normalisation sum: four virtual waves");
    T hq = T(0);
    auto pend_h = [&]() -> T {
        // range-checked buffer loads (zeros past np; adding +0 to a sum of squares changes no bit),
        // all 16 in flight before the sums
        const __amdgpu_buffer_rsrc_t rpp = buf_rsrc(pn.parts, pn.np * (int)sizeof(T));
        T pv[4][4];
#pragma unroll
        for (int vw = 0; vw < 4; ++vw)
#pragma unroll
            for (int j = 0; j < 4; ++j) pv[vw][j] = buf_load<T>(rpp, (64 * vw + ln + j * BS) * (int)sizeof(T));
        T s[4];
#pragma unroll
        for (int vw = 0; vw < 4; ++vw) {
            T a = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) a += pv[vw][j];
            s[vw] = wave_sum(a);
        }
        const T h = sqrt((s[0] + s[1]) + (s[2] + s[3]));
        if (g == 0 && threadIdx.x == 0) {
            pn.hdev[0] = h;
            st_sys(pn.hring, h);
        }
        return h;
    };
    constexpr int NQ = (MAXR - 64 + 64 * W - 1) / (64 * W);   // staging iterations per thread
    constexpr bool QREG = NQ <= 8;               // the staging loads go out at once (registers)
    // branch-free: a range-checked buffer load returns ray 0 past nr (q[0] is read, not stored), so
    // the NQ ray_tab loads and then the NQ gathers each go out with one wait; their stores into the
    // LDS come after the first batches' row pointers are issued (below), so those are in flight
    // with the gathers (round 6)
    T qv[QREG ? NQ : 1];
    if constexpr (QREG) {
        const __amdgpu_buffer_rsrc_t rrt = buf_rsrc(ray_tab + pb, nr * 4);
        int rt[NQ];
#pragma unroll
        for (int u = 0; u < NQ; ++u)
            rt[u] = (int)__builtin_amdgcn_raw_buffer_load_b32(rrt, (int)(threadIdx.x + u * 64 * W) * 4, 0, 0);
#pragma unroll
        for (int u = 0; u < NQ; ++u) qv[u] = q[rt[u]];
    }
    auto stage = [&]() {
        if constexpr (QREG) {
            if (pn.np > 0) hq = pend_h();
            if (hq != T(0)) {                    // (uniform: no divisions without the pending norm)
#pragma unroll
                for (int u = 0; u < NQ; ++u) qv[u] = qv[u] / hq;
            }
#pragma unroll
            for (int u = 0; u < NQ; ++u) {
                const int k = threadIdx.x + u * 64 * W;
                if (k < nr) {
                    qloc[k] = qv[u];
#pragma unroll
                    for (int w = 0; w < W; ++w)
#pragma unroll
                        for (int h = 0; h < NA; ++h) acc[w][h][k] = TA(0);
                }
            }
        } else {
            if (pn.np > 0) hq = pend_h();
            for (int k = threadIdx.x; k < nr; k += 64 * W) {
                const T qq = q[ray_tab[pb + k]];
                qloc[k] = hq != T(0) ? qq / hq : qq;
#pragma unroll
                for (int w = 0; w < W; ++w)
#pragma unroll
                    for (int h = 0; h < NA; ++h) acc[w][h][k] = TA(0);
            }
        }
        if (threadIdx.x < 64) qloc[MAXR - 64 + threadIdx.x] = T(0);
    };
    // the epilogue coefficient: the bits the host takes from the same sum of squares
    const T ea = (GK && easq) ? (T)sqrt((double)*easq) : T(0);
    // (the barrier that publishes the staging sits after the first batches' loads are issued, below:
    // their row pointers and entries are in flight with the staging; round 6)
    TA* __restrict__ ac = &acc[wv][0][0];
    constexpr uint32_t POFF = (uint32_t)(MAXR * sizeof(TA));   // (RP) the second array, in bytes
    int u = ua, o = 0;
    auto next = [&](int& r0, int& cnt) {
        r0 = 0;
        cnt = 0;
        if (u >= ub) return;
        const int rr = __builtin_amdgcn_readlane(runv.x, u - ua), rn = __builtin_amdgcn_readlane(runv.y, u - ua);
        r0 = rr + o;
        cnt = min(G, rn - o);
        o += cnt;
        if (o == rn) {
            ++u;
            o = 0;
        }
    };
    // row pointers of a batch: lane j holds rp[r0 + min(j, cnt)] (rows past cnt are empty)
    auto load_rp = [&](int r0, int cnt) -> int64_t {
        const __amdgpu_buffer_rsrc_t r = buf_rsrc(rp + r0, (cnt + 1) * 8);
        return __builtin_bit_cast(int64_t, __builtin_amdgcn_raw_buffer_load_b64(r, min(ln, cnt) * 8, 0, 0));
    };
    constexpr int GL = 64 / G;                    // lanes per row sum after the butterfly
    struct RB {
        int r0, cnt;
        int len[G], off[G];
        T v[G][NCH][EPL];
        uint32_t s[G][NCH];
        T xv;                                     // x_true of row l / GL at lane l (side dot)
        T evv;                                    // ev of row l / GL at lane l (row epilogue)
    };
    // lane l / GL's row of the batch at the group's first lane, past every range elsewhere
    auto row_off = [&]() { return (ln & (GL - 1)) == 0 ? (ln / GL) * ES : (1 << 30); };
    auto issue = [&](RB& b, int r0, int cnt, int64_t rpv) {
        b.r0 = r0;
        b.cnt = cnt;
        {   // (no xt / ev: an empty range, no memory access)
            const __amdgpu_buffer_rsrc_t rx = buf_rsrc(xt + r0, xt ? cnt * ES : 0);
            b.xv = buf_load<T>(rx, row_off());
            if constexpr (GK) {
                const __amdgpu_buffer_rsrc_t re = buf_rsrc(ev + r0, ev ? cnt * ES : 0);
                b.evv = buf_load<T>(re, row_off());
            } else {
                b.evv = T(0);
            }
        }
        // (pairs) the batch's entries from its first row's first pair; inside a batch the row
        // pointers are 32-bit offsets from it
        const int64_t eb = readlane64(rpv, 0) & ~int64_t(1);
        const int bspan = PR ? (int)((readlane64(rpv, G) - eb + 1) & ~int64_t(1)) : 0;
        const __amdgpu_buffer_rsrc_t rv = buf_rsrc(val + eb, bspan * ES);
        const __amdgpu_buffer_rsrc_t rl = buf_rsrc(lidx + eb, bspan * 2);
        if constexpr (RP == 2) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) {
                // unit u = rows 2u, 2u+1: the first row's pairs from lane 0, the second row's from
                // lane LA at its own pair-aligned start
                const int64_t e0 = readlane64(rpv, 2 * u), e1 = readlane64(rpv, 2 * u + 1),
                              e2 = readlane64(rpv, 2 * u + 2);
                const int lenA = (int)(e1 - e0), lenB = (int)(e2 - e1);
                const int offA = (int)(e0 & 1), offB = (int)(e1 & 1);
                b.len[2 * u] = lenA;
                b.len[2 * u + 1] = lenB;
                b.off[2 * u] = offA;
                b.off[2 * u + 1] = offB;
                const int LA = (lenA + offA + 1) >> 1;
                const int relA = (int)(e0 - eb) - offA, relB = (int)(e1 - eb) - offB;
                const bool isA = ln < LA;
                const int li = isA ? ln : ln - LA;
                const bool in = 2 * li < (isA ? lenA + offA : lenB + offB);
                const int base = (isA ? relA : relB) + 2 * li;      // entry index from eb
                const int vo = in ? base * ES : (1 << 30), lo = in ? base * 2 : (1 << 30);
                if constexpr (ES == 8) {
                    const double2 t = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rv, vo, 0, HGM_RW_AUX));
                    b.v[u][0][0] = t.x;
                    b.v[u][0][EPL - 1] = t.y;
                } else {
                    const float2 t = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rv, vo, 0, HGM_RW_AUX));
                    b.v[u][0][0] = t.x;
                    b.v[u][0][EPL - 1] = t.y;
                }
                b.s[u][0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rl, lo, 0, HGM_RW_AUX);
            }
            return;
        }
        if constexpr (RP == 1 || RP >= 3) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) {
                // unit u = rows 2u, 2u+1 (a single row, or none, at the batch's end: lengths 0)
                const int64_t e0 = readlane64(rpv, 2 * u), e1 = readlane64(rpv, 2 * u + 1),
                              e2 = readlane64(rpv, 2 * u + 2);
                b.len[2 * u] = (int)(e1 - e0);
                b.len[2 * u + 1] = (int)(e2 - e1);
                const int off = (int)(e0 & 1);
                const int rel = (int)(e0 - eb) - off;
                b.off[2 * u] = off;
                const bool in = 2 * ln < (int)(e2 - e0) + off;
                const int vo = in ? 2 * ln * ES : (1 << 30), lo = in ? 2 * ln * 2 : (1 << 30);
                if constexpr (ES == 8) {
                    const double2 t = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rv, vo, rel * ES, HGM_RW_AUX));
                    b.v[u][0][0] = t.x;
                    b.v[u][0][EPL - 1] = t.y;
                } else {
                    const float2 t = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rv, vo, rel * ES, HGM_RW_AUX));
                    b.v[u][0][0] = t.x;
                    b.v[u][0][EPL - 1] = t.y;
                }
                b.s[u][0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rl, lo, rel * 2, HGM_RW_AUX);
            }
            return;
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            if constexpr (PR) {
                // one resource per batch (its rows are consecutive): a row is an SGPR offset into
                // it, and the lanes past the row's last pair get an offset past every range (no
                // memory access, zeros), instead of a resource of their own per row
                const int64_t e0 = readlane64(rpv, j), e1 = readlane64(rpv, j + 1);
                const int len = (int)(e1 - e0);
                b.len[j] = len;
                const int off = (int)(e0 & 1);
                const int rel = (int)(e0 - eb) - off;            // even: the row's first pair
                b.off[j] = off;
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
#ifndef HGM_RW_MASK_LOADS
#define HGM_RW_MASK_LOADS 1
#endif
                    const bool in = !HGM_RW_MASK_LOADS || 2 * ln + CH * c < len + off;
                    const int vo = in ? (2 * ln + CH * c) * ES : (1 << 30), lo = in ? (2 * ln + CH * c) * 2 : (1 << 30);
                    if constexpr (ES == 8) {
                        const double2 t = __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(rv, vo, rel * ES, HGM_RW_AUX));
                        b.v[j][c][0] = t.x;
                        b.v[j][c][EPL - 1] = t.y;
                    } else {
                        const float2 t = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rv, vo, rel * ES, HGM_RW_AUX));
                        b.v[j][c][0] = t.x;
                        b.v[j][c][EPL - 1] = t.y;
                    }
                    b.s[j][c] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rl, lo, rel * 2, HGM_RW_AUX);
                }
            } else {
                const int64_t e0 = readlane64(rpv, j), e1 = readlane64(rpv, j + 1);
                const int len = (int)(e1 - e0);
                b.len[j] = len;
                b.off[j] = 0;
                const __amdgpu_buffer_rsrc_t rv = buf_rsrc(val + e0, len * ES);
                const __amdgpu_buffer_rsrc_t rl = buf_rsrc(lidx + e0, len * 2);
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    if constexpr (ES == 8)
                        b.v[j][c][0] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rv, (ln + CH * c) * 8, 0, 2));
                    else
                        b.v[j][c][0] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rv, (ln + CH * c) * 4, 0, 2));
                    b.s[j][c] = (uint32_t)__builtin_bit_cast(uint16_t, __builtin_amdgcn_raw_buffer_load_b16(rl, (ln + CH * c) * 2, 0, 2));
                }
            }
        }
    };
    // Branch-free: entries outside the row (past its end; with PR also the previous row's entry
    // in the first pair) are pointed at the lane's private dummy slot (MAXR - 64 + lane, q = 0),
    // so every row issues the same instructions and the compiler can interleave the G rows'
    // product and reduction chains (a branch would end the basic block).  The accumulator
    // updates stay in row order (consecutive rows share rays).
    T zx = T(0);                                  // this lane's share of the side sum, batches in order
    const bool first_lane = (ln & (GL - 1)) == 0;
    (void)first_lane;
    auto process = [&](RB& b) {
        T P[G];
        uint32_t k[G][NCH][EPL];
        bool ia[RP ? G / 2 : 1][EPL];             // (RP) entry of its unit's first row
        bool la_[RP == 2 ? G / 2 : 1];            // (RP 2) lane of its unit's first row
        uint32_t kb[RP >= 3 ? G / 2 : 1][EPL];    // (RP 3, 4) the second row's accumulator address
        if constexpr (RP == 2) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) {
                const int offA = b.off[2 * u], offB = b.off[2 * u + 1];
                const int LA = (b.len[2 * u] + offA + 1) >> 1;     // lanes of the first row
                const bool isA = ln < LA;
                la_[u] = isA;
                const int pos0 = isA ? 2 * ln - offA : 2 * (ln - LA) - offB;
                const int len = isA ? b.len[2 * u] : b.len[2 * u + 1];
                const uint32_t aoff = isA ? 0u : POFF;
                T p = T(0);
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const bool ok = (uint32_t)(pos0 + e) < (uint32_t)len;
                    const uint32_t sl = e ? b.s[u][0] >> 16 : b.s[u][0] & 0xffffu;
                    const uint32_t dm = (uint32_t)(MAXR - 64 + ln) * (uint32_t)ES;
                    const uint32_t kq = ok ? sl : dm;
                    p += b.v[u][0][e] * *reinterpret_cast<const T*>(reinterpret_cast<const char*>(qloc) + kq);
                    k[u][0][e] = ok ? sl * AS + aoff : dm * AS;
                }
                P[2 * u] = isA ? p : T(0);
                P[2 * u + 1] = isA ? T(0) : p;
            }
        } else if constexpr (RP == 1 || RP >= 3) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) {
                const int la = b.len[2 * u], lab = la + b.len[2 * u + 1];
                T pa = T(0), pb = T(0);
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const int pos = EPL * ln - b.off[2 * u] + e;
                    const bool inA = (uint32_t)pos < (uint32_t)la;
                    const bool in = (uint32_t)pos < (uint32_t)lab;
                    const uint32_t sl = e ? b.s[u][0] >> 16 : b.s[u][0] & 0xffffu;
                    const uint32_t dm = (uint32_t)(MAXR - 64 + ln) * (uint32_t)ES;
                    if constexpr (RP == 4) {
                        // RP 4 = RP 3 with the q reads through the two accumulator addresses (q = 0
                        // at the dummies): the row split costs a second q read instead of the selects
                        // of the products (AS == 1: the q and accumulator offsets coincide)
                        const uint32_t ka = inA ? sl : dm, kk = (in && !inA) ? sl : dm;
                        const T qa = *reinterpret_cast<const T*>(reinterpret_cast<const char*>(qloc) + ka);
                        const T qb = *reinterpret_cast<const T*>(reinterpret_cast<const char*>(qloc) + kk);
                        if constexpr (HGM_FUSED_FMA) {   // (one rounding per term: half the VALU)
                            pa = fma_t(b.v[u][0][e], qa, pa);
                            pb = fma_t(b.v[u][0][e], qb, pb);
                        } else {
                            pa = pa + b.v[u][0][e] * qa;
                            pb = pb + b.v[u][0][e] * qb;
                        }
                        k[u][0][e] = ka * AS;              // (AS == 2: fp64 accumulators of an fp32 pass)
                        kb[u][e] = kk * AS;
                        ia[u][e] = inA;
                        continue;
                    }
                    const uint32_t kq = in ? sl : dm;
                    const T p = b.v[u][0][e] * *reinterpret_cast<const T*>(reinterpret_cast<const char*>(qloc) + kq);
                    pa = pa + (inA ? p : T(0));
                    pb = pb + (inA ? T(0) : p);
                    // the accumulator: array 0 for the unit's first row, 1 for its second, the dummy
                    // (RP 3: one array, the two rows' adds in two instructions, each other lane on
                    // its dummy)
                    if constexpr (RP == 3) {
                        k[u][0][e] = inA ? sl * AS : dm * AS;
                        kb[u][e] = (in && !inA) ? sl * AS : dm * AS;
                    } else {
                        k[u][0][e] = in ? sl * AS + (inA ? 0u : POFF) : dm * AS;
                    }
                    ia[u][e] = inA;
                }
                P[2 * u] = pa;
                P[2 * u + 1] = pb;
            }
        }
#pragma unroll
        for (int j = 0; j < G && !RP; ++j) {
            T p = T(0);
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    // slots are LDS byte offsets (the plan stores slot * sizeof(T)); pos0 is the lane's
                    // first entry in the row (-1: the previous row's last entry in the first pair)
                    const int pos0 = EPL * ln + CH * c - b.off[j];
                    const bool ok = e == 0 ? (uint32_t)pos0 < (uint32_t)b.len[j] : pos0 < b.len[j] - 1;
                    const uint32_t sl = PR ? (e ? b.s[j][c] >> 16 : b.s[j][c] & 0xffffu) : b.s[j][c];
                    k[j][c][e] = ok ? sl : (uint32_t)(MAXR - 64 + ln) * (uint32_t)ES;
                    if constexpr (DBG & 1) p += b.v[j][c][e] * (T)k[j][c][e];
                    else p += b.v[j][c][e] * *reinterpret_cast<const T*>(reinterpret_cast<const char*>(qloc) + k[j][c][e]);
                }
            P[j] = p;
        }
        T S;                                      // lane l: z of row l / GL
        if constexpr (DBG & 4) S = P[0] + P[G - 1];
        else S = rows_sum_t<G>(P);
        T zs = S;
        if constexpr (GK) {
            const T sa = ea * b.evv;              // row epilogue: zs = z - a*ev (two roundings)
            zs = S - sa;
        }
        {   // z out: each group's first lane, rows past cnt fall outside the range
            const __amdgpu_buffer_rsrc_t rz = buf_rsrc(zraw + b.r0, zraw ? b.cnt * ES : 0);
            buf_store(S, rz, row_off());
            if constexpr (GK) {
                const __amdgpu_buffer_rsrc_t ro = buf_rsrc(zout + b.r0, zout ? b.cnt * ES : 0);
                buf_store(zs, ro, row_off());
            }
        }
        // side: zs * x_true (other lanes: xv = 0), or zs^2 at the first lanes (rows past cnt: zs = 0)
        if constexpr (GK) {
            const T f = side_sq ? (first_lane ? zs : T(0)) : b.xv;
            zx = zx + zs * f;
        } else {
            zx = zx + zs * b.xv;
        }
        if constexpr (RP >= 3) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) {
                const T za = lane_bcast(zs, 2 * u * GL), zb = lane_bcast(zs, (2 * u + 1) * GL);
#pragma unroll
                for (int h = 0; h < 2; ++h) {         // the unit's first row, then its second
                    if constexpr (AM == 1 && EPL == 2) {
                        // read-add-write of the row's two entries per lane with ONE round trip: both
                        // reads, then both writes. Within one pixel row the slots are distinct, so
                        // only a lane whose two entries both sit on its dummy slot reads it twice
                        // (the dummy's value is never used): the same sums as one entry at a time.
                        const T sj = h ? zb : za;
                        TA* p0 = reinterpret_cast<TA*>(reinterpret_cast<char*>(ac) + (h ? kb[u][0] : k[u][0][0]));
                        TA* p1 = reinterpret_cast<TA*>(reinterpret_cast<char*>(ac) + (h ? kb[u][1] : k[u][0][1]));
                        const T o0 = *p0, o1 = *p1;
                        if constexpr (HGM_FUSED_FMA && RP == 4) {
                            *p0 = fma_t(b.v[u][0][0], sj, o0);
                            *p1 = fma_t(b.v[u][0][1], sj, o1);
                        } else {
                            const T t0 = b.v[u][0][0] * sj, t1 = b.v[u][0][1] * sj;
                            *p0 = o0 + t0;
                            *p1 = o1 + t1;
                        }
                        continue;
                    }
#pragma unroll
                    for (int e = 0; e < EPL; ++e) {
                        const T sj = h ? zb : za;
                        TA* pa = reinterpret_cast<TA*>(reinterpret_cast<char*>(ac) + (h ? kb[u][e] : k[u][0][e]));
                        if constexpr (AM == 2) {
                            lds_add(pa, (double)b.v[u][0][e] * (double)sj);
                        } else if constexpr (AM == 1) {
                            const T t = b.v[u][0][e] * sj;
                            *pa = *pa + t;
                        } else {
                            lds_add(pa, b.v[u][0][e] * sj);
                        }
                    }
                }
            }
        } else if constexpr (RP) {
#pragma unroll
            for (int u = 0; u < G / 2; ++u) {
                const T za = lane_bcast(zs, 2 * u * GL), zb = lane_bcast(zs, (2 * u + 1) * GL);
                const T s2 = RP == 2 ? (la_[u] ? za : zb) : T(0);
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    const T sj = RP == 2 ? s2 : (ia[u][e] ? za : zb);
                    TA* pa = reinterpret_cast<TA*>(reinterpret_cast<char*>(ac) + k[u][0][e]);
                    if constexpr (AM == 2) {
                        lds_add(pa, (double)b.v[u][0][e] * (double)sj);
                    } else if constexpr (AM == 1) {
                        const T t = b.v[u][0][e] * sj;
                        *pa = *pa + t;
                    } else {
                        lds_add(pa, b.v[u][0][e] * sj);
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < G && !RP; ++j) {
            const T sj = lane_bcast(zs, j * GL);
#pragma unroll
            for (int c = 0; c < NCH; ++c)
#pragma unroll
                for (int e = 0; e < EPL; ++e) {
                    TA* pa = reinterpret_cast<TA*>(reinterpret_cast<char*>(ac) + k[j][c][e] * AS);
                    if constexpr (DBG & 2) {
                        S += b.v[j][c][e] * sj;
                    } else if constexpr (AM == 2) {
                        lds_add(pa, (double)b.v[j][c][e] * (double)sj);
                    } else if constexpr (AM == 1) {
                        const T t = b.v[j][c][e] * sj;
                        *pa = *pa + t;
                    } else {
                        lds_add(pa, b.v[j][c][e] * sj);
                    }
                }
        }
    };
    // Ring of D batches: while batch i is processed, batches i+1 .. i+D-1 are in flight and the
    // row pointers of batch i+D load.  The loop is unrolled by D so every ring index is static
    // (registers; a register copy of an in-flight load would force a wait), with one exit at the
    // bottom (a rotated loop with two exits had the compiler copy in-flight batches); an empty
    // batch is processed as a no-op (zero-length ranges, dummy slots).  sched_barrier: the
    // scheduler would sink the next batch's loads into the processing.
    RB b[D];
    int a[D], cn[D];
    int64_t r[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        next(a[i], cn[i]);
        r[i] = load_rp(a[i], cn[i]);
    }
    stage();                                      // (the gathers' waits leave the row pointers in flight)
#pragma unroll
    for (int i = 0; i < D - 1; ++i) issue(b[i], a[i], cn[i], r[i]);
    __syncthreads();                              // the staged q and the zeroed accumulators
    do {
#pragma unroll
        for (int t = 0; t < D; ++t) {
            // the row pointers of batch i+D first: issuing batch i+D-1 then waits only for its
            // own row pointers (loaded before batch i+D-2's entries), not for the entries
            const int ti = (t + D - 1) % D;
            next(a[t], cn[t]);
            r[t] = load_rp(a[t], cn[t]);
            issue(b[ti], a[ti], cn[ti], r[ti]);
            __builtin_amdgcn_sched_barrier(0);
            process(b[t]);
            __builtin_amdgcn_sched_barrier(0);
        }
    } while (b[0].cnt > 0);
    if (zx_part) zx = wave_sum(zx);
    __syncthreads();
    // (the waves' side sums go through qloc, free once every wave has left the loop: an
    // array of their own would push the workgroup past half the LDS, one workgroup per CU)
    if (zx_part && ln == 0) qloc[wv] = zx;
    for (int k = threadIdx.x; k < nr; k += 64 * W) {
        TA t = acc[0][0][k];
        if constexpr (NA == 2) t += acc[0][1][k];
#pragma unroll
        for (int w = 1; w < W; ++w) {
            t += acc[w][0][k];
            if constexpr (NA == 2) t += acc[w][1][k];
        }
        if constexpr (HGM_PART_NT) __builtin_nontemporal_store(t, &part[pb + k]);
        else part[pb + k] = t;
    }
    if (zx_part) {
        __syncthreads();
        if (threadIdx.x == 0) {                   // waves in order
            T t = qloc[0];
#pragma unroll
            for (int w = 1; w < W; ++w) t += qloc[w];
            zx_part[g] = t;
        }
    }
}

// ------------------------------------------------------------------------------------------
// plan (host, from B's CSR structure; once per operator)
// ------------------------------------------------------------------------------------------
namespace {
template <typename F>
void parallel_for(int64_t n, F f) {
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt, 16u));
    if (n < 64 || nt == 1) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> th;
    const int64_t step = (n + nt - 1) / nt;
    for (unsigned t = 0; t < nt; ++t) {
        const int64_t a = t * step, b = std::min<int64_t>(n, a + step);
        if (a >= b) break;
        th.emplace_back([=, &f]() {
            for (int64_t i = a; i < b; ++i) f(i);
        });
    }
    for (auto& t : th) t.join();
}

template <typename T>
T* upload(const std::vector<T>& v) {
    T* d = nullptr;
    const size_t bytes = std::max<size_t>(v.size(), 1) * sizeof(T);
    if (hipMalloc(&d, bytes) != hipSuccess) throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
    if (!v.empty()) HGM_HIP(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return d;
}
}  // namespace

// The pixel grid of B's rows: the whole tiled N x N grid (row_order), or a pixel shard of whole
// tile columns of one (row_grid: hgm_mat_row_slice, the multi-GPU path), whose stored positions
// are then shard-local.  Returns the grid (trivial when neither).
static PixOrder fused_grid(const hgm_mat* B) {
    const PixOrder& o = B->row_order;
    if (!o.trivial()) return (int64_t)o.N * o.N == B->rows ? o : PixOrder{};
    const PixOrder& g = B->row_grid;
    if (g.trivial() || g.super > 1 || B->rows % ((int64_t)std::max(g.tile, 1) * g.N) != 0) return PixOrder{};
    return g;
}

// Region (R x R pixel square) of every row of B (rows = pixels in B's stored order; for a shard
// the square grid is laid over the shard's N x W window of pixel columns).
static std::vector<int32_t> row_regions(const hgm_mat* B, int R, int64_t* nreg) {
    const PixOrder o = fused_grid(B);
    HGM_REQUIRE(!o.trivial() && o.N > 0, "fused A*(B*q): B's rows must be the pixels of a tiled N x N grid or a shard of it");
    const int N = o.N;
    const int64_t W = B->rows / N;                     // pixel columns (N for the whole grid)
    const int64_t nbr = (N + R - 1) / R, nbc = (W + R - 1) / R;
    *nreg = nbr * nbc;
    std::vector<int32_t> reg(B->rows);
    if (!B->row_order.trivial()) {
        const std::vector<int64_t> ref = pix_reference_of_stored(o);
        for (int64_t s = 0; s < B->rows; ++s) {
            const int64_t r = ref[s] % N, c = ref[s] / N;
            reg[s] = (int32_t)((c / R) * nbr + r / R);
        }
    } else {
        // shard: whole tile columns, tile x tile tiles in tile-column-major order, column-major
        // inside a tile (ops.hip pixel_rc without super-blocks), from the shard's first column
        const int64_t t = std::max(o.tile, 1), tpc = N / t;
        for (int64_t s = 0; s < B->rows; ++s) {
            const int64_t tl = s / (t * t), w = s % (t * t);
            const int64_t r = (tl % tpc) * t + w % t, c = (tl / tpc) * t + w / t;
            reg[s] = (int32_t)((c / R) * nbr + r / R);
        }
    }
    return reg;
}

FusedPlan* fused_plan_build(hgm_ctx* c, const hgm_mat* B, int R) {
    HGM_REQUIRE(B->dtype == HGM_F64, "fused A*(B*q): fp64 operators");
    HGM_REQUIRE(B->cols < (int64_t(1) << 31) && B->rows < (int64_t(1) << 31), "fused A*(B*q): index range");
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t n = B->rows, m = B->cols, nnz = B->nnz;
    int64_t nreg = 0;
    const std::vector<int32_t> reg = row_regions(B, R, &nreg);
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> ci(std::max<int64_t>(nnz, 1));
    HGM_HIP(hipMemcpy(rp.data(), B->rp, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost));
    if (nnz) HGM_HIP(hipMemcpy(ci.data(), B->ci, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
    // sub-chunks: runs of rows of one region, cut at FCH entries / FROWS rows
    struct Sub { int64_t e0; int32_t r0, reg; int len, nrow; };
    std::vector<Sub> sv;
    for (int64_t s = 0; s < n;) {
        Sub u{rp[s], (int32_t)s, reg[s], 0, 0};
        // (an odd first entry costs one coordinate: see FusedSub)
        while (s < n && reg[s] == u.reg && u.nrow < FROWS && u.len + (rp[s + 1] - rp[s]) <= FCH - (u.e0 & 1)) {
            u.len += (int)(rp[s + 1] - rp[s]);
            ++u.nrow;
            ++s;
        }
        HGM_REQUIRE(u.nrow > 0, "fused A*(B*q): a row longer than the sub-chunk");
        sv.push_back(u);
    }
    // sub-chunks crossed by more than FLRMAX distinct rays (many angles) are halved by rows until
    // none is (a sub-chunk keeps whole rows, so a single row always fits: <= FCH entries)
    auto distinct_rays = [&](const Sub& u) {
        std::vector<int32_t> r(ci.begin() + u.e0, ci.begin() + u.e0 + u.len);
        std::sort(r.begin(), r.end());
        return (int)(std::unique(r.begin(), r.end()) - r.begin());
    };
    for (bool again = true; again;) {
        std::vector<char> big(sv.size(), 0);
        parallel_for((int64_t)sv.size(), [&](int64_t i) { big[i] = distinct_rays(sv[i]) > FLRMAX; });
        again = false;
        std::vector<Sub> nv;
        for (size_t i = 0; i < sv.size(); ++i) {
            if (!big[i] || sv[i].nrow < 2) {
                HGM_REQUIRE(!big[i], "fused A*(B*q): a pixel row is crossed by too many rays");
                nv.push_back(sv[i]);
                continue;
            }
            again = true;
            const Sub& u = sv[i];
            const int h = u.nrow / 2;
            const int l0 = (int)(rp[u.r0 + h] - u.e0);
            nv.push_back(Sub{u.e0, u.r0, u.reg, l0, h});
            nv.push_back(Sub{u.e0 + l0, u.r0 + h, u.reg, u.len - l0, u.nrow - h});
        }
        sv.swap(nv);
    }
    // plan order: by region, storage order inside a region
    std::stable_sort(sv.begin(), sv.end(), [](const Sub& a, const Sub& b) { return a.reg < b.reg; });
    const int64_t nsub = (int64_t)sv.size();
    std::vector<int32_t> reg_sub(nreg + 1, 0);
    for (const Sub& u : sv) reg_sub[u.reg + 1]++;
    for (int64_t g = 0; g < nreg; ++g) reg_sub[g + 1] += reg_sub[g];
    // local CSC of every sub-chunk: perm (entry coordinates in ray order, each sub-chunk's run
    // padded to 4 entries), distinct rays and their starts
    std::vector<int64_t> pbase(nsub + 1, 0);
    for (int64_t i = 0; i < nsub; ++i) pbase[i + 1] = pbase[i] + ((sv[i].len + 3) & ~3);
    HGM_REQUIRE(pbase[nsub] / 4 < (int64_t(1) << 32), "fused A*(B*q): perm index range");
    std::vector<uint16_t> perm(std::max<int64_t>(pbase[nsub], 1), 0);
    std::vector<std::vector<int32_t>> lray(nsub);
    std::vector<std::vector<uint16_t>> lpos(nsub);
    parallel_for(nsub, [&](int64_t i) {
        const Sub& u = sv[i];
        std::vector<uint64_t> key(u.len);
        for (int k = 0; k < u.len; ++k) key[k] = ((uint64_t)(uint32_t)ci[u.e0 + k] << 16) | (uint64_t)k;
        std::sort(key.begin(), key.end());
        auto& lr = lray[i];
        auto& lp = lpos[i];
        for (int k = 0; k < u.len; ++k) {
            const int32_t ray = (int32_t)(key[k] >> 16);
            perm[pbase[i] + k] = (uint16_t)((key[k] & 0xffffu) + (u.e0 & 1));
            if (k == 0 || ray != lr.back()) {
                lr.push_back(ray);
                lp.push_back((uint16_t)k);
            }
        }
    });
    for (int64_t i = 0; i < nsub; ++i)
        HGM_REQUIRE((int)lray[i].size() <= FLRMAX, "fused A*(B*q): a sub-chunk is crossed by too many rays");
    // region ray sets (sorted), their sizes and each local ray's index in its region's set
    std::vector<std::vector<int32_t>> rrays(nreg);
    std::vector<std::vector<uint16_t>> lrr(nsub);
    bool too_many = false;
    parallel_for(nreg, [&](int64_t g) {
        auto& rs = rrays[g];
        for (int32_t i = reg_sub[g]; i < reg_sub[g + 1]; ++i) rs.insert(rs.end(), lray[i].begin(), lray[i].end());
        std::sort(rs.begin(), rs.end());
        rs.erase(std::unique(rs.begin(), rs.end()), rs.end());
        if ((int)rs.size() > FRMAX) {
            too_many = true;
            return;
        }
        for (int32_t i = reg_sub[g]; i < reg_sub[g + 1]; ++i) {
            auto& out = lrr[i];
            out.resize(lray[i].size());
            for (size_t k = 0; k < lray[i].size(); ++k)
                out[k] = (uint16_t)(std::lower_bound(rs.begin(), rs.end(), lray[i][k]) - rs.begin());
        }
    });
    HGM_REQUIRE(!too_many, "fused A*(B*q): a region is crossed by more rays than the LDS holds");
    // flat device arrays
    std::vector<FusedSub> subs(nsub);
    int64_t nlr = 0;
    for (int64_t i = 0; i < nsub; ++i) {
        HGM_REQUIRE(lray[i].size() <= 0xffff, "fused A*(B*q): local rays");
        subs[i] = FusedSub{sv[i].e0, nlr, sv[i].r0, (uint32_t)(pbase[i] / 4), (uint16_t)sv[i].len,
                           (uint16_t)sv[i].nrow, (uint16_t)lray[i].size(), 0};
        nlr += (int64_t)lray[i].size();
    }
    // records: first position (12 bits) | entries (8) | region ray index (12); longest first, so
    // the lanes of a wave walk rays of about the same length (ties: position order)
    std::vector<int32_t> lr_ray(nlr);
    std::vector<uint32_t> lr_pk(nlr);
    bool rec_ok = true;
    parallel_for(nsub, [&](int64_t i) {
        const size_t nl = lray[i].size();
        std::vector<int> ord(nl), lenv(nl);
        for (size_t k = 0; k < nl; ++k) {
            ord[k] = (int)k;
            lenv[k] = (k + 1 < nl ? (int)lpos[i][k + 1] : sv[i].len) - (int)lpos[i][k];
            if (lenv[k] > 0xff || lrr[i][k] > 0xfff) rec_ok = false;
        }
        std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return lenv[a] > lenv[b]; });
        for (size_t k = 0; k < nl; ++k) {
            const int o = ord[k];
            lr_ray[subs[i].lr0 + k] = lray[i][o];
            lr_pk[subs[i].lr0 + k] = (uint32_t)lpos[i][o] | ((uint32_t)lenv[o] << 12) | ((uint32_t)lrr[i][o] << 20);
        }
    });
    HGM_REQUIRE(rec_ok, "fused A*(B*q): a ray's share of a sub-chunk or a region's ray count exceeds the record");
    std::vector<int64_t> reg_base(nreg + 1, 0);
    for (int64_t g = 0; g < nreg; ++g) reg_base[g + 1] = reg_base[g] + (int64_t)rrays[g].size();
    const int64_t nslot = reg_base[nreg];
    HGM_REQUIRE(nslot < (int64_t(1) << 31), "fused A*(B*q): partial slots");
    // ray-major reduction index: ray i's slots in region order
    std::vector<int64_t> rs_ptr(m + 1, 0);
    for (int64_t g = 0; g < nreg; ++g)
        for (int32_t ray : rrays[g]) rs_ptr[ray + 1]++;
    for (int64_t i = 0; i < m; ++i) rs_ptr[i + 1] += rs_ptr[i];
    std::vector<int32_t> rs_slot(std::max<int64_t>(nslot, 1));
    {
        std::vector<int64_t> fill(rs_ptr.begin(), rs_ptr.end() - 1);
        for (int64_t g = 0; g < nreg; ++g)
            for (size_t r = 0; r < rrays[g].size(); ++r) rs_slot[fill[rrays[g][r]]++] = (int32_t)(reg_base[g] + r);
    }
    FusedPlan* P = new FusedPlan;
    try {
        P->region = R;
        P->nreg = nreg;
        P->nsub = nsub;
        P->nlr = nlr;
        P->nslot = nslot;
        P->m = m;
        P->reg_sub = upload(reg_sub);
        P->reg_base = upload(reg_base);
        P->subs = upload(subs);
        P->perm = upload(perm);
        P->lr_ray = upload(lr_ray);
        P->lr_pk = upload(lr_pk);
        P->rs_ptr = upload(rs_ptr);
        P->rs_slot = upload(rs_slot);
        if (hipMalloc(&P->part, sizeof(double) * std::max<int64_t>(nslot, 1)) != hipSuccess)
            throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
    } catch (...) {
        fused_plan_free(P);
        throw;
    }
    (void)c;
    P->build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return P;
}

// The row-wave plan (kind 1): regions of R x R pixels, W waves per region.  Each wave gets a
// contiguous share (by entries) of the region's rows in stored order, as runs of consecutive
// rows; each entry gets its ray's index among the region's rays (sorted ray ids).
namespace {
// (waves, LDS ray slots) of the instantiated kernels, 64 slots of each being the lanes' dummies;
// the plan takes the fewest slots that hold its regions' rays (more workgroups per CU)
#if HGM_EXPERIMENTS
#define HGM_RW_SHAPES(X) X(1, 1088) X(1, 2048) X(1, 4096) X(2, 1088) X(2, 1536) X(2, 2048) X(2, 4096) \
    X(4, 1088) X(4, 1344) X(4, 1536) X(4, 2048)
#else
#define HGM_RW_SHAPES(X) X(4, 1088) X(4, 1344) X(4, 1536) X(4, 2048)
#endif
constexpr int RW_SLOTS_MAX = 4096;
constexpr int RW_ROW_MAX = 255;                   // entries per pixel row (two chunks of 128, pairs)
}  // namespace

template <typename T, bool GK>
static bool fused_rw_launch(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P, const FusedArgs<T>& fa, bool dry);

// ------------------------------------------------------------------------------------------
// Device build of the row-wave plan's ray sets (HGM_OPT_FUSED_PLAN_DEV).  Per
// region, one workgroup marks the rays of the region's entries in an LDS bitmap over the ray
// space (atomic OR: order-free, so the set is the same whatever the schedule); a ray's slot is its
// rank among the set bits.  That is exactly the host build's sorted-unique ray list and
// map[ray] = index, so the plan's bytes are identical (tested).  The bitmap (and, in the fill
// pass, its per-word prefix counts) sit in dynamic LDS: ceil(m / 32) words each, so rays up to
// PLAN_DEV_MAX_M (C4: 272,271 rays, 68 KB).
// ------------------------------------------------------------------------------------------
namespace {
constexpr int PLAN_BS = 1024;
constexpr int64_t PLAN_DEV_MAX_M = int64_t(19) * 1024 * 32;   // 2 x 19 Ki words = 152 KB of LDS

// the region's entries (all its waves' runs), mark their rays in bm
__device__ __forceinline__ void plan_mark(uint32_t* bm, int nwords, const int32_t* __restrict__ wrun,
                                          const int2* __restrict__ runs, int W, const int64_t* __restrict__ rp,
                                          const int32_t* __restrict__ ci) {
    const int g = blockIdx.x;
    for (int i = threadIdx.x; i < nwords; i += PLAN_BS) bm[i] = 0u;
    __syncthreads();
    for (int u = wrun[g * W]; u < wrun[g * W + W]; ++u) {
        const int2 r = runs[u];
        const int64_t e1 = rp[r.x + r.y];
        for (int64_t e = rp[r.x] + threadIdx.x; e < e1; e += PLAN_BS) {
            const int32_t ray = ci[e];
            atomicOr(&bm[ray >> 5], 1u << (ray & 31));
        }
    }
    __syncthreads();
}

// exclusive prefix of v over the workgroup (fixed order), and the total
__device__ __forceinline__ int block_exscan(int v, int* sh, int* total) {
    const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (ln >= d) x += y;
    }
    if (ln == 63) sh[wv] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int a = 0;
        for (int w = 0; w < PLAN_BS / 64; ++w) {
            const int t = sh[w];
            sh[w] = a;
            a += t;
        }
        sh[PLAN_BS / 64] = a;
    }
    __syncthreads();
    *total = sh[PLAN_BS / 64];
    return sh[wv] + x - v;
}

__global__ __launch_bounds__(PLAN_BS) void k_plan_count(const int32_t* __restrict__ wrun, const int2* __restrict__ runs,
                                                        int W, const int64_t* __restrict__ rp,
                                                        const int32_t* __restrict__ ci, int nwords,
                                                        int32_t* __restrict__ cnt) {
    extern __shared__ uint32_t plan_lds[];
    __shared__ int sh[PLAN_BS / 64 + 1];
    plan_mark(plan_lds, nwords, wrun, runs, W, rp, ci);
    int c = 0;
    for (int i = threadIdx.x; i < nwords; i += PLAN_BS) c += __popc(plan_lds[i]);
    int tot = 0;
    (void)block_exscan(c, sh, &tot);
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// ray_tab[reg_base[g] + rank] = ray (ascending), lidx[e] = rank(ci[e]) * es
__global__ __launch_bounds__(PLAN_BS) void k_plan_fill(const int32_t* __restrict__ wrun, const int2* __restrict__ runs,
                                                       int W, const int64_t* __restrict__ rp,
                                                       const int32_t* __restrict__ ci, int nwords,
                                                       const int64_t* __restrict__ reg_base,
                                                       int32_t* __restrict__ ray_tab, uint16_t* __restrict__ lidx,
                                                       int es) {
    extern __shared__ uint32_t plan_lds[];
    __shared__ int sh[PLAN_BS / 64 + 1];
    uint32_t* bm = plan_lds;
    uint32_t* pre = plan_lds + nwords;
    plan_mark(bm, nwords, wrun, runs, W, rp, ci);
    // words in contiguous per-thread chunks, so the exclusive scan of the chunk counts orders them
    const int cw = (nwords + PLAN_BS - 1) / PLAN_BS;
    const int w0 = min(nwords, (int)threadIdx.x * cw), w1 = min(nwords, w0 + cw);
    int c = 0;
    for (int i = w0; i < w1; ++i) c += __popc(bm[i]);
    int tot = 0;
    int a = block_exscan(c, sh, &tot);
    int32_t* rt = ray_tab + reg_base[blockIdx.x];
    for (int i = w0; i < w1; ++i) {
        pre[i] = (uint32_t)a;
        uint32_t b = bm[i];
        while (b) {
            const int k = __ffs(b) - 1;
            rt[a++] = i * 32 + k;
            b &= b - 1;
        }
    }
    __syncthreads();
    const int g = blockIdx.x;
    for (int u = wrun[g * W]; u < wrun[g * W + W]; ++u) {
        const int2 r = runs[u];
        const int64_t e1 = rp[r.x + r.y];
        for (int64_t e = rp[r.x] + threadIdx.x; e < e1; e += PLAN_BS) {
            const int32_t ray = ci[e];
            const uint32_t wd = bm[ray >> 5];
            const int rank = (int)pre[ray >> 5] + __popc(wd & ((1u << (ray & 31)) - 1u));
            lidx[e] = (uint16_t)(rank * es);
        }
    }
}
}  // namespace

// The band runs of k_fused_reduce_band from the plan's region ray lists (regions in order).
static void plan_bands(FusedPlan* P, const std::vector<int32_t>& ray_tab, const std::vector<int64_t>& reg_base) {
    const int64_t m = P->m, nreg = P->nreg, nband = (m + 63) / 64;
    std::vector<int32_t> cnt(nband + 1, 0);
    auto runs_of = [&](auto emit) {
        for (int64_t g = 0; g < nreg; ++g) {
            for (int64_t k = reg_base[g], k1 = reg_base[g + 1]; k < k1;) {
                const int32_t ray = ray_tab[k];
                const int64_t b = ray / 64;
                int64_t e = k + 1;
                while (e < k1 && ray_tab[e] == ray + (int32_t)(e - k) && ray_tab[e] / 64 == b) ++e;
                emit(b, make_int4((int)k, (int)(ray - b * 64), (int)(e - k), 0));
                k = e;
            }
        }
    };
    runs_of([&](int64_t b, int4) { cnt[b + 1]++; });
    for (int64_t b = 0; b < nband; ++b) cnt[b + 1] += cnt[b];
    std::vector<int4> run(std::max<int32_t>(cnt[nband], 1));
    std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
    runs_of([&](int64_t b, int4 r) { run[fill[b]++] = r; });
    P->nband = nband;
    P->nrun = cnt[nband];
    P->band_ptr = upload(cnt);
    P->band_run = upload(run);
}

// The one refusal a smaller region can cure (fused_ab_plan retries it with half the side); every
// other refusal of a plan (option shapes without a kernel, index ranges) goes straight to the
// two-pass path.
static const char* const kLdsCapacityMsg =
    "fused A*(B*q): a region is crossed by more rays than the LDS of its waves holds";

// The device part of the row-wave plan: ray sets, slots (lidx) and ray_tab by k_plan_count /
// k_plan_fill, then the ray-major reduction index by a counting sort of ray_tab on the host
// (slots in increasing order = regions in order, as the host build).
static FusedPlan* fused_plan_dev_finish(hgm_ctx* c, const hgm_mat* B, int R, int W, int G, int rowpair, int es, int64_t nreg,
                                        int64_t maxlen, const std::vector<int32_t>& wrun,
                                        const std::vector<int2>& runs,
                                        std::chrono::steady_clock::time_point t0) {
    const int64_t m = B->cols, nnz = B->nnz;
    const int nwords = (int)((m + 31) / 32);
    FusedPlan* P = new FusedPlan;
    int32_t* cnt_d = nullptr;
    try {
        P->kind = 1;
        P->elem = es;
        P->region = R;
        P->waves = W;
        P->group = G;
        P->depth = c->num.fused_depth;
        P->pairs = c->num.fused_pairs;
        P->rowpair = rowpair;
        P->maxlen = maxlen;
        P->nreg = nreg;
        P->m = m;
        P->wrun = upload(wrun);
        P->runs = upload(runs);
        if (hipMalloc(&cnt_d, sizeof(int32_t) * std::max<int64_t>(nreg, 1)) != hipSuccess)
            throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
        hipLaunchKernelGGL(k_plan_count, dim3((unsigned)nreg), dim3(PLAN_BS), sizeof(uint32_t) * nwords, c->stream,
                           (const int32_t*)P->wrun, (const int2*)P->runs, W, (const int64_t*)B->rp,
                           (const int32_t*)B->ci, nwords, cnt_d);
        HGM_HIP(hipGetLastError());
        std::vector<int32_t> cnt(nreg);
        HGM_HIP(hipMemcpyAsync(cnt.data(), cnt_d, sizeof(int32_t) * nreg, hipMemcpyDeviceToHost, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
        int worst = 0;
        for (int32_t v : cnt) worst = std::max(worst, (int)v);
        int maxr = 0;
#define HGM_RW_PICK(WV, MRV) \
    if (W == WV && worst <= MRV - 64 && (maxr == 0 || MRV < maxr)) maxr = MRV;
        HGM_RW_SHAPES(HGM_RW_PICK)
#undef HGM_RW_PICK
        HGM_REQUIRE(maxr > 0, kLdsCapacityMsg);
        P->maxr = maxr;
        std::vector<int64_t> reg_base(nreg + 1, 0);
        for (int64_t g = 0; g < nreg; ++g) reg_base[g + 1] = reg_base[g] + cnt[g];
        const int64_t nslot = reg_base[nreg];
        HGM_REQUIRE(nslot < (int64_t(1) << 31), "fused A*(B*q): partial slots");
        P->nslot = nslot;
        P->reg_base = upload(reg_base);
        if (hipMalloc(&P->ray_tab, sizeof(int32_t) * std::max<int64_t>(nslot, 1)) != hipSuccess ||
            hipMalloc(&P->lidx, sizeof(uint16_t) * (nnz + 256)) != hipSuccess)
            throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
        HGM_HIP(hipMemsetAsync(P->lidx + nnz, 0, sizeof(uint16_t) * 256, c->stream));   // (the padding)
        hipLaunchKernelGGL(k_plan_fill, dim3((unsigned)nreg), dim3(PLAN_BS), 2 * sizeof(uint32_t) * nwords, c->stream,
                           (const int32_t*)P->wrun, (const int2*)P->runs, W, (const int64_t*)B->rp,
                           (const int32_t*)B->ci, nwords, (const int64_t*)P->reg_base, P->ray_tab, P->lidx, es);
        HGM_HIP(hipGetLastError());
        std::vector<int32_t> ray_tab(std::max<int64_t>(nslot, 1));
        HGM_HIP(hipMemcpyAsync(ray_tab.data(), P->ray_tab, sizeof(int32_t) * nslot, hipMemcpyDeviceToHost, c->stream));
        HGM_HIP(hipStreamSynchronize(c->stream));
        // ray-major reduction index: ray i's slots in region order (= increasing slot)
        std::vector<int64_t> rs_ptr(m + 1, 0);
        for (int64_t k = 0; k < nslot; ++k) rs_ptr[ray_tab[k] + 1]++;
        for (int64_t i = 0; i < m; ++i) rs_ptr[i + 1] += rs_ptr[i];
        std::vector<int32_t> rs_slot(std::max<int64_t>(nslot, 1));
        {
            std::vector<int64_t> fill(rs_ptr.begin(), rs_ptr.end() - 1);
            for (int64_t k = 0; k < nslot; ++k) rs_slot[fill[ray_tab[k]]++] = (int32_t)k;
        }
        P->rs_ptr = upload(rs_ptr);
        P->rs_slot = upload(rs_slot);
        plan_bands(P, ray_tab, reg_base);
        if (hipMalloc(&P->zx_part, sizeof(double) * std::max<int64_t>(nreg, 1)) != hipSuccess ||
            hipMalloc(&P->part, sizeof(double) * std::max<int64_t>(nslot, 1)) != hipSuccess)
            throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
        (void)hipFree(cnt_d);
        cnt_d = nullptr;
    } catch (...) {
        if (cnt_d) (void)hipFree(cnt_d);
        fused_plan_free(P);
        throw;
    }
    P->dev_built = true;
    P->build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool have = es == 4 ? fused_rw_launch<float, true>(c, B, P, FusedArgs<float>{}, true)
                              : fused_rw_launch<double, false>(c, B, P, FusedArgs<double>{}, true);
    if (!have) {
        fused_plan_free(P);
        throw Error{HGM_E_ARG, "fused A*(B*q): no row-wave kernel for this plan's shape and the options"};
    }
    if (std::getenv("HGM_FUSED_VERBOSE"))
        std::fprintf(stderr, "[fused rw plan, device] region %d waves %d: %lld regions, %lld slots, max rays %d (LDS slots %d), %.3f s\n",
                     R, W, (long long)nreg, (long long)P->nslot, 0, P->maxr, P->build_s);
    return P;
}

FusedPlan* fused_plan_build_rw(hgm_ctx* c, const hgm_mat* B, int R, int W, int G) {
    const int es = B->dtype == HGM_F32 ? 4 : 8;       // slots as LDS byte offsets of T

    HGM_REQUIRE(B->cols < (int64_t(1) << 31) && B->rows < (int64_t(1) << 31), "fused A*(B*q): index range");
    HGM_REQUIRE(W == 1 || W == 2 || W == 4, "fused A*(B*q): 1, 2 or 4 waves per region");
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t n = B->rows, m = B->cols, nnz = B->nnz;
    int64_t nreg = 0;
    const std::vector<int32_t> reg = row_regions(B, R, &nreg);
    // the ray sets on the device (no download of the column indices), or on the host (reference)
    const bool dev_build = c->num.fused_plan_dev && m <= PLAN_DEV_MAX_M && nnz > 0;
    std::vector<int64_t> rp(n + 1);
    std::vector<int32_t> ci(dev_build ? 1 : std::max<int64_t>(nnz, 1));
    HGM_HIP(hipMemcpy(rp.data(), B->rp, sizeof(int64_t) * (n + 1), hipMemcpyDeviceToHost));
    if (nnz && !dev_build) HGM_HIP(hipMemcpy(ci.data(), B->ci, sizeof(int32_t) * nnz, hipMemcpyDeviceToHost));
    int64_t maxlen = 0;
    for (int64_t s = 0; s < n; ++s) maxlen = std::max(maxlen, rp[s + 1] - rp[s]);
    HGM_REQUIRE(maxlen <= RW_ROW_MAX, "fused A*(B*q): a pixel row longer than the row-wave pass takes");
    // runs of consecutive stored rows of one region, per region in stored order
    std::vector<std::vector<int2>> rr(nreg);
    for (int64_t s = 0; s < n; ++s) {
        auto& v = rr[reg[s]];
        if (!v.empty() && v.back().x + v.back().y == s) ++v.back().y;
        else v.push_back(make_int2((int)s, 1));
    }
    // split each region's row sequence into W contiguous shares of about equal entries
    std::vector<std::vector<int2>> wr((size_t)nreg * W);
    parallel_for(nreg, [&](int64_t g) {
        int64_t tot = 0;
        for (const int2& r : rr[g]) tot += rp[r.x + r.y] - rp[r.x];
        int w = 0;
        int64_t done = 0;
        for (const int2& r : rr[g]) {
            for (int s = r.x; s < r.x + r.y; ++s) {
                while (w < W - 1 && done * W >= tot * (w + 1)) ++w;
                auto& v = wr[(size_t)g * W + w];
                if (!v.empty() && v.back().x + v.back().y == s) ++v.back().y;
                else v.push_back(make_int2(s, 1));
                done += rp[s + 1] - rp[s];
            }
        }
    });
    // Row pairs (k_fused_rw RP): the kernel pairs rows 2i, 2i+1 of each run (batches start at even
    // offsets) and loads a pair as one chunk of 128 entries from its first row's first pair, so a
    // pair whose span (both rows + the alignment entry) exceeds 128 is not allowed: the run is cut
    // after the pair's first row, which then goes alone (C4: ~2.6 % of the pairs, ~4 cuts per wave).
    // (only for the shape the row-pair kernels exist for: 4 waves, 8-row batches, pairs, depth 2,
    // the production accumulation; any other options keep the plain row-wave plan)
    const int rpmode = c->num.fused_rowpair;
    bool rowpair = rpmode && c->num.fused_pairs && W == 4 && G == 8 && c->num.fused_depth == 2 &&
                         c->num.fused_dbg == 0 &&
                   (es == 8 || c->num.fused_acc32 == 1 || (c->num.fused_acc32 == 2 && rpmode == 4)) &&
                   maxlen + 1 <= 128;
    // does the unit (s, s+1) fit one chunk: mode 1 both rows contiguous from s's first pair (<= 128
    // entries), mode 2 each row from its own first pair (<= 64 lanes of pairs together)
    auto fits = [&](int64_t s) {
        if (rpmode != 2) return (rp[s + 2] - rp[s]) + (rp[s] & 1) <= 128;
        const int64_t la = rp[s + 1] - rp[s] + (rp[s] & 1), lb = rp[s + 2] - rp[s + 1] + (rp[s + 1] & 1);
        return (la + 1) / 2 + (lb + 1) / 2 <= 64;
    };
    // (rows so long that most pairs miss the chunk -- more than 64 runs in a wave after the cuts --
    // keep the plain row-wave plan: every unit would be a single row)
    if (rowpair) {
        std::vector<std::vector<int2>> wr1(wr.size());
        std::atomic<bool> over{false};
        parallel_for((int64_t)wr.size(), [&](int64_t i) {
            std::vector<int2>& out = wr1[(size_t)i];
            for (const int2& r : wr[(size_t)i]) {
                int s0 = r.x;
                const int end = r.x + r.y;
                int s = r.x;
                while (s < end) {
                    if (s + 1 < end && !fits(s)) {
                        out.push_back(make_int2(s0, s + 1 - s0));   // the run ends with row s alone
                        s0 = s + 1;
                        s = s + 1;
                    } else {
                        s += 2;
                    }
                }
                if (s0 < end) out.push_back(make_int2(s0, end - s0));
            }
            if (out.size() > 64) over = true;
        });
        if (over) rowpair = false;
        else wr.swap(wr1);
    }
    std::vector<int32_t> wrun((size_t)nreg * W + 1, 0);
    for (size_t i = 0; i < wr.size(); ++i) {
        HGM_REQUIRE(wr[i].size() <= 64, "fused A*(B*q): more than 64 row runs per wave");
        wrun[i + 1] = wrun[i] + (int32_t)wr[i].size();
    }
    std::vector<int2> runs(std::max<int32_t>(wrun.back(), 1));
    for (size_t i = 0; i < wr.size(); ++i) std::copy(wr[i].begin(), wr[i].end(), runs.begin() + wrun[i]);
    if (dev_build) return fused_plan_dev_finish(c, B, R, W, G, rowpair ? rpmode : 0, es, nreg, maxlen, wrun, runs, t0);
    // region ray sets and every entry's slot among them (a dense map per thread)
    std::vector<std::vector<int32_t>> rrays(nreg);
    std::vector<uint16_t> lidx(std::max<int64_t>(nnz, 1) + 256, 0);
    std::atomic<int> worst{0};
    {
        unsigned nt = std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
        std::vector<std::thread> th;
        std::atomic<int64_t> nextg{0};
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&]() {
                std::vector<int32_t> map(m, -1);
                for (int64_t g; (g = nextg.fetch_add(1)) < nreg;) {
                    auto& rs = rrays[g];
                    for (const int2& r : rr[g])
                        for (int64_t e = rp[r.x]; e < rp[r.x + r.y]; ++e) rs.push_back(ci[e]);
                    std::sort(rs.begin(), rs.end());
                    rs.erase(std::unique(rs.begin(), rs.end()), rs.end());
                    int cur = worst.load();
                    while ((int)rs.size() > cur && !worst.compare_exchange_weak(cur, (int)rs.size())) {}
                    if (rs.size() > (size_t)RW_SLOTS_MAX - 64) continue;
                    for (size_t k = 0; k < rs.size(); ++k) map[rs[k]] = (int32_t)k;
                    for (const int2& r : rr[g])
                        for (int64_t e = rp[r.x]; e < rp[r.x + r.y]; ++e) lidx[e] = (uint16_t)(map[ci[e]] * es);
                    for (int32_t ray : rs) map[ray] = -1;
                }
            });
        for (auto& t : th) t.join();
    }
    int maxr = 0;
#define HGM_RW_PICK(WV, MRV) \
    if (W == WV && worst.load() <= MRV - 64 && (maxr == 0 || MRV < maxr)) maxr = MRV;
    HGM_RW_SHAPES(HGM_RW_PICK)
#undef HGM_RW_PICK
    HGM_REQUIRE(maxr > 0, kLdsCapacityMsg);
    std::vector<int64_t> reg_base(nreg + 1, 0);
    for (int64_t g = 0; g < nreg; ++g) reg_base[g + 1] = reg_base[g] + (int64_t)rrays[g].size();
    const int64_t nslot = reg_base[nreg];
    HGM_REQUIRE(nslot < (int64_t(1) << 31), "fused A*(B*q): partial slots");
    std::vector<int32_t> ray_tab(std::max<int64_t>(nslot, 1));
    for (int64_t g = 0; g < nreg; ++g) std::copy(rrays[g].begin(), rrays[g].end(), ray_tab.begin() + reg_base[g]);
    // ray-major reduction index: ray i's slots in region order
    std::vector<int64_t> rs_ptr(m + 1, 0);
    for (int64_t g = 0; g < nreg; ++g)
        for (int32_t ray : rrays[g]) rs_ptr[ray + 1]++;
    for (int64_t i = 0; i < m; ++i) rs_ptr[i + 1] += rs_ptr[i];
    std::vector<int32_t> rs_slot(std::max<int64_t>(nslot, 1));
    {
        std::vector<int64_t> fill(rs_ptr.begin(), rs_ptr.end() - 1);
        for (int64_t g = 0; g < nreg; ++g)
            for (size_t r = 0; r < rrays[g].size(); ++r) rs_slot[fill[rrays[g][r]]++] = (int32_t)(reg_base[g] + r);
    }
    FusedPlan* P = new FusedPlan;
    try {
        P->kind = 1;
        P->elem = es;
        P->region = R;
        P->waves = W;
        P->group = G;
        P->depth = c->num.fused_depth;
        P->pairs = c->num.fused_pairs;
        P->rowpair = rowpair ? rpmode : 0;
        P->maxr = maxr;
        P->maxlen = maxlen;
        P->nreg = nreg;
        P->nslot = nslot;
        P->m = m;
        P->reg_base = upload(reg_base);
        P->wrun = upload(wrun);
        P->runs = upload(runs);
        P->ray_tab = upload(ray_tab);
        P->lidx = upload(lidx);
        if (hipMalloc(&P->zx_part, sizeof(double) * std::max<int64_t>(nreg, 1)) != hipSuccess)
            throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
        P->rs_ptr = upload(rs_ptr);
        P->rs_slot = upload(rs_slot);
        plan_bands(P, ray_tab, reg_base);
        if (hipMalloc(&P->part, sizeof(double) * std::max<int64_t>(nslot, 1)) != hipSuccess)
            throw Error{HGM_E_NOMEM, "fused plan: hipMalloc failed"};
    } catch (...) {
        fused_plan_free(P);
        throw;
    }
    P->build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const bool have = es == 4 ? fused_rw_launch<float, true>(c, B, P, FusedArgs<float>{}, true)
                              : fused_rw_launch<double, false>(c, B, P, FusedArgs<double>{}, true);
    if (!have) {
        fused_plan_free(P);
        throw Error{HGM_E_ARG, "fused A*(B*q): no row-wave kernel for this plan's shape and the options"};
    }
    if (std::getenv("HGM_FUSED_VERBOSE"))
        std::fprintf(stderr, "[fused rw plan] region %d waves %d group %d: %lld regions, %lld slots, max rays %d (LDS slots %d), longest row %lld, %d runs, %.2f s\n",
                     R, W, G, (long long)nreg, (long long)nslot, worst.load(), maxr, (long long)maxlen, wrun.back(), P->build_s);
    return P;
}

// Whether w = A*(B*q) can run fused for this pair (B = A' value for value, tiled pixels or a shard
// of whole tile columns of them; fp64, or fp32 with the row-wave pass).  On a communicator the
// caller all-reduces w, as it does A*(B*q) of the two-pass form.
bool fused_ab_eligible(const hgm_ctx* c, const hgm_mat* A, const hgm_mat* B) {
    if (!c->num.fused_ab || c->num.parity) return false;
    if (!A || !B || A->dtype != B->dtype) return false;
    if (A->dtype != HGM_F64 && !(A->dtype == HGM_F32 && c->num.fused_kind == 1)) return false;
    if (!(B->transpose_of == A->uid || A->transpose_of == B->uid)) return false;
    return !fused_grid(B).trivial() && B->nnz > 0;
}

// The option tuple a plan is built for (a refused tuple is remembered per operator, so it is not
// re-planned on every solve, while any other tuple plans afresh)
static int64_t fused_key(const Numerics& nu) {
    const bool rw = nu.fused_kind == 1;
    if (!rw) return ((int64_t)nu.fused_region << 1);
    return 1 | ((int64_t)nu.fused_wregion << 1) | ((int64_t)nu.fused_waves << 10) | ((int64_t)nu.fused_group << 13) |
           ((int64_t)nu.fused_depth << 17) | ((int64_t)nu.fused_pairs << 20) | ((int64_t)nu.fused_acc32 << 21) |
           ((int64_t)nu.fused_plan_dev << 23) | ((int64_t)nu.fused_rowpair << 24);
}

// The plan of B, built on first use (a failure to plan leaves the two-pass path in place).
const FusedPlan* fused_ab_plan(hgm_ctx* c, const hgm_mat* A, const hgm_mat* B) {
    if (!fused_ab_eligible(c, A, B)) return nullptr;
    hgm_mat* Bm = const_cast<hgm_mat*>(B);
    const Numerics& nu = c->num;
    const bool rw = nu.fused_kind == 1;
    const int64_t key = fused_key(nu);
    if (Bm->fused && Bm->fused_key != key) {          // options changed since the plan was built
        fused_plan_free(Bm->fused);
        Bm->fused = nullptr;
    }
    if (!Bm->fused && Bm->fused_failed_key != key) {   // (a refused tuple is not re-planned)
        try {
            if (rw) {
                // a region crossed by more rays than the LDS holds (many angles: the fan-beam
                // geometry over a full turn, ~7,400 rays per 32 x 32 region at 180 angles) is
                // retried with regions of half the side (about half the rays) before the pair
                // falls back to the two-pass path
                for (int R = nu.fused_wregion;; R /= 2) {
                    try {
                        Bm->fused = fused_plan_build_rw(c, B, R, nu.fused_waves, nu.fused_group);
                        break;
                    } catch (const Error& e) {
                        if (e.code != HGM_E_ARG || e.msg != kLdsCapacityMsg || R / 2 < 16 || R % 2) throw;
                    }
                }
            } else {
                Bm->fused = fused_plan_build(c, B, nu.fused_region);
            }
            Bm->fused_key = key;
            Bm->fused_failed_key = -1;
        } catch (const Error& e) {
            if (e.code != HGM_E_ARG) throw;
            Bm->fused_failed_key = key;
        }
    }
    return Bm->fused;
}

// kind 1: the row-wave kernel instantiated for the plan's waves, LDS ray slots, row batch and
// chunks per row
// Launch the instantiation for the plan and the options (dry: only report whether one exists;
// the plan is refused at build time when none does, so the two-pass path runs instead).
// T = double, GK = false: every shape and the measured variants (the GMRES family); GK = true
// (the row epilogue of the Golub-Kahan step, and every fp32 pass): the production kernel with
// four waves per region (a plan of another shape keeps the two-pass path).
#define HGM_RW_SHAPES_GK(X) X(4, 1088) X(4, 1344) X(4, 1536) X(4, 2048)
template <typename T, bool GK>
static bool fused_rw_launch(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P, const FusedArgs<T>& fa, bool dry) {
    const int W = P->waves, MR = P->maxr, G = P->group, D = c->num.fused_depth;
    const bool PRm = c->num.fused_pairs;
    // chunks per row: 64 entries (128 with pairs, whose first pair may start one entry early)
    const int64_t ml = P->maxlen + (PRm ? 1 : 0);
    const int NC = ml <= (PRm ? 128 : 64) ? 1 : ml <= (PRm ? 256 : 128) ? 2 : 4;
    const int dbg = c->num.fused_dbg;
    const int am = sizeof(T) == 4 ? c->num.fused_acc32 : 0;   // accumulation mode (k_fused_rw AM)
    const bool side = fa.side_out != nullptr && (fa.xt != nullptr || fa.side_sq);
#define HGM_RWL(AMV, WV, MRV, GV, NCV, DV, PV, DBV) HGM_RWLR(AMV, WV, MRV, GV, NCV, DV, PV, DBV, 0)
#define HGM_RWLR(AMV, WV, MRV, GV, NCV, DV, PV, DBV, RPV)                                                            \
    {                                                                                                                 \
        if (!dry)                                                                                                     \
            launch(c, false, k_fused_rw<T, GK, AMV, WV, MRV, GV, NCV, DV, PV, DBV, RPV>, dim3((unsigned)P->nreg),   \
                   dim3(64 * WV), (const int64_t*)P->reg_base, (const int32_t*)P->ray_tab, (const int32_t*)P->wrun, \
                   (const int2*)P->runs, (const int64_t*)B->rp, (const T*)B->val, (const uint16_t*)P->lidx, fa.q,  \
                   fa.zraw, (typename AccT<T, AMV>::t*)P->part, side ? fa.xt : nullptr,                            \
                   side ? (T*)P->zx_part : nullptr, fa.ev, fa.easq, fa.zout, fa.side_sq ? 1 : 0, fa.pn);           \
        return true;                                                                                                  \
    }
    if (P->rowpair) {
        // row pairs: the production accumulation, four waves, one chunk, 8-row batches, depth 2
        constexpr int AMP = sizeof(T) == 4 ? 1 : 0;
#if HGM_EXPERIMENTS
        if constexpr (sizeof(T) == 4)            // fp64 accumulators (ds_add_f64) with mode 4: measured variant
            if (am == 2 && P->rowpair == 4 && !dbg && W == 4 && G == 8 && NC == 1 && PRm && D == 2 && MR == 2048)
                HGM_RWLR(2, 4, 2048, 8, 1, 2, true, 0, 4)
#endif
        if (dbg || W != 4 || G != 8 || NC != 1 || !PRm || D != 2 || am != AMP) {
            if (dry) return false;
            throw Error{HGM_E_ARG, "fused A*(B*q): row pairs take 4 waves, 8 rows, one chunk, pairs, depth 2, "
                                   "the production accumulation"};
        }
        // mode 4 (the default) for every four-wave shape; modes 1-3 (measured variants)
        // for the C4/C5 shape only
        if (P->rowpair == 4) {
            if (MR == 1088) HGM_RWLR(AMP, 4, 1088, 8, 1, 2, true, 0, 4)
            if (MR == 1344) HGM_RWLR(AMP, 4, 1344, 8, 1, 2, true, 0, 4)
            if (MR == 1536) HGM_RWLR(AMP, 4, 1536, 8, 1, 2, true, 0, 4)
            if (MR == 2048) HGM_RWLR(AMP, 4, 2048, 8, 1, 2, true, 0, 4)
        }
#if HGM_EXPERIMENTS
        if (P->rowpair == 3 && MR == 2048) HGM_RWLR(AMP, 4, 2048, 8, 1, 2, true, 0, 3)
        if (P->rowpair == 1 && MR == 2048) HGM_RWLR(AMP, 4, 2048, 8, 1, 2, true, 0, 1)
        if (P->rowpair == 2 && MR == 2048) HGM_RWLR(AMP, 4, 2048, 8, 1, 2, true, 0, 2)
#endif
        if (dry) return false;
        throw Error{HGM_E_ARG, "fused A*(B*q): no row-pair kernel for this plan's shape and the options"};
    }
    if constexpr (GK) {
        constexpr int AMP = sizeof(T) == 4 ? 1 : 0;    // the production accumulation of this T
        const bool dshape = W == 4 && MR == 2048 && G == 8 && NC == 1 && PRm && D == 2;
        if (dbg) {   // timing experiments (hgm_spmv_ab only): the default shape
#if HGM_EXPERIMENTS
            if (dshape && am == AMP) {
#define HGM_RWD(DV) if (dbg == DV) HGM_RWL(AMP, 4, 2048, 8, 1, 2, true, DV)
                HGM_RWD(1) HGM_RWD(2) HGM_RWD(4) HGM_RWD(7)
#undef HGM_RWD
            }
#endif
            if (dry) return false;
            throw Error{HGM_E_ARG, "fused_dbg (Golub-Kahan / fp32 pass): waves 4, 2048 slots, 8 rows, pairs, depth 2, one chunk; 1, 2, 4 or 7"};
        }
#if HGM_EXPERIMENTS
        if constexpr (sizeof(T) == 4) {   // the other fp32 accumulations: the default shape (measurements)
            if (dshape && am == 0) HGM_RWL(0, 4, 2048, 8, 1, 2, true, 0)
            if (dshape && am == 2) HGM_RWL(2, 4, 2048, 8, 1, 2, true, 0)
        }
#endif
        (void)dshape;
        if (am == AMP) {
#define HGM_RW(WV, MRV)                                                                                              \
    if (W == WV && MR == MRV && G == 8 && PRm && D == 2) {                                                           \
        if (NC == 1) HGM_RWL(AMP, WV, MRV, 8, 1, 2, true, 0)                                                        \
        if (NC == 2) HGM_RWL(AMP, WV, MRV, 8, 2, 2, true, 0)                                                        \
    }
            HGM_RW_SHAPES_GK(HGM_RW)
#undef HGM_RW
        }
    } else {
        if (dbg) {   // timing experiments: the default shape only
#if HGM_EXPERIMENTS
            if (W == 4 && MR == 2048 && G == 8 && NC == 1 && PRm && D == 2) {
#define HGM_RWD(DV) if (dbg == DV) HGM_RWL(0, 4, 2048, 8, 1, 2, true, DV)
                HGM_RWD(1) HGM_RWD(2) HGM_RWD(3) HGM_RWD(4) HGM_RWD(5) HGM_RWD(6) HGM_RWD(7)
#undef HGM_RWD
            }
#endif
            if (dry) return false;
            throw Error{HGM_E_ARG, "fused_dbg with the row-wave pass: waves 4, 2048 slots, 8 rows, pairs, depth 2, one chunk"};
        }
        // production: pairs, 8-row batches, depth 2 (every shape, 1 or 2 chunks); the other
        // variants for the default shape only (measurements)
#define HGM_RW(WV, MRV)                                                                                              \
    if (W == WV && MR == MRV && G == 8 && PRm && D == 2) {                                                           \
        if (NC == 1) HGM_RWL(0, WV, MRV, 8, 1, 2, true, 0)                                                          \
        if (NC == 2) HGM_RWL(0, WV, MRV, 8, 2, 2, true, 0)                                                          \
    }
        HGM_RW_SHAPES(HGM_RW)
#undef HGM_RW
#if HGM_EXPERIMENTS
        if (W == 4 && MR == 2048 && NC == 1 && PRm) {
            if (G == 8 && D == 3) HGM_RWL(0, 4, 2048, 8, 1, 3, true, 0)
            if (G == 4 && D == 2) HGM_RWL(0, 4, 2048, 4, 1, 2, true, 0)
            if (G == 4 && D == 3) HGM_RWL(0, 4, 2048, 4, 1, 3, true, 0)
        }
        if (W == 4 && MR == 2048 && NC == 2 && !PRm && D == 2) {
            if (G == 8) HGM_RWL(0, 4, 2048, 8, 2, 2, false, 0)
            if (G == 4) HGM_RWL(0, 4, 2048, 4, 2, 2, false, 0)
        }
#endif
    }
#undef HGM_RWL
#undef HGM_RWLR
    if (dry) return false;
    throw Error{HGM_E_ARG, "fused A*(B*q): no row-wave kernel for this plan and options"};
}

// Whether the Golub-Kahan form of the pass (row epilogue, side sum of squares; every fp32 pass)
// has a kernel for this plan and the options.
bool fused_gk_ok(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P) {
    if (!P || P->kind != 1) return false;
    if (P->elem == 4) return fused_rw_launch<float, true>(c, B, P, FusedArgs<float>{}, true);
    return fused_rw_launch<double, true>(c, B, P, FusedArgs<double>{}, true);
}

__global__ void k_copy_sys(const double* __restrict__ src, double* dst) {
    if (threadIdx.x == 0) st_sys(dst, *src);
}
void copy_sys(hgm_ctx* c, const double* src, double* dst) {
    hipLaunchKernelGGL(k_copy_sys, dim3(1), dim3(64), 0, c->stream, src, dst);
    HGM_HIP(hipGetLastError());
}

// One pass over B (fa: internal.h FusedArgs): z = B*q, the row epilogue zs, w = A*zs, the side sum.
template <typename T>
bool fused_pass(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P, const FusedArgs<T>& fa) {
    HGM_REQUIRE((int)sizeof(T) == P->elem && (int)sizeof(T) == (B->dtype == HGM_F32 ? 4 : 8), "fused pass: dtype");
    const bool gk = fa.ev || fa.zout || fa.side_sq || sizeof(T) == 4;
    const bool side = fa.side_out != nullptr && (fa.xt != nullptr || fa.side_sq) && P->kind == 1;
    hipEvent_t t0 = nullptr;
    timing_begin(c, KC_FUSED, &t0);
    if (P->kind == 1) {
        if (gk) fused_rw_launch<T, true>(c, B, P, fa, false);
        else if constexpr (sizeof(T) == 8) fused_rw_launch<T, false>(c, B, P, fa, false);
    } else {
        HGM_REQUIRE(!gk && sizeof(T) == 8, "fused pass: the sub-chunk kernel is fp64 without epilogues");
#if !HGM_EXPERIMENTS
        HGM_REQUIRE(false, "fused pass: the sub-chunk kernel (kind 0) is in the experiments build only");
#else
        if constexpr (sizeof(T) == 8) {
#define HGM_FUSED_LAUNCH(FB, FGV, PFV)                                                                          \
    launch(c, false, k_fused_ab<FB, FGV, PFV>, dim3((unsigned)P->nreg), dim3(FB), (const FusedSub*)P->subs,      \
           (const int32_t*)P->reg_sub, (const int64_t*)P->reg_base, (const uint16_t*)P->perm,                    \
           (const int32_t*)P->lr_ray, (const uint32_t*)P->lr_pk, (const int64_t*)B->rp, (const double*)B->val, fa.q, \
           fa.zraw, P->part, c->num.fused_dbg)
            // (one lane count per row sum for every variant: the same summation order, the same bits)
            const int d = c->num.fused_pf;
            if (c->num.fused_bs == 512) {
                if (d <= 1) HGM_FUSED_LAUNCH(512, HGM_FUSED_FGR, 1);
                else if (d == 2) HGM_FUSED_LAUNCH(512, HGM_FUSED_FGR, 2);
                else if (d == 3) HGM_FUSED_LAUNCH(512, HGM_FUSED_FGR, 3);
                else HGM_FUSED_LAUNCH(512, HGM_FUSED_FGR, 4);
            } else {
                if (d <= 1) HGM_FUSED_LAUNCH(1024, HGM_FUSED_FGR, 1);
                else if (d == 2) HGM_FUSED_LAUNCH(1024, HGM_FUSED_FGR, 2);
                else if (d == 3) HGM_FUSED_LAUNCH(1024, HGM_FUSED_FGR, 3);
                else HGM_FUSED_LAUNCH(1024, HGM_FUSED_FGR, 4);
            }
#undef HGM_FUSED_LAUNCH
        }
#endif
    }
    // one lane group per ray, no grid-stride cap (C4: 8,508 blocks; the 4,096 cap measured 5 us slower)
    const unsigned rgrid = (unsigned)std::max<int64_t>(1, (P->m * HGM_FUSED_RG + BS - 1) / BS);
    const bool f64p = sizeof(T) == 4 && P->kind == 1 && c->num.fused_acc32 == 2;   // fp64 partials of the fp32 pass
    if (P->kind == 1 && P->band_ptr && c->num.fused_reduce == 1) {
        const unsigned bgrid = (unsigned)std::max<int64_t>(1, (P->nband + BS / 64 - 1) / (BS / 64));
        if (f64p)
            launch(c, true, k_fused_reduce_band<T, double>, dim3(bgrid), dim3(BS), P->m, P->nband,
                   (const int32_t*)P->band_ptr, (const int4*)P->band_run, (const double*)P->part, fa.w,
                   (const T*)P->zx_part, (int)P->nreg, side ? fa.side_out : nullptr);
        else
            launch(c, true, k_fused_reduce_band<T, T>, dim3(bgrid), dim3(BS), P->m, P->nband,
                   (const int32_t*)P->band_ptr, (const int4*)P->band_run, (const T*)P->part, fa.w,
                   (const T*)P->zx_part, (int)P->nreg, side ? fa.side_out : nullptr);
#if HGM_EXPERIMENTS
    } else if (f64p) {
        launch(c, true, k_fused_reduce<HGM_FUSED_RG, T, double>, dim3(rgrid), dim3(BS), P->m,
               (const int64_t*)P->rs_ptr, (const int32_t*)P->rs_slot, (const double*)P->part, fa.w,
               (const T*)P->zx_part, (int)P->nreg, side ? fa.side_out : nullptr);
    } else if (c->num.fused_reduce >= 2) {
        // measured variants: fewer lanes per ray (the lanes of a wave then read adjacent rays' slots
        // of one region: coalesced partial gathers), more loads in flight
        const int rg = c->num.fused_reduce == 2 ? 1 : c->num.fused_reduce == 3 ? 2 : 4;
        const unsigned g2 = (unsigned)std::max<int64_t>(1, (P->m * rg + BS - 1) / BS);
#define HGM_RED(RGV, RBV)                                                                                        \
    launch(c, true, k_fused_reduce<RGV, T, T, RBV>, dim3(g2), dim3(BS), P->m, (const int64_t*)P->rs_ptr,          \
           (const int32_t*)P->rs_slot, (const T*)P->part, fa.w, (const T*)P->zx_part, (int)P->nreg,               \
           side ? fa.side_out : nullptr)
        if (rg == 1) HGM_RED(1, 8);
        else if (rg == 2) HGM_RED(2, 8);
        else HGM_RED(4, 4);
#undef HGM_RED
#endif
    } else {
        // partials per lane: C4 ~14 (RB 16); rank g's shard of an 8-way cut ~1.8 (RB 4: the batch of
        // 16 issued 8x the loads it adds; round 6)
        const double ppl = (double)P->nslot / (double)std::max<int64_t>(1, P->m) / HGM_FUSED_RG;
#define HGM_RED_RB(RBV)                                                                                         \
    launch(c, true, k_fused_reduce<HGM_FUSED_RG, T, T, RBV>, dim3(rgrid), dim3(BS), P->m,                       \
           (const int64_t*)P->rs_ptr, (const int32_t*)P->rs_slot, (const T*)P->part, fa.w, (const T*)P->zx_part, \
           (int)P->nreg, side ? fa.side_out : nullptr)
        if (ppl <= 4.0) HGM_RED_RB(4);
        else if (ppl <= 8.0) HGM_RED_RB(8);
        else HGM_RED_RB(16);
#undef HGM_RED_RB
    }
    HGM_HIP(hipGetLastError());
    // algorithmic bytes of the fused pass: B's CSR once (values, 32-bit indices, row pointers),
    // q read, z and w written (SURVEY.md §8(d)'s SpMV count for one pass over the operator), and
    // with the row epilogue its read of ev (the two-pass form's EPI_SUB operand)
    const double s = (double)sizeof(T);
    const double bytes = (s + 4.0) * (double)B->nnz + 8.0 * (B->rows + 1) + s * B->cols + s * B->rows + s * B->cols +
                         (fa.ev ? s * B->rows : 0.0);
    timing_end(c, KC_FUSED, t0, bytes);
    return side;
}
template bool fused_pass<double>(hgm_ctx*, const hgm_mat*, const FusedPlan*, const FusedArgs<double>&);
template bool fused_pass<float>(hgm_ctx*, const hgm_mat*, const FusedPlan*, const FusedArgs<float>&);

// Bq = B*q (n), ABq = A*(B*q) (m), one pass over B.
bool fused_ab(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P, const double* q, double* Bq, double* ABq,
              const double* xt, double* zx_out, const PendNorm<double>* pn) {
    FusedArgs<double> fa;
    fa.q = q;
    fa.zraw = Bq;
    fa.w = ABq;
    fa.xt = xt;
    fa.side_out = zx_out;
    if (pn && pn->np > 0) {
        HGM_REQUIRE(fused_pend_ok(c, P) && pn->hdev && pn->hring && pn->np <= MAX_PARTS,
                    "fused A*(B*q): pending normalisation needs the row-wave pass");
        fa.pn = *pn;
    }
    return fused_pass<double>(c, B, P, fa);
}

// (the row-wave pass; every wave re-forms reduce_parts' BS-thread order, whatever its waves)
bool fused_pend_ok(const hgm_ctx* c, const FusedPlan* P) {
    return P && P->kind == 1 && c->num.fused_dbg == 0;
}

}  // namespace hgm

namespace hgm {
// FNV-1a over the plan's arrays (hgm_fused_plan_info): two builds compare byte for byte
uint64_t fused_plan_checksum(hgm_ctx* c, const hgm_mat* B, const FusedPlan* P) {
    HGM_REQUIRE(P->kind == 1, "plan checksum: the row-wave plan");
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* dev, size_t bytes) {
        std::vector<unsigned char> v(bytes);
        if (bytes) HGM_HIP(hipMemcpy(v.data(), dev, bytes, hipMemcpyDeviceToHost));
        for (unsigned char b : v) h = (h ^ b) * 1099511628211ull;
    };
    int32_t nrun = 0;
    HGM_HIP(hipMemcpy(&nrun, P->wrun + P->nreg * P->waves, sizeof(int32_t), hipMemcpyDeviceToHost));
    mix(P->wrun, sizeof(int32_t) * (P->nreg * P->waves + 1));
    mix(P->runs, sizeof(int2) * nrun);
    mix(P->reg_base, sizeof(int64_t) * (P->nreg + 1));
    mix(P->ray_tab, sizeof(int32_t) * P->nslot);
    mix(P->lidx, sizeof(uint16_t) * B->nnz);
    mix(P->rs_ptr, sizeof(int64_t) * (P->m + 1));
    mix(P->rs_slot, sizeof(int32_t) * P->nslot);
    if (P->band_ptr) {
        mix(P->band_ptr, sizeof(int32_t) * (P->nband + 1));
        mix(P->band_run, sizeof(int4) * P->nrun);
    }
    const int64_t meta[6] = {P->elem, P->region, P->waves, P->maxr, P->maxlen, P->nslot};
    for (int64_t v : meta)
        for (int k = 0; k < 8; ++k) h = (h ^ (unsigned char)(v >> (8 * k))) * 1099511628211ull;
    (void)c;
    return h;
}
double fused_plan_build_seconds(const FusedPlan* P) { return P->build_s; }
int64_t fused_plan_slots(const FusedPlan* P) { return P->nslot; }
bool fused_plan_device_built(const FusedPlan* P) { return P->dev_built; }
}  // namespace hgm
