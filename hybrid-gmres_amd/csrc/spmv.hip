// Sparse matrix-vector products of the Arnoldi / Golub-Kahan loop, hand-written for
// gfx950 (CDNA4).  Three kernels, chosen per operator (ops.hip: finalize_operator):
//  * k_spmv        one G-lane group per CSR row (G = 32 for the long ray-major rows of A,
//                  G = 8 for the short pixel-major rows of B = A'), optional 16-byte
//                  paired loads / nontemporal loads / XCD-aware block order;
//  * k_spmv_band   the same over column bands of A (cache blocking of the x gather: the
//                  blocks in flight gather from one L2-resident x-slice), followed by a
//                  fixed-order band reduction;
//  * k_spmv_stream nnz-balanced: fixed 2048-entry chunks streamed with 16-byte loads,
//                  products staged in LDS, per-segment reduction, fixed-order fix-up.
// Every reduction is a fixed tree (no atomics): repeated products are bitwise equal.
// Epilogues of the reference's operator closures are fused into the final store:
// `B*(A*v) + lambda*v` (hybrid_*_rtp.m:6), `A*v - alpha*u` (lsqr_solver.m:22),
// `A'*u - beta*v` (lsqr_solver.m:26), `b - A*x` (hybrid_*_rtp.m:32/35).
#include "device_common.h"

namespace hgm {

// XCD-aware block order (speed only, never correctness): consecutive logical row blocks
// run on the same XCD so neighbouring rays share x lines in that XCD's L2
// (cdna_hip_programming.md §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
    const int64_t q = nb / 8, r = nb % 8, xcd = b % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// One G-lane group per CSR row.  VEC: each lane streams pairs of entries with 16-byte
// value loads and 8-byte index loads (row heads/tails peeled to keep them aligned).
// NT: nontemporal (streaming) loads for val/col so they do not evict x from L2/MALL.
// Per-lane partial of the dot product of entries [s, e) with x, lane gl of a G-lane group.
#ifndef HGM_SPMV_U
#define HGM_SPMV_U 4   // pairs per lane per iteration of the VEC row loop (C2 A: 4 beats 2 and 8)
#endif
// IX: column index type (int32_t, or uint16_t for the narrow copy ci16; scalar path only).
template <typename T, int G, bool VEC, bool NT, typename IX = int32_t>
__device__ __forceinline__ T seg_partial(int64_t s, int64_t e, int gl, const IX* __restrict__ ci,
                                         const T* __restrict__ val, const T* __restrict__ x) {
    static_assert(!VEC || sizeof(IX) == 4, "paired loads need 32-bit column indices");
    T a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    {
        if constexpr (!VEC) {
            int64_t i = s + gl;
            for (; i + 3 * G < e; i += 4 * G) {
                const int32_t c0 = ld<NT>(ci + i), c1 = ld<NT>(ci + i + G), c2 = ld<NT>(ci + i + 2 * G),
                              c3 = ld<NT>(ci + i + 3 * G);
                const T v0 = ld<NT>(val + i), v1 = ld<NT>(val + i + G), v2 = ld<NT>(val + i + 2 * G),
                        v3 = ld<NT>(val + i + 3 * G);
                a0 += v0 * x[c0];
                a1 += v1 * x[c1];
                a2 += v2 * x[c2];
                a3 += v3 * x[c3];
            }
            for (; i < e; i += G) a0 += ld<NT>(val + i) * x[ld<NT>(ci + i)];
        } else {
            using T2 = typename NV2<T>::t;
            using I2 = ni2;
            static_assert(sizeof(IX) == 4, "");
            const int64_t s2 = (s + 1) & ~int64_t(1);     // first even index >= s
            const int64_t e2 = e & ~int64_t(1);           // last even bound <= e
            if (gl == 0 && s < s2 && s < e) a0 += ld<NT>(val + s) * x[ld<NT>(ci + s)];
            if (gl == G - 1 && e2 < e && e2 >= s2) a1 += ld<NT>(val + e2) * x[ld<NT>(ci + e2)];
            int64_t i = s2 + 2 * gl;
#if HGM_SPMV_U > 2
            // U pairs per lane per iteration (all index/value loads, then all gathers)
            for (; i + (HGM_SPMV_U - 1) * 2 * G < e2; i += HGM_SPMV_U * 2 * G) {
                I2 cc[HGM_SPMV_U];
                T2 vv[HGM_SPMV_U];
#pragma unroll
                for (int u = 0; u < HGM_SPMV_U; ++u) {
                    cc[u] = ld<NT>(reinterpret_cast<const I2*>(ci + i + u * 2 * G));
                    vv[u] = ld<NT>(reinterpret_cast<const T2*>(val + i + u * 2 * G));
                }
                T xx[2 * HGM_SPMV_U];
#pragma unroll
                for (int u = 0; u < HGM_SPMV_U; ++u) {
                    xx[2 * u] = x[cc[u].x];
                    xx[2 * u + 1] = x[cc[u].y];
                }
#pragma unroll
                for (int u = 0; u < HGM_SPMV_U; u += 2) {
                    a0 += vv[u].x * xx[2 * u];
                    a1 += vv[u].y * xx[2 * u + 1];
                    a2 += vv[u + 1].x * xx[2 * u + 2];
                    a3 += vv[u + 1].y * xx[2 * u + 3];
                }
            }
#endif
            for (; i + 2 * G < e2; i += 4 * G) {
                const I2 c0 = ld<NT>(reinterpret_cast<const I2*>(ci + i));
                const I2 c1 = ld<NT>(reinterpret_cast<const I2*>(ci + i + 2 * G));
                const T2 v0 = ld<NT>(reinterpret_cast<const T2*>(val + i));
                const T2 v1 = ld<NT>(reinterpret_cast<const T2*>(val + i + 2 * G));
                a0 += v0.x * x[c0.x];
                a1 += v0.y * x[c0.y];
                a2 += v1.x * x[c1.x];
                a3 += v1.y * x[c1.y];
            }
            for (; i < e2; i += 2 * G) {
                const I2 c0 = ld<NT>(reinterpret_cast<const I2*>(ci + i));
                const T2 v0 = ld<NT>(reinterpret_cast<const T2*>(val + i));
                a0 += v0.x * x[c0.x];
                a1 += v0.y * x[c0.y];
            }
        }
    }
    return (a0 + a1) + (a2 + a3);
}

// NRM: also write the block's sum of y_r^2 (rows in increasing order) to nparts[blk] —
// the residual monitor norm(b - A*x) (hybrid_*_rtp.m:32/35) without re-reading y.
template <typename T, int G, int EPI, bool VEC, bool NT, bool NRM = false, typename IX = int32_t>
__global__ __launch_bounds__(BS) void k_spmv(int64_t rows, const int64_t* __restrict__ rp,
                                             const IX* __restrict__ ci,
                                             const T* __restrict__ val, const T* __restrict__ x,
                                             T* __restrict__ y, T a, const T* __restrict__ z, int xcd,
                                             T* __restrict__ nparts, PendNorm<T> pn) {
    constexpr int RPB = BS / G;
    const int64_t blk = xcd ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t row = blk * RPB + threadIdx.x / G;
    const int gl = threadIdx.x & (G - 1);
    const T hpre = pn_pre<T, EPI>(pn);
    if constexpr (EPI == EPI_ADD || EPI == EPI_SUB) a = pn_coef<T>(pn, a);
    T zr = T(0);   // epilogue operand, loaded up front
    if constexpr (EPI != EPI_NONE && EPI != EPI_DIVH) {
        if (gl == 0 && row < rows) zr = z[row];
    }
    T acc = 0;
    if (row < rows) acc = seg_partial<T, G, VEC, NT, IX>(rp[row], rp[row + 1], gl, ci, val, x);
    acc = group_sum<T, G>(acc);
    __shared__ T hsh[4];
    const T h = pn_fin<T, EPI>(pn, hpre, hsh);
    T r = 0;
    if (gl == 0 && row < rows) {
        r = apply_epi_zv<T, EPI>(acc, a, zr, row, pn, h);
        y[row] = r;
    }
    if (NRM) {
        __shared__ T rs[RPB];
        if (gl == 0) rs[threadIdx.x / G] = r * r;
        __syncthreads();
        if (threadIdx.x == 0) {
            T s = 0;
            for (int j = 0; j < RPB; ++j) s += rs[j];
            nparts[blk] = s;
        }
    }
}

// fixed-order sum of np partials by one block
template <typename T>
__global__ __launch_bounds__(BS) void k_sum_parts(const T* __restrict__ parts, int64_t np, T* out) {
    __shared__ T sh[4];
    T a = 0;
    for (int64_t i = threadIdx.x; i < np; i += BS) a += parts[i];
    const T r = block_sum_all(a, sh);
    if (threadIdx.x == 0) st_sys(out, r);
}

// Column-banded SpMV: work items (band b, block of RPB rows) in band-major order, grid-
// stride, so the blocks resident at any moment gather x from one band's slice (L2-
// resident).  Writes the per-band partial ypart[b*rows + r]; k_band_reduce sums them.
template <typename T, int G, bool VEC, bool NT>
__global__ __launch_bounds__(BS) void k_spmv_band(int64_t rows, int nbands, const int64_t* __restrict__ brp,
                                                  const int32_t* __restrict__ ci, const T* __restrict__ val,
                                                  const T* __restrict__ x, T* __restrict__ ypart) {
    constexpr int RPB = BS / G;
    const int64_t rb_per_band = (rows + RPB - 1) / RPB;
    const int64_t items = rb_per_band * nbands;
    const int gl = threadIdx.x & (G - 1);
    for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {
        const int64_t b = it / rb_per_band;
        const int64_t row = (it - b * rb_per_band) * RPB + threadIdx.x / G;
        T acc = 0;
        if (row < rows) {
            const int64_t* p = brp + b * rows + row;
            acc = seg_partial<T, G, VEC, NT>(p[0], p[1], gl, ci, val, x);
        }
        acc = group_sum<T, G>(acc);
        if (gl == 0 && row < rows) ypart[b * rows + row] = acc;
    }
}

// ------------------------------------------------------------------------------
// nnz-balanced streaming SpMV over segments (rows, or (band,row) pairs).
// Block k owns entries [k*CH, (k+1)*CH): it streams them with 16-byte loads, stages the
// products in LDS, then G-lane groups reduce every segment that STARTS in the chunk
// (fo[k] .. fo[k+1]) plus the head part of the segment that started earlier.  Complete
// segments are written (with the epilogue); a segment running past the chunk leaves its
// partial in tail[k] and every later chunk's share in head[j]; k_stream_fixup adds them
// in chunk order.  Fixed chunking => fixed summation order => bitwise reproducible.
// ------------------------------------------------------------------------------
// Paged x gathers (SPMV_PAGED, hgm_mat::pg_*).  PMC at C4 (profiles/r2_pmc_spmv/): with one
// global gather per entry the A and B stream kernels make ~1 L1 tag lookup per entry and keep
// the TA 80-90 % busy -- the address path, not HBM, bounds them (420 G entries/s in fp64 and
// only 500 G/s in fp32 on a third fewer bytes).  A 4096-entry chunk touches 87 (B) / 235 (A)
// distinct 128-B lines of x on average (scripts/page_stats.py), so the chunk stages those pages
// in LDS with coalesced 16-B loads and gathers from LDS through 16-bit page-local indices:
// ~L1 lookups per chunk drop from ~4096 to the page count and the index stream from 4 to 2
// bytes per entry.  Products and summation order are unchanged (same bits as the unpaged kernel).
template <typename T>
struct Paged {
    const int32_t* pptr = nullptr;
    const int32_t* pids = nullptr;
    const uint16_t* lidx = nullptr;
    int64_t xlen = 0;
    int xcd = 0;   // SPMV_XCD: workgroups of one XCD take one contiguous eighth of the chunks
};

// 16 bytes of page `pid` for lane `pl` of the page's loaders, zero past the end of x
template <typename V16, typename T>
__device__ __forceinline__ V16 load_page16(const T* __restrict__ x, int64_t pid, int pl, int64_t xlen) {
    constexpr int PGV = PG_BYTES / (int)sizeof(T), VE = 16 / (int)sizeof(T);
    const int64_t e0 = pid * PGV + (int64_t)pl * VE;
    if (e0 + VE <= xlen) return *reinterpret_cast<const V16*>(x + e0);
    V16 v;
    const T* vp = reinterpret_cast<const T*>(&v);
    T tmp[VE];
#pragma unroll
    for (int i = 0; i < VE; ++i) tmp[i] = e0 + i < xlen ? x[e0 + i] : T(0);
    (void)vp;
    __builtin_memcpy(&v, tmp, 16);
    return v;
}

// CLS: the operator class (KC_SPMV_A ray-major / KC_SPMV_B pixel-major) only names the
// instantiation, so kernel traces (rocprofv3 --stats) report A and B separately.
template <typename T, int G, int EPI, bool NT, typename IX = int32_t, bool PG = false, int CLS = 0>
__global__ __launch_bounds__(BS) void k_spmv_stream(int64_t nnz, int64_t nseg, const int64_t* __restrict__ sp,
                                                    const int32_t* __restrict__ fo, const IX* __restrict__ ci,
                                                    const T* __restrict__ val, const T* __restrict__ x,
                                                    T* __restrict__ out, T a, const T* __restrict__ z,
                                                    T* __restrict__ head, T* __restrict__ tail, PendNorm<T> pn,
                                                    Paged<T> pg) {
    static_assert(EPI != EPI_DIVH, "EPI_DIVH is applied by the band reduction or the row kernel");
    using T2 = typename NV2<T>::t;
    using IV2 = std::conditional_t<sizeof(IX) == 2, nus2, ni2>;   // index pair / quad of the type
    using IV4 = std::conditional_t<sizeof(IX) == 2, nus4, ni4>;
    __shared__ __attribute__((aligned(16))) unsigned char smem[stream_lds_bytes<T>(PG)];
    T* prod = reinterpret_cast<T*>(smem);
    // chunk of this workgroup: in launch order, or (pg.xcd) XCD-contiguous -- workgroups are
    // dispatched to the 8 XCDs round-robin, so XCD j then streams the j-th eighth of the chunks
    // (band-major: its own bands, whose x-slices only its L2 fetches)
    const int64_t k = pg.xcd ? xcd_block(blockIdx.x, gridDim.x) : (int64_t)blockIdx.x;
    const int64_t c0 = k * SCH;
    const int64_t c1 = (c0 + SCH < nnz) ? c0 + SCH : nnz;
    const int n = (int)(c1 - c0);
    // Segment bookkeeping of the reduction phase (the chunk's segment range, sp at its first
    // segment for the head test and, per group, sp around its first task's segment) is
    // loaded while the chunk's value/index loads are in flight, so its two dependent round
    // trips (fo -> sp) overlap the product phase instead of following the barrier.  The
    // scheduling barriers keep the compiler from hoisting its waits above those loads.
    const int gid = threadIdx.x / G, gl = threadIdx.x & (G - 1);
    int64_t s_begin, s_end, q, sp_b, pm, p0, p1;
    T h = T(1);
    auto bookkeeping = [&]() {
        h = pn_pre<T, EPI>(pn);
        if constexpr (EPI == EPI_ADD || EPI == EPI_SUB) a = pn_coef<T>(pn, a);
        s_begin = fo[k];
        s_end = fo[k + 1];
        q = s_begin + gid;
        sp_b = s_begin <= nseg ? sp[s_begin] : 0;
        pm = (q >= 1 && q - 1 <= nseg) ? sp[q - 1] : 0;
        p0 = q <= nseg ? sp[q] : 0;
        p1 = q + 1 <= nseg ? sp[q + 1] : 0;
    };
    bool staged = false;
    if constexpr (PG) {
        // ---- paged gathers: x pages -> LDS (prod[] doubles as the page buffer), then products ----
        const int pp0 = pg.pptr[k];
        const int npg = n == SCH ? pg.pptr[k + 1] - pp0 : 0;      // 0: gather through ci (below)
        if (npg > 0) {
            constexpr int LPP = PG_BYTES / 16;                       // lanes per page, 16 B each
            constexpr int PPP = BS / LPP;                            // pages per pass
            constexpr int NPASS = (pg_max<T>() + PPP - 1) / PPP;
            using V16 = std::conditional_t<sizeof(T) == 8, nd2, nf4>;
            using VV = std::conditional_t<sizeof(T) == 8, nd2, nf4>;        // values per lane per step
            using LV = std::conditional_t<sizeof(T) == 8, nus2, nus4>;      // their page-local indices
            constexpr int VE = 16 / (int)sizeof(T);                  // entries per lane per step
            constexpr int U = SCH / (VE * BS);
            const int pl = threadIdx.x % LPP, ps = threadIdx.x / LPP;
            VV vv[U];
            LV lc[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = VE * threadIdx.x + u * VE * BS;
                vv[u] = ld<NT>(reinterpret_cast<const VV*>(val + c0 + j));
                lc[u] = ld<NT>(reinterpret_cast<const LV*>(pg.lidx + c0 + j));
            }
            int pid[NPASS];
#pragma unroll
            for (int i = 0; i < NPASS; ++i) {
                const int sl = ps + i * PPP;
                pid[i] = sl < npg ? pg.pids[pp0 + sl] : -1;
            }
            V16 pv[NPASS];
#pragma unroll
            for (int i = 0; i < NPASS; ++i)
                if (pid[i] >= 0) pv[i] = load_page16<V16>(x, pid[i], pl, pg.xlen);
            __builtin_amdgcn_sched_barrier(0);
            bookkeeping();
            __builtin_amdgcn_sched_barrier(0);
            V16* pages = reinterpret_cast<V16*>(prod);
#pragma unroll
            for (int i = 0; i < NPASS; ++i)
                if (pid[i] >= 0) pages[(ps + i * PPP) * LPP + pl] = pv[i];
            __syncthreads();
            if constexpr (pg_rounds<T>() == 1) {
                T pr[U * VE];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < VE; ++e) pr[u * VE + e] = vv[u][e] * prod[lc[u][e]];
                __syncthreads();                                      // pages no longer read
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < VE; ++e) prod[VE * threadIdx.x + u * VE * BS + e] = pr[u * VE + e];
            } else {
                // (a one-round fast path beside this loop measured slower: 66 vs 62 VGPRs,
                // C5 A 1.33-1.35 vs 1.32-1.33 ms, profiles/r2_tworound_c5.jsonl)
                // more than PGM pages: later rounds restage the buffer with the next PGM pages;
                // each entry is multiplied in its page's round (products: the same bits)
                constexpr int PGM = pg_max<T>(), LIM = PGM * (PG_BYTES / (int)sizeof(T));
                T pr[U * VE];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < VE; ++e) pr[u * VE + e] = vv[u][e];
                const int nround = (npg + PGM - 1) / PGM;             // block-uniform
#pragma unroll 1
                for (int r = 0; r < nround; ++r) {
                    if (r > 0) {
                        // in quarters: the products and the segment bookkeeping are live here
                        constexpr int NQ = NPASS >= 4 ? NPASS / 4 : 1;
                        __syncthreads();                              // the previous round's pages no longer read
#pragma unroll 1
                        for (int i0 = 0; i0 < NPASS; i0 += NQ) {
                            int qid[NQ];
                            V16 qv[NQ];
#pragma unroll
                            for (int i = 0; i < NQ; ++i) {
                                const int sl = r * PGM + ps + (i0 + i) * PPP;
                                qid[i] = sl < npg ? pg.pids[pp0 + sl] : -1;
                            }
#pragma unroll
                            for (int i = 0; i < NQ; ++i)
                                if (qid[i] >= 0) qv[i] = load_page16<V16>(x, qid[i], pl, pg.xlen);
#pragma unroll
                            for (int i = 0; i < NQ; ++i)
                                if (qid[i] >= 0) pages[(ps + (i0 + i) * PPP) * LPP + pl] = qv[i];
                        }
                        __syncthreads();
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int e = 0; e < VE; ++e) {
                            const int li = lc[u][e] - r * LIM;
                            if (li >= 0 && li < LIM) pr[u * VE + e] = pr[u * VE + e] * prod[li];
                        }
                }
                __syncthreads();                                      // pages no longer read
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < VE; ++e) prod[VE * threadIdx.x + u * VE * BS + e] = pr[u * VE + e];
            }
            staged = true;
        }
    }
    if (staged) {
        // products are in prod[]
    } else if (n == SCH && sizeof(T) == 4) {
        // fp32: four entries per lane per step (16-B value and 16-B index loads, both fully
        // coalesced across the wave)
        constexpr int U = SCH / (4 * BS);
        IV4 cc[U];
        nf4 vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = 4 * threadIdx.x + u * 4 * BS;
            cc[u] = ld<NT>(reinterpret_cast<const IV4*>(ci + c0 + j));
            vv[u] = ld<NT>(reinterpret_cast<const nf4*>(val + c0 + j));
        }
        __builtin_amdgcn_sched_barrier(0);
        bookkeeping();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = 4 * threadIdx.x + u * 4 * BS;
            prod[j] = vv[u].x * x[cc[u].x];
            prod[j + 1] = vv[u].y * x[cc[u].y];
            prod[j + 2] = vv[u].z * x[cc[u].z];
            prod[j + 3] = vv[u].w * x[cc[u].w];
        }
    } else if (n == SCH) {
        // fp64: a pair per lane per step (16-B value loads; four entries per lane would leave
        // every 16-B wave load half-coalesced: measured 17% slower at C4)
        constexpr int U = SCH / (2 * BS);
        IV2 cc[U];
        T2 vv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = 2 * threadIdx.x + u * 2 * BS;
            vv[u] = ld<NT>(reinterpret_cast<const T2*>(val + c0 + j));
            cc[u] = ld<NT>(reinterpret_cast<const IV2*>(ci + c0 + j));
        }
        __builtin_amdgcn_sched_barrier(0);
        bookkeeping();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = 2 * threadIdx.x + u * 2 * BS;
            prod[j] = vv[u].x * x[cc[u].x];
            prod[j + 1] = vv[u].y * x[cc[u].y];
        }
    } else {
        bookkeeping();
        for (int j = threadIdx.x; j < n; j += BS) prod[j] = val[c0 + j] * x[ci[c0 + j]];
    }
    __syncthreads();
    const int has_head = (s_begin > 0 && sp_b > c0) ? 1 : 0;
    const int64_t ntasks = (s_end - s_begin) + has_head;
    constexpr int NG = BS / G;
    for (int64_t t = gid; t < ntasks; t += NG) {
        int64_t s, lo, send;
        if (t == gid) {             // first task: prefetched bounds
            s = q - has_head;
            lo = (has_head && t == 0) ? c0 : (has_head ? pm : p0);
            send = has_head ? p0 : p1;
        } else {
            s = s_begin + t - has_head;
            lo = sp[s];
            send = sp[s + 1];
        }
        const int64_t hi = send < c1 ? send : c1;
        T acc = 0;
        for (int64_t i = lo + gl; i < hi; i += G) acc += prod[i - c0];
        acc = group_sum<T, G>(acc);
        if (gl == 0) {
            if (has_head && t == 0) head[k] = acc;
            else if (send > c1) tail[k] = acc;
            else out[s] = apply_epi_pn<T, EPI>(acc, a, z, s, pn, h);
        }
    }
}

template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_stream_fixup(int64_t nnz, int64_t nchunks, const int64_t* __restrict__ sp,
                                                     const int32_t* __restrict__ fo, T* __restrict__ out, T a,
                                                     const T* __restrict__ z, const T* __restrict__ head,
                                                     const T* __restrict__ tail, PendNorm<T> pn) {
    static_assert(EPI != EPI_DIVH, "EPI_DIVH is applied by the band reduction or the row kernel");
    const T h = pn_pre<T, EPI>(pn);
    if constexpr (EPI == EPI_ADD || EPI == EPI_SUB) a = pn_coef<T>(pn, a);
    for (int64_t k = (int64_t)blockIdx.x * BS + threadIdx.x; k < nchunks; k += (int64_t)gridDim.x * BS) {
        const int64_t s_begin = fo[k], s_end = fo[k + 1];
        if (s_end <= s_begin) continue;
        const int64_t s = s_end - 1;
        const int64_t c1 = (k + 1) * SCH < nnz ? (k + 1) * SCH : nnz;
        if (sp[s + 1] <= c1) continue;
        T sum = tail[k];
        for (int64_t j = k + 1; j < nchunks; ++j) {
            sum += head[j];
            const int64_t cj1 = (j + 1) * SCH < nnz ? (j + 1) * SCH : nnz;
            if (sp[s + 1] <= cj1) break;
        }
        out[s] = apply_epi_pn<T, EPI>(sum, a, z, s, pn, h);
    }
}

template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_fill_epi(int64_t n, T* __restrict__ out, T a, const T* __restrict__ z) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        out[i] = apply_epi<T, EPI>(T(0), a, z, i);
}

// y[r] = epi( sum_b ypart[b*rows + r] ), bands summed in increasing b (deterministic)
template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_band_reduce(int64_t rows, int nbands, const T* __restrict__ ypart,
                                                    T* __restrict__ y, T a, const T* __restrict__ z,
                                                    PendNorm<T> pn) {
    __shared__ T hsh[4];
    const T h = pn_fin<T, EPI>(pn, pn_pre<T, EPI>(pn), hsh);
    if constexpr (EPI == EPI_ADD || EPI == EPI_SUB) a = pn_coef<T>(pn, a);
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BS) {
        // eight independent (read-once, nontemporal) loads in flight, summed in band order
        T s = 0;
        int b = 0;
        for (; b + 8 <= nbands; b += 8) {
            T v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = __builtin_nontemporal_load(ypart + (int64_t)(b + i) * rows + r);
#pragma unroll
            for (int i = 0; i < 8; ++i) s += v[i];
        }
        for (; b < nbands; ++b) s += ypart[(int64_t)b * rows + r];
        y[r] = apply_epi_pn<T, EPI>(s, a, z, r, pn, h);
    }
}

// Parity mode (HGM_OPT_PARITY): one thread per row, entries summed sequentially in stored
// order with a separate multiply and add: s = ((0 + a_0 x_0) + a_1 x_1) + ...  This is
// scipy's csr_matvec (the oracle's `A @ v`), and, for B = A' from the stable device
// transpose, its csc_matvec of `A.T @ u` too; the epilogue keeps the closures' two roundings.
template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_spmv_seq(int64_t rows, const int64_t* __restrict__ rp,
                                                 const int32_t* __restrict__ ci, const T* __restrict__ val,
                                                 const T* __restrict__ x, T* y, T a, const T* z) {
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BS) {
        T s = 0;
        for (int64_t j = rp[r]; j < rp[r + 1]; ++j) {
            const T p = val[j] * x[ci[j]];
            s = s + p;
        }
        y[r] = apply_epi<T, EPI>(s, a, z, r);
    }
}

template <typename T>
static void spmv_seq(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z) {
    HGM_REQUIRE(epi == EPI_NONE || epi == EPI_ADD || epi == EPI_SUB || epi == EPI_RSUB,
                "parity mode: pending-normalisation epilogues are not used");
    const T* val = reinterpret_cast<const T*>(M->val);
    const dim3 g((unsigned)grid_for(M->rows)), b(BS);
    switch (epi) {
        case EPI_NONE: launch(c, true, k_spmv_seq<T, EPI_NONE>, g, b, M->rows, M->rp, M->ci, val, x, y, a, z); break;
        case EPI_ADD: launch(c, true, k_spmv_seq<T, EPI_ADD>, g, b, M->rows, M->rp, M->ci, val, x, y, a, z); break;
        case EPI_SUB: launch(c, true, k_spmv_seq<T, EPI_SUB>, g, b, M->rows, M->rp, M->ci, val, x, y, a, z); break;
        default: launch(c, true, k_spmv_seq<T, EPI_RSUB>, g, b, M->rows, M->rp, M->ci, val, x, y, a, z); break;
    }
}

int pick_group(int64_t rows, int64_t nnz) {
    const double avg = rows > 0 ? (double)nnz / (double)rows : 0.0;
    if (avg >= 128) return 64;
    if (avg >= 40) return 32;
    if (avg >= 16) return 16;
    if (avg >= 6) return 8;
    return 4;
}


template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_epi(int64_t n, T* __restrict__ y, T a, const T* __restrict__ z) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        y[i] = apply_epi<T, EPI>(y[i], a, z, i);
}


// ------------------------------------------------------------------------------
// launchers (every SpMV launch goes through hgm::launch so armed timing events ride
// in the dispatch packets of the first / last kernel of the product)
// ------------------------------------------------------------------------------
template <typename T, int G, int EPI, bool NT, typename IX, int CLS>
static void launch_stream_e(hgm_ctx* c, bool last, const SegIndex& si, const IX* ci, const T* val, const T* x,
                            T* out, T a, const T* z, T* head, T* tail, const PendNorm<T>& pn, const Paged<T>& pg) {
    if (si.nnz == 0) {
        int64_t g = (si.nseg + BS - 1) / BS;
        if (g > 4096) g = 4096;
        if (g > 0) launch(c, last, k_fill_epi<T, EPI>, dim3(g), dim3(BS), si.nseg, out, a, z);
        return;
    }
    if constexpr (std::is_same<IX, int32_t>::value) {
        if (pg.pptr)
            launch(c, false, k_spmv_stream<T, G, EPI, NT, IX, true, CLS>, dim3(si.nchunks), dim3(BS), si.nnz, si.nseg,
                   si.sp, si.fo, ci, val, x, out, a, z, head, tail, pn, pg);
        else
            launch(c, false, k_spmv_stream<T, G, EPI, NT, IX, false, CLS>, dim3(si.nchunks), dim3(BS), si.nnz, si.nseg,
                   si.sp, si.fo, ci, val, x, out, a, z, head, tail, pn, pg);
    } else {
        launch(c, false, k_spmv_stream<T, G, EPI, NT, IX, false, CLS>, dim3(si.nchunks), dim3(BS), si.nnz, si.nseg, si.sp,
               si.fo, ci, val, x, out, a, z, head, tail, pn, pg);
    }
    int64_t g = (si.nchunks + BS - 1) / BS;
    if (g > 4096) g = 4096;
    launch(c, last, k_stream_fixup<T, EPI>, dim3(g), dim3(BS), si.nnz, si.nchunks, si.sp, si.fo, out, a, z,
           (const T*)head, (const T*)tail, pn);
}

template <typename T, int G, bool NT, typename IX, int CLS>
static void launch_stream_g(hgm_ctx* c, bool last, const SegIndex& si, const IX* ci, const T* val, const T* x,
                            T* out, int epi, T a, const T* z, T* head, T* tail, const PendNorm<T>& pn,
                            const Paged<T>& pg) {
    switch (epi) {
        case EPI_NONE: launch_stream_e<T, G, EPI_NONE, NT, IX, CLS>(c, last, si, ci, val, x, out, a, z, head, tail, pn, pg); break;
        case EPI_ADD: launch_stream_e<T, G, EPI_ADD, NT, IX, CLS>(c, last, si, ci, val, x, out, a, z, head, tail, pn, pg); break;
        case EPI_SUB: launch_stream_e<T, G, EPI_SUB, NT, IX, CLS>(c, last, si, ci, val, x, out, a, z, head, tail, pn, pg); break;
        case EPI_ADDQ: launch_stream_e<T, G, EPI_ADDQ, NT, IX, CLS>(c, last, si, ci, val, x, out, a, z, head, tail, pn, pg); break;
        default: launch_stream_e<T, G, EPI_RSUB, NT, IX, CLS>(c, last, si, ci, val, x, out, a, z, head, tail, pn, pg); break;
    }
}

template <typename T, typename IX = int32_t>
static void spmv_stream(hgm_ctx* c, bool last, const SegIndex& si, int G, bool nt, const IX* ci, const T* val,
                        const T* x, T* out, int epi, T a, const T* z, const PendNorm<T>& pn = PendNorm<T>{},
                        const Paged<T>& pg = Paged<T>{}, int kclass = KC_SPMV_A) {
    T* head = c->buf<T>("stream_head", si.nchunks + 1);
    T* tail = c->buf<T>("stream_tail", si.nchunks + 1);
#define HGM_SG(GG)                                                                                          \
    if (kclass == KC_SPMV_B) {                                                                              \
        if (nt) launch_stream_g<T, GG, true, IX, KC_SPMV_B>(c, last, si, ci, val, x, out, epi, a, z, head, tail, pn, pg); \
        else launch_stream_g<T, GG, false, IX, KC_SPMV_B>(c, last, si, ci, val, x, out, epi, a, z, head, tail, pn, pg); \
    } else {                                                                                                \
        if (nt) launch_stream_g<T, GG, true, IX, KC_SPMV_A>(c, last, si, ci, val, x, out, epi, a, z, head, tail, pn, pg); \
        else launch_stream_g<T, GG, false, IX, KC_SPMV_A>(c, last, si, ci, val, x, out, epi, a, z, head, tail, pn, pg); \
    }
    switch (G) {
        case 64: HGM_SG(64) break;
        case 32: HGM_SG(32) break;
        case 16: HGM_SG(16) break;
        case 8: HGM_SG(8) break;
        case 2: HGM_SG(2) break;
        default: HGM_SG(4) break;
    }
#undef HGM_SG
}

template <typename T, int G, bool VEC, bool NT, typename IX = int32_t>
static void launch_spmv_v(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z,
                          const PendNorm<T>& pn) {
    const int64_t nb = (M->rows + (BS / G) - 1) / (BS / G);
    if (nb == 0) return;
    const T* val = reinterpret_cast<const T*>(M->val);
    const IX* ci = sizeof(IX) == 2 ? reinterpret_cast<const IX*>(M->ci16) : reinterpret_cast<const IX*>(M->ci);
    const int xcd = (M->variant & SPMV_XCD) ? 1 : 0;
    const dim3 g((unsigned)nb), b(BS);
    T* np_ = nullptr;
    switch (epi) {
        case EPI_NONE: launch(c, true, k_spmv<T, G, EPI_NONE, VEC, NT, false, IX>, g, b, M->rows, M->rp, ci, val, x, y, a, z, xcd, np_, pn); break;
        case EPI_ADD: launch(c, true, k_spmv<T, G, EPI_ADD, VEC, NT, false, IX>, g, b, M->rows, M->rp, ci, val, x, y, a, z, xcd, np_, pn); break;
        case EPI_SUB: launch(c, true, k_spmv<T, G, EPI_SUB, VEC, NT, false, IX>, g, b, M->rows, M->rp, ci, val, x, y, a, z, xcd, np_, pn); break;
        case EPI_DIVH: launch(c, true, k_spmv<T, G, EPI_DIVH, VEC, NT, false, IX>, g, b, M->rows, M->rp, ci, val, x, y, a, z, xcd, np_, pn); break;
        case EPI_ADDQ: launch(c, true, k_spmv<T, G, EPI_ADDQ, VEC, NT, false, IX>, g, b, M->rows, M->rp, ci, val, x, y, a, z, xcd, np_, pn); break;
        default: launch(c, true, k_spmv<T, G, EPI_RSUB, VEC, NT, false, IX>, g, b, M->rows, M->rp, ci, val, x, y, a, z, xcd, np_, pn); break;
    }
}

// row kernel with the fused sum of squares of the output (EPI_SUB / EPI_RSUB)
template <typename T, int G, bool VEC, bool NT>
static void launch_spmv_nrm_v(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z, T* out) {
    const int64_t nb = (M->rows + (BS / G) - 1) / (BS / G);
    if (nb == 0) {
        HGM_HIP(hipMemsetAsync(out, 0, sizeof(T), c->stream));
        return;
    }
    const T* val = reinterpret_cast<const T*>(M->val);
    const int xcd = (M->variant & SPMV_XCD) ? 1 : 0;
    T* parts = c->buf<T>("spmv_nparts", nb + 1);
    const dim3 g((unsigned)nb), b(BS);
    if (epi == EPI_SUB)
        launch(c, true, k_spmv<T, G, EPI_SUB, VEC, NT, true>, g, b, M->rows, M->rp, M->ci, val, x, y, a, z, xcd, parts,
               PendNorm<T>{});
    else
        launch(c, true, k_spmv<T, G, EPI_RSUB, VEC, NT, true>, g, b, M->rows, M->rp, M->ci, val, x, y, a, z, xcd, parts,
               PendNorm<T>{});
    hipLaunchKernelGGL(k_sum_parts<T>, dim3(1), dim3(BS), 0, c->stream, (const T*)parts, nb, out);
}

template <typename T, int G>
static void launch_spmv_g(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z, T* nrm,
                          const PendNorm<T>& pn) {
    const bool vec = M->variant & SPMV_VEC, nt = M->variant & SPMV_NT;
    if (nrm) {
        if (vec && nt) launch_spmv_nrm_v<T, G, true, true>(c, M, x, y, epi, a, z, nrm);
        else if (vec) launch_spmv_nrm_v<T, G, true, false>(c, M, x, y, epi, a, z, nrm);
        else if (nt) launch_spmv_nrm_v<T, G, false, true>(c, M, x, y, epi, a, z, nrm);
        else launch_spmv_nrm_v<T, G, false, false>(c, M, x, y, epi, a, z, nrm);
        return;
    }
    if (vec && nt) launch_spmv_v<T, G, true, true>(c, M, x, y, epi, a, z, pn);
    else if (vec) launch_spmv_v<T, G, true, false>(c, M, x, y, epi, a, z, pn);
    else if (M->ci16 && nt) launch_spmv_v<T, G, false, true, uint16_t>(c, M, x, y, epi, a, z, pn);
    else if (M->ci16) launch_spmv_v<T, G, false, false, uint16_t>(c, M, x, y, epi, a, z, pn);
    else if (nt) launch_spmv_v<T, G, false, true>(c, M, x, y, epi, a, z, pn);
    else launch_spmv_v<T, G, false, false>(c, M, x, y, epi, a, z, pn);
}

template <typename T, int G, bool VEC, bool NT>
static void launch_band_v(hgm_ctx* c, const hgm_mat* M, const T* x, T* yp) {
    constexpr int RPB = BS / G;
    const int64_t items = (M->rows + RPB - 1) / RPB * M->nbands;
    int64_t grid = 256 * 8;                      // ~all resident blocks, grid-stride in band-major order
    if (grid > items) grid = items;
    if (grid < 1) return;
    launch(c, false, k_spmv_band<T, G, VEC, NT>, dim3((unsigned)grid), dim3(BS), M->rows, M->nbands, M->brp, M->bci,
           reinterpret_cast<const T*>(M->bval), x, yp);
}

template <typename T, int G>
static void launch_band_g(hgm_ctx* c, const hgm_mat* M, const T* x, T* yp) {
    const bool vec = M->variant & SPMV_VEC, nt = M->variant & SPMV_NT;
    if (vec && nt) launch_band_v<T, G, true, true>(c, M, x, yp);
    else if (vec) launch_band_v<T, G, true, false>(c, M, x, yp);
    else if (nt) launch_band_v<T, G, false, true>(c, M, x, yp);
    else launch_band_v<T, G, false, false>(c, M, x, yp);
}

template <typename T, int EPI>
static void launch_band_reduce(hgm_ctx* c, const hgm_mat* M, const T* yp, T* y, T a, const T* z,
                               const PendNorm<T>& pn) {
    launch(c, true, k_band_reduce<T, EPI>, dim3(grid_for(M->rows)), dim3(BS), M->rows, M->nbands, yp, y, a, z, pn);
}

template <typename T>
static void band_reduce(hgm_ctx* c, const hgm_mat* M, const T* yp, T* y, int epi, T a, const T* z,
                        const PendNorm<T>& pn) {
    switch (epi) {
        case EPI_NONE: launch_band_reduce<T, EPI_NONE>(c, M, yp, y, a, z, pn); break;
        case EPI_ADD: launch_band_reduce<T, EPI_ADD>(c, M, yp, y, a, z, pn); break;
        case EPI_SUB: launch_band_reduce<T, EPI_SUB>(c, M, yp, y, a, z, pn); break;
        case EPI_DIVH: launch_band_reduce<T, EPI_DIVH>(c, M, yp, y, a, z, pn); break;
        case EPI_ADDQ: launch_band_reduce<T, EPI_ADDQ>(c, M, yp, y, a, z, pn); break;
        default: launch_band_reduce<T, EPI_RSUB>(c, M, yp, y, a, z, pn); break;
    }
}

template <typename T>
static void spmv_banded(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z,
                        const PendNorm<T>& pn) {
    T* yp = c->buf<T>("band_part", (size_t)M->nbands * M->rows + 1);
    switch (M->bgroup) {
        case 64: launch_band_g<T, 64>(c, M, x, yp); break;
        case 32: launch_band_g<T, 32>(c, M, x, yp); break;
        case 16: launch_band_g<T, 16>(c, M, x, yp); break;
        case 8: launch_band_g<T, 8>(c, M, x, yp); break;
        default: launch_band_g<T, 4>(c, M, x, yp); break;
    }
    band_reduce<T>(c, M, yp, y, epi, a, z, pn);
}

template <typename T>
static void spmv_streamed(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z,
                          const PendNorm<T>& pn, int kclass) {
    const int kc = kclass == KC_SPMV_B ? KC_SPMV_B : KC_SPMV_A;
    const bool nt = M->variant & SPMV_NT;
    // paged x gathers need the page index and a 16-B aligned x (vector page loads)
    Paged<T> pg;
    pg.xcd = (M->variant & SPMV_XCD) ? 1 : 0;
    if ((M->variant & SPMV_PAGED) && M->pg_ptr && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        pg.pptr = M->pg_ptr;
        pg.pids = M->pg_ids;
        pg.lidx = M->pg_lidx;
        pg.xlen = M->cols;
    }
    if (M->nbands > 1) {
        T* yp = c->buf<T>("band_part", (size_t)M->nbands * M->rows + 1);
        SegIndex si{M->nnz, (int64_t)M->nbands * M->rows, stream_chunks(M->nnz), M->brp, M->bcfo};
        spmv_stream<T>(c, false, si, M->bsgroup, nt, M->bci, reinterpret_cast<const T*>(M->bval), x, yp, EPI_NONE,
                       T(0), nullptr, PendNorm<T>{}, pg, kc);
        band_reduce<T>(c, M, yp, y, epi, a, z, pn);
    } else {
        SegIndex si{M->nnz, M->rows, stream_chunks(M->nnz), M->rp, M->cfo};
        // 16-bit column indices (<= 65,536 columns) unless the paged gathers are on: those read
        // 16-bit page-local indices instead, and only chunks past the page limit read M->ci
        if (M->ci16 && !(pg.pptr && c->num.paged16))
            spmv_stream<T, uint16_t>(c, true, si, M->sgroup, nt, M->ci16, reinterpret_cast<const T*>(M->val), x, y,
                                     epi, a, z, pn, pg, kc);
        else
            spmv_stream<T>(c, true, si, M->sgroup, nt, M->ci, reinterpret_cast<const T*>(M->val), x, y, epi, a, z, pn,
                           pg, kc);
    }
}

bool spmv_pn_ok(const hgm_mat* M, int epi) {
    if (M->nnz == 0) return false;
    const bool stream = (M->variant & SPMV_STREAM) && (M->nbands > 1 ? M->bcfo != nullptr : M->cfo != nullptr);
    if (epi == EPI_DIVH) return !(stream && M->nbands <= 1);   // row kernel or band reduction
    return epi == EPI_ADDQ;
}

template <typename T>
void spmv(hgm_ctx* c, const hgm_mat* M, const T* x, T* y, int epi, T a, const T* z, int kclass, T* sumsq_out,
          const PendNorm<T>* pnp) {
    const PendNorm<T> pn = pnp ? *pnp : PendNorm<T>{};
    HGM_REQUIRE((epi != EPI_DIVH && epi != EPI_ADDQ) || (pnp && spmv_pn_ok(M, epi)), "spmv: pending-norm epilogue");
    hipEvent_t t0 = nullptr;
    timing_begin(c, kclass, &t0);
    const bool stream = (M->variant & SPMV_STREAM) && (M->nbands > 1 ? M->bcfo != nullptr : M->cfo != nullptr);
    const bool rowk = !stream && M->nbands <= 1;
    T* nrm = (rowk && !c->num.parity && (epi == EPI_SUB || epi == EPI_RSUB)) ? sumsq_out : nullptr;
    if (c->num.parity) {
        spmv_seq<T>(c, M, x, y, epi, a, z);
    } else if (stream) {
        spmv_streamed<T>(c, M, x, y, epi, a, z, pn, kclass);
    } else if (M->nbands > 1) {
        spmv_banded<T>(c, M, x, y, epi, a, z, pn);
    } else {
        switch (M->group) {
            case 64: launch_spmv_g<T, 64>(c, M, x, y, epi, a, z, nrm, pn); break;
            case 32: launch_spmv_g<T, 32>(c, M, x, y, epi, a, z, nrm, pn); break;
            case 16: launch_spmv_g<T, 16>(c, M, x, y, epi, a, z, nrm, pn); break;
            case 8: launch_spmv_g<T, 8>(c, M, x, y, epi, a, z, nrm, pn); break;
            default: launch_spmv_g<T, 4>(c, M, x, y, epi, a, z, nrm, pn); break;
        }
    }
    // other kernels: separate fixed-order reduction of the output
    if (sumsq_out && !nrm) sumsq<T>(c, M->rows, y, sumsq_out);
    HGM_HIP(hipGetLastError());
    // algorithmic bytes: nnz*(s+4) + 8(rows+1) + s*cols + s*rows (+ s*rows epilogue operand)
    const double s = sizeof(T);
    // 16-bit indices read (row kernel without paired loads, or the unbanded streaming kernel)
    // (the paged kernel also reads 2-byte indices, plus its page lists; the roofline keeps
    // SURVEY.md §8(d)'s 4-byte CSR definition of the work and reports the physical bytes as traffic)
    const bool narrow = M->ci16 && ((rowk && !nrm && !(M->variant & SPMV_VEC)) || (stream && M->nbands <= 1));
    double bytes = (double)M->nnz * (s + (narrow ? 2 : 4)) + 8.0 * (M->rows + 1) + s * M->cols + s * M->rows;
    if (epi != EPI_NONE && epi != EPI_DIVH) bytes += s * M->rows;   // epilogue operand read
    if (epi == EPI_ADDQ) bytes += s * M->rows;                       // ... and the normalised q written back
    timing_end(c, kclass, t0, bytes);
}

template <typename T>
void epilogue(hgm_ctx* c, int64_t n, T* y, int epi, T a, const T* z) {
    const int g = grid_for(n);
    switch (epi) {
        case EPI_ADD: k_epi<T, EPI_ADD><<<g, BS, 0, c->stream>>>(n, y, a, z); break;
        case EPI_SUB: k_epi<T, EPI_SUB><<<g, BS, 0, c->stream>>>(n, y, a, z); break;
        case EPI_RSUB: k_epi<T, EPI_RSUB><<<g, BS, 0, c->stream>>>(n, y, a, z); break;
        default: return;
    }
    HGM_HIP(hipGetLastError());
}

template <typename T, int EPI>
__global__ __launch_bounds__(BS) void k_epi_to(int64_t n, const T* __restrict__ in, T* out, T a, const T* z) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS)
        out[i] = apply_epi<T, EPI>(in[i], a, z, i);
}

template <typename T>
void epilogue_to(hgm_ctx* c, int64_t n, const T* in, T* out, int epi, T a, const T* z) {
    const int g = grid_for(n);
    switch (epi) {
        case EPI_ADD: k_epi_to<T, EPI_ADD><<<g, BS, 0, c->stream>>>(n, in, out, a, z); break;
        case EPI_SUB: k_epi_to<T, EPI_SUB><<<g, BS, 0, c->stream>>>(n, in, out, a, z); break;
        case EPI_RSUB: k_epi_to<T, EPI_RSUB><<<g, BS, 0, c->stream>>>(n, in, out, a, z); break;
        default:
            if (in != out) HGM_HIP(hipMemcpyAsync(out, in, sizeof(T) * n, hipMemcpyDeviceToDevice, c->stream));
            return;
    }
    HGM_HIP(hipGetLastError());
}
template void epilogue_to<double>(hgm_ctx*, int64_t, const double*, double*, int, double, const double*);
template void epilogue_to<float>(hgm_ctx*, int64_t, const float*, float*, int, float, const float*);

template void spmv<double>(hgm_ctx*, const hgm_mat*, const double*, double*, int, double, const double*, int, double*,
                           const PendNorm<double>*);
template void spmv<float>(hgm_ctx*, const hgm_mat*, const float*, float*, int, float, const float*, int, float*,
                          const PendNorm<float>*);
template void epilogue<double>(hgm_ctx*, int64_t, double*, int, double, const double*);
template void epilogue<float>(hgm_ctx*, int64_t, float*, int, float, const float*);

}  // namespace hgm
