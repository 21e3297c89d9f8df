// Sparse operator construction on the device (gfx950):
//  * deterministic CSR transpose (ray-major A <-> pixel-major A^T / MATLAB CSC hand-over),
//  * parallel-beam Siddon projector generated ray-per-thread directly into CSR
//    (same geometry and floating-point operation order as
//    hgmres/problems.py so the two generators agree bit for bit).
#include <hipcub/hipcub.hpp>

#include <atomic>
#include <climits>
#include <cmath>
#include <cstdlib>

#include "internal.h"

namespace hgm {

hgm_mat* mat_alloc(hgm_ctx* c, int64_t rows, int64_t cols, int64_t nnz, int dtype) {
    static std::atomic<uint64_t> next_uid{0};
    hgm_mat* M = new hgm_mat();
    M->uid = ++next_uid;
    M->ctx = c;
    M->rows = rows;
    M->cols = cols;
    M->nnz = nnz;
    M->dtype = dtype;
    const size_t vs = dtype == HGM_F32 ? 4 : 8;
    if (hipMalloc(&M->rp, sizeof(int64_t) * (rows + 1)) != hipSuccess ||
        hipMalloc(&M->ci, sizeof(int32_t) * (nnz > 0 ? nnz : 1)) != hipSuccess ||
        hipMalloc(&M->val, vs * (nnz + 4)) != hipSuccess) {   // (+4: whole 16-byte loads at the end, fused.hip)
        mat_free(M);
        throw Error{HGM_E_NOMEM, "hipMalloc failed for sparse matrix"};
    }
    M->group = pick_group(rows, nnz);
    M->variant = SPMV_VEC;
    return M;
}

static int grid_cap(int64_t n);

__global__ __launch_bounds__(BS) void k_rebase(int64_t n, const int64_t* __restrict__ in, int64_t base,
                                               int64_t* __restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = in[i] - base;
}

// rows [lo, hi) of M as a new operator (same columns): B_g = B(P_g,:) of a pixel shard
hgm_mat* row_slice(hgm_ctx* c, const hgm_mat* M, int64_t lo, int64_t hi) {
    HGM_REQUIRE(0 <= lo && lo <= hi && hi <= M->rows, "row_slice: need 0 <= lo <= hi <= rows");
    // tiled rows: [lo, hi) are STORED positions, and the slice numbers its rows in that stored
    // order (a shard-local index space, reported as the trivial order)
    hipStream_t st = c->stream;
    int64_t b[2];
    HGM_HIP(hipMemcpy(&b[0], M->rp + lo, sizeof(int64_t), hipMemcpyDeviceToHost));
    HGM_HIP(hipMemcpy(&b[1], M->rp + hi, sizeof(int64_t), hipMemcpyDeviceToHost));
    hgm_mat* S = mat_alloc(c, hi - lo, M->cols, b[1] - b[0], M->dtype);
    S->col_order = M->col_order;
    // a window of whole tile columns keeps the grid's strip geometry (dual bands of A_g = S')
    const PixOrder& ro = !M->row_order.trivial() ? M->row_order : M->row_grid;
    if (!ro.trivial() && ro.super <= 1 && lo % ((int64_t)std::max(ro.tile, 1) * ro.N) == 0) S->row_grid = ro;
    try {
        k_rebase<<<grid_cap(hi - lo + 1), BS, 0, st>>>(hi - lo + 1, M->rp + lo, b[0], S->rp);
        HGM_HIP(hipGetLastError());
        const size_t vs = M->dtype == HGM_F32 ? 4 : 8;
        if (S->nnz) {
            HGM_HIP(hipMemcpyAsync(S->ci, M->ci + b[0], sizeof(int32_t) * S->nnz, hipMemcpyDeviceToDevice, st));
            HGM_HIP(hipMemcpyAsync(S->val, static_cast<const char*>(M->val) + vs * b[0], vs * S->nnz,
                                   hipMemcpyDeviceToDevice, st));
        }
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        mat_free(S);
        throw;
    }
    return S;
}

// fo[k] = first segment starting at or after chunk k's first entry; fo[nchunks] = nseg
__global__ void k_chunk_fo(int64_t nchunks, int64_t nseg, const int64_t* __restrict__ sp, int32_t* __restrict__ fo) {
    for (int64_t k = (int64_t)blockIdx.x * BS + threadIdx.x; k <= nchunks; k += (int64_t)gridDim.x * BS) {
        if (k == nchunks) {
            fo[k] = (int32_t)nseg;
            continue;
        }
        const int64_t c0 = k * SCH;
        int64_t lo = 0, hi = nseg;          // lower_bound over sp[0..nseg]
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (sp[mid] < c0) lo = mid + 1;
            else hi = mid;
        }
        fo[k] = (int32_t)lo;
    }
}

static int32_t* build_chunk_index(hgm_ctx* c, const int64_t* sp, int64_t nseg, int64_t nnz) {
    const int64_t nch = stream_chunks(nnz);
    int32_t* fo = nullptr;
    HGM_HIP(hipMalloc(&fo, sizeof(int32_t) * (nch + 1)));
    k_chunk_fo<<<grid_cap(nch + 1), BS, 0, c->stream>>>(nch, nseg, sp, fo);
    HGM_HIP(hipGetLastError());
    return fo;
}

static int stream_group(double avg) {
    return avg >= 512 ? 64 : (avg >= 128 ? 32 : (avg >= 40 ? 16 : 8));
}

void build_stream_index(hgm_ctx* c, hgm_mat* M) {
    HGM_REQUIRE(M->rows < (int64_t)INT32_MAX, "stream index: rows must be < 2^31");
    if (M->cfo) (void)hipFree(M->cfo);
    M->cfo = build_chunk_index(c, M->rp, M->rows, M->nnz);
    M->sgroup = stream_group(M->rows ? (double)M->nnz / M->rows : 0.0);
    HGM_HIP(hipStreamSynchronize(c->stream));
}

// --------------------------------------------------------------------------
// x-page index of the paged streaming kernel (spmv.hip).  One 256-thread block per chunk of
// SCH entries: block radix sort of (page, position) pairs, head flags, block scan -> slots.
// Pass 0 counts the distinct pages (0 when more than PGMAX, the LDS budget times pg_rounds: the
// chunk keeps the 32-bit gathers); pass 1 writes the page list and the page-local 16-bit indices
// (slot x values per page + offset; the kernel stages slots [0, pg_max) first, then the rest).
// --------------------------------------------------------------------------
template <int PGV, int PGMAX, bool FILL>
__global__ __launch_bounds__(256) void k_page_index(int64_t nnz, const int32_t* __restrict__ ci,
                                                    int32_t* __restrict__ cnt, const int32_t* __restrict__ pptr,
                                                    int32_t* __restrict__ pids, uint16_t* __restrict__ lidx) {
    constexpr int IPT = SCH / 256;
    using Sort = hipcub::BlockRadixSort<int, 256, IPT, int>;
    using Scan = hipcub::BlockScan<int, 256>;
    __shared__ typename Sort::TempStorage ts;
    __shared__ typename Scan::TempStorage tsc;
    __shared__ int last_key[256];
    const int64_t k = blockIdx.x, c0 = k * SCH;
    int keys[IPT], vals[IPT];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const int pos = threadIdx.x * IPT + i;
        const int64_t e = c0 + pos;
        if (e < nnz) {
            const int col = ci[e];
            keys[i] = col / PGV;
            vals[i] = (pos << 6) | (col % PGV);
        } else {
            keys[i] = INT_MAX;
            vals[i] = -1;
        }
    }
    Sort(ts).Sort(keys, vals);            // blocked: thread t holds sorted items [IPT t, IPT t + IPT)
    last_key[threadIdx.x] = keys[IPT - 1];
    __syncthreads();
    int flag[IPT], heads = 0;
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        const int prev = i > 0 ? keys[i - 1] : (threadIdx.x > 0 ? last_key[threadIdx.x - 1] : -1);
        flag[i] = (keys[i] != INT_MAX && keys[i] != prev) ? 1 : 0;
        heads += flag[i];
    }
    int excl = 0, total = 0;
    Scan(tsc).ExclusiveSum(heads, excl, total);
    const bool fits = total <= PGMAX && c0 + SCH <= nnz;   // full chunks only
    if (!FILL) {
        if (threadIdx.x == 0) cnt[k] = fits ? total : 0;
        return;
    }
    if (!fits) return;
    int slot = excl - 1;
    const int base = pptr[k];
#pragma unroll
    for (int i = 0; i < IPT; ++i) {
        if (keys[i] == INT_MAX) continue;
        if (flag[i]) {
            ++slot;
            pids[base + slot] = keys[i];
        }
        lidx[c0 + (vals[i] >> 6)] = (uint16_t)(slot * PGV + (vals[i] & 63));
    }
}

void free_page_index(hgm_mat* M) {
    if (M->pg_ptr) (void)hipFree(M->pg_ptr);
    if (M->pg_ids) (void)hipFree(M->pg_ids);
    if (M->pg_lidx) (void)hipFree(M->pg_lidx);
    M->pg_ptr = M->pg_ids = nullptr;
    M->pg_lidx = nullptr;
    M->variant &= ~SPMV_PAGED;
}

template <int PGV, int PGMAX>
static void build_page_index_t(hgm_ctx* c, hgm_mat* M) {
    const bool banded = M->nbands > 1;
    const int32_t* ci = banded ? M->bci : M->ci;
    const int64_t nch = stream_chunks(M->nnz);
    hipStream_t st = c->stream;
    int32_t* cnt = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    try {
        HGM_HIP(hipMalloc(&cnt, sizeof(int32_t) * (nch + 1)));
        HGM_HIP(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (nch + 1), st));
        HGM_HIP(hipMalloc(&M->pg_ptr, sizeof(int32_t) * (nch + 1)));
        k_page_index<PGV, PGMAX, false><<<(unsigned)nch, 256, 0, st>>>(M->nnz, ci, cnt, nullptr, nullptr, nullptr);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, M->pg_ptr, (int)(nch + 1), st));
        HGM_HIP(hipMalloc(&tmp, tmp_bytes));
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, M->pg_ptr, (int)(nch + 1), st));
        int32_t total = 0;
        HGM_HIP(hipMemcpyAsync(&total, M->pg_ptr + nch, sizeof(int32_t), hipMemcpyDeviceToHost, st));
        HGM_HIP(hipStreamSynchronize(st));
        HGM_HIP(hipMalloc(&M->pg_ids, sizeof(int32_t) * (total > 0 ? total : 1)));
        HGM_HIP(hipMalloc(&M->pg_lidx, sizeof(uint16_t) * M->nnz));
        k_page_index<PGV, PGMAX, true><<<(unsigned)nch, 256, 0, st>>>(M->nnz, ci, nullptr, M->pg_ptr, M->pg_ids,
                                                                     M->pg_lidx);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        (void)hipFree(cnt);
        (void)hipFree(tmp);
        free_page_index(M);
        throw;
    }
    (void)hipFree(cnt);
    (void)hipFree(tmp);
}

void build_page_index(hgm_ctx* c, hgm_mat* M) {
    free_page_index(M);
    HGM_REQUIRE(stream_chunks(M->nnz) < (int64_t)INT32_MAX, "page index: too many chunks");
    if (M->nnz < SCH) return;
    // (PGMAX: the pages a chunk may touch, over all its LDS rounds)
    if (M->dtype == HGM_F32) build_page_index_t<PG_BYTES / 4, pg_max<float>() * pg_rounds<float>()>(c, M);
    else build_page_index_t<PG_BYTES / 8, pg_max<double>() * pg_rounds<double>()>(c, M);
    M->variant |= SPMV_PAGED;
}

static void free_bands(hgm_mat* M) {
    if (M->bcfo) (void)hipFree(M->bcfo);
    M->bcfo = nullptr;
    if (M->brp) (void)hipFree(M->brp);
    if (M->bci) (void)hipFree(M->bci);
    if (M->bval) (void)hipFree(M->bval);
    M->brp = nullptr;
    M->bci = nullptr;
    M->bval = nullptr;
    M->nbands = 0;
    M->band_w = 0;
    M->band_dual = false;
}

void mat_free(hgm_mat* M) {
    if (!M) return;
    fused_plan_free(M->fused);
    free_page_index(M);
    free_bands(M);
    if (M->ci16) (void)hipFree(M->ci16);
    if (M->cfo) (void)hipFree(M->cfo);
    if (M->rp) (void)hipFree(M->rp);
    if (M->ci) (void)hipFree(M->ci);
    if (M->val) (void)hipFree(M->val);
    delete M;
}

// --------------------------------------------------------------------------
// column bands (cache blocking of the x gather for long-row operators)
// --------------------------------------------------------------------------
// Band of a stored column.  Column strips: s / W.  Dual (tiled N x N grid): a
// steep row (pixel-row span > pixel-column span) takes the strip of h = W / N pixel ROWS its
// pixel lies in instead; in the tile-column-major order that is (s mod tile*N) / (h*tile).
struct BandKey {
    int64_t W = 0;
    int dual = 0, tile = 1;
    int64_t N = 0, tN = 0, rdiv = 1;
};

__device__ __forceinline__ bool row_steep(const BandKey& k, const int64_t* __restrict__ rp,
                                          const int32_t* __restrict__ ci, int64_t r) {
    if (!k.dual) return false;
    const int64_t t = k.tile, Nt = k.N / t;
    int64_t rmin = INT64_MAX, rmax = -1, cmin = INT64_MAX, cmax = -1;
    for (int64_t i = rp[r]; i < rp[r + 1]; ++i) {
        const int64_t s = ci[i], q = s / (t * t);
        const int64_t pr = (q % Nt) * t + s % t, pc = (q / Nt) * t + (s / t) % t;
        rmin = pr < rmin ? pr : rmin;
        rmax = pr > rmax ? pr : rmax;
        cmin = pc < cmin ? pc : cmin;
        cmax = pc > cmax ? pc : cmax;
    }
    return rmax >= 0 && rmax - rmin > cmax - cmin;
}

__device__ __forceinline__ int64_t band_of(const BandKey& k, int64_t s, bool steep) {
    return steep ? (s % k.tN) / k.rdiv : s / k.W;
}

// one thread per row, sequential over the row (each row is owned by one thread: no races)
__global__ void k_band_count(int64_t rows, BandKey key, const int64_t* __restrict__ rp,
                             const int32_t* __restrict__ ci, int64_t* __restrict__ cnt) {
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BS) {
        const bool steep = row_steep(key, rp, ci, r);
        for (int64_t i = rp[r]; i < rp[r + 1]; ++i) cnt[band_of(key, ci[i], steep) * rows + r] += 1;
    }
}

template <typename T>
__global__ void k_band_fill(int64_t rows, BandKey key, const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                            const T* __restrict__ val, int64_t* __restrict__ cur, int32_t* __restrict__ bci,
                            T* __restrict__ bval) {
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < rows; r += (int64_t)gridDim.x * BS) {
        const bool steep = row_steep(key, rp, ci, r);
        for (int64_t i = rp[r]; i < rp[r + 1]; ++i) {
            const int64_t p = cur[band_of(key, ci[i], steep) * rows + r]++;
            bci[p] = ci[i];
            bval[p] = val[i];
        }
    }
}

// Kernel defaults from the gfx950 sweep (profiles/):
//   long rows (ray-major A), x within one XCD's L2  -> row kernel, 32 lanes/row, 16-B loads
//   long rows, x beyond L2                          -> 128 Ki-pixel column bands + streaming kernel
//   short rows (pixel-major B), < 5e7 nnz           -> row kernel, 8 lanes/row, 8-B loads
//   short rows, >= 5e7 nnz                          -> streaming kernel, nontemporal loads
__global__ void k_narrow_ci(int64_t nnz, const int32_t* __restrict__ ci, uint16_t* __restrict__ o) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * BS)
        o[i] = (uint16_t)ci[i];
}

// 16-bit column indices for operators with <= 65536 columns (the pixel-major B of C2/C3,
// whose columns are rays): 10 instead of 12 bytes per fp64 entry for the row kernel.
static void build_ci16(hgm_ctx* c, hgm_mat* M) {
    if (M->ci16) (void)hipFree(M->ci16);
    M->ci16 = nullptr;
    if (M->nnz == 0 || M->cols > 65536) return;
    HGM_HIP(hipMalloc(&M->ci16, sizeof(uint16_t) * M->nnz));
    k_narrow_ci<<<grid_cap(M->nnz), BS, 0, c->stream>>>(M->nnz, M->ci, M->ci16);
    HGM_HIP(hipGetLastError());
}

#ifndef HGM_A_BSGROUP
#define HGM_A_BSGROUP 4
#endif
#ifndef HGM_B_SGROUP
#define HGM_B_SGROUP 2
#endif
void finalize_operator(hgm_ctx* c, hgm_mat* M) {
    if (M->nnz > 0) build_stream_index(c, M);
    build_ci16(c, M);
    const double avg = M->rows ? (double)M->nnz / (double)M->rows : 0.0;
    set_bands(c, M, auto_band_width(M));
    if (avg >= 64) {
        if (M->nbands > 1) {
            // the streaming kernel over the (band,row) segments, 4 lanes per segment (set_bands);
            // the wider bands also gain from nontemporal val/col loads (C4 sweeps,
            // profiles/r1_spmv_sweep_c4_*.jsonl; reference order 2.96 ms vs 4.18 ms at 32 lanes)
            M->variant = SPMV_STREAM | SPMV_NT;
            // XCD-contiguous chunk order: each XCD streams its own bands, so a band's x-slice is
            // fetched into one L2 instead of eight (paged kernel, alternating runs: C4 A 2.36 ->
            // 2.31 ms, C3 A 252 -> 238 us, bitwise equal; profiles/r2_c{3,4}_xcd.log)
            M->variant |= SPMV_XCD;
        } else if (M->nnz >= 50000000 && avg <= 256 &&
                   (double)M->cols * (M->dtype == HGM_F64 ? 8.0 : 4.0) <= 4.0 * 1024 * 1024) {
            // long rows over an L2-resident x at >= 5e7 nnz: the unmatched pixel-driven
            // back-projector of C4 (94 entries per pixel row, 1.6e9 nnz; bench.py --unmatched).
            // Paged streaming with 4 lanes per row: 4.10 -> 2.61 ms (row kernel, 16 lanes), 2 / 8
            // lanes 2.79 / 2.87 ms, unpaged 3.74 ms (profiles/r4_unmatched_c4_b_variants.log).
            // Gated on the shape it was measured on: rows of <= 256 entries and an
            // x (2.2 MB there) that fits one XCD's 4 MiB L2; other single-band operators keep the
            // row kernel below.
            M->variant = SPMV_STREAM | SPMV_NT;
            M->sgroup = 4;
        } else {
            // C2 A (460-entry rays, x L2-resident): 16 lanes per row beats 32 in the solve
            // (33.0 vs 34.6 us, alternating runs, scripts/ab_compare.sh)
            M->variant = SPMV_VEC;
            M->group = avg < 1024 ? 16 : 32;
        }
    } else {
        if (M->nnz >= 50000000) {
            // C3/C4 sweeps: nontemporal val/col loads, and 2 lanes per pixel row in the segment
            // reduction (round 3, isolated paged kernel: C4 B 2.02 -> 1.93 ms, C3 B 210 -> 207 us
            // against 4 lanes; profiles/r3_stream_g2.log)
            M->variant = SPMV_STREAM | SPMV_NT;
            M->sgroup = HGM_B_SGROUP;
        } else {
            M->variant = 0;
            M->group = avg >= 6 ? 8 : 4;
        }
    }
    // streaming operators gather x through LDS-staged pages
    if (M->variant & SPMV_STREAM) build_page_index(c, M);
}

int64_t auto_band_width(const hgm_mat* M) {
    const size_t vs = M->dtype == HGM_F32 ? 4 : 8;
    // x fits comfortably in one XCD's 4 MiB L2: no banding
    if ((double)M->cols * vs <= 4.0 * 1024 * 1024) return 0;
    // only long-row operators benefit (the short pixel-major rows of B gather an L2-resident y)
    if (M->rows > 0 && (double)M->nnz / (double)M->rows < 64) return 0;
    // tiled pixel order (tile-column-major): a strip of 64 pixel columns, 64 N pixels.  The paged
    // stream kernel's sweeps (profiles/r2_c{3,4}_bands*.log) put the optimum there at both sizes:
    // C4 (N = 4096) 262,144 pixels, 2.20 ms against 2.25 (128 Ki) and 2.38 (512 Ki); C3
    // (N = 2048) 131,072 pixels, 254-257 us against 269 (256 Ki) and 259 (64 Ki).
    if (!M->col_order.trivial() && M->col_order.super == 0) return (int64_t)64 * M->col_order.N;
    // super-blocks: 256 Ki pixels (2 MiB fp64 x-slice)
    if (!M->col_order.trivial()) return (int64_t)(1 << 18);
    return (int64_t)(1 << 17);   // 128 Ki pixels = 1 MiB fp64 x-slice per band
}

void set_bands(hgm_ctx* c, hgm_mat* M, int64_t W) {
    free_page_index(M);   // it indexes the stream the bands replace; the caller rebuilds it
    free_bands(M);
    if (W <= 0 || W >= M->cols || M->nnz == 0) return;
    // dual strips: the columns are a window of whole tile columns of a tiled
    // N x N grid (the full grid, or a pixel shard's slice of it).  Steep rows take strips of h
    // pixel rows of the same pixel count as a column strip: h = W N / cols (64 on the full grid).
    BandKey key;
    key.W = W;
    int64_t nb = (M->cols + W - 1) / W;
    const PixOrder& o = !M->col_order.trivial() ? M->col_order : M->col_grid;
    if (c->num.band_dual && !o.trivial() && o.super <= 1 && o.N > 0) {
        const int64_t t = o.tile > 1 ? o.tile : 1, tN = t * o.N;
        int64_t h = (int64_t)((double)W * o.N / (double)M->cols + 0.5);
        h = (h + t - 1) / t * t;
        // narrow shards: strips of h >= 4 W / N rows are as slow as the column strips (4 shards of
        // C4) or slower (8 shards: A_g 0.305 -> 0.336 ms); strips of W / N rows there multiply
        // the band count (4-6x slower).  Full grid and halves gain (C4 A 2.27 -> 2.11 ms, half
        // 1.14-1.18 -> 1.11 ms; profiles/r2_shard_kernels_dual.log)
        if (o.N % t == 0 && M->cols % tN == 0 && M->cols <= (int64_t)o.N * o.N && h >= t && h < o.N &&
            h * o.N <= 2 * W) {
            key.dual = 1;
            key.tile = (int)t;
            key.N = o.N;
            key.tN = tN;
            key.rdiv = h * t;
            nb = std::max(nb, (o.N + h - 1) / h);
        }
    }
    HGM_REQUIRE(nb * M->rows + 1 < (int64_t)INT32_MAX, "set_bands: too many (band,row) segments");
    hipStream_t st = c->stream;
    const size_t vs = M->dtype == HGM_F32 ? 4 : 8;
    const int64_t nseg = nb * M->rows;
    int64_t* cnt = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    try {
        HGM_HIP(hipMalloc(&M->brp, sizeof(int64_t) * (nseg + 1)));
        HGM_HIP(hipMalloc(&M->bci, sizeof(int32_t) * M->nnz));
        HGM_HIP(hipMalloc(&M->bval, vs * M->nnz));
        HGM_HIP(hipMalloc(&cnt, sizeof(int64_t) * (nseg + 1)));
        HGM_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (nseg + 1), st));
        const int g = grid_cap(M->rows);
        k_band_count<<<g, BS, 0, st>>>(M->rows, key, M->rp, M->ci, cnt);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, cnt, M->brp, (int)(nseg + 1), st));
        HGM_HIP(hipMalloc(&tmp, tmp_bytes));
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, cnt, M->brp, (int)(nseg + 1), st));
        HGM_HIP(hipMemcpyAsync(cnt, M->brp, sizeof(int64_t) * (nseg + 1), hipMemcpyDeviceToDevice, st));
        if (M->dtype == HGM_F32)
            k_band_fill<float><<<g, BS, 0, st>>>(M->rows, key, M->rp, M->ci, (const float*)M->val, cnt, M->bci, (float*)M->bval);
        else
            k_band_fill<double><<<g, BS, 0, st>>>(M->rows, key, M->rp, M->ci, (const double*)M->val, cnt, M->bci, (double*)M->bval);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        (void)hipFree(cnt);
        (void)hipFree(tmp);
        free_bands(M);
        throw;
    }
    (void)hipFree(cnt);
    (void)hipFree(tmp);
    M->band_w = W;
    M->nbands = (int)nb;
    M->band_dual = key.dual != 0;
    const double avg = (double)M->nnz / (double)nseg;
    M->bgroup = avg >= 96 ? 32 : (avg >= 24 ? 16 : 8);
    // streaming index over the (band,row) segments; ~2/3 of them are non-empty for a
    // parallel-beam operator, hence the 1.5 factor in the average segment length
    M->bcfo = build_chunk_index(c, M->brp, nseg, M->nnz);
    const double row_avg = (double)M->nnz / (double)(M->rows > 0 ? M->rows : 1);
    M->bsgroup = stream_group(row_avg / (double)(nb > 0 ? nb : 1) * 1.5);
    // long-row (ray-major) operators: band segments are short ray chords (tens to hundreds of
    // entries), and 4 lanes per segment keeps every lane busy (C4 sweeps,
    // profiles/r1_spmv_sweep_c4_*.jsonl: 2.90 ms vs 3.31 ms at 16 lanes).  Set here so that
    // hgm_mat_set_bands keeps it too (a 64-column re-band at 8/16 lanes cost the C4 shards
    // 2.57 vs 2.27 ms, profiles/r2_shard_order.log)
    // (round 3: 2 lanes helps fp32 only: C5 A 1.274 -> 1.258 ms in the solve, but C4 A 2.12 ->
    // 2.17 ms and C3 A 226 -> 230 us in fp64; profiles/r3_ab_a2.log)
    if (row_avg >= 64) M->bsgroup = M->dtype == HGM_F32 ? 2 : HGM_A_BSGROUP;
    HGM_HIP(hipStreamSynchronize(st));
}

// --------------------------------------------------------------------------
// transpose
// --------------------------------------------------------------------------
__global__ void k_expand_rows(int64_t rows, const int64_t* __restrict__ rp, int32_t* __restrict__ ridx) {
    // one wave per row
    const int64_t row = (int64_t)blockIdx.x * (BS / 64) + threadIdx.x / 64;
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    for (int64_t i = rp[row] + lane; i < rp[row + 1]; i += 64) ridx[i] = (int32_t)row;
}

__global__ void k_iota(int64_t n, int32_t* out) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) out[i] = (int32_t)i;
}

// row pointer of the transpose from the sorted column keys: rp[c] = first index with key >= c
__global__ void k_bounds(int64_t nnz, int64_t cols, const int32_t* __restrict__ keys, int64_t* __restrict__ rp) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i <= nnz; i += (int64_t)gridDim.x * BS) {
        const int64_t kprev = (i == 0) ? -1 : (int64_t)keys[i - 1];
        const int64_t kcur = (i == nnz) ? cols : (int64_t)keys[i];
        for (int64_t cc = kprev + 1; cc <= kcur; ++cc) rp[cc] = i;
    }
}

template <typename T>
__global__ void k_gather_t(int64_t nnz, const int32_t* __restrict__ perm, const int32_t* __restrict__ ridx,
                           const T* __restrict__ vin, int32_t* __restrict__ ci_out, T* __restrict__ vout) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nnz; i += (int64_t)gridDim.x * BS) {
        const int32_t p = perm[i];
        ci_out[i] = ridx[p];
        vout[i] = vin[p];
    }
}

static int grid_cap(int64_t n) {
    int64_t g = (n + BS - 1) / BS;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return (int)g;
}

hgm_mat* transpose(hgm_ctx* c, const hgm_mat* M) {
    HGM_REQUIRE(M->nnz < (int64_t)INT32_MAX, "transpose: nnz must be < 2^31");
    HGM_REQUIRE(M->cols < (int64_t)INT32_MAX && M->rows < (int64_t)INT32_MAX, "transpose: dims must be < 2^31");
    hipStream_t st = c->stream;
    const int64_t nnz = M->nnz;
    hgm_mat* T = mat_alloc(c, M->cols, M->rows, nnz, M->dtype);
    T->row_order = M->col_order;
    T->col_order = M->row_order;
    T->row_grid = M->col_grid;
    T->col_grid = M->row_grid;
    T->transpose_of = M->uid;
    if (nnz == 0) {
        HGM_HIP(hipMemsetAsync(T->rp, 0, sizeof(int64_t) * (T->rows + 1), st));
        HGM_HIP(hipStreamSynchronize(st));
        return T;
    }
    int32_t *ridx = nullptr, *keys_out = nullptr, *perm_in = nullptr, *perm_out = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    int bits = 1;
    while ((int64_t(1) << bits) < M->cols) ++bits;
    try {
        HGM_HIP(hipMalloc(&ridx, sizeof(int32_t) * nnz));
        HGM_HIP(hipMalloc(&keys_out, sizeof(int32_t) * nnz));
        HGM_HIP(hipMalloc(&perm_in, sizeof(int32_t) * nnz));
        HGM_HIP(hipMalloc(&perm_out, sizeof(int32_t) * nnz));
        k_expand_rows<<<(M->rows + 3) / 4, BS, 0, st>>>(M->rows, M->rp, ridx);
        k_iota<<<grid_cap(nnz), BS, 0, st>>>(nnz, perm_in);
        HGM_HIP(hipGetLastError());
        // stable LSD radix sort by column keeps row order inside every output row
        HGM_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, M->ci, keys_out, perm_in, perm_out,
                                                  (int)nnz, 0, bits, st));
        HGM_HIP(hipMalloc(&tmp, tmp_bytes));
        HGM_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, M->ci, keys_out, perm_in, perm_out,
                                                  (int)nnz, 0, bits, st));
        k_bounds<<<grid_cap(nnz + 1), BS, 0, st>>>(nnz, M->cols, keys_out, T->rp);
        if (M->dtype == HGM_F32)
            k_gather_t<float><<<grid_cap(nnz), BS, 0, st>>>(nnz, perm_out, ridx, (const float*)M->val, T->ci, (float*)T->val);
        else
            k_gather_t<double><<<grid_cap(nnz), BS, 0, st>>>(nnz, perm_out, ridx, (const double*)M->val, T->ci, (double*)T->val);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        (void)hipFree(ridx); (void)hipFree(keys_out); (void)hipFree(perm_in); (void)hipFree(perm_out); (void)hipFree(tmp);
        mat_free(T);
        throw;
    }
    (void)hipFree(ridx); (void)hipFree(keys_out); (void)hipFree(perm_in); (void)hipFree(perm_out); (void)hipFree(tmp);
    return T;
}

// --------------------------------------------------------------------------
// Siddon parallel-beam projector (mirrors hgmres/problems.py::_siddon_chunk)
// --------------------------------------------------------------------------
struct RayGeom {
    double x0, y0, c, s, tmin, tmax;
    bool cx, cy, hit;
};

// a ray x(t) = (x0, y0) + t (c, s_) (unit direction; hgmres/problems.py::_siddon_rays)
__device__ __forceinline__ RayGeom ray_geom_xy(int N, double x0, double y0, double c, double s_) {
    RayGeom g;
    const double half = N / 2.0;
    g.c = c;
    g.s = s_;
    g.x0 = x0;
    g.y0 = y0;
    g.cx = fabs(c) > 1e-12;
    g.cy = fabs(s_) > 1e-12;
    const double inf = INFINITY;
    double txmin, txmax, tymin, tymax;
    if (g.cx) {
        const double a = ((0.0 - half) - g.x0) / c, b = (((double)N - half) - g.x0) / c;
        txmin = fmin(a, b); txmax = fmax(a, b);
    } else {
        const bool in = fabs(g.x0) < half;
        txmin = in ? -inf : inf; txmax = in ? inf : -inf;
    }
    if (g.cy) {
        const double a = ((0.0 - half) - g.y0) / s_, b = (((double)N - half) - g.y0) / s_;
        tymin = fmin(a, b); tymax = fmax(a, b);
    } else {
        const bool in = fabs(g.y0) < half;
        tymin = in ? -inf : inf; tymax = in ? inf : -inf;
    }
    g.tmin = fmax(txmin, tymin);
    g.tmax = fmin(txmax, tymax);
    g.hit = g.tmin < g.tmax;
    return g;
}
// parallel ray at signed detector offset sd (_siddon_chunk: x0 = -s sin, y0 = s cos)
__device__ __forceinline__ RayGeom ray_geom(int N, double c, double s_, double sd) {
    return ray_geom_xy(N, -sd * s_, sd * c, c, s_);
}

// Walk the merged, sorted crossing sequence [tmin, x/y-plane crossings in range, tmax]
// and emit segments with length > 1e-10 (problems.py: valid = isfinite & L > 1e-10).
// pixel (row r, column c) -> column index: column-major r + c*N (the reference's
// x(:) order) or, for tile > 1, tile-major over tile x tile blocks (column-major inside)
__device__ __forceinline__ int64_t tiled_index(int64_t S, int tile, int64_t r, int64_t c) {
    if (tile <= 1) return r + c * S;
    const int64_t tr = r / tile, tc = c / tile;
    return ((tc * (S / tile) + tr) * tile + (c % tile)) * tile + (r % tile);
}
// super > 1: super x super blocks (column-major over blocks), each contiguous, tiled inside
__host__ __device__ __forceinline__ int64_t pixel_index(int N, int tile, int64_t r, int64_t c, int super = 0) {
    if (super <= 1) return tiled_index(N, tile, r, c);
    const int64_t sr = r / super, sc = c / super;
    return (sc * (N / super) + sr) * (int64_t)super * super + tiled_index(super, tile, r % super, c % super);
}

// inverse of pixel_index: stored index -> (r, c)
__host__ __device__ __forceinline__ void pixel_rc(int N, int tile, int super, int64_t idx, int64_t& r, int64_t& c) {
    const int64_t S = super > 1 ? super : N;
    const int64_t blk = idx / (S * S), rem = idx % (S * S);
    const int64_t nb = N / S;
    const int64_t sc = blk / nb, sr = blk % nb;
    int64_t rr, cc;
    if (tile > 1) {
        const int64_t t = rem / ((int64_t)tile * tile), w = rem % ((int64_t)tile * tile);
        const int64_t tc = t / (S / tile), tr = t % (S / tile);
        rr = tr * tile + w % tile;
        cc = tc * tile + w / tile;
    } else {
        rr = rem % S;
        cc = rem / S;
    }
    r = sr * S + rr;
    c = sc * S + cc;
}

// reference index p = r + c*N <-> stored index pixel_index(r, c)
template <typename T>
__global__ __launch_bounds__(BS) void k_pix_permute(int N, int tile, int super, const T* __restrict__ in,
                                                    T* __restrict__ out, int dir) {
    const int64_t n = (int64_t)N * N;
    for (int64_t p = (int64_t)blockIdx.x * BS + threadIdx.x; p < n; p += (int64_t)gridDim.x * BS) {
        const int64_t s = pixel_index(N, tile, p % N, p / N, super);
        if (dir == 0) out[s] = in[p];
        else out[p] = in[s];
    }
}

__global__ __launch_bounds__(BS) void k_pix_unmap(int N, int tile, int super, int32_t* __restrict__ idx, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (int64_t)gridDim.x * BS) {
        int64_t r, c;
        pixel_rc(N, tile, super, idx[i], r, c);
        idx[i] = (int32_t)(r + c * N);
    }
}

// The same permutation for the default order (tiles of a power-of-two side, no super-blocks,
// N^2 < 2^32), swept in STORED order with 32-bit index math (round 6): a wave's 64 stored
// entries are 64 / tile^2 consecutive tiles of one tile column, i.e. tile full runs of 64 / tile
// consecutive reference entries, so both sides move whole cache lines, and no 64-bit division is
// left (k_pix_permute walks the reference order and divides in 64 bits: at C4, 67-89 us for the
// 134 MB each way, on the critical path of every solve's input and output hand-over).
template <typename T>
__global__ __launch_bounds__(BS) void k_pix_permute_t(uint32_t N, uint32_t nt, int tsh, const T* __restrict__ in,
                                                      T* __restrict__ out, int dir, uint32_t n) {
    const uint32_t tm = (1u << tsh) - 1u, wm = (1u << (2 * tsh)) - 1u;
    for (uint32_t s = blockIdx.x * BS + threadIdx.x; s < n; s += gridDim.x * BS) {
        const uint32_t t = s >> (2 * tsh), w = s & wm;            // tile, position in it (column-major)
        const uint32_t tc = t / nt, tr = t - tc * nt;              // tile-column-major tiles
        const uint32_t col = (tc << tsh) + (w >> tsh), row = (tr << tsh) + (w & tm);
        const uint32_t p = row + col * N;
        if (dir == 0) out[s] = in[p];
        else out[p] = in[s];
    }
}

template <typename T>
void pix_permute(hgm_ctx* c, const PixOrder& o, const T* in, T* out, int dir) {
    HGM_REQUIRE(!o.trivial(), "pix_permute: trivial order");
    const int64_t n = (int64_t)o.N * o.N;
    const bool pow2 = o.tile >= 2 && (o.tile & (o.tile - 1)) == 0;
    if (o.super <= 1 && pow2 && o.N % o.tile == 0 && n < ((int64_t)1 << 32)) {
        int tsh = 0;
        while ((1 << tsh) < o.tile) ++tsh;
        k_pix_permute_t<T><<<grid_cap(n), BS, 0, c->stream>>>((uint32_t)o.N, (uint32_t)(o.N / o.tile), tsh, in, out,
                                                             dir, (uint32_t)n);
    } else {
        k_pix_permute<T><<<grid_cap(n), BS, 0, c->stream>>>(o.N, o.tile, o.super, in, out, dir);
    }
    HGM_HIP(hipGetLastError());
}
template void pix_permute<double>(hgm_ctx*, const PixOrder&, const double*, double*, int);
template void pix_permute<float>(hgm_ctx*, const PixOrder&, const float*, float*, int);

void pix_unmap_indices(hgm_ctx* c, const PixOrder& o, int32_t* idx, int64_t n) {
    if (o.trivial() || n == 0) return;
    k_pix_unmap<<<grid_cap(n), BS, 0, c->stream>>>(o.N, o.tile, o.super, idx, n);
    HGM_HIP(hipGetLastError());
}

std::vector<int64_t> pix_reference_of_stored(const PixOrder& o) {
    const int64_t n = (int64_t)o.N * o.N;
    std::vector<int64_t> ref(n);
    for (int64_t s = 0; s < n; ++s) {
        int64_t r, c;
        pixel_rc(o.N, o.tile, o.super, s, r, c);
        ref[s] = r + c * o.N;
    }
    return ref;
}

template <bool FILL, typename T>
__device__ int64_t siddon_walk(int N, const RayGeom& g, int64_t out0, int32_t* ci, T* val, int tile = 1,
                               int super = 0) {
    if (!g.hit) return 0;
    const double half = N / 2.0;
    // next in-range crossing of each family in increasing t
    int kx = 0, dkx = 1, ky = 0, dky = 1;
    if (g.cx) { if (g.c > 0) { kx = 0; dkx = 1; } else { kx = N; dkx = -1; } }
    if (g.cy) { if (g.s > 0) { ky = 0; dky = 1; } else { ky = N; dky = -1; } }
    auto tx_at = [&](int k) { return (((double)k - half) - g.x0) / g.c; };
    auto ty_at = [&](int k) { return (((double)k - half) - g.y0) / g.s; };
    // skip crossings below tmin
    double tx = INFINITY, ty = INFINITY;
    bool hx = g.cx, hy = g.cy;
    if (hx) { while (kx >= 0 && kx <= N && !(tx_at(kx) >= g.tmin)) kx += dkx; hx = (kx >= 0 && kx <= N); if (hx) tx = tx_at(kx); }
    if (hy) { while (ky >= 0 && ky <= N && !(ty_at(ky) >= g.tmin)) ky += dky; hy = (ky >= 0 && ky <= N); if (hy) ty = ty_at(ky); }
    if (hx && !(tx <= g.tmax)) { hx = false; tx = INFINITY; }
    if (hy && !(ty <= g.tmax)) { hy = false; ty = INFINITY; }
    double t0 = g.tmin;
    int64_t cnt = 0;
    bool done = false;
    while (!done) {
        double t1;
        if (hx && (!hy || tx <= ty)) {
            t1 = tx;
            kx += dkx;
            hx = (kx >= 0 && kx <= N);
            if (hx) { tx = tx_at(kx); if (!(tx <= g.tmax)) { hx = false; tx = INFINITY; } }
        } else if (hy) {
            t1 = ty;
            ky += dky;
            hy = (ky >= 0 && ky <= N);
            if (hy) { ty = ty_at(ky); if (!(ty <= g.tmax)) { hy = false; ty = INFINITY; } }
        } else {
            t1 = g.tmax;
            done = true;
        }
        const double L = t1 - t0;
        if (L > 1e-10) {
            if (FILL) {
                const double mid = 0.5 * (t0 + t1);
                const double xm = g.x0 + mid * g.c;
                const double ym = g.y0 + mid * g.s;
                double fx = floor(xm + half), fy = floor(ym + half);
                fx = fmin(fmax(fx, 0.0), (double)(N - 1));
                fy = fmin(fmax(fy, 0.0), (double)(N - 1));
                const int64_t ix = (int64_t)fx, iy = (int64_t)fy;
                ci[out0 + cnt] = (int32_t)pixel_index(N, tile, N - 1 - iy, ix, super);
                val[out0 + cnt] = (T)L;
            }
            ++cnt;
        }
        t0 = t1;
    }
    return cnt;
}

template <bool FILL, typename T>
__global__ __launch_bounds__(BS) void k_siddon(int N, int p, int64_t m, const double* __restrict__ cth,
                                               const double* __restrict__ sth, const double* __restrict__ sdet,
                                               int64_t* __restrict__ counts, const int64_t* __restrict__ rp,
                                               int32_t* __restrict__ ci, T* __restrict__ val, int tile,
                                               int super) {
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < m; r += (int64_t)gridDim.x * BS) {
        const int a = (int)(r / p), d = (int)(r % p);
        const RayGeom g = ray_geom(N, cth[a], sth[a], sdet[d]);
        if (FILL) siddon_walk<true, T>(N, g, rp[r], ci, val, tile, super);
        else counts[r] = siddon_walk<false, T>(N, g, 0, nullptr, nullptr);
    }
}

// Fan-beam, curved (equiangular) detector (hgmres/problems.py::fan_geometry; the CTtype
// 'fancurved' of run_2D_phantom.m:12-13): ray r = a*p + d leaves the source D (cos b_a, sin b_a)
// towards the centre rotated by omega_d, u = -(cos(b+w), sin(b+w)) by the angle-addition formula
// from the host's libm cos / sin of b_a and omega_d (no FMA: -ffp-contract=off), so the rays
// are bitwise those of the numpy twin.
template <bool FILL, typename T>
__global__ __launch_bounds__(BS) void k_fanbeam(int N, int p, int64_t m, double D, const double* __restrict__ cb,
                                                const double* __restrict__ sb, const double* __restrict__ co,
                                                const double* __restrict__ so, int64_t* __restrict__ counts,
                                                const int64_t* __restrict__ rp, int32_t* __restrict__ ci,
                                                T* __restrict__ val, int tile, int super) {
    for (int64_t r = (int64_t)blockIdx.x * BS + threadIdx.x; r < m; r += (int64_t)gridDim.x * BS) {
        const int a = (int)(r / p), d = (int)(r % p);
        const double x0 = D * cb[a], y0 = D * sb[a];
        const double ux = -(cb[a] * co[d] - sb[a] * so[d]);
        const double uy = -(sb[a] * co[d] + cb[a] * so[d]);
        const RayGeom g = ray_geom_xy(N, x0, y0, ux, uy);
        if (FILL) siddon_walk<true, T>(N, g, rp[r], ci, val, tile, super);
        else counts[r] = siddon_walk<false, T>(N, g, 0, nullptr, nullptr);
    }
}

// --------------------------------------------------------------------------
// Unmatched pixel-driven back-projector (mirrors hgmres/problems.py::pixel_driven_backprojector,
// the role of PRtomo_mismatched in run_2D_phantom.m:13-14): for every pixel centre and angle,
// linear interpolation between the two nearest detector bins.  One thread per STORED pixel row
// (the rows follow the pixel order, so B pairs with a tiled A); entries in increasing column.
// --------------------------------------------------------------------------
template <bool FILL, typename T>
__global__ __launch_bounds__(BS) void k_backproj(int N, int p, int na, const double* __restrict__ cth,
                                                 const double* __restrict__ sth, double doff, int tile, int super,
                                                 int64_t* __restrict__ counts, const int64_t* __restrict__ rp,
                                                 int32_t* __restrict__ ci, T* __restrict__ val) {
    const int64_t n = (int64_t)N * N;
    const double half = N / 2.0;
    for (int64_t s = (int64_t)blockIdx.x * BS + threadIdx.x; s < n; s += (int64_t)gridDim.x * BS) {
        int64_t r, c;
        if (tile > 1 || super > 1) pixel_rc(N, tile, super, s, r, c);
        else { r = s % N; c = s / N; }
        const double xc = ((double)c - half) + 0.5;
        const double yc = ((double)(N - 1 - r) - half) + 0.5;
        const double mxc = -xc;
        int64_t cnt = 0;
        const int64_t o = FILL ? rp[s] : 0;
        for (int a = 0; a < na; ++a) {
            const double t0 = mxc * sth[a], t1 = yc * cth[a];
            const double sa = t0 + t1;
            const double df = (sa + (p - 1) / 2.0) - doff;
            const double fd = floor(df);
            const double w1 = df - fd, w0 = 1.0 - w1;
            const int64_t d0 = (int64_t)fd;
            if (d0 >= 0 && d0 < p && w0 > 0) {
                if (FILL) { ci[o + cnt] = (int32_t)((int64_t)a * p + d0); val[o + cnt] = (T)w0; }
                ++cnt;
            }
            if (d0 + 1 >= 0 && d0 + 1 < p && w1 > 0) {
                if (FILL) { ci[o + cnt] = (int32_t)((int64_t)a * p + d0 + 1); val[o + cnt] = (T)w1; }
                ++cnt;
            }
        }
        if (!FILL) counts[s] = cnt;
    }
}

hgm_mat* backprojector(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, int tile, int super) {
    HGM_REQUIRE(N > 0 && n_angles > 0, "backprojector: N and n_angles must be positive");
    if (tile < 1) tile = 1;
    if (super < 2) super = 0;
    HGM_REQUIRE(N % tile == 0 && (super == 0 || (N % super == 0 && super % tile == 0)),
                "backprojector: tile must divide N (and super), super must divide N");
    hipStream_t st = c->stream;
    const int p = (int)std::ceil(std::sqrt(2.0) * N);
    const int64_t n = (int64_t)N * N, m = (int64_t)p * n_angles;
    std::vector<double> cth(n_angles), sth(n_angles);
    const double dth = M_PI / n_angles;
    for (int a = 0; a < n_angles; ++a) {
        const double th = (double)a * dth;
        cth[a] = std::cos(th);
        sth[a] = std::sin(th);
    }
    double *dc = nullptr, *ds = nullptr;
    int64_t *counts = nullptr, *rp = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hgm_mat* M = nullptr;
    try {
        HGM_HIP(hipMalloc(&dc, 8 * n_angles));
        HGM_HIP(hipMalloc(&ds, 8 * n_angles));
        HGM_HIP(hipMalloc(&counts, 8 * (n + 1)));
        HGM_HIP(hipMalloc(&rp, 8 * (n + 1)));
        HGM_HIP(hipMemcpyAsync(dc, cth.data(), 8 * n_angles, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemcpyAsync(ds, sth.data(), 8 * n_angles, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemsetAsync(counts, 0, 8 * (n + 1), st));
        const int g = grid_cap(n);
        k_backproj<false, double><<<g, BS, 0, st>>>(N, p, n_angles, dc, ds, det_offset, tile, super, counts, nullptr,
                                                    nullptr, nullptr);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, rp, (int)(n + 1), st));
        HGM_HIP(hipMalloc(&tmp, tmp_bytes));
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, counts, rp, (int)(n + 1), st));
        int64_t nnz = 0;
        HGM_HIP(hipMemcpyAsync(&nnz, rp + n, 8, hipMemcpyDeviceToHost, st));
        HGM_HIP(hipStreamSynchronize(st));
        M = mat_alloc(c, n, m, nnz, dtype);
        if (tile > 1 || super > 1) M->row_order = PixOrder{N, tile, super};
        HGM_HIP(hipMemcpyAsync(M->rp, rp, 8 * (n + 1), hipMemcpyDeviceToDevice, st));
        if (dtype == HGM_F32)
            k_backproj<true, float><<<g, BS, 0, st>>>(N, p, n_angles, dc, ds, det_offset, tile, super, nullptr, M->rp,
                                                      M->ci, (float*)M->val);
        else
            k_backproj<true, double><<<g, BS, 0, st>>>(N, p, n_angles, dc, ds, det_offset, tile, super, nullptr,
                                                       M->rp, M->ci, (double*)M->val);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        (void)hipFree(dc); (void)hipFree(ds); (void)hipFree(counts); (void)hipFree(rp); (void)hipFree(tmp);
        mat_free(M);
        throw;
    }
    (void)hipFree(dc); (void)hipFree(ds); (void)hipFree(counts); (void)hipFree(rp); (void)hipFree(tmp);
    return M;
}

hgm_mat* siddon(hgm_ctx* c, int N, int n_angles, double det_offset, int dtype, int tile, int super) {
    HGM_REQUIRE(N > 0 && n_angles > 0, "siddon: N and n_angles must be positive");
    if (tile < 1) tile = 1;
    if (super < 2) super = 0;
    HGM_REQUIRE(N % tile == 0 && (super == 0 || (N % super == 0 && super % tile == 0)),
                "siddon: tile must divide N (and super), super must divide N");
    hipStream_t st = c->stream;
    const int p = (int)std::ceil(std::sqrt(2.0) * N);
    const int64_t m = (int64_t)p * n_angles;
    // geometry on the host with C libm (problems.py uses math.cos / math.sin, same libm)
    std::vector<double> cth(n_angles), sth(n_angles), sdet(p);
    const double dth = M_PI / n_angles;
    for (int a = 0; a < n_angles; ++a) {
        const double th = (double)a * dth;
        cth[a] = std::cos(th);
        sth[a] = std::sin(th);
    }
    for (int d = 0; d < p; ++d) sdet[d] = ((double)d - (p - 1) / 2.0) + det_offset;
    double *dc = nullptr, *ds = nullptr, *dd = nullptr;
    int64_t *counts = nullptr, *rp = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hgm_mat* M = nullptr;
    try {
        HGM_HIP(hipMalloc(&dc, 8 * n_angles));
        HGM_HIP(hipMalloc(&ds, 8 * n_angles));
        HGM_HIP(hipMalloc(&dd, 8 * p));
        HGM_HIP(hipMalloc(&counts, 8 * (m + 1)));
        HGM_HIP(hipMalloc(&rp, 8 * (m + 1)));
        HGM_HIP(hipMemcpyAsync(dc, cth.data(), 8 * n_angles, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemcpyAsync(ds, sth.data(), 8 * n_angles, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemcpyAsync(dd, sdet.data(), 8 * p, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemsetAsync(counts, 0, 8 * (m + 1), st));
        const int g = grid_cap(m);
        k_siddon<false, double><<<g, BS, 0, st>>>(N, p, m, dc, ds, dd, counts, nullptr, nullptr, nullptr, 1, 0);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, rp, (int)(m + 1), st));
        HGM_HIP(hipMalloc(&tmp, tmp_bytes));
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, counts, rp, (int)(m + 1), st));
        int64_t nnz = 0;
        HGM_HIP(hipMemcpyAsync(&nnz, rp + m, 8, hipMemcpyDeviceToHost, st));
        HGM_HIP(hipStreamSynchronize(st));
        HGM_REQUIRE(nnz < (int64_t)INT32_MAX * 2, "siddon: nnz overflow");
        M = mat_alloc(c, m, (int64_t)N * N, nnz, dtype);
        HGM_HIP(hipMemcpyAsync(M->rp, rp, 8 * (m + 1), hipMemcpyDeviceToDevice, st));
        if (tile > 1 || super > 1) M->col_order = PixOrder{N, tile, super};
        if (dtype == HGM_F32)
            k_siddon<true, float><<<g, BS, 0, st>>>(N, p, m, dc, ds, dd, nullptr, M->rp, M->ci, (float*)M->val, tile,
                                                    super);
        else
            k_siddon<true, double><<<g, BS, 0, st>>>(N, p, m, dc, ds, dd, nullptr, M->rp, M->ci, (double*)M->val,
                                                     tile, super);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        (void)hipFree(dc); (void)hipFree(ds); (void)hipFree(dd); (void)hipFree(counts); (void)hipFree(rp); (void)hipFree(tmp);
        mat_free(M);
        throw;
    }
    (void)hipFree(dc); (void)hipFree(ds); (void)hipFree(dd); (void)hipFree(counts); (void)hipFree(rp); (void)hipFree(tmp);
    return M;
}

hgm_mat* fanbeam(hgm_ctx* c, int N, int n_angles, double R, double span, double det_offset, int dtype, int tile,
                 int super) {
    HGM_REQUIRE(N > 0 && n_angles > 0, "fanbeam: N and n_angles must be positive");
    HGM_REQUIRE(R > 1.0 / std::sqrt(2.0), "fanbeam: the source must lie outside the image (R > 1/sqrt(2))");
    if (tile < 1) tile = 1;
    if (super < 2) super = 0;
    HGM_REQUIRE(N % tile == 0 && (super == 0 || (N % super == 0 && super % tile == 0)),
                "fanbeam: tile must divide N (and super), super must divide N");
    if (!(span > 0)) span = 2.0 * std::asin(1.0 / (std::sqrt(2.0) * R));
    HGM_REQUIRE(span < M_PI, "fanbeam: span must be below pi");
    hipStream_t st = c->stream;
    const int p = (int)std::ceil(std::sqrt(2.0) * N);
    const int64_t m = (int64_t)p * n_angles;
    const double D = R * N, dom = span / p;
    // geometry on the host with C libm (problems.py fan_geometry: math.cos / math.sin, same libm)
    std::vector<double> cb(n_angles), sb(n_angles), co(p), so(p);
    for (int a = 0; a < n_angles; ++a) {
        const double b = a * (2.0 * M_PI / n_angles);
        cb[a] = std::cos(b);
        sb[a] = std::sin(b);
    }
    for (int d = 0; d < p; ++d) {
        const double w = (((double)d - (p - 1) / 2.0) + det_offset) * dom;
        co[d] = std::cos(w);
        so[d] = std::sin(w);
    }
    double* geo = nullptr;
    int64_t *counts = nullptr, *rp = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    hgm_mat* M = nullptr;
    auto release = [&]() {
        (void)hipFree(geo); (void)hipFree(counts); (void)hipFree(rp); (void)hipFree(tmp);
    };
    try {
        HGM_HIP(hipMalloc(&geo, 8 * (2 * (size_t)n_angles + 2 * (size_t)p)));
        double *dcb = geo, *dsb = geo + n_angles, *dco = geo + 2 * n_angles, *dso = geo + 2 * n_angles + p;
        HGM_HIP(hipMalloc(&counts, 8 * (m + 1)));
        HGM_HIP(hipMalloc(&rp, 8 * (m + 1)));
        HGM_HIP(hipMemcpyAsync(dcb, cb.data(), 8 * n_angles, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemcpyAsync(dsb, sb.data(), 8 * n_angles, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemcpyAsync(dco, co.data(), 8 * p, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemcpyAsync(dso, so.data(), 8 * p, hipMemcpyHostToDevice, st));
        HGM_HIP(hipMemsetAsync(counts, 0, 8 * (m + 1), st));
        const int g = grid_cap(m);
        k_fanbeam<false, double><<<g, BS, 0, st>>>(N, p, m, D, dcb, dsb, dco, dso, counts, nullptr, nullptr, nullptr,
                                                   1, 0);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, rp, (int)(m + 1), st));
        HGM_HIP(hipMalloc(&tmp, tmp_bytes));
        HGM_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, counts, rp, (int)(m + 1), st));
        int64_t nnz = 0;
        HGM_HIP(hipMemcpyAsync(&nnz, rp + m, 8, hipMemcpyDeviceToHost, st));
        HGM_HIP(hipStreamSynchronize(st));
        HGM_REQUIRE(nnz < (int64_t)INT32_MAX * 2, "fanbeam: nnz overflow");
        M = mat_alloc(c, m, (int64_t)N * N, nnz, dtype);
        HGM_HIP(hipMemcpyAsync(M->rp, rp, 8 * (m + 1), hipMemcpyDeviceToDevice, st));
        if (tile > 1 || super > 1) M->col_order = PixOrder{N, tile, super};
        if (dtype == HGM_F32)
            k_fanbeam<true, float><<<g, BS, 0, st>>>(N, p, m, D, dcb, dsb, dco, dso, nullptr, M->rp, M->ci,
                                                     (float*)M->val, tile, super);
        else
            k_fanbeam<true, double><<<g, BS, 0, st>>>(N, p, m, D, dcb, dsb, dco, dso, nullptr, M->rp, M->ci,
                                                      (double*)M->val, tile, super);
        HGM_HIP(hipGetLastError());
        HGM_HIP(hipStreamSynchronize(st));
    } catch (...) {
        release();
        mat_free(M);
        throw;
    }
    release();
    return M;
}

}  // namespace hgm
