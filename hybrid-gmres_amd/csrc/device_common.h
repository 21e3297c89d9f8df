// Device-side helpers shared by the HIP translation units of libhgmres (gfx950).
#pragma once

#include <hip/hip_ext.h>

#include "internal.h"

namespace hgm {

template <typename T> struct V2;
template <> struct V2<double> { using t = double2; };
template <> struct V2<float> { using t = float2; };

// native clang vectors (the nontemporal builtin does not take HIP_vector_type)
typedef double nd2 __attribute__((ext_vector_type(2)));
typedef float nf2 __attribute__((ext_vector_type(2)));
typedef int ni2 __attribute__((ext_vector_type(2)));
typedef int ni4 __attribute__((ext_vector_type(4)));
typedef float nf4 __attribute__((ext_vector_type(4)));
typedef unsigned short nus2 __attribute__((ext_vector_type(2)));
typedef unsigned short nus4 __attribute__((ext_vector_type(4)));
template <typename T> struct NV2;
template <> struct NV2<double> { using t = nd2; };
template <> struct NV2<float> { using t = nf2; };
// 16-byte vectors of the elementwise kernels: W elements of T per access
template <typename T> struct V16;
template <> struct V16<double> { using t = nd2; static constexpr int W = 2; };
template <> struct V16<float> { using t = nf4; static constexpr int W = 4; };
static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

template <bool NT, typename V>
__device__ __forceinline__ V ld(const V* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// DPP lane permutations within a 16-lane row (no LDS traffic, no lane-index VGPRs).
// Each step pairs every lane with a lane of the other half of its group, so the sums
// differ only by commutation and every lane of the row ends with the same bits.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <typename T>
__device__ __forceinline__ T row16_sum(T v) {
    v += dpp_mov<0xB1>(v);    // quad_perm [1,0,3,2]: lane ^ 1
    v += dpp_mov<0x4E>(v);    // quad_perm [2,3,0,1]: lane ^ 2
    v += dpp_mov<0x141>(v);   // row_half_mirror: other quad of the 8-lane half
    v += dpp_mov<0x140>(v);   // row_mirror: other half of the row
    return v;
}
__device__ __forceinline__ double lane_bcast(double v, int l) {
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ float lane_bcast(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// 64-lane sum: row sums by DPP, then the four rows combined in fixed order from
// scalar broadcasts — identical bits in every lane.
template <typename T>
__device__ __forceinline__ T wave_sum_dpp(T v) {
    v = row16_sum(v);
    return (lane_bcast(v, 0) + lane_bcast(v, 16)) + (lane_bcast(v, 32) + lane_bcast(v, 48));
}

// 64-lane sum, the same bits in every lane.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) { return wave_sum_dpp(v); }

// Sum over aligned groups of G lanes (G a power of two <= 64), the same bits in every
// lane of a group: DPP within 16-lane rows, xor shuffles across rows.
template <typename T, int G>
__device__ __forceinline__ T group_sum(T acc) {
    if constexpr (G >= 2) acc += dpp_mov<0xB1>(acc);
    if constexpr (G >= 4) acc += dpp_mov<0x4E>(acc);
    if constexpr (G >= 8) acc += dpp_mov<0x141>(acc);
    if constexpr (G >= 16) acc += dpp_mov<0x140>(acc);
    if constexpr (G >= 32) acc += __shfl_xor(acc, 16);
    if constexpr (G >= 64) acc += __shfl_xor(acc, 32);
    return acc;
}

// Store of a result scalar that the host may read from pinned host memory (the
// per-iteration ring): system scope, written through to memory, so the host needs no
// system-scope fence on the event it waits for (capi.cpp sync_event_flags).
template <typename T>
__device__ __forceinline__ void st_sys(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Block (256 threads) sum, result broadcast to every thread.  Fixed order.  REUSE=false
// drops the trailing barrier that protects `sh` for a later call (the caller then never
// writes `sh` again in this launch).
template <typename T, bool REUSE = true>
__device__ __forceinline__ T block_sum_all(T v, T* sh) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    T r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    if (REUSE) __syncthreads();
    return r;
}

// Sum of np partials (np <= MAX_PARTS) — same bits in every block that calls it.
template <typename T, bool REUSE = true>
__device__ __forceinline__ T reduce_parts(const T* __restrict__ p, int np, T* sh) {
    T a = 0;
    for (int i = threadIdx.x; i < np; i += BS) a += p[i];
    return block_sum_all<T, REUSE>(a, sh);
}

// Fused epilogues of the reference's operator closures, two roundings each (the
// library is compiled with -ffp-contract=off): t + a*z, t - a*z, z - t.
template <typename T, int EPI>
__device__ __forceinline__ T apply_epi(T t, T a, const T* __restrict__ z, int64_t i) {
    if (EPI == EPI_ADD) { T s = a * z[i]; return t + s; }
    if (EPI == EPI_SUB) { T s = a * z[i]; return t - s; }
    if (EPI == EPI_RSUB) return z[i] - t;
    return t;
}

// Epilogues with the pending normalisation (internal.h PendNorm); h from pn_pre / pn_fin.
template <typename T, int EPI>
__device__ __forceinline__ T apply_epi_pn(T t, T a, const T* __restrict__ z, int64_t i, const PendNorm<T>& pn, T h) {
    if constexpr (EPI == EPI_DIVH) {
        return h != T(0) ? t / h : t;
    } else if constexpr (EPI == EPI_ADDQ) {
        const T v = z[i];
        const T q = h != T(0) ? v / h : v;   // a zero norm (breakdown) leaves v as k_mgs_normalize does
        if (pn.q) pn.q[i] = q;
        const T s = a * q;
        return t + s;
    } else {
        return apply_epi<T, EPI>(t, a, z, i);
    }
}

// The same epilogues with the operand z_i already loaded (zi; the row kernel issues that
// load at kernel start so it overlaps the product instead of following it).
template <typename T, int EPI>
__device__ __forceinline__ T apply_epi_zv(T t, T a, T zi, int64_t i, const PendNorm<T>& pn, T h) {
    if constexpr (EPI == EPI_ADD) { T s = a * zi; return t + s; }
    if constexpr (EPI == EPI_SUB) { T s = a * zi; return t - s; }
    if constexpr (EPI == EPI_RSUB) return zi - t;
    if constexpr (EPI == EPI_DIVH) return h != T(0) ? t / h : t;
    if constexpr (EPI == EPI_ADDQ) {
        const T q = h != T(0) ? zi / h : zi;
        if (pn.q) pn.q[i] = q;
        const T s = a * q;
        return t + s;
    }
    return t;
}

// The epilogue coefficient: the host's scalar, or sqrt of a device sum of squares (PendNorm::asq)
template <typename T>
__device__ __forceinline__ T pn_coef(const PendNorm<T>& pn, T a) {
    return pn.asq ? (T)sqrt((double)*pn.asq) : a;
}

// h of the pending normalisation, in two halves so that its loads are issued at kernel
// start and overlap the product: pn_pre returns this thread's share (EPI_DIVH: its
// strided partial sum, the order of reduce_parts; EPI_ADDQ: h itself), pn_fin the value.
// EPI_DIVH: every thread of the block must call pn_fin (block sum, same bits as
// k_mgs_normalize's sqrt(sum)); block 0 publishes h to hdev and the host ring.
template <typename T, int EPI>
__device__ __forceinline__ T pn_pre(const PendNorm<T>& pn) {
    if constexpr (EPI == EPI_DIVH) {
        T a = 0;
        for (int i = threadIdx.x; i < pn.np; i += BS) a += pn.parts[i];
        return a;
    } else if constexpr (EPI == EPI_ADDQ) {
        return *pn.hdev;
    } else {
        return T(1);
    }
}
template <typename T, int EPI>
__device__ __forceinline__ T pn_fin(const PendNorm<T>& pn, T pre, T* sh) {
    if constexpr (EPI == EPI_DIVH) {
        const T h = sqrt(block_sum_all<T, true>(pre, sh));
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            pn.hdev[0] = h;
            st_sys(pn.hring, h);
        }
        return h;
    } else {
        return pre;
    }
}

// Raw buffer access (gfx9 resource word 3 = 0x00020000): the range check against
// `bytes` returns 0 for loads and drops stores past the end, and one 32-bit lane
// offset serves every resource, so unrolled strided loops keep one address VGPR.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes < 0 ? 0 : bytes, 0x00020000);
}
template <typename T> __device__ __forceinline__ T buf_load(__amdgpu_buffer_rsrc_t r, int off);
template <> __device__ __forceinline__ double buf_load<double>(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
template <> __device__ __forceinline__ float buf_load<float>(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
// a pair (double2 / float2) through a buffer resource
template <typename T2> __device__ __forceinline__ T2 buf_load2(__amdgpu_buffer_rsrc_t r, int off);
template <> __device__ __forceinline__ double2 buf_load2<double2>(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
template <> __device__ __forceinline__ float2 buf_load2<float2>(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}
__device__ __forceinline__ void buf_store(double x, __amdgpu_buffer_rsrc_t r, int off) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b64(r, 0, 0, 0)), x),
                                          r, off, 0, 0);
}
__device__ __forceinline__ void buf_store(float x, __amdgpu_buffer_rsrc_t r, int off) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(decltype(__builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 0)), x),
                                          r, off, 0, 0);
}

static inline int grid_for(int64_t n) {
    int64_t nb = (n + BS - 1) / BS;
    if (nb > 4096) nb = 4096;
    if (nb < 1) nb = 1;
    return (int)nb;
}

// Launch `kern` on the context stream.  When kernel timing is armed (timing_begin of
// an SpMV class), the first launch carries the start event and the launch flagged
// `last` the stop event inside their dispatch packets (hipExtLaunchKernelGGL), so the
// measured interval is kernel execution only, as rocprofv3's kernel trace sees it.
template <typename... KArgs, typename... Args>
static inline void launch(hgm_ctx* c, bool last, void (*kern)(KArgs...), dim3 grid, dim3 block, Args... args) {
    static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel argument count");
    hipEvent_t s = c->arm_start, e = last ? c->arm_stop : nullptr;
    if (s || e) {
        hipExtLaunchKernelGGL(kern, grid, block, 0, c->stream, s, e, 0, static_cast<KArgs>(args)...);
        c->arm_start = nullptr;
        if (last) c->arm_stop = nullptr;
    } else {
        hipLaunchKernelGGL(kern, grid, block, 0, c->stream, static_cast<KArgs>(args)...);
    }
}

}  // namespace hgm
