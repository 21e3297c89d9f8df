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
template <typename T> struct NV2;
template <> struct NV2<double> { using t = nd2; };
template <> struct NV2<float> { using t = nf2; };

template <bool NT, typename V>
__device__ __forceinline__ V ld(const V* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}

// 64-lane xor butterfly: every lane ends with the same, fixed-order sum.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

template <typename T, int G>
__device__ __forceinline__ T group_sum(T acc) {
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    return acc;
}

// Block (256 threads) sum, result broadcast to every thread.  Fixed order.
template <typename T>
__device__ __forceinline__ T block_sum_all(T v, T* sh) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[w] = v;
    __syncthreads();
    T r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    return r;
}

// Sum of np partials (np <= MAX_PARTS) — same bits in every block that calls it.
template <typename T>
__device__ __forceinline__ T reduce_parts(const T* __restrict__ p, int np, T* sh) {
    T a = 0;
    for (int i = threadIdx.x; i < np; i += BS) a += p[i];
    return block_sum_all(a, sh);
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
