// Microbenchmark (gfx950): cost of one grid-wide exchange of block partials, the step
// between two MGS passes.  Build: hipcc -O3 --offload-arch=gfx950 barrier_bench.hip -o /tmp/bb
//   mode 0: K dependent kernel launches (each block re-reduces the previous partials)
//   mode 1: one cooperative kernel, K flat atomic-counter barriers
//   mode 2: one cooperative kernel, K two-level (8 groups) barriers
//   mode 3: one cooperative kernel, K sentinel exchanges: partials are published with
//           coherent stores into slots pre-filled with a signalling-NaN sentinel, every
//           block polls the np slots until none is the sentinel (no atomics at all)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

constexpr int BS = 256;
constexpr unsigned long long SENT = 0x7FF0DEADBEEF0001ull;

__device__ __forceinline__ double wave_sum(double v) {
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double block_sum(double v, double* sh) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    return r;
}

__global__ void k_step(const double* pin, double* pout, int np, int first) {
    __shared__ double sh[4];
    double a = 0;
    if (!first)
        for (int i = threadIdx.x; i < np; i += BS) a += pin[i];
    double h = block_sum(a, sh);
    if (threadIdx.x == 0) pout[blockIdx.x] = h * 0.5 + blockIdx.x;
}

__device__ void flat_barrier(unsigned long long* bar, unsigned long long target) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        while (__hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__device__ void tree_barrier(unsigned long long* bar, unsigned long long e, int np) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const int g = blockIdx.x & 7;
        const unsigned long long gsize = (np - g + 7) / 8;
        unsigned long long old = __hip_atomic_fetch_add(bar + g * 16, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        if (old + 1 == e * gsize) {
            unsigned long long o2 =
                __hip_atomic_fetch_add(bar + 8 * 16, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            if (o2 + 1 == e * 8)
                for (int gg = 0; gg < 8; ++gg)
                    __hip_atomic_store(bar + (9 + gg) * 16, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        while (__hip_atomic_load(bar + (9 + g) * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e)
            __builtin_amdgcn_s_sleep(1);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
}

__global__ void k_coop(int mode, int K, double* parts, unsigned long long* bar, unsigned long long* slots) {
    __shared__ double sh[4];
    __shared__ int pending;
    const int np = gridDim.x;
    double h = 0;
    for (int j = 0; j < K; ++j) {
        const double mine = h * 0.5 + blockIdx.x;
        if (mode == 3) {
            unsigned long long* s = slots + (size_t)j * np;
            if (threadIdx.x == 0)
                __hip_atomic_store(s + blockIdx.x, __double_as_longlong(mine), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            double a = 0;
            // poll own slots until published (each lane owns slots t, t+BS, ...)
            for (;;) {
                int miss = 0;
                a = 0;
                for (int i = threadIdx.x; i < np; i += BS) {
                    unsigned long long v = __hip_atomic_load(s + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (v == SENT) miss = 1;
                    a += __longlong_as_double(v);
                }
                if (!__syncthreads_or(miss)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            h = block_sum(a, sh);
        } else {
            if (threadIdx.x == 0) parts[(size_t)(j & 1) * 1024 + blockIdx.x] = mine;
            if (mode == 1) flat_barrier(bar, (unsigned long long)np * (j + 1));
            else tree_barrier(bar, j + 1, np);
            double a = 0;
            for (int i = threadIdx.x; i < np; i += BS) a += parts[(size_t)(j & 1) * 1024 + i];
            h = block_sum(a, sh);
        }
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) parts[2048] = h;
    (void)pending;
}

int main(int argc, char** argv) {
    const int np = argc > 1 ? std::atoi(argv[1]) : 512;
    const int K = 64;
    double* parts;
    unsigned long long *bar, *slots;
    CK(hipMalloc(&parts, sizeof(double) * 4096));
    CK(hipMalloc(&bar, sizeof(unsigned long long) * 17 * 16));
    CK(hipMalloc(&slots, sizeof(unsigned long long) * (size_t)K * np));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> sent((size_t)K * np, SENT);
    for (int mode = 0; mode <= 3; ++mode) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipMemset(bar, 0, sizeof(unsigned long long) * 17 * 16));
            CK(hipMemcpy(slots, sent.data(), sizeof(unsigned long long) * sent.size(), hipMemcpyHostToDevice));
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st));
            if (mode == 0) {
                for (int j = 0; j < K; ++j)
                    hipLaunchKernelGGL(k_step, dim3(np), dim3(BS), 0, st, parts + (j & 1) * 1024,
                                       parts + ((j + 1) & 1) * 1024, np, j == 0);
            } else {
                int m = mode, kk = K;
                void* args[] = {&m, &kk, &parts, &bar, &slots};
                CK(hipLaunchCooperativeKernel(reinterpret_cast<const void*>(k_coop), dim3(np), dim3(BS), args, 0, st));
            }
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        std::printf("{\"mode\": %d, \"np\": %d, \"K\": %d, \"us_per_exchange\": %.3f}\n", mode, np, K, best * 1e3 / K);
    }
    return 0;
}
