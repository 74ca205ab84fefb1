// sorted_probe.hip — cfg4 gather pattern with every row's 32 ids sorted ascending (diagnostic).
// Variants: one-shot (all 32 gathers in flight), staged sweeps (G groups of 32/G gathers with a
// wait between groups), persistent generations with a soft per-group re-sync, block size.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t N = 1u << 20;

template <int STAGES, int BS>
__global__ __launch_bounds__(BS) void k_sorted(const u32x4* ell, const double* x, double* out) {
    const uint32_t i = blockIdx.x * BS + threadIdx.x;
    const u32x4* cp = ell + (uint64_t)(i >> 6) * 512 + (i & 63);
    uint32_t col[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        u32x4 c = cp[q * 64];
        col[4 * q] = c.x; col[4 * q + 1] = c.y; col[4 * q + 2] = c.z; col[4 * q + 3] = c.w;
    }
    double v[32];
    constexpr int PER = 32 / STAGES;
#pragma unroll
    for (int s = 0; s < STAGES; ++s) {
#pragma unroll
        for (int t = 0; t < PER; ++t) v[s * PER + t] = x[col[s * PER + t]];
        if (STAGES > 1 && s + 1 < STAGES) {
            // keep the next stage behind this one: consume the values (forces the wait)
            double z = 0;
#pragma unroll
            for (int t = 0; t < PER; ++t) z += v[s * PER + t];
            asm volatile("" ::"v"(z));
        }
    }
    double acc = 0;
#pragma unroll
    for (int t = 0; t < 32; ++t) acc += v[t];
    out[i] = acc;
}

__device__ __forceinline__ void soft_barrier(uint32_t* ctr, uint32_t target, int spin_limit) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int k = 0; k < spin_limit; ++k) {
            if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
}

template <int SYNC>
__global__ __launch_bounds__(256) void k_gen(const u32x4* ell, const double* x, double* out, uint32_t* ctr) {
    const uint32_t nb = gridDim.x, g = blockIdx.x % 8, rho = blockIdx.x / 8, per_group = nb / 8;
    uint32_t epoch = 0;
    for (uint32_t sl = blockIdx.x; sl < N / 256; sl += nb) {
        const uint32_t i = sl * 256 + threadIdx.x;
        const u32x4* cp = ell + (uint64_t)(i >> 6) * 512 + (i & 63);
        double v[32];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            u32x4 c = cp[q * 64];
            v[4 * q] = x[c.x]; v[4 * q + 1] = x[c.y]; v[4 * q + 2] = x[c.z]; v[4 * q + 3] = x[c.w];
        }
        double acc = 0;
#pragma unroll
        for (int t = 0; t < 32; ++t) acc += v[t];
        out[i] = acc;
        if (SYNC) soft_barrier(ctr + g * 64, (++epoch) * per_group, 4000);
    }
    (void)rho;
}

int main() {
    std::vector<uint32_t> ell(N * 32);
    uint64_t s = 88172645463325252ull;
    uint32_t r[32];
    for (uint32_t i = 0; i < N; ++i) {
        for (int t = 0; t < 32; ++t) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; r[t] = (uint32_t)(s >> 20) & (N - 1); }
        std::sort(r, r + 32);
        for (int t = 0; t < 32; ++t) ell[(((i >> 6) * 8 + t / 4) * 64 + (i & 63)) * 4 + (t & 3)] = r[t];
    }
    u32x4* dell; uint32_t* ctr; double *x, *out;
    CK(hipMalloc(&dell, N * 128));
    CK(hipMalloc(&x, N * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMalloc(&ctr, 8 * 64 * 4));
    CK(hipMemcpy(dell, ell.data(), N * 128, hipMemcpyHostToDevice));
    CK(hipMemset(x, 0, N * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto fn) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipEventRecord(a));
        const int reps = 30;
        for (int rr = 0; rr < reps; ++rr) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipGetLastError());
        const float us = ms * 1000.f / reps;
        printf("%s,%.1f,%.0f\n", name, us, 400.0 * N / (us * 1e-6) / 1e9);
    };
    printf("variant,us,alg_GBps\n");
    timeit("sorted_oneshot_bs256", [&] { hipLaunchKernelGGL((k_sorted<1, 256>), dim3(N / 256), dim3(256), 0, 0, dell, x, out); });
    timeit("sorted_oneshot_bs64", [&] { hipLaunchKernelGGL((k_sorted<1, 64>), dim3(N / 64), dim3(64), 0, 0, dell, x, out); });
    timeit("sorted_oneshot_bs1024", [&] { hipLaunchKernelGGL((k_sorted<1, 1024>), dim3(N / 1024), dim3(1024), 0, 0, dell, x, out); });
    timeit("sorted_2stage", [&] { hipLaunchKernelGGL((k_sorted<2, 256>), dim3(N / 256), dim3(256), 0, 0, dell, x, out); });
    timeit("sorted_4stage", [&] { hipLaunchKernelGGL((k_sorted<4, 256>), dim3(N / 256), dim3(256), 0, 0, dell, x, out); });
    timeit("sorted_8stage", [&] { hipLaunchKernelGGL((k_sorted<8, 256>), dim3(N / 256), dim3(256), 0, 0, dell, x, out); });
    for (int nb : {256, 512, 1024}) {
        char name[64];
        snprintf(name, 64, "gen_nosync_nb%d", nb);
        timeit(name, [&] { hipLaunchKernelGGL((k_gen<0>), dim3(nb), dim3(256), 0, 0, dell, x, out, ctr); });
        snprintf(name, 64, "gen_sync_nb%d", nb);
        timeit(name, [&] {
            CK(hipMemsetAsync(ctr, 0, 8 * 64 * 4));
            hipLaunchKernelGGL((k_gen<1>), dim3(nb), dim3(256), 0, 0, dell, x, out, ctr);
        });
    }
    return 0;
}
