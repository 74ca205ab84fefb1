// stream_probe.hip — random 8-byte gathers over an 8 MiB table with in-kernel random ids
// (murmur-mixed, uniform) plus an id stream of S bytes per node (XORed into the ids so it is
// live).  Separates "table too big for L2" from "id stream pollutes L2".  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t N = 1u << 20;

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// NQ = uint4 loads of id-stream per lane (0..8), TB = table bits
template <int NQ, int TB, int SC1STORE>
__global__ __launch_bounds__(256) void k(const u32x4* __restrict__ ell, const double* __restrict__ x,
                                         double* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t salt = 0;
    if (NQ) {
        const u32x4* cp = ell + (uint64_t)(i >> 6) * (NQ * 64) + (i & 63);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const u32x4 c = cp[q * 64];
            salt ^= c.x ^ c.y ^ c.z ^ c.w;
        }
        salt &= 1u;   // keep the loads live without changing the id distribution
    }
    double v[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) v[t] = x[(mix(i * 32u + t) ^ salt) & ((1u << TB) - 1)];
    double acc = 0;
#pragma unroll
    for (int t = 0; t < 32; ++t) acc += v[t];
    if (SC1STORE) __hip_atomic_store(out + i, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else out[i] = acc;
}

int main() {
    u32x4* ell; double *x, *out;
    CK(hipMalloc(&ell, N * 128));
    CK(hipMalloc(&x, (size_t)(1u << 24) * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMemset(ell, 1, N * 128));
    CK(hipMemset(x, 0, (size_t)(1u << 24) * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto fn) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipEventRecord(a));
        const int reps = 40;
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipGetLastError());
        const float us = ms * 1000.f / reps;
        printf("%s,%.1f,%.0f\n", name, us, 400.0 * N / (us * 1e-6) / 1e9);
    };
#define R(NQ, TB, SC) timeit("ids" #NQ "x16B_table2^" #TB "_sc1st" #SC, [&] { hipLaunchKernelGGL((k<NQ, TB, SC>), dim3(N / 256), dim3(256), 0, 0, ell, x, out); })
    printf("case,us,alg_GBps\n");
    R(0, 14, 0); R(0, 17, 0); R(0, 19, 0); R(0, 20, 0); R(0, 21, 0); R(0, 23, 0);
    R(2, 20, 0); R(4, 20, 0); R(5, 20, 0); R(6, 20, 0); R(8, 20, 0);
    R(8, 19, 0); R(8, 18, 0); R(8, 17, 0);
    R(0, 20, 1); R(8, 20, 1);
    return 0;
}
