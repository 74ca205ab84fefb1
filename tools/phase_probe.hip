// phase_probe.hip — best-case emulation of source-partitioned cfg4 round designs (diagnostic).
//  base   : one kernel, 32 ids + 32 gathers from the whole 8 MiB table (today's design)
//  2phase : KA gathers 16 values from the low 4 MiB half and stages them (coalesced rows),
//           KB gathers 16 from the high half + reads the staged 16
//  8part  : KP (grid = 8 x slices, block%8 = partition) gathers 4 values from a 1 MiB slice and
//           stages them; KC reads the 32 staged values (coalesced rows)
//  8part_lds: as 8part, but KC stages through LDS with full-line loads
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t N = 1u << 20, HALF = N / 2, PART = N / 8;

__global__ __launch_bounds__(256) void k_base(const u32x4* ell, const double* x, double* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const u32x4* cp = ell + (uint64_t)(i >> 6) * 512 + (i & 63);
    double acc = 0;
    double v[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        u32x4 c = cp[q * 64];
        v[4 * q] = x[c.x & (N - 1)]; v[4 * q + 1] = x[c.y & (N - 1)]; v[4 * q + 2] = x[c.z & (N - 1)]; v[4 * q + 3] = x[c.w & (N - 1)];
    }
#pragma unroll
    for (int t = 0; t < 32; ++t) acc += v[t];
    out[i] = acc;
}

template <int PHASE>
__global__ __launch_bounds__(256) void k_phase(const u32x4* ell, const double* x, double* stage, double* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const u32x4* cp = ell + (uint64_t)(i >> 6) * 512 + (i & 63) + PHASE * 4 * 64;
    const uint32_t base = PHASE ? HALF : 0;
    double v[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        u32x4 c = cp[q * 64];
        v[4 * q] = x[base + (c.x & (HALF - 1))]; v[4 * q + 1] = x[base + (c.y & (HALF - 1))];
        v[4 * q + 2] = x[base + (c.z & (HALF - 1))]; v[4 * q + 3] = x[base + (c.w & (HALF - 1))];
    }
    double* sp = stage + (uint64_t)(i >> 6) * 16 * 64 + (i & 63);
    if (PHASE == 0) {
#pragma unroll
        for (int t = 0; t < 16; ++t) sp[t * 64] = v[t];
    } else {
        double acc = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) acc += v[t] + sp[t * 64];
        out[i] = acc;
    }
}

__global__ __launch_bounds__(256) void k_part(const u32x4* ell, const double* x, double* stage) {
    const uint32_t q = blockIdx.x & 7, slice4 = blockIdx.x >> 3;   // 4 slices of 64 per block
    const uint32_t i = slice4 * 256 + threadIdx.x;
    const u32x4 c = ell[((uint64_t)q * (N / 64) + (i >> 6)) * 64 + (i & 63)];
    const uint32_t base = q * PART;
    double v0 = x[base + (c.x & (PART - 1))], v1 = x[base + (c.y & (PART - 1))];
    double v2 = x[base + (c.z & (PART - 1))], v3 = x[base + (c.w & (PART - 1))];
    double* sp = stage + ((uint64_t)(i >> 6) * 32 + q * 4) * 64 + (i & 63);
    sp[0] = v0; sp[64] = v1; sp[128] = v2; sp[192] = v3;
}

__global__ __launch_bounds__(256) void k_combine(const double* stage, double* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const double* sp = stage + (uint64_t)(i >> 6) * 32 * 64 + (i & 63);
    double acc = 0;
#pragma unroll
    for (int t = 0; t < 32; ++t) acc += sp[t * 64];
    out[i] = acc;
}

int main() {
    std::vector<uint32_t> h(N * 32);
    uint64_t s = 88172645463325252ull;
    for (auto& v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint32_t)(s >> 11); }
    std::vector<double> hx(N);
    for (uint32_t k = 0; k < N; ++k) hx[k] = k * 1e-7;
    u32x4* ell; double *x, *out, *stage;
    CK(hipMalloc(&ell, N * 32 * 4));
    CK(hipMalloc(&x, N * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMalloc(&stage, (size_t)N * 32 * 8));
    CK(hipMemcpy(ell, h.data(), N * 32 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(x, hx.data(), N * 8, hipMemcpyHostToDevice));
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
    printf("design,us_per_round,alg_GBps\n");
    timeit("base", [&] { hipLaunchKernelGGL(k_base, dim3(N / 256), dim3(256), 0, 0, ell, x, out); });
    timeit("2phase", [&] {
        hipLaunchKernelGGL(k_phase<0>, dim3(N / 256), dim3(256), 0, 0, ell, x, stage, out);
        hipLaunchKernelGGL(k_phase<1>, dim3(N / 256), dim3(256), 0, 0, ell, x, stage, out);
    });
    timeit("2phase_A_only", [&] { hipLaunchKernelGGL(k_phase<0>, dim3(N / 256), dim3(256), 0, 0, ell, x, stage, out); });
    timeit("8part", [&] {
        hipLaunchKernelGGL(k_part, dim3(8 * N / 256), dim3(256), 0, 0, ell, x, stage);
        hipLaunchKernelGGL(k_combine, dim3(N / 256), dim3(256), 0, 0, stage, out);
    });
    timeit("8part_P_only", [&] { hipLaunchKernelGGL(k_part, dim3(8 * N / 256), dim3(256), 0, 0, ell, x, stage); });
    timeit("8part_C_only", [&] { hipLaunchKernelGGL(k_combine, dim3(N / 256), dim3(256), 0, 0, stage, out); });
    return 0;
}
