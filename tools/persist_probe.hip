// persist_probe.hip — emulation of a "phase-pure" cfg4 round (diagnostic).
// Each receiver's 32 neighbour ids are stored sorted by source half (count c_A of low-half ids).
// A persistent grid (4 blocks/CU) walks the receivers in generations; within a generation every
// block first gathers its low-half neighbours, meets the other blocks of its XCD group at a soft
// (bounded) barrier, then gathers the high-half neighbours.  No data crosses blocks, so the
// barrier only shapes the per-XCD L2 working set (4 MiB instead of 8 MiB); correctness would not
// depend on it.  Compared with the one-pass design ("base").
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
constexpr uint32_t N = 1u << 20, HALF = N / 2;

__global__ __launch_bounds__(256) void k_base(const uint32_t* ids, const double* x, double* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const uint32_t* cp = ids + (uint64_t)(i >> 6) * 32 * 64 + (i & 63);
    double v[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) v[t] = x[cp[t * 64]];
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

template <int PHASED, int GROUPS>
__global__ __launch_bounds__(256, 1) void k_persist(const uint32_t* ids, const uint8_t* cA, const double* x,
                                                    double* out, uint32_t* ctr, int spin_limit) {
    const uint32_t nb = gridDim.x, g = blockIdx.x % GROUPS, rho = blockIdx.x / GROUPS;
    const uint32_t per_group = nb / GROUPS;
    const uint32_t slices_per_group = N / 256 / GROUPS;
    uint32_t epoch = 0;
    for (uint32_t s = rho; s < slices_per_group; s += per_group) {
        const uint32_t i = (g * slices_per_group + s) * 256 + threadIdx.x;
        const uint32_t* cp = ids + (uint64_t)(i >> 6) * 32 * 64 + (i & 63);
        const uint32_t ca = cA[i];
        double v[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) {     // phase A: low-half ids (t < c_A), else own value
            const uint32_t j = cp[t * 64];
            v[t] = x[(uint32_t)t < ca ? j : i];
        }
        if (PHASED) soft_barrier(ctr + g * 64, (++epoch) * per_group, spin_limit);
#pragma unroll
        for (int t = 0; t < 32; ++t) {     // phase B: high-half ids
            const uint32_t j = cp[t * 64];
            const bool hb = (uint32_t)t >= ca;
            const double vb = x[hb ? j : i];
            v[t] = hb ? vb : v[t];
        }
        double acc = 0;
#pragma unroll
        for (int t = 0; t < 32; ++t) acc += v[t];
        out[i] = acc;
        if (PHASED) soft_barrier(ctr + g * 64, (++epoch) * per_group, spin_limit);
    }
}

int main() {
    // random neighbour ids, each row sorted so low-half ids come first
    std::vector<uint32_t> rows(N * 32), ell(N * 32);
    std::vector<uint8_t> ca(N);
    uint64_t s = 88172645463325252ull;
    for (uint32_t i = 0; i < N; ++i) {
        uint32_t* r = &rows[i * 32];
        for (int t = 0; t < 32; ++t) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; r[t] = (uint32_t)(s >> 20) & (N - 1); }
        std::stable_partition(r, r + 32, [](uint32_t v) { return v < HALF; });
        ca[i] = (uint8_t)std::count_if(r, r + 32, [](uint32_t v) { return v < HALF; });
        for (int t = 0; t < 32; ++t) ell[((i >> 6) * 32 + t) * 64 + (i & 63)] = r[t];
    }
    uint32_t *ids, *ctr; uint8_t* dca; double *x, *out;
    CK(hipMalloc(&ids, N * 128));
    CK(hipMalloc(&dca, N));
    CK(hipMalloc(&x, N * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMalloc(&ctr, 8 * 64 * 4));
    CK(hipMemcpy(ids, ell.data(), N * 128, hipMemcpyHostToDevice));
    CK(hipMemcpy(dca, ca.data(), N, hipMemcpyHostToDevice));
    CK(hipMemset(x, 0, N * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timeit = [&](const char* name, auto fn) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipEventRecord(a));
        const int reps = 30;
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        CK(hipGetLastError());
        const float us = ms * 1000.f / reps;
        printf("%s,%.1f,%.0f\n", name, us, 400.0 * N / (us * 1e-6) / 1e9);
    };
    printf("design,us,alg_GBps\n");
    timeit("base_sorted_ids", [&] { hipLaunchKernelGGL(k_base, dim3(N / 256), dim3(256), 0, 0, ids, x, out); });
    for (int nb : {512, 1024}) {
        char name[64];
        snprintf(name, 64, "persist_nophase_nb%d", nb);
        timeit(name, [&] { hipLaunchKernelGGL((k_persist<0, 8>), dim3(nb), dim3(256), 0, 0, ids, dca, x, out, ctr, 0); });
        for (int sl : {200, 2000, 20000}) {
            snprintf(name, 64, "persist_phased_nb%d_spin%d", nb, sl);
            timeit(name, [&] {
                CK(hipMemsetAsync(ctr, 0, 8 * 64 * 4));
                hipLaunchKernelGGL((k_persist<1, 8>), dim3(nb), dim3(256), 0, 0, ids, dca, x, out, ctr, sl);
            });
        }
    }
    return 0;
}
