// hybrid_probe.hip — can per-lane random gathers from an L2-sized table run BESIDE a streaming
// kernel without slowing it?  Diagnostic for a hybrid cfg4 round (part of the deliveries gathered
// directly from an L2-resident slice of x, the rest through the binned stage).
//   stream : 64 MiB read (16-B loads) + 256 MiB written (16-B stores), the shape of phase A
//   gather : 2^20 lanes x G random 8-byte gathers from a T-byte table + one 8-byte store per lane
//   both   : the two kernels on two streams, launched together
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

template <int NT>
__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16in) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16in; i += (uint64_t)gridDim.x * 256) {
        u4 v;
        if (NT) v = __builtin_nontemporal_load(reinterpret_cast<const u4*>(in) + i);
        else { const uint4 t = in[i]; v = u4{t.x, t.y, t.z, t.w}; }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            u4 w = v + (unsigned)q;
            if (NT) __builtin_nontemporal_store(w, reinterpret_cast<u4*>(out) + i * 4 + q);
            else out[i * 4 + q] = make_uint4(w.x, w.y, w.z, w.w);
        }
    }
}

template <int G>
__global__ __launch_bounds__(256) void k_gather(const double* __restrict__ tab, uint32_t mask, double* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    double v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) v[g] = tab[mix(i * G + g) & mask];
    double acc = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) acc += v[g];
    out[i] = acc;
}

int main() {
    const uint64_t MiB = 1ull << 20;
    uint4 *in, *out;
    double *tab, *gout;
    CK(hipMalloc(&in, 64 * MiB));
    CK(hipMalloc(&out, 256 * MiB));
    CK(hipMalloc(&tab, 8 * MiB));
    CK(hipMalloc(&gout, 8 * MiB));
    CK(hipMemset(in, 1, 64 * MiB));
    CK(hipMemset(tab, 0, 8 * MiB));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint64_t n16 = 64 * MiB / 16;
    auto timeit = [&](auto fn) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipDeviceSynchronize());
        const int reps = 20;
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3f / reps;
    };
    auto stream = [&](int nt, hipStream_t s) {
        if (nt) hipLaunchKernelGGL(k_stream<1>, dim3(2048), dim3(256), 0, s, in, out, n16);
        else hipLaunchKernelGGL(k_stream<0>, dim3(2048), dim3(256), 0, s, in, out, n16);
    };
    auto gather = [&](int G, uint32_t tmask, hipStream_t s) {
        if (G == 8) hipLaunchKernelGGL(k_gather<8>, dim3(4096), dim3(256), 0, s, tab, tmask, gout);
        else if (G == 16) hipLaunchKernelGGL(k_gather<16>, dim3(4096), dim3(256), 0, s, tab, tmask, gout);
        else hipLaunchKernelGGL(k_gather<4>, dim3(4096), dim3(256), 0, s, tab, tmask, gout);
    };
    printf("case,us\n");
    for (int nt = 0; nt < 2; ++nt) printf("stream_nt%d,%.1f\n", nt, timeit([&] { stream(nt, s1); }));
    for (uint32_t tmb : {1u, 2u, 4u}) {
        const uint32_t mask = tmb * MiB / 8 - 1;
        for (int G : {4, 8, 16}) {
            printf("gather_T%uMiB_G%d,%.1f\n", tmb, G, timeit([&] { gather(G, mask, s2); }));
            for (int nt = 0; nt < 2; ++nt)
                printf("both_nt%d_T%uMiB_G%d,%.1f\n", nt, tmb, G, timeit([&] { stream(nt, s1); gather(G, mask, s2); }));
        }
        fflush(stdout);
    }
    return 0;
}
