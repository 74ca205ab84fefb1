// mall_probe.hip — does the 256 MiB Infinity Cache (MALL) serve a streamed buffer that was just
// written, and does rewriting a resident buffer avoid HBM write-back?  Diagnostic only: decides
// whether receiver-range chunking of the binned exchange (a stage that stays on-die) can pay.
//   read  S : 16-B loads over S bytes, repeated (steady state: resident iff S fits)
//   write S : 16-B stores over S bytes, repeated
//   w+r   S : write S then read S, repeated (the stage hand-off of phase A -> phase B)
//   ldsdma S: 16-B LDS-DMA loads of S bytes (phase B's transfer form), after a write of S
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ p, uint64_t n16, uint32_t salt) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, salt, 0u, 1u);
}

// phase-B shaped: each workgroup copies 64 KiB chunks into LDS by 16-B LDS-DMA, then touches them
__global__ __launch_bounds__(256) void k_ldsdma(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint4 lds[4096];   // 64 KiB
    uint32_t acc = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * 4096; c < n16; c += (uint64_t)gridDim.x * 4096) {
        const uint32_t w = threadIdx.x >> 6;
        for (uint32_t o = w * 64; o < 4096; o += 256)
            if (c + o + (threadIdx.x & 63) < n16)
                __builtin_amdgcn_global_load_lds(p + c + o + (threadIdx.x & 63), lds + o, 16, 0, 0);
        __syncthreads();
        acc ^= lds[threadIdx.x * 16].x;
        __syncthreads();
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const uint64_t MiB = 1ull << 20;
    uint4* buf;
    uint32_t* sink;
    const uint64_t cap = 1024 * MiB;
    CK(hipMalloc(&buf, cap));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, cap));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = 256 * 8;
    auto timeit = [&](auto fn, int reps) {
        for (int w = 0; w < 3; ++w) fn();
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) fn();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms / reps;
    };
    printf("mode,MiB,us,GBps\n");
    const uint64_t sizes[] = {32, 64, 96, 128, 160, 192, 224, 256, 320, 384, 512, 1024};
    for (uint64_t s : sizes) {
        const uint64_t n16 = s * MiB / 16;
        const double by = (double)s * MiB;
        float t = timeit([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, buf, n16, sink); }, 20);
        printf("read,%llu,%.2f,%.1f\n", (unsigned long long)s, t * 1e3, by / t / 1e6);
        t = timeit([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, buf, n16, 7u); }, 20);
        printf("write,%llu,%.2f,%.1f\n", (unsigned long long)s, t * 1e3, by / t / 1e6);
        // write then read: time the pair, and the read alone after a write (events in between)
        float tw = 0, tr = 0;
        for (int r = 0; r < 13; ++r) {
            hipEvent_t e0, e1, e2;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipEventCreate(&e2));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, buf, n16, (uint32_t)r);
            CK(hipEventRecord(e1));
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, buf, n16, sink);
            CK(hipEventRecord(e2));
            CK(hipEventSynchronize(e2));
            float x, y;
            CK(hipEventElapsedTime(&x, e0, e1));
            CK(hipEventElapsedTime(&y, e1, e2));
            if (r >= 3) { tw += x; tr += y; }
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(e1));
            CK(hipEventDestroy(e2));
        }
        printf("w+r:write,%llu,%.2f,%.1f\n", (unsigned long long)s, tw / 10 * 1e3, by / (tw / 10) / 1e6);
        printf("w+r:read,%llu,%.2f,%.1f\n", (unsigned long long)s, tr / 10 * 1e3, by / (tr / 10) / 1e6);
        t = timeit([&] { hipLaunchKernelGGL(k_ldsdma, dim3(1024), dim3(256), 0, 0, buf, n16, sink); }, 20);
        printf("ldsdma,%llu,%.2f,%.1f\n", (unsigned long long)s, t * 1e3, by / t / 1e6);
        fflush(stdout);
    }
    return 0;
}
