// run_probe.hip — how fast can phase B's transfer form read the stage, as a function of the run
// length?  Diagnostic only.  The stage is 256 MiB laid out tile-major like the
// binned plan's: Q receiver blocks, 64 source blocks, tile (a, b) = RUN bytes at a * Q * RUN + b * RUN.
// Each 256-thread workgroup (36 KiB of LDS: 4 per CU, as k_bin_gather<32, 5, ..., 2>) copies its
// block's 64 runs into LDS by 16-B LDS-DMA, 32 KiB per part with a barrier after each part, and
// touches one word per lane; no pick-up, no sort.  The stage is rewritten before every timed read
// (phase A's stores, then phase B's reads), and only the read kernel is timed.
//   usage: run_probe [reps]   -> CSV: layout,run_B,blocks,us,GBps
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr uint64_t kStage = 256ull << 20;   // bytes
constexpr uint32_t kPart16 = 2048;          // 32 KiB per part, in 16-B units
constexpr uint32_t kRuns = 64;              // source blocks (runs per receiver block)

__global__ __launch_bounds__(256) void k_write(uint4* __restrict__ p, uint64_t n16, uint32_t salt) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        p[i] = make_uint4((uint32_t)i, salt, 0u, 1u);
}

// run16: run length in 16-B units; Q: receiver blocks; contig: the block's 64 runs adjacent
// (b * 64 * run + a * run) instead of tile-major (a * Q * run + b * run)
__global__ __launch_bounds__(256) void k_runs(const uint4* __restrict__ p, uint32_t run16, uint32_t Q, int contig,
                                              uint32_t* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kPart16 + 256];
    const uint32_t Qc = Q / 8;
    const uint32_t b = (blockIdx.x & 7u) * Qc + (blockIdx.x >> 3);   // XCD-aware, as k_bin_gather
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t rpp = kPart16 / run16;                             // runs per part
    uint32_t acc = 0;
    for (uint32_t a0 = 0; a0 < kRuns; a0 += rpp) {
        for (uint32_t a = a0 + w; a < a0 + rpp; a += 4) {              // wave w: every 4th run of the part
            const uint64_t off = contig ? ((uint64_t)b * kRuns + a) * run16 : ((uint64_t)a * Q + b) * run16;
            uint4* d = lds + (a - a0) * run16;
            for (uint32_t o = 0; o < run16; o += 64)
                if (o + lane < run16) __builtin_amdgcn_global_load_lds(p + off + o + lane, d + o + lane, 16, 0, 0);
        }
        __syncthreads();
        acc ^= lds[threadIdx.x * 8].x;
        __syncthreads();
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    uint4* p;
    uint32_t* sink;
    CK(hipMalloc(&p, kStage));
    CK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const uint64_t n16 = kStage / 16;
    printf("layout,run_B,blocks,us,GBps\n");
    const uint32_t runs[] = {512, 1024, 2048, 4096, 8192};
    for (int contig = 0; contig < 2; ++contig)
        for (uint32_t rb : runs) {
            const uint32_t run16 = rb / 16;
            const uint32_t Q = (uint32_t)(kStage / ((uint64_t)kRuns * rb));
            if (Q % 8 || kPart16 % run16) continue;
            float best = 1e30f, sum = 0.f;
            for (int r = 0; r < reps + 1; ++r) {
                hipLaunchKernelGGL(k_write, dim3(2048), dim3(256), 0, 0, p, n16, (uint32_t)r);
                CK(hipEventRecord(e0, 0));
                hipLaunchKernelGGL(k_runs, dim3(Q), dim3(256), 0, 0, p, run16, Q, contig, sink);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0.f;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r) {   // the first is a warm-up
                    best = ms < best ? ms : best;
                    sum += ms;
                }
            }
            const float us = sum / reps * 1e3f;
            printf("%s,%u,%u,%.2f,%.1f\n", contig ? "contiguous" : "tile-major", rb, Q, us,
                   (double)kStage / (us * 1e-6) / 1e9);
            fflush(stdout);
        }
    CK(hipFree(p));
    CK(hipFree(sink));
    return 0;
}
