// mall_chunk_probe.hip — VERDICT r04 item 7: does phase B's transfer form read a
// stage chunk that phase A has JUST written, small enough to stay in the 256 MiB Infinity Cache
// (MALL), faster than the ~6.4 TB/s it reads the whole 256 MiB stage at?  Diagnostic only.
// The cfg4 stage (256 MiB, tile-major: 64 source blocks x Q receiver blocks of 1 KiB runs) is
// written and read in C receiver chunks: for c: write chunk c (phase A's streaming stores,
// write-through like the one-level default), then read chunk c (k_runs: 4 workgroups per CU,
// 16-B LDS-DMA, 32 KiB parts, as k_bin_gather's transfer).  C = 1 is today's round.  With
// `overlap`, chunk c + 1's write runs on a second stream beside chunk c's read (the pipelined
// form a chunked round would need, since a chunk's read launch alone fills 1 / C of the CU slots).
//   usage: mall_chunk_probe [reps]   -> CSV: C,overlap,chunk_MB,write_us,read_us,read_GBps,total_us
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr uint64_t kStage = 256ull << 20;   // bytes
constexpr uint32_t kPart16 = 2048;          // 32 KiB per part, in 16-B units
constexpr uint32_t kRuns = 64;              // source blocks (runs per receiver block)
constexpr uint32_t kRun16 = 64;             // 1 KiB runs (cfg4's tiles hold ~128 fp64 values)
constexpr uint32_t kQ = (uint32_t)(kStage / 16 / kRuns / kRun16);   // 4096 receiver blocks

// write-through (sc1) streaming stores of a chunk, 16 B per lane, 1 KiB per wave-instruction
__global__ __launch_bounds__(512) void k_write(uint4* __restrict__ p, uint64_t n16, uint32_t salt) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7FFFFFF0, 0x00020000);
    for (uint64_t i = (uint64_t)blockIdx.x * 512 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 512) {
        using UV = unsigned int __attribute__((ext_vector_type(4)));
        const UV v = {(uint32_t)i, salt, 0u, 1u};
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, (uint32_t)(i * 16), 0, 16);
    }
}

// read receiver blocks [0, Qc) of a chunk whose tiles are (a, b) at (a * Qc + b) * RUN
__global__ __launch_bounds__(256) void k_runs(const uint4* __restrict__ p, uint32_t Qc, uint32_t* __restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint4 lds[kPart16 + 256];
    const uint32_t q8 = Qc / 8;
    const uint32_t b = (blockIdx.x & 7u) * q8 + (blockIdx.x >> 3);   // XCD-aware, as k_bin_gather
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr uint32_t rpp = kPart16 / kRun16;
    uint32_t acc = 0;
    for (uint32_t a0 = 0; a0 < kRuns; a0 += rpp) {
        for (uint32_t a = a0 + w; a < a0 + rpp; a += 4) {
            const uint64_t off = ((uint64_t)a * Qc + b) * kRun16;
            __builtin_amdgcn_global_load_lds(p + off + lane, lds + (a - a0) * kRun16 + lane, 16, 0, 0);
        }
        __syncthreads();
        acc ^= lds[threadIdx.x * 8].x;
        __syncthreads();
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 5;
    uint4* p;
    uint32_t* sink;
    CK(hipMalloc(&p, kStage));
    CK(hipMalloc(&sink, 4));
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t ev[64];
    for (auto& evk : ev) CK(hipEventCreate(&evk));
    printf("C,overlap,chunk_MB,write_us,read_us,read_GBps,total_us\n");
    const uint32_t Cs[] = {1, 2, 4, 8};
    for (int overlap = 0; overlap < 2; ++overlap)
        for (uint32_t C : Cs) {
            if (overlap && C == 1) continue;
            const uint64_t cb = kStage / C, c16 = cb / 16;
            const uint32_t Qc = kQ / C;
            for (int r = 0; r < reps + 1; ++r) {
                // ev[4c]: write start, ev[4c+1]: write end, ev[4c+2]: read start, ev[4c+3]: read end
                CK(hipDeviceSynchronize());
                for (uint32_t c = 0; c < C; ++c) {
                    uint4* pc = p + c * c16;
                    hipStream_t ws = overlap ? s1 : s0;
                    if (overlap && c) CK(hipStreamWaitEvent(ws, ev[4 * (c - 1) + 1], 0));   // writes in order
                    CK(hipEventRecord(ev[4 * c], ws));
                    hipLaunchKernelGGL(k_write, dim3(256), dim3(512), 0, ws, pc, c16, (uint32_t)(r * 16 + c));
                    CK(hipEventRecord(ev[4 * c + 1], ws));
                    if (overlap) CK(hipStreamWaitEvent(s0, ev[4 * c + 1], 0));
                    CK(hipEventRecord(ev[4 * c + 2], s0));
                    hipLaunchKernelGGL(k_runs, dim3(Qc), dim3(256), 0, s0, pc, Qc, sink);
                    CK(hipEventRecord(ev[4 * c + 3], s0));
                }
                CK(hipDeviceSynchronize());
                if (r == 0) continue;   // warm-up
                float wsum = 0.f, rsum = 0.f, tot = 0.f, ms;
                for (uint32_t c = 0; c < C; ++c) {
                    CK(hipEventElapsedTime(&ms, ev[4 * c], ev[4 * c + 1]));
                    wsum += ms;
                    CK(hipEventElapsedTime(&ms, ev[4 * c + 2], ev[4 * c + 3]));
                    rsum += ms;
                }
                CK(hipEventElapsedTime(&tot, ev[0], ev[4 * (C - 1) + 3]));
                printf("%u,%d,%.1f,%.2f,%.2f,%.1f,%.2f\n", C, overlap, cb / 1e6, wsum * 1e3, rsum * 1e3,
                       kStage / (rsum * 1e-3) / 1e9, tot * 1e3);
                fflush(stdout);
            }
        }
    return 0;
}
