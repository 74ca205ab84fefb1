// dma_asm_check.hip — does an asm `global_load_lds_dwordx4 voffset, saddr` with M0 set in the same
// statement copy a run into LDS like the compiler's __builtin_amdgcn_global_load_lds?  Diagnostic for
// DESIGN.md §5.11 (the phase-B asm DMA variant failed its bit-exactness tests).  One workgroup of 256
// threads copies 4 runs per wave (lengths 1..150 16-B units, random source offsets) both ways into
// LDS, dumps both images, and the host compares them.   usage: dma_asm_check
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kUnits = 4096;   // 64 KiB image

__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ src, const uint2* __restrict__ runs,
                                              int nruns, int use_asm, uint4* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint4 img[kUnits];
    for (int i = threadIdx.x; i < kUnits; i += 256) img[i] = make_uint4(0xdeadbeef, 0, 0, 0);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t lb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)img;
    uint32_t pre = 0;
    for (int k = 0; k < nruns; ++k) {          // run k: (source unit offset, length in units)
        const uint2 r = runs[k];
        if ((int)w == k % 4) {
            for (uint32_t o = 0; o < r.y; o += 64) {
                if (lane < r.y - o) {
                    if (use_asm) {
                        const uint64_t sb = (uint64_t)(uintptr_t)(src + r.x + o);
                        const uint32_t m0 = lb + (pre + o) * 16u;
                        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                                     :: "v"(lane * 16u), "s"(sb), "s"(m0) : "memory");
                    } else {
                        __builtin_amdgcn_global_load_lds(src + r.x + o + lane, img + pre + o, 16, 0, 0);
                    }
                }
            }
        }
        pre += r.y;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < kUnits; i += 256) out[i] = img[i];
}

int main() {
    const int nsrc = 1 << 20;
    uint4* h = (uint4*)malloc(nsrc * 16);
    for (int i = 0; i < nsrc; ++i) h[i] = make_uint4(i, i * 3u, ~i, 7);
    const int nruns = 48;
    uint2 hr[nruns];
    srand(1);
    int tot = 0;
    for (int k = 0; k < nruns; ++k) {
        hr[k] = make_uint2(rand() % (nsrc - 256), 1 + rand() % 150);
        if (tot + (int)hr[k].y > kUnits) hr[k].y = 0;
        tot += hr[k].y;
    }
    uint4 *src, *o0, *o1;
    uint2* dr;
    CK(hipMalloc(&src, nsrc * 16));
    CK(hipMalloc(&o0, kUnits * 16));
    CK(hipMalloc(&o1, kUnits * 16));
    CK(hipMalloc(&dr, sizeof hr));
    CK(hipMemcpy(src, h, nsrc * 16, hipMemcpyHostToDevice));
    CK(hipMemcpy(dr, hr, sizeof hr, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, 0, src, dr, nruns, 0, o0);
    hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, 0, src, dr, nruns, 1, o1);
    CK(hipDeviceSynchronize());
    uint4* a = (uint4*)malloc(kUnits * 16);
    uint4* b = (uint4*)malloc(kUnits * 16);
    CK(hipMemcpy(a, o0, kUnits * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b, o1, kUnits * 16, hipMemcpyDeviceToHost));
    int bad = 0, badref = 0, first = -1, pre = 0;
    for (int k = 0; k < nruns; ++k) {
        for (uint32_t u = 0; u < hr[k].y; ++u) {
            const uint4 e = h[hr[k].x + u];
            const uint4 x = a[pre + u], y = b[pre + u];
            badref += x.x != e.x || x.y != e.y;
            if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) { if (first < 0) first = pre + u; ++bad; }
        }
        pre += hr[k].y;
    }
    printf("units %d: builtin vs expected mismatches %d; asm vs builtin mismatches %d (first at %d)\n", tot, badref, bad, first);
    if (first >= 0) printf("builtin %08x asm %08x\n", a[first].x, b[first].x);
    return bad || badref;
}
