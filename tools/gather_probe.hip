// gather_probe.hip — microbenchmark of the cfg4 access pattern (diagnostic tool, not product).
// Each lane = one receiver: D=32 neighbour ids from the ELL slice layout ([N/64][8][64] uint4),
// then 32 random 8-byte gathers from a table of T doubles.  Variants isolate the id stream,
// the gathers, cache policy bits (buffer-load aux), packed 20-bit ids and XCD-partitioned
// source tables.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/gather_probe tools/gather_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum { M_PLAIN = 0, M_IDS_ONLY = 2, M_HASH = 3, M_BUF = 5, M_PACKED = 6, M_HALF = 7, M_XCDPART = 8, M_PAIR16 = 9 };

template <int AUX>
__device__ __forceinline__ u32x4 bufload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}

template <int MODE, int AUX, int GAUX>
__global__ __launch_bounds__(256) void k_probe(const u32x4* __restrict__ ell, const double* __restrict__ x,
                                              double* __restrict__ out, uint32_t N, uint32_t tmask) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    uint32_t col[32];
    if (MODE == M_PACKED) {
        // 20-bit ids, 32 per row = 20 words = 5 uint4 per lane
        const u32x4* cp = ell + (uint64_t)(i >> 6) * 320 + (i & 63);
        uint32_t w[20];
#pragma unroll
        for (int q = 0; q < 5; ++q) {
            u32x4 c = cp[q * 64];
            w[4 * q] = c.x; w[4 * q + 1] = c.y; w[4 * q + 2] = c.z; w[4 * q + 3] = c.w;
        }
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const int bit = t * 20, wd = bit >> 5, sh = bit & 31;
            uint64_t v = w[wd];
            if (wd + 1 < 20) v |= (uint64_t)w[wd + 1] << 32;
            col[t] = (uint32_t)(v >> sh) & 0xFFFFF;
        }
    } else {
        const u32x4* cp = ell + (uint64_t)(i >> 6) * 512 + (i & 63);
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)ell, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            u32x4 c;
            if (MODE == M_HASH || (MODE == M_HALF && q >= 4))
                c = u32x4{i * 2654435761u + q, i * 40503u + 7u * q, i ^ (q * 977u), i * 69069u + q};
            else if (MODE == M_BUF)
                c = bufload<AUX>(rs, (uint32_t)(((i >> 6) * 512 + (i & 63) + q * 64) * 16));
            else
                c = cp[q * 64];
            col[4 * q] = c.x; col[4 * q + 1] = c.y; col[4 * q + 2] = c.z; col[4 * q + 3] = c.w;
        }
    }
    double acc = 0.0;
    if (MODE == M_IDS_ONLY) {
        uint32_t s = 0;
#pragma unroll
        for (int t = 0; t < 32; ++t) s += col[t];
        acc = (double)s;
    } else if (MODE == M_PAIR16) {
        typedef double d2 __attribute__((ext_vector_type(2)));
        d2 v[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) v[t] = *reinterpret_cast<const d2*>(x + ((col[t] & tmask) & ~1u));
#pragma unroll
        for (int t = 0; t < 32; ++t) acc += v[t].x + v[t].y;
    } else {
        uint32_t part = 0, pmask = tmask;
        if (MODE == M_XCDPART) {   // each XCD group gathers only from its own 1/8 of the table
            pmask = tmask >> 3;
            part = (blockIdx.x & 7u) * (pmask + 1);
        }
        __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, 0x7FFFFFF0, 0x00020000);
        double v[32];
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            const uint32_t j = part + (col[t] & pmask);
            if (GAUX) v[t] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, j * 8, 0, GAUX));
            else v[t] = x[j];
        }
#pragma unroll
        for (int t = 0; t < 32; ++t) acc += v[t];
    }
    out[i] = acc;
}

template <int MODE, int AUX = 0, int GAUX = 0>
float run(const u32x4* ell, const double* x, double* out, uint32_t N, uint32_t tmask, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_probe<MODE, AUX, GAUX>), dim3(N / 256), dim3(256), 0, 0, ell, x, out, N, tmask);
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((k_probe<MODE, AUX, GAUX>), dim3(N / 256), dim3(256), 0, 0, ell, x, out, N, tmask);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGetLastError());
    return ms * 1000.f / reps;
}

int main() {
    const uint32_t N = 1u << 20;
    const uint32_t TMAX = 1u << 24;
    std::vector<uint32_t> h(N * 32);
    uint64_t s = 88172645463325252ull;
    for (auto& v : h) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; v = (uint32_t)s & 0xFFFFF; }
    std::vector<double> hx(TMAX);
    for (uint32_t k = 0; k < TMAX; ++k) hx[k] = k * 1e-7;
    u32x4* ell; double *x, *out;
    CK(hipMalloc(&ell, N * 32 * 4));
    CK(hipMalloc(&x, (size_t)TMAX * 8));
    CK(hipMalloc(&out, N * 8));
    CK(hipMemcpy(ell, h.data(), N * 32 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(x, hx.data(), (size_t)TMAX * 8, hipMemcpyHostToDevice));
    const int reps = 40;
    const uint32_t T = 1u << 20, m = T - 1;
    printf("mode,us_per_launch,alg_GBps(400B/node)\n");
    auto rep = [&](const char* name, float us) { printf("%s,%.1f,%.0f\n", name, us, 400.0 * N / (us * 1e-6) / 1e9); };
    rep("plain_8MiB", run<M_PLAIN>(ell, x, out, N, m, reps));
    rep("ids_only", run<M_IDS_ONLY>(ell, x, out, N, m, reps));
    rep("hash_8MiB", run<M_HASH>(ell, x, out, N, m, reps));
    rep("buf_aux0", run<M_BUF, 0>(ell, x, out, N, m, reps));
    rep("buf_aux1_sc0", run<M_BUF, 1>(ell, x, out, N, m, reps));
    rep("buf_aux2_nt", run<M_BUF, 2>(ell, x, out, N, m, reps));
    rep("buf_aux3_sc0nt", run<M_BUF, 3>(ell, x, out, N, m, reps));
    rep("buf_aux16_sc1", run<M_BUF, 16>(ell, x, out, N, m, reps));
    rep("buf_aux17_sc0sc1", run<M_BUF, 17>(ell, x, out, N, m, reps));
    rep("buf_aux18_sc1nt", run<M_BUF, 18>(ell, x, out, N, m, reps));
    rep("buf_aux19_sc0sc1nt", run<M_BUF, 19>(ell, x, out, N, m, reps));
    rep("packed20_8MiB", run<M_PACKED>(ell, x, out, N, m, reps));
    rep("half_ids_8MiB", run<M_HALF>(ell, x, out, N, m, reps));
    rep("xcdpart_8MiB", run<M_XCDPART>(ell, x, out, N, m, reps));
    rep("pair16_8MiB", run<M_PAIR16>(ell, x, out, N, m, reps));
    rep("gather_aux1_sc0", run<M_PLAIN, 0, 1>(ell, x, out, N, m, reps));
    rep("gather_aux2_nt", run<M_PLAIN, 0, 2>(ell, x, out, N, m, reps));
    rep("buf19_gather1", run<M_BUF, 19, 1>(ell, x, out, N, m, reps));
    rep("xcdpart_buf19", run<M_XCDPART, 0, 0>(ell, x, out, N, m, reps));
    return 0;
}
