// setup.hip — one-time device setup: initial values, the Feistel
// graph as an ELL slice layout, and the fault schedule.  Not timed as the hot path, but
// bit-exact with the spec like everything else.
#include <cstdlib>
#include <hipcub/hipcub.hpp>

#include "engine.hpp"
#include "sortnet.hpp"

namespace acs {

// §A.2: x_i^0 = u53(draw(INIT,b,0,2i), draw(INIT,b,0,2i+1)); both words come from one Philox
// call (counter (2i)>>2 = i>>1, words 2(i&1) and 2(i&1)+1).
// fp32 mode: x_i = (draw(INIT, b, 0, 2i) >> 8) * 2^-24, exact in binary32
__global__ __launch_bounds__(256) void k_init_values(double* x, uint64_t N, Key key, uint64_t inst_offset,
                                                     uint32_t f32) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t lb = blockIdx.y;
    if (i >= N) return;
    const uint32_t b = (uint32_t)(inst_offset + lb);
    const U4 w = philox10((uint32_t)(i >> 1), 0u, b, kStreamInit, key);
    const uint32_t sel = (uint32_t)((i & 1u) << 1);
    if (f32)
        reinterpret_cast<float*>(x)[lb * N + i] = (float)(pick(w, sel) >> 8) * 0x1p-24f;
    else
        x[lb * N + i] = u53(pick(w, sel), pick(w, sel + 1));
}

// §A.3: column t of node i is π_{t/2}(i) (t even) or π_{t/2}^{-1}(i) (t odd).  Builds the rows
// [row0, row0 + nrows) (a node partition; 0, N otherwise) into a local ELL.
__global__ __launch_bounds__(256) void k_build_ell(uint32_t* ell, uint64_t N, uint64_t row0, uint64_t nrows,
                                                   uint32_t d, uint32_t dp, Feistel f) {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t half = d >> 1;
    const uint64_t li = gid / half;
    const uint32_t k = (uint32_t)(gid % half);
    const uint64_t i = row0 + li;
    if (li >= nrows || i >= N) return;
    const uint32_t fw = feistel_fwd(f, k, (uint32_t)i);
    const uint32_t iv = feistel_inv(f, k, (uint32_t)i);
    const uint64_t base = ((li >> 6) * (dp >> 2)) * 256 + (li & 63) * 4;
    const uint32_t t0 = 2 * k, t1 = 2 * k + 1;
    ell[base + (uint64_t)(t0 >> 2) * 256 + (t0 & 3)] = fw;
    ell[base + (uint64_t)(t1 >> 2) * 256 + (t1 & 3)] = iv;
}

// Sort every row of the ELL ascending (rows of D ids, D a compile-time multiple of 4).  Used
// only for clean configs under order-independent rules (trimmed mean / midpoint / DLPSW sort the
// received values anyway, and a clean config has no slot-dependent drop or fault decisions), so
// the round's result is unchanged; the gathers of one wave instruction then fall into a narrow
// band of x (the t-th smallest neighbour of every lane), which measurably improves L2 reuse.
template <int D>
__global__ __launch_bounds__(256) void k_sort_ell_rows(uint32_t* ell, uint64_t N) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    uint4* cp = reinterpret_cast<uint4*>(ell) + (i >> 6) * (D / 4) * 64 + (i & 63);
    uint32_t v[D];
#pragma unroll
    for (int q = 0; q < D / 4; ++q) {
        const uint4 c = cp[q * 64];
        v[4 * q] = c.x; v[4 * q + 1] = c.y; v[4 * q + 2] = c.z; v[4 * q + 3] = c.w;
    }
    select_sort<D>(v);
#pragma unroll
    for (int q = 0; q < D / 4; ++q) cp[q * 64] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
}

hipError_t launch_sort_ell_rows(uint32_t* ell, uint64_t N, uint32_t d, hipStream_t s) {
    const dim3 grid((unsigned)((N + 255) / 256));
    switch (d) {
        case 4: hipLaunchKernelGGL(k_sort_ell_rows<4>, grid, dim3(256), 0, s, ell, N); break;
        case 8: hipLaunchKernelGGL(k_sort_ell_rows<8>, grid, dim3(256), 0, s, ell, N); break;
        case 16: hipLaunchKernelGGL(k_sort_ell_rows<16>, grid, dim3(256), 0, s, ell, N); break;
        case 32: hipLaunchKernelGGL(k_sort_ell_rows<32>, grid, dim3(256), 0, s, ell, N); break;
        default: return hipErrorNotSupported;
    }
    return hipGetLastError();
}

// §8(f) row 1: CSR rows as the padded ELL slice layout of the register / binned paths.
__global__ __launch_bounds__(256) void k_csr_to_ell(const uint64_t* __restrict__ rowptr, const uint32_t* __restrict__ colidx,
                                                    uint64_t N, uint32_t d, uint32_t* __restrict__ ell,
                                                    uint8_t* __restrict__ deg) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const uint64_t rp = rowptr[i];
    const uint64_t dg64 = rowptr[i + 1] - rp;
    const bool hub = dg64 > d;   // served by the generic kernel: an empty ELL row
    const uint32_t dg = hub ? 0u : (uint32_t)dg64;
    deg[i] = hub ? kDegHub : (uint8_t)dg;
    for (uint32_t t = 0; t < d; ++t)
        ell[(((i >> 6) * (d >> 2) + (t >> 2)) * 64 + (i & 63)) * 4 + (t & 3)] = t < dg ? colidx[rp + t] : kEllNone;
}

// SELL-64 slice widths: 4-wide column groups used by the longest row of each 64-row slice
__global__ __launch_bounds__(256) void k_slice_width(const uint8_t* __restrict__ deg, uint64_t N, uint8_t* __restrict__ sw) {
    const uint64_t sl = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (sl * 64 >= N) return;
    uint32_t mx = 0;
    for (uint64_t k = sl * 64; k < N && k < sl * 64 + 64; ++k)
        if (deg[k] != kDegHub) mx = deg[k] > mx ? deg[k] : mx;
    sw[sl] = (uint8_t)((mx + 3) / 4);
}

hipError_t launch_csr_to_ell(const uint64_t* rowptr, const uint32_t* colidx, uint64_t N, uint32_t d, uint32_t* ell,
                             uint8_t* deg, uint8_t* sw, hipStream_t s) {
    hipLaunchKernelGGL(k_csr_to_ell, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rowptr, colidx, N, d, ell, deg);
    const uint64_t ns = (N + 63) / 64;
    hipLaunchKernelGGL(k_slice_width, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, s, deg, N, sw);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_fault_keys(uint64_t* keys, uint64_t N, Key key, uint64_t inst_offset) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint32_t lb = blockIdx.y;
    if (i >= N) return;
    const uint32_t b = (uint32_t)(inst_offset + lb);
    keys[lb * N + i] = ((uint64_t)draw(key, kStreamFaultset, b, 0, i) << 32) | i;
}

__global__ __launch_bounds__(256) void k_fill_u32(uint32_t* p, uint64_t n, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) p[i] = v;
}

// §A.4: the f smallest (key, i) pairs of each instance are faulty.
__global__ __launch_bounds__(256) void k_mark_faults(uint32_t* status, const uint64_t* sorted, uint64_t N,
                                                     uint32_t f, uint32_t model, uint32_t W, Key key,
                                                     uint64_t inst_offset) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    const uint32_t lb = blockIdx.y;
    if (k >= f) return;
    const uint32_t b = (uint32_t)(inst_offset + lb);
    const uint32_t v = (uint32_t)(sorted[lb * N + k] & 0xFFFFFFFFu);
    status[lb * N + v] = model == 2 ? kByz : draw(key, kStreamCrashRound, b, 0, v) % W;
}

struct SegOffset {
    uint64_t N;
    __host__ __device__ uint64_t operator()(uint64_t b) const { return b * N; }
};

hipError_t launch_init_values(double* x, uint64_t B, uint64_t N, Key key, uint64_t inst_offset, bool f32,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_init_values, dim3((unsigned)((N + 255) / 256), (unsigned)B), dim3(256), 0, s, x, N,
                       key, inst_offset, f32 ? 1u : 0u);
    return hipGetLastError();
}

hipError_t launch_build_ell(uint32_t* ell, uint64_t N, uint64_t row0, uint64_t nrows, uint32_t d, uint32_t dp,
                            const Feistel& f, hipStream_t s) {
    const uint64_t work = nrows * (d >> 1);
    hipLaunchKernelGGL(k_build_ell, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, s, ell, N, row0, nrows, d,
                       dp, f);
    return hipGetLastError();
}

// §A.4 fault schedule of B instances.  The segmented radix sort takes int sizes, so instances are
// processed in batches of nb with nb * N < 2^31 (and at most 2^28 keys, 4 GiB of key buffers);
// ACSIM_FAULT_BATCH caps nb (tests force several batches on small configs).  Needs N < 2^31.
hipError_t build_fault_status(uint32_t* status, uint64_t B, uint64_t N, uint32_t f,
                              uint32_t fault_model, uint32_t crash_window, Key key,
                              uint64_t inst_offset, hipStream_t s) {
    hipError_t e;
    hipLaunchKernelGGL(k_fill_u32, dim3(1024), dim3(256), 0, s, status, B * N, kHonest);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (fault_model == 0 || f == 0) return hipSuccess;
    if (N >= (1ull << 31)) return hipErrorNotSupported;
    uint64_t nb = ((1ull << 28) + N - 1) / N;   // instances per batch
    if (nb * N >= (1ull << 31)) nb = ((1ull << 31) - 1) / N;
    if (const char* v = getenv("ACSIM_FAULT_BATCH")) {
        const uint64_t cap = strtoull(v, nullptr, 10);
        if (cap && cap < nb) nb = cap;
    }
    if (nb > B) nb = B;
    if (nb > 65535) nb = 65535;   // grid y
    const uint64_t n = nb * N;
    uint64_t *keys = nullptr, *sorted = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    if ((e = hipMalloc(&keys, n * sizeof(uint64_t))) != hipSuccess) return e;
    if ((e = hipMalloc(&sorted, n * sizeof(uint64_t))) != hipSuccess) { (void)hipFree(keys); return e; }
    auto offs = hipcub::TransformInputIterator<uint64_t, SegOffset, hipcub::CountingInputIterator<uint64_t>>(
        hipcub::CountingInputIterator<uint64_t>(0), SegOffset{N});
    e = hipcub::DeviceSegmentedRadixSort::SortKeys(nullptr, temp_bytes, keys, sorted, (int)n, (int)nb, offs,
                                                   offs + 1, 0, 64, s);
    if (e == hipSuccess) e = hipMalloc(&temp, temp_bytes ? temp_bytes : 16);
    for (uint64_t b0 = 0; e == hipSuccess && b0 < B; b0 += nb) {
        const uint64_t bn = B - b0 < nb ? B - b0 : nb;
        hipLaunchKernelGGL(k_fault_keys, dim3((unsigned)((N + 255) / 256), (unsigned)bn), dim3(256), 0, s, keys, N,
                           key, inst_offset + b0);
        size_t tb = temp_bytes;
        e = hipcub::DeviceSegmentedRadixSort::SortKeys(temp, tb, keys, sorted, (int)(bn * N), (int)bn, offs,
                                                       offs + 1, 0, 64, s);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_mark_faults, dim3((f + 255) / 256, (unsigned)bn), dim3(256), 0, s, status + b0 * N,
                               sorted, N, f, fault_model, crash_window, key, inst_offset + b0);
            e = hipGetLastError();
        }
    }
    hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    (void)hipFree(temp);
    (void)hipFree(sorted);
    (void)hipFree(keys);
    return e;
}

}  // namespace acs
