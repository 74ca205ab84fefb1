// reduce.hip — ε-spread test and termination.
//
// The round kernels leave one honest (min, max) partial per block; k_finalize (one workgroup per
// instance) folds them, records spread^{r+1}, sets converged / done and bumps the device-side
// done counter.  Every later round kernel reads the done flag first and exits, so the final x
// of an instance is exactly x^{rounds} however many rounds the host enqueued ahead.
#include "finalize.hpp"

namespace acs {

constexpr int kReduceBlock = 256;

template <typename VT>
__global__ __launch_bounds__(kReduceBlock) void k_partials_from_x(const VT* __restrict__ x,
                                                                  const uint32_t* __restrict__ status,
                                                                  uint64_t N, double2* partial,
                                                                  uint32_t nblk) {
    const uint32_t lb = blockIdx.y;
    const VT* xb = x + lb * N;
    const uint32_t* sb = status ? status + lb * N : nullptr;
    const uint64_t per = (N + nblk - 1) / nblk;
    const uint64_t beg = (uint64_t)blockIdx.x * per;
    const uint64_t end = beg + per < N ? beg + per : N;
    double mn = kInf, mx = -kInf;
    for (uint64_t i = beg + threadIdx.x; i < end; i += kReduceBlock) {
        if (sb && sb[i] != kHonest) continue;
        const double v = (double)xb[i];
        mn = __builtin_fmin(mn, v);
        mx = __builtin_fmax(mx, v);
    }
    block_minmax_store<kReduceBlock>(mn, mx, partial + (uint64_t)lb * nblk + blockIdx.x);
}

__global__ __launch_bounds__(kReduceBlock) void k_finalize(const FinalizeArgs a) {
    const uint32_t lb = blockIdx.x;
    if (!a.init_mode && a.st[lb].done) return;
    finalize_instance<false>(a, lb);
}

// acs_run's summary over the B instance states (rounds_max, converged count, Σ rounds, max final
// spread) folded on the device, so a run returns 32 bytes instead of copying B states to the host.
// Spreads are >= +0.0, so their bit patterns order as unsigned integers.
__global__ __launch_bounds__(kReduceBlock) void k_run_summary(const InstState* __restrict__ st, uint64_t B,
                                                              RunSummary* out) {
    uint32_t rmax = 0, conv = 0;
    uint64_t rsum = 0, smax = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * kReduceBlock + threadIdx.x; b < B; b += (uint64_t)gridDim.x * kReduceBlock) {
        const InstState e = st[b];
        rmax = e.rounds > rmax ? e.rounds : rmax;
        conv += e.converged;
        rsum += e.rounds;
        const uint64_t sb = (uint64_t)__double_as_longlong(e.spread);
        smax = sb > smax ? sb : smax;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint32_t r2 = __shfl_xor(rmax, o, 64);
        const uint64_t s2 = __shfl_xor(smax, o, 64);
        rmax = r2 > rmax ? r2 : rmax;
        smax = s2 > smax ? s2 : smax;
        conv += __shfl_xor(conv, o, 64);
        rsum += __shfl_xor(rsum, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&out->rounds_max, rmax);
        atomicAdd(&out->n_converged, (unsigned long long)conv);
        atomicAdd(&out->rounds_sum, (unsigned long long)rsum);
        atomicMax(&out->spread_max_bits, (unsigned long long)smax);
    }
}

hipError_t launch_run_summary(const InstState* st, uint64_t B, RunSummary* out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(RunSummary), s);
    if (e != hipSuccess) return e;
    const uint64_t g = (B + kReduceBlock - 1) / kReduceBlock;
    hipLaunchKernelGGL(k_run_summary, dim3((unsigned)(g < 1024 ? g : 1024)), dim3(kReduceBlock), 0, s, st, B, out);
    return hipGetLastError();
}

hipError_t launch_partials_from_x(const double* x, const uint32_t* status, uint64_t B, uint64_t N,
                                  double2* partial, uint32_t nblk, bool f32, hipStream_t s) {
    if (f32)
        hipLaunchKernelGGL(k_partials_from_x<float>, dim3(nblk, (unsigned)B), dim3(kReduceBlock), 0, s,
                           reinterpret_cast<const float*>(x), status, N, partial, nblk);
    else
        hipLaunchKernelGGL(k_partials_from_x<double>, dim3(nblk, (unsigned)B), dim3(kReduceBlock), 0, s, x,
                           status, N, partial, nblk);
    return hipGetLastError();
}

hipError_t launch_finalize(const FinalizeArgs& a, uint64_t B, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)B), dim3(kReduceBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace acs
