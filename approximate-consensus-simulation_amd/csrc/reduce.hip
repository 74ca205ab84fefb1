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
