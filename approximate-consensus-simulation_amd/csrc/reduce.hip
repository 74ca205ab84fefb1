// reduce.hip — ε-spread test and termination.
//
// The round kernels leave one honest (min, max) partial per block; k_finalize (one workgroup per
// instance) folds them, records spread^{r+1}, sets converged / done and bumps the device-side
// done counter.  Every later round kernel reads the done flag first and exits, so the final x
// of an instance is exactly x^{rounds} however many rounds the host enqueued ahead.
#include "resolve.hpp"

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
    InstState* S = a.st + lb;
    if (!a.init_mode && S->done) return;
    const double2* p = a.partial + (uint64_t)lb * a.nblk;
    double mn = kInf, mx = -kInf;
    // 8 independent loads in flight per lane: a serial load->min chain over thousands of
    // partials costs one memory latency per step (≈7 µs at 4096 partials, measured)
    constexpr uint32_t U = 8;
    uint32_t k = threadIdx.x;
    for (; k + (U - 1) * kReduceBlock < a.nblk; k += U * kReduceBlock) {
        double2 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = p[k + u * kReduceBlock];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            mn = __builtin_fmin(mn, a.negmin ? -v[u].x : v[u].x);
            mx = __builtin_fmax(mx, v[u].y);
        }
    }
    for (; k < a.nblk; k += kReduceBlock) {
        const double2 v = p[k];
        mn = __builtin_fmin(mn, a.negmin ? -v.x : v.x);
        mx = __builtin_fmax(mx, v.y);
    }
    __shared__ double2 red[kReduceBlock / 64];
    mn = wave_min(mn);
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_double2(mn, mx);
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 1; k < kReduceBlock / 64; ++k) {
            mn = __builtin_fmin(mn, red[k].x);
            mx = __builtin_fmax(mx, red[k].y);
        }
        mn = __builtin_fmin(mn, red[0].x);
        mx = __builtin_fmax(mx, red[0].y);
        if (a.fold_out) {   // node partition: hand (-min, max) to the all-reduce
            *a.fold_out = make_double2(-mn, mx);
            return;
        }
        const double spread = a.f32 ? (double)(float)(mx - mn) : mx - mn;   // binary32 subtraction
        S->lo = mn;
        S->hi = mx;
        S->spread = spread;
        S->rounds = a.r_next;
        const bool conv = spread <= a.eps;
        const bool done = (a.term_eps && conv) || a.r_next >= a.max_rounds;
        S->converged = conv ? 1u : 0u;
        S->done = done ? 1u : 0u;
        if (a.trace) a.trace[(uint64_t)lb * a.trace_stride + a.r_next] = spread;
        if (done) atomicAdd(a.n_done, 1u);
    }
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
