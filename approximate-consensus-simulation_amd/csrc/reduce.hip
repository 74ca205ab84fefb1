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
// One-launch summary (launch_run_summary_mapped): per-block partial -> agent-scope release ->
// arrival counter; the last block acquires, folds the partials and writes `out` (host memory).
struct SumPart {
    uint32_t rmax, conv;
    uint64_t rsum, smax;
    uint32_t ndone, pad;
};
__global__ __launch_bounds__(kReduceBlock) void k_run_summary_mapped(const InstState* __restrict__ st, uint64_t B,
                                                                     unsigned char* scratch, RunSummary* out,
                                                                     unsigned long long seq) {
    uint32_t* cnt = reinterpret_cast<uint32_t*>(scratch);
    SumPart* part = reinterpret_cast<SumPart*>(scratch + 64);
    __shared__ SumPart red[kReduceBlock / 64];
    __shared__ uint32_t last;
    uint32_t rmax = 0, conv = 0, dn = 0;
    uint64_t rsum = 0, smax = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * kReduceBlock + threadIdx.x; b < B; b += (uint64_t)gridDim.x * kReduceBlock) {
        const InstState e = st[b];
        rmax = e.rounds > rmax ? e.rounds : rmax;
        conv += e.converged;
        dn += e.done != 0u;
        rsum += e.rounds;
        const uint64_t sb = (uint64_t)__double_as_longlong(e.spread);
        smax = sb > smax ? sb : smax;
    }
    auto fold_wave = [&]() {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t r2 = __shfl_xor(rmax, o, 64);
            const uint64_t s2 = __shfl_xor(smax, o, 64);
            rmax = r2 > rmax ? r2 : rmax;
            smax = s2 > smax ? s2 : smax;
            conv += __shfl_xor(conv, o, 64);
            dn += __shfl_xor(dn, o, 64);
            rsum += __shfl_xor(rsum, o, 64);
        }
    };
    auto fold_block = [&]() {   // -> thread 0
        fold_wave();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = SumPart{rmax, conv, rsum, smax, dn, 0u};
        __syncthreads();
        if (threadIdx.x == 0)
            for (uint32_t w = 1; w < kReduceBlock / 64; ++w) {
                rmax = red[w].rmax > rmax ? red[w].rmax : rmax;
                smax = red[w].smax > smax ? red[w].smax : smax;
                conv += red[w].conv;
                dn += red[w].ndone;
                rsum += red[w].rsum;
            }
    };
    fold_block();
    if (threadIdx.x == 0) {
        part[blockIdx.x] = SumPart{rmax, conv, rsum, smax, dn, 0u};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 == gridDim.x;
    }
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    rmax = 0, conv = 0, dn = 0, rsum = 0, smax = 0;
    for (uint32_t k = threadIdx.x; k < gridDim.x; k += kReduceBlock) {
        const SumPart q = part[k];
        rmax = q.rmax > rmax ? q.rmax : rmax;
        smax = q.smax > smax ? q.smax : smax;
        conv += q.conv;
        dn += q.ndone;
        rsum += q.rsum;
    }
    __syncthreads();   // (red[] reuse)
    fold_block();
    if (threadIdx.x == 0) {
        out->rounds_max = rmax;
        out->n_done = dn;
        out->n_converged = conv;
        out->rounds_sum = rsum;
        out->spread_max_bits = smax;
        *cnt = 0;   // ready for the next launch (stream-ordered)
        // last: the sequence number, released at system scope after the fields above (the host polls it)
        __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_run_summary_mapped(const InstState* st, uint64_t B, void* scratch, RunSummary* out,
                                     unsigned long long seq, hipStream_t s) {
    const uint64_t g = (B + kReduceBlock - 1) / kReduceBlock;
    static_assert(64 + 1024 * sizeof(SumPart) <= kSummaryScratch, "summary scratch");
    hipLaunchKernelGGL(k_run_summary_mapped, dim3((unsigned)(g == 0 ? 1 : g < 1024 ? g : 1024)), dim3(kReduceBlock), 0, s,
                       st, B, reinterpret_cast<unsigned char*>(scratch), out, seq);
    return hipGetLastError();
}

// One thread copies the B <= kMappedStates states (its own stores, so the release below orders them)
__global__ __launch_bounds__(64) void k_states_mapped(const InstState* __restrict__ st,
                                                      const uint32_t* __restrict__ n_done, uint32_t B,
                                                      MappedStates* out, unsigned long long seq) {
    if (threadIdx.x != 0) return;
    for (uint32_t b = 0; b < B; ++b) out->st[b] = st[b];
    out->n_done = *n_done;
    __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_states_mapped(const InstState* st, const uint32_t* n_done, uint32_t B, MappedStates* out,
                                unsigned long long seq, hipStream_t s) {
    if (B > kMappedStates) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_states_mapped, dim3(1), dim3(64), 0, s, st, n_done, B, out, seq);
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
