// finalize.hpp — §A.8 spread / ε test of one instance from its block partials,
// shared by k_finalize (reduce.hip) and the last workgroup of a fused round kernel
// (round_binned.hip).  Called by a whole 256-thread workgroup.
#pragma once

#include "resolve.hpp"

namespace acs {

// SC1: the partials were handed over inside this launch by other workgroups (any XCD): each was
// stored with sc1 (agent-scope) stores and drained before the hand-off counter, so it is read back
// with sc1 loads too (MI355X_MICROARCH.md, correctness boundaries: inter-workgroup visibility).
template <bool SC1>
__device__ __forceinline__ double2 load_partial(const double2* p) {
    if constexpr (SC1) {
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        const unsigned long long lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_double2(__longlong_as_double((long long)lo), __longlong_as_double((long long)hi));
    } else {
        return *p;
    }
}

__device__ __forceinline__ void store_partial_sc1(double2* p, double2 v) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, (unsigned long long)__double_as_longlong(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, (unsigned long long)__double_as_longlong(v.y), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Fold the block partials of instance lb and evaluate §A.8.  Called by all NT threads of a
// workgroup; every thread returns the same verdict (done).  With `record`, thread 0 stores lo / hi /
// spread / rounds / converged / done, the trace entry and the done counter (a partition fold
// instead hands (-min, max) to fold_out and returns false).
template <bool SC1, uint32_t NT = 256>
__device__ __forceinline__ bool fold_partials(const FinalizeArgs& a, uint32_t lb, bool record) {
    InstState* S = a.st + lb;
    const double2* p = a.partial + (uint64_t)lb * a.nblk;
    double mn = kInf, mx = -kInf;
    // 8 independent loads in flight per lane: a serial load->min chain over thousands of
    // partials costs one memory latency per step (≈7 µs at 4096 partials, measured)
    constexpr uint32_t U = 8;
    uint32_t k = threadIdx.x;
    for (; k + (U - 1) * NT < a.nblk; k += U * NT) {
        double2 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = load_partial<SC1>(p + k + u * NT);
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            mn = __builtin_fmin(mn, a.negmin ? -v[u].x : v[u].x);
            mx = __builtin_fmax(mx, v[u].y);
        }
    }
    for (; k < a.nblk; k += NT) {
        const double2 v = load_partial<SC1>(p + k);
        mn = __builtin_fmin(mn, a.negmin ? -v.x : v.x);
        mx = __builtin_fmax(mx, v.y);
    }
    __shared__ double2 red[NT / 64];
    mn = wave_min(mn);
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_double2(mn, mx);
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < NT / 64; ++q) {
        mn = __builtin_fmin(mn, red[q].x);
        mx = __builtin_fmax(mx, red[q].y);
    }
    if (a.fold_out) {   // node partition: hand (-min, max) to the all-reduce
        if (record && threadIdx.x == 0) *a.fold_out = make_double2(-mn, mx);
        return false;
    }
    const double spread = a.f32 ? (double)(float)(mx - mn) : mx - mn;   // binary32 subtraction
    const bool conv = spread <= a.eps;
    const bool done = (a.term_eps && conv) || a.r_next >= a.max_rounds;
    if (record && threadIdx.x == 0) {
        S->lo = mn;
        S->hi = mx;
        S->spread = spread;
        S->rounds = a.r_next;
        S->converged = conv ? 1u : 0u;
        S->done = done ? 1u : 0u;
        if (a.trace) a.trace[(uint64_t)lb * a.trace_stride + a.r_next] = spread;
        if (done) atomicAdd(a.n_done, 1u);
    }
    return done;
}

template <bool SC1>
__device__ __forceinline__ void finalize_instance(const FinalizeArgs& a, uint32_t lb) {
    (void)fold_partials<SC1>(a, lb, true);
}

}  // namespace acs
