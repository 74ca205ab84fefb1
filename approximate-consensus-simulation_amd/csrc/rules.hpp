// rules.hpp — the §A.7 update rules over a register-resident entry array (SURVEY §8(a) a7+a8),
// shared by the register round kernels (round_regular.hip, round_binned.hip).
#pragma once

#include "sortnet.hpp"

namespace acs {

// v[0..D] holds the m = D+1 resolved entries (entry order for AVERAGE; any order for the
// sort-based rules, whose result depends only on the multiset).
// W-MSR over the m = D+1 entries, v[0] = the receiver's own value: full sort,
// drop min(T, #below) from the bottom and min(T, #above) from the top, tree_sum the window.
// The window start is a runtime value in [0, T]; zero padding past the window leaves the
// stride-halving sum unchanged (no -0.0 values), so the compile-time tree over next_pow2(M)
// equals the spec's tree over next_pow2(window).
template <int D, int T, typename VT>
__device__ __forceinline__ VT wmsr_reg(VT (&v)[D + 1]) {
    constexpr int M = D + 1;
    const VT xi = v[0];
    select_sort<M>(v);
    uint32_t nl = 0, ng = 0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        nl += v[k] < xi;
        ng += v[k] > xi;
    }
    const uint32_t lo = nl < (uint32_t)T ? nl : (uint32_t)T, hi = ng < (uint32_t)T ? ng : (uint32_t)T;
    const uint32_t nw = M - lo - hi;
    VT w[M];
#pragma unroll
    for (int k = 0; k < M; ++k) {
        VT s = v[k];
#pragma unroll
        for (int q = 1; q <= T; ++q)
            if (k + q < M && lo == (uint32_t)q) s = v[k + q];
        w[k] = (uint32_t)k < nw ? s : VT(0);
    }
    return tree_sum_const<M>(w) / (VT)nw;
}

// WMSR = true instantiates the W-MSR rule only (a separate kernel instantiation, so the other
// rules' kernels carry none of its registers).
template <int D, int T, bool WMSR = false, typename VT>
__device__ __forceinline__ VT apply_rule_reg(uint32_t rule, VT (&v)[D + 1]) {
    constexpr int M = D + 1;
    if constexpr (WMSR) {
        return wmsr_reg<D, T>(v);
    }
    if constexpr (T == 0) {
        if (rule == 0) return tree_sum_const<M>(v) / (VT)M;       // AVERAGE: entry order
    }
    select_sort<M, T, M - T>(v);
    constexpr int NR = M - 2 * T;
    if (rule == 2) return (v[T] + v[M - T - 1]) * VT(0.5);            // MIDPOINT
    if constexpr (T >= 1) {
        if (rule == 3) {                                             // DLPSW: R[0], R[T], ...
            constexpr int NQ = (NR + T - 1) / T;
            return tree_sum_const<NQ, T, T>(v) / (VT)NQ;
        }
    }
    return tree_sum_const<NR, T>(v) / (VT)NR;                        // TRIMMED_MEAN
}

}  // namespace acs
