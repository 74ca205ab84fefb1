// rules.hpp — the §A.7 update rules over a register-resident entry array (SURVEY §8(a) a7+a8),
// shared by the register round kernels (round_regular.hip, round_binned.hip).
#pragma once

#include "sortnet.hpp"

namespace acs {

// v[0..D] holds the m = D+1 resolved entries (entry order for AVERAGE; any order for the
// sort-based rules, whose result depends only on the multiset).
template <int D, int T>
__device__ __forceinline__ double apply_rule_reg(uint32_t rule, double (&v)[D + 1]) {
    constexpr int M = D + 1;
    if constexpr (T == 0) {
        if (rule == 0) return tree_sum_const<M>(v) / (double)M;   // AVERAGE: entry order
    }
    select_sort<M, T, M - T>(v);
    constexpr int NR = M - 2 * T;
    if (rule == 2) return (v[T] + v[M - T - 1]) * 0.5;                // MIDPOINT
    if constexpr (T >= 1) {
        if (rule == 3) {                                             // DLPSW: R[0], R[T], ...
            constexpr int NQ = (NR + T - 1) / T;
            return tree_sum_const<NQ, T, T>(v) / (double)NQ;
        }
    }
    return tree_sum_const<NR, T>(v) / (double)NR;                    // TRIMMED_MEAN
}

}  // namespace acs
