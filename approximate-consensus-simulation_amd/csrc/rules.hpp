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
// nmiss entries are absent (missing_policy = OMIT or a CSR receiver below the compiled degree):
// they hold +inf, sort last and are neither counted above x_i nor part of the window.
template <int D, int T, typename VT>
__device__ __forceinline__ VT wmsr_reg(VT (&v)[D + 1], uint32_t nmiss = 0) {
    constexpr int M = D + 1;
    const VT xi = v[0];
    select_sort<M>(v);
    uint32_t nl = 0, ng = 0;
#pragma unroll
    for (int k = 0; k < M; ++k) {
        nl += v[k] < xi;
        ng += v[k] > xi;
    }
    ng -= nmiss;
    const uint32_t lo = nl < (uint32_t)T ? nl : (uint32_t)T, hi = ng < (uint32_t)T ? ng : (uint32_t)T;
    const uint32_t nw = M - nmiss - lo - hi;
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
// rules' kernels carry none of its registers).  NZ: no value is -0.0 (tree_sum_const).
template <int D, int T, bool WMSR = false, bool NZ = false, typename VT>
__device__ __forceinline__ VT apply_rule_reg(uint32_t rule, VT (&v)[D + 1]) {
    constexpr int M = D + 1;
    if constexpr (WMSR) {
        return wmsr_reg<D, T>(v);
    }
    if constexpr (T == 0) {
        if (rule == 0) return tree_sum_const<M, 0, 1, NZ>(v) / (VT)M;       // AVERAGE: entry order
    }
    select_sort<M, T, M - T>(v);
    constexpr int NR = M - 2 * T;
    if (rule == 2) return (v[T] + v[M - T - 1]) * VT(0.5);            // MIDPOINT
    if constexpr (T >= 1) {
        if (rule == 3) {                                             // DLPSW: R[0], R[T], ...
            constexpr int NQ = (NR + T - 1) / T;
            return tree_sum_const<NQ, T, T, NZ>(v) / (VT)NQ;
        }
    }
    return tree_sum_const<NR, T, 1, NZ>(v) / (VT)NR;                        // TRIMMED_MEAN
}

// The rules over a receiver with nmiss absent entries (DESIGN.md §9 missing_policy = OMIT; CSR
// receivers with fewer than D senders): v[0] = x_i, absent entries hold omit_fill (+0.0 for
// AVERAGE, +inf otherwise), m' = D + 1 - nmiss.  With nmiss = 0 every result equals
// apply_rule_reg's bit for bit.  Windows of runtime size are taken by masking the compile-time
// window with +0.0 past the end, which leaves the stride-halving sum unchanged; TRIMMED /
// MIDPOINT / DLPSW keep x_i when m' <= 2t.
template <int D, int T, bool WMSR = false, typename VT>
__device__ __forceinline__ VT apply_rule_reg_omit(uint32_t rule, VT (&v)[D + 1], uint32_t nmiss) {
    constexpr int M = D + 1;
    const uint32_t mp = M - nmiss;
    if constexpr (WMSR) {
        return wmsr_reg<D, T>(v, nmiss);
    }
    if constexpr (T == 0) {
        if (rule == 0) return tree_sum_const<M>(v) / (VT)mp;
    }
    const VT xi = v[0];
    if (mp <= 2u * T) return xi;
    select_sort<M, T, M - T>(v);
    constexpr int NR = M - 2 * T;
    const uint32_t nr = mp - 2 * T;
    if (rule == 2) {                                                  // MIDPOINT: R[0] + R[nr - 1]
        VT top = v[T];
#pragma unroll
        for (int k = T; k < M - T; ++k)
            if ((uint32_t)(k - T) == nr - 1) top = v[k];
        return (v[T] + top) * VT(0.5);
    }
    if constexpr (T >= 1) {
        if (rule == 3) {                                              // DLPSW: R[0], R[T], ...
            constexpr int NQ = (NR + T - 1) / T;
            const uint32_t nq = (nr + T - 1) / T;
            VT w[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) w[q] = (uint32_t)q < nq ? v[T + q * T] : VT(0);
            return tree_sum_const<NQ>(w) / (VT)nq;
        }
    }
    VT w[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) w[k] = (uint32_t)k < nr ? v[T + k] : VT(0);
    return tree_sum_const<NR>(w) / (VT)nr;                            // TRIMMED_MEAN
}

}  // namespace acs
