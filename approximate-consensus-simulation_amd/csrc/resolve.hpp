// resolve.hpp — device helpers shared by the round kernels.
#pragma once

#include "engine.hpp"
#include "sortnet.hpp"

namespace acs {

constexpr double kInf = __builtin_huge_val();

// §A.6 resolution of one non-self entry (i <- j, slot s, round r), given the sender's status
// word, its value x_j, the receiver's x_i and the precomputed §A.5 drop decision.  `miss`
// reports a missing message (x_i is returned for it: the §A.6 self-substitution).
// VT = double, or float in fp32 mode.
template <typename VT>
__device__ __forceinline__ VT resolve_entry_m(const MsgParams& mp, uint32_t stj, VT xj, VT xi, bool dropped,
                                              uint32_t b, uint32_t r, uint32_t i, uint64_t s, VT lo, VT hi,
                                              bool& miss) {
    miss = dropped || crash_missing(mp, stj, b, r, s);
    if (miss) return xi;
    if (stj == kByz) return byz_value_t(mp, b, r, i, s, lo, hi);
    return xj;
}

template <typename VT>
__device__ __forceinline__ VT resolve_entry(const MsgParams& mp, uint32_t stj, VT xj, VT xi, bool dropped,
                                            uint32_t b, uint32_t r, uint32_t i, uint64_t s, VT lo, VT hi) {
    bool miss;
    return resolve_entry_m(mp, stj, xj, xi, dropped, b, r, i, s, lo, hi, miss);
}

// The value a missing entry takes under missing_policy = OMIT: +0.0 in AVERAGE's
// entry-order tree sum (it keeps its place, adds nothing), +inf for the sorting rules (it sorts
// past every present entry and the rule's window, sized by the present count, excludes it).
template <typename VT>
__device__ __forceinline__ VT omit_fill(uint32_t rule) {
    return rule == 0 ? VT(0) : (VT)__builtin_huge_val();
}

// DESIGN.md §9 bounded delay: sender j's value as delivered on slot s in round r, given the
// slot's DELAY draw w: x_j^{r - min(r, w mod (D + 1))}.
template <typename VT = double>
__device__ __forceinline__ VT delayed_x(const RoundArgs& a, uint32_t lb, uint32_t r, uint32_t w, uint64_t j) {
    uint32_t dl = w % (a.delay + 1);
    dl = dl < r ? dl : r;
    return reinterpret_cast<const VT*>(a.xh)[(uint64_t)((r - dl) % a.H) * a.xstride + (uint64_t)lb * a.N + j];
}

__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = __builtin_fmin(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = __builtin_fmax(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
// Wave-wide fp64 min / max through DPP instead of ds_bpermute butterflies (round 5, DESIGN.md
// §5.11): quad swaps, row rotations by 4 and 8, then row_bcast15 / row_bcast31 fold the four rows
// into lane 63, which is read back wave-uniform.  No LDS round trips on the block's exit path,
// 3 VALU per step.  Every lane must hold a non-NaN value (the callers pass +-inf for idle lanes).
template <bool MAX, int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_minmax_step(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), CTRL, ROW_MASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), CTRL, ROW_MASK, 0xF, false);
    const double u = __hiloint2double(hi, lo);
    return MAX ? ce_max(v, u) : ce_min(v, u);
#else
    return v;
#endif
}
template <bool MAX>
__device__ __forceinline__ double wave_minmax_dpp(double v) {
    v = dpp_minmax_step<MAX, 0xB1, 0xF>(v);    // quad_perm [1,0,3,2]
    v = dpp_minmax_step<MAX, 0x4E, 0xF>(v);    // quad_perm [2,3,0,1]
    v = dpp_minmax_step<MAX, 0x124, 0xF>(v);   // row_ror:4
    v = dpp_minmax_step<MAX, 0x128, 0xF>(v);   // row_ror:8   (every lane: its row of 16)
    v = dpp_minmax_step<MAX, 0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
    v = dpp_minmax_step<MAX, 0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3 (lane 63: all four rows)
    return readlane_f64(v, 63);
}

// EPS verdict publication (RoundArgs::eacc): a double's bits mapped so that unsigned order is numeric
// order (for non-NaN values), and back.  Block b folds into pair b % kEaccSlots (one 128-B line each,
// so the blocks' device-scope atomics spread over 32 addresses instead of queueing on one); word 0
// holds max ~ord(min), word 1 max ord(max), both with identity 0.  A reader takes the max over the
// pairs; if nothing was published the pair decodes to NaNs, whose spread never passes the ε test.
__device__ __forceinline__ unsigned long long ord_of(double v) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    return (u >> 63) ? ~u : (u | (1ull << 63));
}
__device__ __forceinline__ double ord_inv(unsigned long long o) {
    return __longlong_as_double((long long)((o >> 63) ? (o & ~(1ull << 63)) : ~o));
}
__device__ __forceinline__ void publish_minmax(unsigned long long* eacc, double mn, double mx) {
    unsigned long long* p = eacc + (blockIdx.x % kEaccSlots) * kEaccStride;
    __hip_atomic_fetch_max(p, ~ord_of(mn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(p + 1, ord_of(mx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide honest (min, max) -> one partial per block (§A.8; min/max are exact and
// order-free, so any reduction tree gives the oracle's value).  eacc: also publish it (above).
template <int BS>
__device__ __forceinline__ void block_minmax_store(double mn, double mx, double2* out,
                                                   unsigned long long* eacc = nullptr) {
    static_assert(BS % 64 == 0, "block must be whole wavefronts");
    constexpr int NW = BS / 64;
    mn = wave_minmax_dpp<false>(mn);
    mx = wave_minmax_dpp<true>(mx);
    if constexpr (NW == 1) {
        if (threadIdx.x == 0) {
            *out = make_double2(mn, mx);
            if (eacc) publish_minmax(eacc, mn, mx);
        }
    } else {
        __shared__ double2 red[NW];
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) red[w] = make_double2(mn, mx);
        __syncthreads();
        if (threadIdx.x == 0) {
            double a = red[0].x, c = red[0].y;
#pragma unroll
            for (int k = 1; k < NW; ++k) {
                a = __builtin_fmin(a, red[k].x);
                c = __builtin_fmax(c, red[k].y);
            }
            *out = make_double2(a, c);
            if (eacc) publish_minmax(eacc, a, c);
        }
    }
}

__device__ __forceinline__ double readlane_v(double v, int lane) { return readlane_f64(v, lane); }
__device__ __forceinline__ float readlane_v(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

}  // namespace acs
