// batched_small.hip — persistent batched kernel for COMPLETE graphs with N <= 64 (cfg1, cfg3).
//
// One wavefront = one instance, lane i = node i.  x stays in a VGPR across rounds; a sender's
// value reaches every receiver with v_readlane (compile-time lane index -> SGPR broadcast), so a
// round touches no memory at all.  Per lane and round:
//   - the §A.5 drop mask of its N slots (one Philox call per 4 slots) and §A.4 crash bits;
//   - AVERAGE (cfg3): the §A.7 tree sum over entries in entry order, evaluated as an adjacent-
//     pair stack over the bit-reversed entry sequence (stride-halving over a[] == adjacent
//     pairing over a[bitrev(k)]; fp add is commutative, so the sum is bit-identical), using
//     log2(P) registers instead of P;
//   - sorting rules (cfg1 MIDPOINT): a compile-time P-wire network in registers, then the
//     runtime-t window read back from a lane-private LDS column;
//   - honest (min, max) by wavefront shuffles, ε test, early exit per instance (§A.8).
// HBM traffic: 8N bytes in and out per instance per launch.  Bound: integer VALU (Philox).
#include <stdio.h>

#include "resolve.hpp"
#include "sortnet.hpp"

namespace acs {

template <int L>
constexpr int bitrev(int q) {
    int r = 0;
    for (int b = 0; b < L; ++b)
        if (q & (1 << b)) r |= 1 << (L - 1 - b);
    return r;
}

constexpr int ilog2(int p) {
    int l = 0;
    while ((1 << l) < p) ++l;
    return l;
}

template <int P, int Q, int LOG2P, typename VT>
__device__ __forceinline__ void push_leaf(VT (&acc)[LOG2P + 1], VT v) {
    // combine while bit l of Q is set (compile-time), then park at level l
    if constexpr ((Q & 1) && LOG2P > 0) {
        v = acc[0] + v;
        if constexpr ((Q & 2) && LOG2P > 1) {
            v = acc[1] + v;
            if constexpr ((Q & 4) && LOG2P > 2) {
                v = acc[2] + v;
                if constexpr ((Q & 8) && LOG2P > 3) {
                    v = acc[3] + v;
                    if constexpr ((Q & 16) && LOG2P > 4) {
                        v = acc[4] + v;
                        if constexpr ((Q & 32) && LOG2P > 5) {
                            v = acc[5] + v;
                            acc[6] = v;
                        } else acc[5] = v;
                    } else acc[4] = v;
                } else acc[3] = v;
            } else acc[2] = v;
        } else acc[1] = v;
    } else {
        acc[0] = v;
    }
}

template <typename VT>
struct LaneCtx {
    const MsgParams* mp;
    uint32_t N, lane, b, r;
    VT xi, lo, hi;
    uint32_t sti;
    const VT* xs;          // this round's x of every node of the instance (LDS, broadcast reads)
    const uint32_t* ss;    // every node's status word (LDS)
    uint64_t miss;   // bit j: message from j missing (crash or drop)
    VT fill;         // missing_policy = OMIT: the value a missing entry takes (omit_fill)
};

// Byzantine value kept out of line: inlined into each of the P unrolled leaves it multiplied the
// code (one Philox call per leaf) and spilled registers.
template <typename VT>
__device__ __noinline__ VT byz_value_ool(const MsgParams& mp, uint32_t b, uint32_t r, uint32_t i, uint64_t s, VT lo,
                                         VT hi) {
    return byz_value_t(mp, b, r, i, s, lo, hi);   // binary32 arithmetic for float
}


// §A.6 entry j of receiver `lane` (valid for j < N).  FAULTS = false: no fault schedule, so a
// sender is never Byzantine and only the drop bits matter (cfg3).
// Sender values come from an LDS copy of the instance's x (a wave-uniform address: one broadcast
// read per entry) rather than v_readlane: 64 readlane pairs per round held 128 SGPRs live, which
// spilled to VGPR lanes and cost more VALU than the Philox draws.
template <bool FAULTS, typename VT>
__device__ __forceinline__ VT entry_value(const LaneCtx<VT>& c, int j) {
    const VT xj = c.xs[j];
    if ((uint32_t)j == c.lane) return c.xi;
    if ((c.miss >> j) & 1ull) return c.mp->omit ? c.fill : c.xi;   // OMIT: +0.0 / +inf
    if constexpr (FAULTS) {
        const uint32_t stj = c.ss[j];
        if (stj == kByz) return byz_value_ool(*c.mp, c.b, c.r, c.lane, (uint64_t)c.lane * c.N + j, c.lo, c.hi);
    }
    return xj;
}

template <int P, bool FAULTS, typename VT, int... Q>
__device__ __forceinline__ VT average_tree(const LaneCtx<VT>& c, std::integer_sequence<int, Q...>) {
    constexpr int LOG2P = ilog2(P);
    VT acc[LOG2P + 1];
    (push_leaf<P, Q, LOG2P>(acc, (bitrev<LOG2P>(Q) < (int)c.N) ? entry_value<FAULTS>(c, bitrev<LOG2P>(Q)) : VT(0)), ...);
    return acc[LOG2P];
}

// Bit-select of two values of the same width: (m & a) | (~m & b) per 32-bit word (v_bfi_b32), m all
// ones or all zeros.  No lane-mask (SGPR pair) per entry: 64 entries' compare masks held live
// otherwise spill SGPRs to VGPR lanes.
// v_bfi_b32 written out: given a mask it can prove is 0 / -1 the compiler turns the and/or form
// into a compare plus two v_cndmask per value (one VALU op more per leaf).
__device__ __forceinline__ uint32_t bfi32(uint32_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double bitsel(uint32_t m, double a, double b) {
    const uint64_t ua = (uint64_t)__double_as_longlong(a), ub = (uint64_t)__double_as_longlong(b);
    const uint32_t lo = bfi32(m, (uint32_t)ua, (uint32_t)ub);
    const uint32_t hi = bfi32(m, (uint32_t)(ua >> 32), (uint32_t)(ub >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ float bitsel(uint32_t m, float a, float b) {
    return __uint_as_float(bfi32(m, __float_as_uint(a), __float_as_uint(b)));
}

// AVERAGE without a fault schedule (cfg3): entry j is x_i when bit j of `usexi` is set (missing
// messages under §A.6 substitution), +0.0 when bit j of `use0` is set (missing messages under
// OMIT), else x_j from the LDS copy — which for j = lane IS x_i, so the self entry
// needs no lane-dependent test (use0 never holds the self bit).  FULL: N == P (no padding test).
template <int P, bool OMIT, bool FULL, typename VT, int... Q>
__device__ __forceinline__ VT average_tree_sel(const VT* xs, VT xi, uint64_t usexi, uint64_t use0, uint32_t N,
                                               std::integer_sequence<int, Q...>) {
    constexpr int LOG2P = ilog2(P);
    VT acc[LOG2P + 1];
    const uint32_t w0 = (uint32_t)usexi, w1 = (uint32_t)(usexi >> 32);
    const uint32_t z0 = (uint32_t)use0, z1 = (uint32_t)(use0 >> 32);
    auto leaf = [&](int j) -> VT {
        if (!FULL && j >= (int)N) return VT(0);
        VT v = xs[j];
        // all-ones / all-zeros select mask of bit j: one signed 1-bit field extract (v_bfe_i32)
        if constexpr (OMIT) v = bitsel((uint32_t)__builtin_amdgcn_sbfe((int)(j < 32 ? z0 : z1), j & 31, 1), VT(0), v);
        return bitsel((uint32_t)__builtin_amdgcn_sbfe((int)(j < 32 ? w0 : w1), j & 31, 1), xi, v);
    };
    // scheduling fence every 8 leaves: unfenced, the compiler hoists all 64 LDS reads (128 VGPRs
    // live, one wave per SIMD); fenced, a group's reads overlap only the previous group's adds
    auto fence = [](int q) {
        if ((q & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    };
    ((push_leaf<P, Q, LOG2P>(acc, leaf(bitrev<LOG2P>(Q))), fence(Q)), ...);
    return acc[LOG2P];
}

#ifndef ACS_BATCHED_WPE
#define ACS_BATCHED_WPE 4   // waves per SIMD asked of the compiler (VGPR budget 512 / WPE)
#endif
// VT = double, or float in fp32 mode: every §A.7 step in binary32, spread =
// binary32(hi - lo) compared as a double, lo / hi / spread kept as doubles in InstState.
template <int P, bool SORT, bool FAULTS, typename VT = double>
__global__ __launch_bounds__(64, (!SORT && !FAULTS) ? ACS_BATCHED_WPE : 1) void k_batched_small(const BatchArgs a, uint32_t kmax) {
    const uint32_t lb = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    InstState* S = a.st + lb;
    if (S->done) return;
    const uint32_t N = a.N;
    const MsgParams& mp = a.mp;
    uint32_t r = S->rounds;
    double lo = S->lo, hi = S->hi, spread = S->spread;
    const uint32_t b = (uint32_t)(mp.inst_offset + lb);
    const uint32_t bG = b - b % mp.mask_group;
    const bool valid = lane < N;
    const VT* xin = reinterpret_cast<const VT*>((r & 1u) ? a.x1 : a.x0) + (uint64_t)lb * N;
    VT xi = valid ? xin[lane] : VT(0);
    const uint32_t sti = valid ? (a.status ? a.status[(uint64_t)lb * N + lane] : kHonest) : kByz;
    const bool honest = sti == kHonest;
    __shared__ VT colbuf[SORT ? P * 64 : 1];
    __shared__ VT xs[64];
    __shared__ uint32_t ss[64];
    ss[lane] = sti;   // read after the first round's barrier
    bool done = false, conv = spread <= a.eps;
    for (uint32_t q = 0; q < kmax; ++q) {
        const bool act = valid && is_active(sti, r);
        LaneCtx<VT> c;
        c.mp = &mp; c.N = N; c.lane = lane; c.b = b; c.r = r; c.xi = xi; c.lo = (VT)lo; c.hi = (VT)hi;
        c.sti = sti;
        __syncthreads();   // (one wave: orders the previous round's reads before this write)
        xs[lane] = xi;
        __syncthreads();
        c.xs = xs;
        c.ss = ss;
        c.miss = 0;
        // drop mask (§A.5): slot s = lane*N + j
        if (mp.thr && act) {
            if ((N & 3u) == 0) {
                c.miss = drop_mask_n4(lane, N >> 2, r, bG, mp.key, mp.thr);
            } else {
                for (uint32_t j = 0; j < N; ++j)
                    if (draw(mp.key, kStreamDrop, bG, r, (uint64_t)lane * N + j) < mp.thr) c.miss |= 1ull << j;
            }
        }
        // crash bits (§A.4): sender status is uniform per j
        if (FAULTS && mp.fault == 1 && act) {
            for (uint32_t j = 0; j < N; ++j) {
                const uint32_t stj = (uint32_t)__builtin_amdgcn_readlane((int)sti, (int)j);
                if (stj < kByz && r >= stj && crash_missing(mp, stj, b, r, (uint64_t)lane * N + j))
                    c.miss |= 1ull << j;
            }
        }
        c.miss &= ~(1ull << lane);   // the self entry is never missing
        c.fill = omit_fill<VT>(a.rule);
        // m' = entries present (missing_policy = OMIT); N under §A.6 substitution
        const uint32_t mn_ = mp.omit ? N - (uint32_t)__builtin_popcountll(c.miss) : N;
        VT res;
        if constexpr (!SORT) {
            if constexpr (!FAULTS) {
                constexpr auto seq = std::make_integer_sequence<int, P>{};
                if (mp.omit)
                    res = (N == P ? average_tree_sel<P, true, true>(xs, xi, 0ull, c.miss, N, seq)
                                  : average_tree_sel<P, true, false>(xs, xi, 0ull, c.miss, N, seq)) / (VT)mn_;
                else
                    res = (N == P ? average_tree_sel<P, false, true>(xs, xi, c.miss, 0ull, N, seq)
                                  : average_tree_sel<P, false, false>(xs, xi, c.miss, 0ull, N, seq)) / (VT)mn_;
            } else {
                res = average_tree<P, FAULTS>(c, std::make_integer_sequence<int, P>{}) / (VT)mn_;
            }
        } else {
            VT v[P];
#pragma unroll
            for (int j = 0; j < P; ++j) v[j] = j < (int)N ? entry_value<FAULTS>(c, j) : (VT)kInf;
            select_sort<P>(v);
#pragma unroll
            for (int k = 0; k < P; ++k) colbuf[k * 64 + lane] = v[k];
            const uint32_t t = a.trim, nr = mn_ - 2 * t;
            if (a.rule != 4 && mn_ <= 2 * t) {   // OMIT: too few entries to trim, keep x_i
                res = xi;
            } else if (a.rule == 2) {
                res = (colbuf[t * 64 + lane] + colbuf[(mn_ - t - 1) * 64 + lane]) * VT(0.5);
            } else {
                uint32_t start = t, step = a.rule == 3 ? t : 1;
                uint32_t cnt = a.rule == 3 ? (nr + t - 1) / t : nr;
                if (a.rule == 4) {   // W-MSR: window [min(t, #below), N - min(t, #above))
                    uint32_t nl = 0, ng = 0;
                    for (uint32_t k = 0; k < mn_; ++k) {
                        const VT u = colbuf[k * 64 + lane];
                        nl += u < xi;
                        ng += u > xi;
                    }
                    const uint32_t wlo = nl < t ? nl : t, whi = ng < t ? ng : t;
                    start = wlo;
                    step = 1;
                    cnt = mn_ - wlo - whi;
                }
                uint32_t P2 = 1;
                while (P2 < cnt) P2 <<= 1;
                for (uint32_t k = 0; k < P2; ++k)   // in place: source index start + k*step >= k
                    colbuf[k * 64 + lane] = k < cnt ? colbuf[(start + k * step) * 64 + lane] : VT(0);
                for (uint32_t s2 = P2 >> 1; s2 >= 1; s2 >>= 1)
                    for (uint32_t k = 0; k < s2; ++k)
                        colbuf[k * 64 + lane] = colbuf[k * 64 + lane] + colbuf[(k + s2) * 64 + lane];
                res = colbuf[lane] / (VT)cnt;
            }
        }
        xi = act ? res : xi;
        r += 1;
        lo = wave_min(honest ? (double)xi : kInf);
        hi = wave_max(honest ? (double)xi : -kInf);
        spread = (double)((VT)hi - (VT)lo);   // binary32 subtraction in fp32 mode
        if (a.trace && lane == 0) a.trace[(uint64_t)lb * a.trace_stride + r] = spread;
        conv = spread <= a.eps;
        done = (a.term_eps && conv) || r >= a.max_rounds;
        if (done) break;
    }
    VT* xout = reinterpret_cast<VT*>((r & 1u) ? a.x1 : a.x0) + (uint64_t)lb * N;
    if (valid) xout[lane] = xi;
    if (lane == 0) {
        S->lo = lo;
        S->hi = hi;
        S->spread = spread;
        S->rounds = r;
        S->converged = conv ? 1u : 0u;
        S->done = done ? 1u : 0u;
    }
}

// ------------------------------------------------------------------------------ split instances
// cfg3 (N = 64, AVERAGE, no fault schedule) with F lanes per receiver: one instance = F waves of one
// workgroup; wave w holds receivers [w*R, (w+1)*R) (R = 64/F), lane l of it receiver w*R + l % R,
// part f = l / R.  Why: at one wave per instance the batch is dealt in whole-instance units, and
// a shard of 12 500 instances fills 3.05 generations of the resident waves (the fourth nearly
// empty); F lanes per receiver make the unit 1/F of an instance's time.
// Per round and lane:
//   - Philox calls [f*16/F, (f+1)*16/F) of receiver i's drop slots (64/F drop bits); the F parts'
//     bits are all-gathered over the F lanes of the receiver by lane shuffles;
//   - the §A.7 tree restricted to entries j ≡ f (mod F): the stride-halving tree over 64 entries
//     first combines the residue classes mod F as a stride-halving tree over the F class sums
//     ((c0 + c2) + (c1 + c3) at F = 4), and each class sum is the same tree over its 64/F entries
//     (adjacent pairs over bit-reversed order, as average_tree_sel); the F lanes then combine the
//     class sums in that order by shuffles, so every lane holds the spec's sum bit for bit;
//   - honest (min, max) by wave shuffles and an LDS word per wave; x through LDS.
template <int F, bool OMIT, typename VT, int... Q>
__device__ __forceinline__ VT class_tree(const VT* xs, uint32_t f, VT xi, uint64_t usexi, uint64_t use0,
                                         std::integer_sequence<int, Q...>) {
    constexpr int L = 64 / F;
    constexpr int LOG2L = ilog2(L);
    VT acc[LOG2L + 1];
    const uint64_t u = usexi >> f, z = use0 >> f;   // bit F*k: entry F*k + f
    const uint32_t w0 = (uint32_t)u, w1 = (uint32_t)(u >> 32), z0 = (uint32_t)z, z1 = (uint32_t)(z >> 32);
    const VT* xf = xs + f;
    auto leaf = [&](int k) -> VT {   // entry F*k + f
        const int bit = F * k;
        VT v = xf[bit];
        if constexpr (OMIT) v = bitsel((uint32_t)__builtin_amdgcn_sbfe((int)(bit < 32 ? z0 : z1), bit & 31, 1), VT(0), v);
        return bitsel((uint32_t)__builtin_amdgcn_sbfe((int)(bit < 32 ? w0 : w1), bit & 31, 1), xi, v);
    };
    auto fence = [](int q) {
        if ((q & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    };
    ((push_leaf<L, Q, LOG2L>(acc, leaf(bitrev<LOG2L>(Q))), fence(Q)), ...);
    return acc[LOG2L];
}

template <int F, typename VT>
__device__ __forceinline__ VT shfl_xor_v(VT v, int m) {
    return __shfl_xor(v, m, 64);
}

#ifndef ACS_SPLIT_WPE
#define ACS_SPLIT_WPE 0   // variant builds: waves per SIMD asked of the fp64 F = 2 kernel (unbounded: 98 VGPRs, 4)
#endif
template <int F, typename VT = double>
__global__ __launch_bounds__(64 * F, (F == 2 && sizeof(VT) == 8 && ACS_SPLIT_WPE) ? ACS_SPLIT_WPE : 1) void k_batched_split(
    const BatchArgs a, uint32_t kmax) {
    constexpr int R = 64 / F;        // receivers per wave
    constexpr int CPL = 16 / F;      // Philox calls (4 slots each) per lane and round
    const uint32_t lb = blockIdx.x;
    InstState* S = a.st + lb;
    if (S->done) return;
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t f = lane / R, i = w * R + lane % R;
    const MsgParams& mp = a.mp;
    uint32_t r = S->rounds;
    double lo = S->lo, hi = S->hi, spread = S->spread;
    const uint32_t b = (uint32_t)(mp.inst_offset + lb);
    const uint32_t bG = b - b % mp.mask_group;
    const VT* xin = reinterpret_cast<const VT*>((r & 1u) ? a.x1 : a.x0) + (uint64_t)lb * 64;
    VT xi = xin[i];
    __shared__ VT xs[64];
    __shared__ double2 red[F];
    bool done = false, conv = spread <= a.eps;
    for (uint32_t q = 0; q < kmax; ++q) {
        __syncthreads();   // the previous round's reads of xs and red are done
        if (f == 0) xs[i] = xi;
        __syncthreads();
        uint64_t miss = 0;
        if (mp.thr) {   // drop bits of entries [f*4*CPL, (f+1)*4*CPL) of receiver i, then all-gathered
            uint32_t m = 0;
#pragma unroll
            for (int g = 0; g < CPL; ++g) {
                const U4 wd = philox10(i * 16u + f * CPL + g, r, bG, kStreamDrop, mp.key);
#pragma unroll
                for (int e = 0; e < 4; ++e) m = shift_in_lt(m, wd.v[e], mp.thr);
            }
            miss = (uint64_t)(__builtin_bitreverse32(m) >> (32 - 4 * CPL)) << (f * 4 * CPL);
#pragma unroll
            for (int sh = R; sh < 64; sh <<= 1) {
                const uint32_t lo32 = (uint32_t)__shfl_xor((int)(uint32_t)miss, sh, 64);
                const uint32_t hi32 = (uint32_t)__shfl_xor((int)(uint32_t)(miss >> 32), sh, 64);
                miss |= (uint64_t)hi32 << 32 | lo32;
            }
        }
        miss &= ~(1ull << i);   // the self entry is never missing
        constexpr auto seq = std::make_integer_sequence<int, 64 / F>{};
        VT c = mp.omit ? class_tree<F, true>(xs, f, xi, 0ull, miss, seq) : class_tree<F, false>(xs, f, xi, miss, 0ull, seq);
#pragma unroll
        for (int st = F / 2; st >= 1; st >>= 1) {   // stride-halving over the class sums
            const VT o = shfl_xor_v<F>(c, st * R);
            c = (f & st) ? o + c : c + o;
        }
        const uint32_t mn_ = mp.omit ? 64u - (uint32_t)__builtin_popcountll(miss) : 64u;
        xi = c / (VT)mn_;
        r += 1;
        const double wmn = wave_min((double)xi), wmx = wave_max((double)xi);
        if (lane == 0) red[w] = make_double2(wmn, wmx);
        __syncthreads();
        lo = red[0].x;
        hi = red[0].y;
#pragma unroll
        for (int k = 1; k < F; ++k) {
            lo = __builtin_fmin(lo, red[k].x);
            hi = __builtin_fmax(hi, red[k].y);
        }
        spread = (double)((VT)hi - (VT)lo);   // binary32 subtraction in fp32 mode
        if (a.trace && threadIdx.x == 0) a.trace[(uint64_t)lb * a.trace_stride + r] = spread;
        conv = spread <= a.eps;
        done = (a.term_eps && conv) || r >= a.max_rounds;
        if (done) break;
    }
    VT* xout = reinterpret_cast<VT*>((r & 1u) ? a.x1 : a.x0) + (uint64_t)lb * 64;
    if (f == 0) xout[i] = xi;
    if (threadIdx.x == 0) {
        S->lo = lo;
        S->hi = hi;
        S->spread = spread;
        S->rounds = r;
        S->converged = conv ? 1u : 0u;
        S->done = done ? 1u : 0u;
    }
}

// Lanes per receiver for a clean AVERAGE batch of 64-node instances: ACSIM_BATCH_SPLIT (1, 2, 4)
// or the default.
uint32_t batched_split_factor(uint32_t N, uint32_t rule, bool faults) {
    if (N != 64 || rule != 0 || faults) return 1;
    // default 2: at 10^5 instances as fast as one lane per receiver (2.08 ms either way), and the
    // 8-rank shard's tail shrinks (0.300 -> 0.281 ms); 4 costs about 25 % more work (re-measured in
    // round 5 beside the default: profiles/r05_cfg3_split_factor.jsonl, tools/cfg3_shard_probe.py)
    uint32_t F = 2;
    if (const char* v = getenv("ACSIM_BATCH_SPLIT")) F = (uint32_t)strtoul(v, nullptr, 10);
    return F == 2 || F == 4 ? F : 1;
}

static int pick_p(uint32_t N) {
    int P = 2;
    while ((uint32_t)P < N) P <<= 1;
    return P;
}

const char* batched_small_name(uint32_t N, uint32_t rule, bool faults) {
    static char names[2][2][7][40];
    const int P = pick_p(N), lp = ilog2(P), so = rule != 0, fa = faults ? 1 : 0;
    char* nm = names[so][fa][lp];
    if (!nm[0]) snprintf(nm, 40, "k_batched_small<%d,%s,%s>", P, so ? "sort" : "avg", fa ? "faulty" : "clean");
    return nm;
}

template <typename VT>
static hipError_t launch_batched_small_t(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s) {
    const int P = pick_p(a.N);
    const bool sort = a.rule != 0, faults = a.status != nullptr;
    const dim3 grid((unsigned)B), block(64);
#define L(PP)                                                                                                  \
    case PP:                                                                                                   \
        if (sort && faults) hipLaunchKernelGGL((k_batched_small<PP, true, true, VT>), grid, block, 0, s, a, k);   \
        else if (sort) hipLaunchKernelGGL((k_batched_small<PP, true, false, VT>), grid, block, 0, s, a, k);       \
        else if (faults) hipLaunchKernelGGL((k_batched_small<PP, false, true, VT>), grid, block, 0, s, a, k);     \
        else hipLaunchKernelGGL((k_batched_small<PP, false, false, VT>), grid, block, 0, s, a, k);                \
        break;
    switch (P) {
        L(2) L(4) L(8) L(16) L(32) L(64)
        default: return hipErrorNotSupported;
    }
#undef L
    return hipGetLastError();
}

hipError_t launch_batched_small(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s) {
    if (a.N < 1 || a.N > kBatchedMaxN) return hipErrorNotSupported;
    const uint32_t F = batched_split_factor(a.N, a.rule, a.status != nullptr);
    if (F > 1) {
        const dim3 grid((unsigned)B), block(64 * F);
        if (F == 2 && a.f32) hipLaunchKernelGGL((k_batched_split<2, float>), grid, block, 0, s, a, k);
        else if (F == 2) hipLaunchKernelGGL((k_batched_split<2, double>), grid, block, 0, s, a, k);
        else if (a.f32) hipLaunchKernelGGL((k_batched_split<4, float>), grid, block, 0, s, a, k);
        else hipLaunchKernelGGL((k_batched_split<4, double>), grid, block, 0, s, a, k);
        return hipGetLastError();
    }
    return a.f32 ? launch_batched_small_t<float>(a, B, k, s) : launch_batched_small_t<double>(a, B, k, s);
}

}  // namespace acs
