// round_dense.hip — complete-graph rounds with one shared sort per round (cfg2 shape).
//
// On a complete graph without message loss, every active receiver i sees the same base multiset
// B = { x_j : j honest or crash-active } (its own entry x_i is one of them) plus receiver-specific
// constant blocks: n_byz copies of its Byzantine value c_i (SPLIT: hi^r+Δ / lo^r−Δ by receiver
// parity; CONSTANT: c) and n_silent copies of x_i (crash-silent senders, missing -> x_i).  So:
//   k_dense_sort  : one workgroup sorts B once per round (LDS bitonic, +inf padding) and counts
//                   the silent / Byzantine senders;
//   k_dense_recv  : one wavefront per receiver reads its window R = M[t, m-t) of the merged
//                   sequence M = B ⊕ {c_i}^n_byz ⊕ {x_i}^n_silent directly by index arithmetic
//                   (two ranks found by binary search), and applies the rule with the §A.7
//                   stride-halving tree sum, spread over the wavefront's 64 lanes.
// The sorted value sequence of S_i is unique (no -0, no NaN), so this equals sorting S_i per
// receiver (the generic kernel) bit for bit, at O(N log^2 N + N·|R|/64) instead of
// O(N^2 log^2 N) work per round.  Rounds in which a crash sender delivers partially (r == r_v),
// message loss, AVERAGE and RANDOM Byzantine values keep the generic kernel.
#include <mutex>
#include <type_traits>
#include "resolve.hpp"

namespace acs {

constexpr int kDenseSortBlock = 1024;
constexpr int kDenseRecvBlock = 256;   // 4 receivers (wavefronts) per block

// Ascending bitonic sort of sh[0..P) (P a power of two, +inf padded) by a 1024-thread block.
// Thread t owns wires t + 1024e (e < E = P/1024) in registers; on return v[e] holds wire
// t + 1024e of the sorted sequence (sh is scratch).  Compare distance j < 64: partner in the same
// wavefront (shuffle, no barrier); 64 <= j < 1024: partner in another wavefront (LDS exchange,
// one barrier pair); j >= 1024: partner in the same thread (register swap).  55 stages at
// P = 1024, of which only 10 touch LDS.
__device__ __forceinline__ double vmin(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ double vmax(double a, double b) { return __builtin_fmax(a, b); }
__device__ __forceinline__ float vmin(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ float vmax(float a, float b) { return __builtin_fmaxf(a, b); }

// VT = double, or float for the fp32 persistent kernel
template <int EMAX, typename VT>
__device__ __forceinline__ void dense_bitonic(VT* sh, uint32_t P, VT (&v)[EMAX]) {
    const uint32_t E = (P + kDenseSortBlock - 1) / kDenseSortBlock;
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
        const uint32_t idx = tid + kDenseSortBlock * e;
        v[e] = ((uint32_t)e < E && idx < P) ? sh[idx] : (VT)kInf;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j < 64) {
#pragma unroll
                for (int e = 0; e < EMAX; ++e) {
                    if ((uint32_t)e >= E) break;
                    const uint32_t idx = tid + kDenseSortBlock * e;
                    const VT p = __shfl_xor(v[e], (int)j, 64);
                    const bool keep_min = ((idx & j) == 0) == ((idx & k) == 0);
                    v[e] = keep_min ? vmin(v[e], p) : vmax(v[e], p);
                }
            } else if (j < (uint32_t)kDenseSortBlock) {
#pragma unroll
                for (int e = 0; e < EMAX; ++e)
                    if ((uint32_t)e < E) sh[tid + kDenseSortBlock * e] = v[e];
                __syncthreads();
#pragma unroll
                for (int e = 0; e < EMAX; ++e) {
                    if ((uint32_t)e >= E) break;
                    const uint32_t idx = tid + kDenseSortBlock * e;
                    const VT p = sh[idx ^ j];
                    const bool keep_min = ((idx & j) == 0) == ((idx & k) == 0);
                    v[e] = keep_min ? vmin(v[e], p) : vmax(v[e], p);
                }
                __syncthreads();
            } else {
                const uint32_t ej = j / kDenseSortBlock;   // 1, 2 or 4: partner element e ^ ej
#define ACS_SWAP_STAGE(EJ)                                                                      \
    _Pragma("unroll") for (int e = 0; e < EMAX; ++e) {                                          \
        if ((e ^ EJ) > e && (uint32_t)(e ^ EJ) < E) {                                           \
            const uint32_t idx = tid + kDenseSortBlock * e;                                     \
            const VT lo_ = vmin(v[e], v[e ^ EJ]), hi_ = vmax(v[e], v[e ^ EJ]);                 \
            const bool asc = (idx & k) == 0;                                                    \
            v[e] = asc ? lo_ : hi_;                                                             \
            v[e ^ EJ] = asc ? hi_ : lo_;                                                        \
        }                                                                                       \
    }
                if (ej == 1) { ACS_SWAP_STAGE(1) }
                else if (ej == 2) { ACS_SWAP_STAGE(2) }
                else { ACS_SWAP_STAGE(4) }
#undef ACS_SWAP_STAGE
            }
        }
    }
}

// VT = double, or float in fp32 mode (binary32 values, the same sorted multiset)
template <typename VT = double>
__global__ __launch_bounds__(kDenseSortBlock) void k_dense_sort(const DenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sh_raw[];
    VT* sh = reinterpret_cast<VT*>(sh_raw);
    const VT* x = reinterpret_cast<const VT*>(a.x);
    InstState* S = a.st;
    if (S->done) return;
    const uint32_t N = a.N, P = a.P, r = a.r;
    __shared__ uint32_t cnt[3];   // base, byz, silent
    if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t nb = 0, nz = 0, ns = 0;
    for (uint32_t j = threadIdx.x; j < P; j += kDenseSortBlock) {
        VT v = (VT)kInf;
        if (j < N) {
            const uint32_t st = a.status ? a.status[j] : kHonest;
            if (st == kHonest || (st != kByz && r < st)) {
                v = x[j];
                ++nb;
            } else if (st == kByz) {
                ++nz;
            } else if (r > st) {
                ++ns;
            }
        }
        sh[j] = v;
    }
    // wavefront sums first: 1024 LDS atomics on one address serialise
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        nb += __shfl_xor(nb, o, 64);
        nz += __shfl_xor(nz, o, 64);
        ns += __shfl_xor(ns, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&cnt[0], nb);
        atomicAdd(&cnt[1], nz);
        atomicAdd(&cnt[2], ns);
    }
    __syncthreads();
    constexpr int EMAX = kGenericMaxM / kDenseSortBlock;   // 8
    const uint32_t E = (P + kDenseSortBlock - 1) / kDenseSortBlock;
    const uint32_t tid = threadIdx.x;
    VT v[EMAX];
    dense_bitonic<EMAX>(sh, P, v);
    VT* sorted = reinterpret_cast<VT*>(a.sorted);
#pragma unroll
    for (int e = 0; e < EMAX; ++e) {
        const uint32_t idx = tid + kDenseSortBlock * e;
        if ((uint32_t)e < E && idx < cnt[0]) sorted[idx] = v[e];
    }
    if (threadIdx.x == 0) {
        a.counts[0] = cnt[0];
        a.counts[1] = cnt[1];
        a.counts[2] = cnt[2];
    }
}

// number of elements of sorted b[0..n) strictly below v
template <typename VT>
__device__ __forceinline__ uint32_t rank_below(const VT* b, uint32_t n, VT v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (b[mid] < v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

template <typename VT = double>
struct Merged {   // M = B with two constant blocks (v1 <= v2) spliced in at their ranks
    using value_type = VT;
    const VT* b;
    uint32_t r1, n1, r2, n2;
    VT v1, v2;
    __device__ __forceinline__ VT at(uint32_t k) const {
        if (k < r1) return b[k];
        if (k < r1 + n1) return v1;
        if (k < r2 + n1) return b[k - n1];
        if (k < r2 + n1 + n2) return v2;
        return b[k - n1 - n2];
    }
};

// A sorted sequence made of three constant runs: v[0] on [0, e[0]), v[1] on [e[0], e[1]), v[2] on
// [e[1], m).  After one persistent round every active node holds its class value, so a
// receiver's sequence is the class values of the base plus its Byzantine block: three runs.
template <typename VT = double>
struct Runs3 {
    using value_type = VT;
    VT v0, v1, v2;
    uint32_t e0, e1;
    // A bitwise blend of all three values, not a select of two loads: the compiler folds the
    // latter into a load through a selected address, which pins the struct in scratch memory.
    __device__ __forceinline__ VT at(uint32_t k) const {
        using U = __UINT64_TYPE__;
        using B = typename std::conditional<sizeof(VT) == 8, U, uint32_t>::type;
        const B m0 = (B)0 - (B)(k < e0), m1 = (B)0 - (B)(k < e1);
        const B b0 = __builtin_bit_cast(B, v0), b1 = __builtin_bit_cast(B, v1), b2 = __builtin_bit_cast(B, v2);
        return __builtin_bit_cast(VT, (b0 & m0) | (~m0 & ((b1 & m1) | (~m1 & b2))));
    }
};

// Lane l receives lane l + O's 32-bit value (O = 32, 16: v_permlane32_swap / v_permlane16_swap,
// whose second result carries the upper half / odd rows into the lower half / even rows; O <= 8:
// DPP row_shl within a 16-lane row).  Only the lanes l < O are meaningful.
template <int O>
__device__ __forceinline__ uint32_t lane_up_u32(uint32_t x) {
    if constexpr (O == 32) return __builtin_amdgcn_permlane32_swap(x, x, false, false)[1];
    else if constexpr (O == 16) return __builtin_amdgcn_permlane16_swap(x, x, false, false)[1];
    else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x100 + O, 0xF, 0xF, false);
}
template <int O>
__device__ __forceinline__ double lane_up(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint64_t lo = lane_up_u32<O>((uint32_t)b), hi = lane_up_u32<O>((uint32_t)(b >> 32));
    return __builtin_bit_cast(double, lo | (hi << 32));
}
template <int O>
__device__ __forceinline__ float lane_up(float v) {
    return __builtin_bit_cast(float, lane_up_u32<O>(__builtin_bit_cast(uint32_t, v)));
}

// The rule over the window R = M[t, m - t) of one receiver's merged sorted sequence, by one
// wavefront (§A.7 stride-halving tree sum spread over the 64 lanes); every lane returns the result.
template <typename Seq, typename VT = typename Seq::value_type>
__device__ __forceinline__ VT dense_window(const Seq& M, uint32_t rule, uint32_t m, uint32_t t, uint32_t lane) {
    const uint32_t nr = m - 2 * t;
    VT res;
    if (rule == 2) {
        res = (M.at(t) + M.at(m - t - 1)) * VT(0.5);
    } else {
        const uint32_t step = rule == 3 ? t : 1;
        const uint32_t cnt = rule == 3 ? (nr + t - 1) / t : nr;
        uint32_t P2 = 64;
        while (P2 < cnt) P2 <<= 1;
        // §A.7 stride halving over P2 slots: this lane owns w[lane + 64a]
        const uint32_t per = P2 / 64;   // <= 128 for m <= 8192
        VT w[8];
        // levels with stride >= 64 fold in registers: accumulate slot groups in tree order
        // (per <= 8 keeps the whole lane column in registers; larger P2 folds first)
        uint32_t per_eff = per;
        if (per <= 8) {
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const uint32_t k = lane + 64u * g;
                w[g] = (g < (int)per && k < cnt) ? M.at(t + k * step) : VT(0);
            }
            for (uint32_t s = per >> 1; s >= 1; s >>= 1) {
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    if ((uint32_t)g < s) w[g] = w[g] + w[g + s];
            }
        } else {
            // large windows: strided partial trees per lane, folded in the same order
            // (position k = lane + 64*g pairs with k + P2/2 = lane + 64*(g + per/2))
            VT col[128];
            for (uint32_t g = 0; g < per_eff; ++g) {
                const uint32_t k = lane + 64u * g;
                col[g] = k < cnt ? M.at(t + k * step) : VT(0);
            }
            for (uint32_t s = per_eff >> 1; s >= 1; s >>= 1)
                for (uint32_t g = 0; g < s; ++g) col[g] = col[g] + col[g + s];
            w[0] = col[0];
        }
        // strides 32 .. 1 across lanes: lane l < o adds lane l + o (lanes >= o compute values
        // nobody reads).  Register-to-register moves instead of LDS permutes: the gfx950 permlane
        // swaps for 32 and 16, DPP row shifts within a 16-lane row for 8 .. 1.
        VT v = w[0];
        v = v + lane_up<32>(v);
        v = v + lane_up<16>(v);
        v = v + lane_up<8>(v);
        v = v + lane_up<4>(v);
        v = v + lane_up<2>(v);
        v = v + lane_up<1>(v);
        res = readlane_v(v, 0) / (VT)cnt;
    }
    return res;
}

// receiver i's Byzantine value (SPLIT by parity, or CONSTANT): fp64 as §A.4, fp32 as spec.hpp
// byz_value_f32 (Δ and c rounded to binary32 once, a binary32 add)
__device__ __forceinline__ double dense_recv_byz(const DenseArgs& a, uint32_t i, double lo, double hi, double) {
    return a.byz == 0 ? ((i & 1u) == 0 ? hi + a.delta : lo - a.delta) : a.bconst;
}
__device__ __forceinline__ float dense_recv_byz(const DenseArgs& a, uint32_t i, double lo, double hi, float) {
    const float dl = (float)a.delta;
    return a.byz == 0 ? ((i & 1u) == 0 ? (float)hi + dl : (float)lo - dl) : (float)a.bconst + 0.0f;
}

template <typename VT = double>
__global__ __launch_bounds__(kDenseRecvBlock) void k_dense_recv(const DenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char shB_raw[];
    VT* shB = reinterpret_cast<VT*>(shB_raw);   // the sorted base multiset
    InstState* S = a.st;
    if (S->done) return;
    {
        const uint32_t nb = a.counts[0];
        const VT* sorted = reinterpret_cast<const VT*>(a.sorted);
        for (uint32_t k = threadIdx.x; k < nb; k += kDenseRecvBlock) shB[k] = sorted[k];
        __syncthreads();
    }
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = blockIdx.x * (kDenseRecvBlock / 64) + (threadIdx.x >> 6);
    double mn = kInf, mx = -kInf;
    if (i < a.N) {
        const VT xi = reinterpret_cast<const VT*>(a.x)[i];
        const uint32_t st = a.status ? a.status[i] : kHonest;
        VT res = xi;
        if (st == kHonest || (st != kByz && a.r < st)) {
            const uint32_t nb = a.counts[0], nz = a.counts[1], ns = a.counts[2];
            const VT c = dense_recv_byz(a, i, S->lo, S->hi, VT(0));
            // blocks (c, nz) and (xi, ns), ordered by value
            Merged<VT> M;
            M.b = shB;
            const bool cfirst = c <= xi;
            M.v1 = cfirst ? c : xi;
            M.n1 = cfirst ? nz : ns;
            M.v2 = cfirst ? xi : c;
            M.n2 = cfirst ? ns : nz;
            M.r1 = M.n1 ? rank_below(shB, nb, M.v1) : 0;
            M.r2 = M.n2 ? rank_below(shB, nb, M.v2) : M.r1;
            if (M.r2 < M.r1) M.r2 = M.r1;
            res = dense_window(M, a.rule, a.N, a.trim, lane);
            if (st == kHonest) {
                mn = res;
                mx = res;
            }
        }
        if (lane == 0) reinterpret_cast<VT*>(a.xo)[i] = res;
    }
    // lanes of a receiver agree; fold the block's receivers
    block_minmax_store<kDenseRecvBlock>(mn, mx, a.partial + blockIdx.x);
}

// Persistent variant: one 1024-thread workgroup per instance runs k rounds in one launch with x
// resident in LDS (N <= kDensePersistMaxN).  dense_supported() excludes crash faults, so no
// sender is ever silent and S_i depends on receiver i only through its Byzantine value c_i: the
// window rule is evaluated once per distinct c (SPLIT: two, by receiver parity; CONSTANT or no
// faults: one) and broadcast, instead of once per receiver.  Per round: base multiset -> LDS,
// bitonic sort (dense_bitonic), ≤ 2 window rules, update, honest (min, max), ε test — no
// launches, no host round trips (cfg2: ≈ 900 rounds).
// The rounds' Byzantine class value: SPLIT hi + Δ (class 0) / lo - Δ (class 1), or CONSTANT c;
// in fp32 mode Δ and c are rounded to binary32 once and the add is binary32 (spec.hpp byz_value_f32).
__device__ __forceinline__ double dense_byz(const MsgParams& mp, uint32_t w, double lo, double hi, double) {
    return mp.byz == 0 ? (w == 0 ? hi + mp.delta : lo - mp.delta) : mp.bconst;
}
__device__ __forceinline__ float dense_byz(const MsgParams& mp, uint32_t w, double lo, double hi, float) {
    const float dl = (float)mp.delta;
    return mp.byz == 0 ? (w == 0 ? (float)hi + dl : (float)lo - dl) : (float)mp.bconst + 0.0f;
}

template <typename VT = double>
__global__ __launch_bounds__(kDenseSortBlock) void k_dense_persist(const BatchArgs a, uint32_t kmax) {
    __shared__ __attribute__((aligned(16))) VT xs[kDensePersistMaxN];
    __shared__ __attribute__((aligned(16))) VT sb[kDensePersistMaxN];
    __shared__ uint8_t byz[kDensePersistMaxN];   // 1: Byzantine (never updates, never in the base)
    __shared__ uint32_t cnt[4];                  // base size, #Byzantine, #honest-or-active per parity
    __shared__ VT cls[2][2];                     // class values of a round, double-buffered by round parity
    const uint32_t lb = blockIdx.x;
    InstState* S = a.st + lb;
    if (S->done) return;
    const uint32_t N = a.N, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t P = 64;
    while (P < N) P <<= 1;
    const uint32_t* stv = a.status ? a.status + (uint64_t)lb * N : nullptr;
    const MsgParams& mp = a.mp;
    uint32_t r = S->rounds;
    double lo = S->lo, hi = S->hi, spread = S->spread;
    bool conv = S->converged != 0, done = false;
    if (tid < 4) cnt[tid] = 0;
    __syncthreads();
    {
        const VT* xin = reinterpret_cast<const VT*>((r & 1u) ? a.x1 : a.x0) + (uint64_t)lb * N;
        uint32_t nz = 0, ne = 0, no = 0;
        for (uint32_t j = tid; j < N; j += kDenseSortBlock) {
            xs[j] = xin[j];
            const bool bz = stv && stv[j] == kByz;
            byz[j] = bz ? 1 : 0;
            nz += bz;
            ne += !bz && !(j & 1u);
            no += !bz && (j & 1u);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            nz += __shfl_xor(nz, o, 64);
            ne += __shfl_xor(ne, o, 64);
            no += __shfl_xor(no, o, 64);
        }
        if (lane == 0) {
            atomicAdd(&cnt[1], nz);
            atomicAdd(&cnt[2], ne);
            atomicAdd(&cnt[3], no);
        }
        __syncthreads();
    }
    const uint32_t nzv = cnt[1], nbv = N - nzv;
    const uint32_t ncls = (nzv && mp.byz == 0) ? 2u : 1u;   // SPLIT: parity classes
    // (scalars, not arrays: a runtime-indexed array lands in scratch, and the per-round class loop
    // then waited on two dependent scratch round trips per class)
    const uint32_t ncnt0 = ncls == 2 ? cnt[2] : nbv, ncnt1 = ncls == 2 ? cnt[3] : 0u;
    // After any round every non-Byzantine node holds its class's value (its multiset is the base,
    // which contains its own entry, plus its class's Byzantine block), and in these configs every
    // non-Byzantine node is honest (dense_supported admits no crash schedules).  So after the first
    // round of a launch (the base sort) a round is ≤ 2 window rules on three constant runs, one
    // wave per class, and the honest (min, max) is the (min, max) of the populated classes: one
    // barrier per round, and x is written out once at the end.  (Wave 0 alone evaluating both
    // windows without a barrier measured slower: cfg2 2.25 against 2.0 ms, and again 1.35 against
    // 0.98 ms once the class values stayed in registers and the tree used permlane / DPP moves.)
    bool classed = false;   // cl0 / cl1 hold every non-Byzantine node's value
    VT cl0 = VT(0), cl1 = VT(0);
    // (the class values come in as arguments, not by reference: a select between two referenced
    // locals also becomes a load through a selected address)
    auto window_classed = [&](uint32_t wc, VT cl0, VT cl1) -> VT {   // base = {cl0 x n0, cl1 x n1} + {c x nz}
        const VT c = dense_byz(mp, wc, lo, hi, VT(0));
        const bool sw = ncls == 2 && cl1 < cl0;   // base runs in value order
        const VT b0 = sw ? cl1 : cl0, b1 = sw ? cl0 : cl1;
        const uint32_t n0 = sw ? ncnt1 : ncnt0, n1 = sw ? ncnt0 : ncnt1;
        // insert the Byzantine block before the first base run with a value >= c
        const uint32_t pos = (nzv == 0 || c <= b0) ? 0u : (ncls == 1 || c <= b1) ? 1u : 2u;
        Runs3<VT> R;
        R.v0 = pos == 0 ? c : b0;
        R.v1 = pos == 0 ? b0 : pos == 1 ? c : b1;
        R.v2 = pos == 2 ? c : b1;
        R.e0 = pos == 0 ? nzv : n0;
        R.e1 = pos == 0 ? nzv + n0 : pos == 1 ? n0 + nzv : n0 + n1;
        return dense_window(R, a.rule, N, a.trim, lane);
    };
    for (uint32_t q = 0; q < kmax && !done; ++q) {
        if (!classed) {
            // base multiset B = values of the non-Byzantine senders, sorted (every wave)
            for (uint32_t j = tid; j < P; j += kDenseSortBlock) sb[j] = (j < N && !byz[j]) ? xs[j] : (VT)kInf;
            __syncthreads();
            constexpr int EP = kDensePersistMaxN / kDenseSortBlock;
            VT v[EP];
            dense_bitonic<EP>(sb, P, v);
            __syncthreads();
#pragma unroll
            for (int e = 0; e < EP; ++e) {
                const uint32_t idx = tid + kDenseSortBlock * e;
                if (idx < P) sb[idx] = v[e];
            }
            __syncthreads();
            if (w < ncls) {
                Merged<VT> M;
                M.b = sb;
                M.v1 = dense_byz(mp, w, lo, hi, VT(0));
                M.n1 = nzv;
                M.r1 = nzv ? rank_below(sb, nbv, M.v1) : 0;
                M.v2 = (VT)kInf;
                M.n2 = 0;
                M.r2 = M.r1;
                const VT res = dense_window(M, a.rule, N, a.trim, lane);
                if (lane == 0) cls[q & 1u][w] = res;
            }
        } else if (w < ncls) {
            const VT res = window_classed(w, cl0, cl1);
            if (lane == 0) cls[q & 1u][w] = res;
        }
        __syncthreads();   // (round q + 1 writes the other buffer; round q + 2 writes this one
                           // only after every wave has passed round q + 1's barrier)
        cl0 = cls[q & 1u][0];
        cl1 = ncls == 2 ? cls[q & 1u][1] : cl0;
        classed = true;
        double mn = kInf, mx = -kInf;
        if (ncnt0) {   // classes with members
            mn = __builtin_fmin(mn, (double)cl0);
            mx = __builtin_fmax(mx, (double)cl0);
        }
        if (ncls == 2 && ncnt1) {
            mn = __builtin_fmin(mn, (double)cl1);
            mx = __builtin_fmax(mx, (double)cl1);
        }
        r += 1;
        lo = mn;
        hi = mx;
        spread = (double)((VT)hi - (VT)lo);   // binary32 subtraction in fp32 mode
        if (a.trace && tid == 0) a.trace[(uint64_t)lb * a.trace_stride + r] = spread;
        conv = spread <= a.eps;
        done = (a.term_eps && conv) || r >= a.max_rounds;
    }
    VT* xout = reinterpret_cast<VT*>((r & 1u) ? a.x1 : a.x0) + (uint64_t)lb * N;
    for (uint32_t j = tid; j < N; j += kDenseSortBlock)
        xout[j] = (classed && !byz[j]) ? ((ncls == 2 && (j & 1u)) ? cl1 : cl0) : xs[j];
    if (tid == 0) {
        S->lo = lo;
        S->hi = hi;
        S->spread = spread;
        S->rounds = r;
        S->converged = conv ? 1u : 0u;
        S->done = done ? 1u : 0u;
        if (done) atomicAdd(a.n_done, 1u);
    }
}

hipError_t launch_dense_persist(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s) {
    if (a.N > kDensePersistMaxN) return hipErrorNotSupported;
    if (a.f32)
        hipLaunchKernelGGL(k_dense_persist<float>, dim3((unsigned)B), dim3(kDenseSortBlock), 0, s, a, k);
    else
        hipLaunchKernelGGL(k_dense_persist<double>, dim3((unsigned)B), dim3(kDenseSortBlock), 0, s, a, k);
    return hipGetLastError();
}

bool dense_supported(uint32_t fault_model, uint32_t byz, uint32_t rule, uint32_t thr, uint64_t N) {
    if (thr != 0 || rule == 0 || rule == 4 || N > kGenericMaxM || N < 2) return false;   // W-MSR: per-x_i windows
    if (fault_model == 1) return false;   // crash rounds deliver per slot: generic kernel
    if (fault_model == 2 && byz == 1) return false;   // RANDOM Byzantine values are per slot
    return true;
}

uint32_t dense_nblk(uint64_t N) { return (uint32_t)((N + (kDenseRecvBlock / 64) - 1) / (kDenseRecvBlock / 64)); }

hipError_t launch_round_dense(const DenseArgs& a, hipStream_t s) {
    // >64 KiB dynamic LDS: the attribute belongs to the current device, so it is set once per
    // device ordinal (a process may drive several devices from several threads)
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static hipError_t status[kMaxDev];
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    std::call_once(once[dev], [dev] {
        hipError_t e = hipSuccess;
        for (const void* f : {(const void*)k_dense_sort<double>, (const void*)k_dense_recv<double>,
                              (const void*)k_dense_sort<float>, (const void*)k_dense_recv<float>})
            if (e == hipSuccess)
                e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kGenericMaxM * sizeof(double)));
        status[dev] = e;
    });
    if (status[dev] != hipSuccess) return status[dev];
    if (a.N > kGenericMaxM || a.P > kGenericMaxM) return hipErrorNotSupported;   // (LDS images of P values)
    const size_t es = a.f32 ? sizeof(float) : sizeof(double);
    if (a.f32)
        hipLaunchKernelGGL(k_dense_sort<float>, dim3(1), dim3(kDenseSortBlock), a.P * es, s, a);
    else
        hipLaunchKernelGGL(k_dense_sort<double>, dim3(1), dim3(kDenseSortBlock), a.P * es, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (a.f32)
        hipLaunchKernelGGL(k_dense_recv<float>, dim3(dense_nblk(a.N)), dim3(kDenseRecvBlock), a.N * es, s, a);
    else
        hipLaunchKernelGGL(k_dense_recv<double>, dim3(dense_nblk(a.N)), dim3(kDenseRecvBlock), a.N * es, s, a);
    return hipGetLastError();
}

}  // namespace acs
