// sortnet.hpp — compile-time sorting / selection networks kept entirely in VGPRs.
//
// Batcher's odd–even merge sort on P = 2^k wires, pruned in two ways at compile time:
//  1. to M <= P live inputs (comparators touching wires >= M are dropped; the network still
//     sorts the first M wires because padding wires would hold +inf and never move);
//  2. to an output window [LO, HI): comparators whose outputs never reach a window position
//     are dropped (backward liveness).  SURVEY §8(a) a7: the trimmed mean needs only the sorted
//     middle R = S[t .. m-t), e.g. 239 instead of 246 comparators for m = 33, t = 5.
// Every comparator index is a template constant, so the value array never leaves registers.
#pragma once

#include <stdint.h>

#include <utility>

namespace acs {

struct CE {
    int16_t a, b;
};

template <int CAP>
struct CEList {
    CE c[CAP];
    int n;
};

constexpr int ce_cap(int P) { return P * P / 2 + 8; }

template <int P>
constexpr CEList<ce_cap(P)> batcher_all() {
    CEList<ce_cap(P)> L{};
    L.n = 0;
    for (int p = 1; p < P; p <<= 1)
        for (int k = p; k >= 1; k >>= 1)
            for (int j = k % p; j + k < P; j += 2 * k)
                for (int i = 0; i < (k < P - j - k ? k : P - j - k); ++i)
                    if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        L.c[L.n].a = (int16_t)(i + j);
                        L.c[L.n].b = (int16_t)(i + j + k);
                        ++L.n;
                    }
    return L;
}

// Green's 60-comparator sorting network on 16 wires (M. W. Green, 1969; Knuth, TAOCP vol. 3,
// §5.3.4), against Batcher's 63.  Checked by the 0-1 principle (tests/test_sortnet_host.py).
constexpr CE kGreen16[60] = {
    {0, 13}, {1, 12}, {2, 15}, {3, 14}, {4, 8}, {5, 6}, {7, 11}, {9, 10},
    {0, 5}, {1, 7}, {2, 9}, {3, 4}, {6, 13}, {8, 14}, {10, 15}, {11, 12},
    {0, 1}, {2, 3}, {4, 5}, {6, 8}, {7, 9}, {10, 11}, {12, 13}, {14, 15},
    {0, 2}, {1, 3}, {4, 10}, {5, 11}, {6, 7}, {8, 9}, {12, 14}, {13, 15},
    {1, 2}, {3, 12}, {4, 6}, {5, 7}, {8, 10}, {9, 11}, {13, 14},
    {1, 4}, {2, 6}, {5, 8}, {7, 10}, {9, 13}, {11, 14},
    {2, 4}, {3, 6}, {9, 12}, {11, 13},
    {3, 5}, {6, 8}, {7, 9}, {10, 12},
    {3, 4}, {5, 6}, {7, 8}, {9, 10}, {11, 12},
    {6, 7}, {8, 9}};

// Batcher's odd-even merge of the sorted halves of wires [lo, lo + n) (n a power of two)
template <int CAP>
constexpr void oem_merge(CEList<CAP>& L, int lo, int n, int r) {
    const int m = r * 2;
    if (m < n) {
        oem_merge(L, lo, n, m);
        oem_merge(L, lo + r, n, m);
        for (int i = lo + r; i + r < lo + n; i += m) {
            L.c[L.n].a = (int16_t)i;
            L.c[L.n].b = (int16_t)(i + r);
            ++L.n;
        }
    } else {
        L.c[L.n].a = (int16_t)lo;
        L.c[L.n].b = (int16_t)(lo + r);
        ++L.n;
    }
}

// A network and the wire that holds each rank at its end (perm[k]: rank k's wire).
template <int P>
struct NetPerm {
    CEList<ce_cap(P)> list;
    int16_t perm[P];
};

template <int CAP>
constexpr void push_ce(CEList<CAP>& L, int a, int b) {
    L.c[L.n].a = (int16_t)a;
    L.c[L.n].b = (int16_t)b;
    ++L.n;
}

// M = 2^k + 1 entries (the d + 1 entries of a d-regular receiver, d = 8 / 16 / 32).
//  d = 8: Batcher's network on entries 1..8, then entry 0 inserted by a compare-exchange chain
//    (0,1), (1,2), ...
//  d = 16: the same with Green's network on entries 1..16.
//  d = 32: entries 0..16 sorted as for d = 16, entries 17..32 by Green's network,
//    and the two runs merged by Batcher's odd-even merge of 2 x 32 wires whose 31 padding wires hold
//    +inf: a comparator whose upper wire is padding is dropped, one whose lower wire is padding
//    becomes a relabelling (the finite value moves to the padding's place).  The ranks end on
//    permuted wires (perm).  For the t = 5 window of 33 entries: 200 compare-exchanges after
//    pruning, against 218 for Batcher's 32-wire network plus the insertion chain and 239 for the
//    pruned 64-wire Batcher network (full sort: 206, 223 and 246).
#ifndef ACS_SORTNET_INSERT
#define ACS_SORTNET_INSERT 1
#endif
#ifndef ACS_SORTNET_GREEN   // 0: Batcher's network on entries 1..M-1 for d = 16 / 32 too (round 4; A/B builds)
#define ACS_SORTNET_GREEN 1
#endif
constexpr bool insert_net_applies(int M) { return ACS_SORTNET_INSERT && M >= 5 && ((M - 1) & (M - 2)) == 0; }

template <int P, int M>
constexpr NetPerm<P> full_net() {
    NetPerm<P> R{};
    R.list.n = 0;
    for (int w = 0; w < P; ++w) R.perm[w] = (int16_t)w;
    if constexpr (ACS_SORTNET_GREEN && insert_net_applies(M) && M == 33) {
        // entries 0..16: Green on 1..16, entry 0 inserted
        for (int q = 0; q < 60; ++q) push_ce(R.list, kGreen16[q].a + 1, kGreen16[q].b + 1);
        for (int i = 0; i < 16; ++i) push_ce(R.list, i, i + 1);
        // entries 17..32: Green
        for (int q = 0; q < 60; ++q) push_ce(R.list, kGreen16[q].a + 17, kGreen16[q].b + 17);
        // merge: virtual wires 0..16 = entries 0..16, 32..47 = entries 17..32, the rest +inf
        CEList<ce_cap(64)> mg{};
        mg.n = 0;
        oem_merge(mg, 0, 64, 1);
        int content[64] = {};
        bool inf[64] = {};
        for (int v = 0; v < 64; ++v) {
            inf[v] = !(v < 17 || (v >= 32 && v < 48));
            content[v] = v < 17 ? v : v >= 32 && v < 48 ? v - 15 : -1;
        }
        for (int q = 0; q < mg.n; ++q) {
            const int a = mg.c[q].a, b = mg.c[q].b;
            if (inf[b]) continue;   // +inf above: no exchange
            if (inf[a]) {           // +inf below a finite value: they trade places
                const int t = content[a];
                content[a] = content[b];
                content[b] = t;
                inf[a] = false;
                inf[b] = true;
                continue;
            }
            push_ce(R.list, content[a], content[b]);
        }
        for (int k = 0; k < M; ++k) R.perm[k] = (int16_t)content[k];
    } else if constexpr (ACS_SORTNET_GREEN && insert_net_applies(M) && M == 17) {
        for (int q = 0; q < 60; ++q) push_ce(R.list, kGreen16[q].a + 1, kGreen16[q].b + 1);
        for (int i = 0; i < 16; ++i) push_ce(R.list, i, i + 1);
    } else if constexpr (insert_net_applies(M)) {
        const auto all = batcher_all<M - 1>();
        for (int q = 0; q < all.n; ++q) push_ce(R.list, all.c[q].a + 1, all.c[q].b + 1);
        for (int i = 0; i + 1 < M; ++i) push_ce(R.list, i, i + 1);
    } else {
        const auto all = batcher_all<P>();
        for (int q = 0; q < all.n; ++q)
            if (all.c[q].b < M) R.list.c[R.list.n++] = all.c[q];
    }
    return R;
}

template <int P, int M, int LO, int HI>
constexpr NetPerm<P> pruned_net() {
    const NetPerm<P> F = full_net<P, M>();
    bool need[P] = {};
    for (int k = LO; k < HI; ++k) need[F.perm[k]] = true;
    bool keep[ce_cap(P)] = {};
    for (int q = F.list.n - 1; q >= 0; --q) {
        const int a = F.list.c[q].a, b = F.list.c[q].b;
        if (need[a] || need[b]) {
            keep[q] = true;
            need[a] = need[b] = true;
        }
    }
    NetPerm<P> out{};
    out.list.n = 0;
    for (int q = 0; q < F.list.n; ++q)
        if (keep[q]) out.list.c[out.list.n++] = F.list.c[q];
    for (int w = 0; w < P; ++w) out.perm[w] = F.perm[w];
    return out;
}

constexpr int next_pow2(int n) {
    int p = 1;
    while (p < n) p <<= 1;
    return p;
}

template <int M, int LO, int HI>
struct SelectNet {
    static constexpr int P = next_pow2(M);
    static constexpr auto net = pruned_net<P, M, LO, HI>();
    static constexpr auto list = net.list;
    static constexpr int count = list.n;
    static constexpr bool permuted = [] {
        for (int k = 0; k < M; ++k)
            if (net.perm[k] != k) return true;
        return false;
    }();
};

// fp64 compare-exchange halves as raw v_min_f64 / v_max_f64: every value the engine sorts is a
// finite, non-NaN double (inputs are validated), so the sNaN-quieting canonicalisation that
// __builtin_fmin / fmax add for values loaded from memory (one extra v_max_f64 per input) is dead
// work.  -0.0 never occurs (§A.4 canonicalises the constant), so min/max are exact.
// (The host pass — and the host build of tests/host/sortnet_check.cpp — takes the plain comparison.)
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double ce_min(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double ce_max(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float ce_min(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float ce_max(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
#else
__device__ __forceinline__ double ce_min(double a, double b) { return b < a ? b : a; }
__device__ __forceinline__ double ce_max(double a, double b) { return b < a ? a : b; }
__device__ __forceinline__ float ce_min(float a, float b) { return b < a ? b : a; }
__device__ __forceinline__ float ce_max(float a, float b) { return b < a ? a : b; }
#endif
__device__ __forceinline__ uint32_t ce_min(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t ce_max(uint32_t a, uint32_t b) { return a < b ? b : a; }

template <int A, int B, typename T, int M>
__device__ __forceinline__ void cmpx(T (&v)[M]) {
    const T a = v[A], b = v[B];
    v[A] = ce_min(a, b);
    v[B] = ce_max(a, b);
}

template <typename Net, typename T, int M, size_t... I>
__device__ __forceinline__ void run_net(T (&v)[M], std::index_sequence<I...>) {
    (cmpx<Net::list.c[I].a, Net::list.c[I].b>(v), ...);
}

template <typename Net, typename T, int M, size_t... K>
__device__ __forceinline__ void apply_perm(T (&v)[M], std::index_sequence<K...>) {
    const T t[M] = {v[Net::net.perm[K]]...};   // compile-time register renaming
    ((v[K] = t[K]), ...);
}

// Sort v[0..M) so that positions [LO, HI) hold the ascending order statistics LO..HI-1.
template <int M, int LO = 0, int HI = M, typename T>
__device__ __forceinline__ void select_sort(T (&v)[M]) {
    using Net = SelectNet<M, LO, HI>;
    run_net<Net>(v, std::make_index_sequence<Net::count>{});
    if constexpr (Net::permuted) apply_perm<Net>(v, std::make_index_sequence<M>{});
}

// §A.7 tree_sum over N values a[OFF], a[OFF+STRIDE], ...: pad to a power of two with +0.0,
// stride-halving pairwise adds.  Compile-time indices only.  NZ: the adds of a
// padding +0.0 are skipped and the root gets one +0.0 instead — 23 instead of 31 adds for the t = 5
// window of 33 entries.  Exact for every input: x + (+0.0) == x except for x = -0.0, so by induction
// every node differs from the spec's at most in the sign of a zero, and the spec's root is never
// -0.0 when N < P (a sum is -0.0 only if both operands are, and some node below the root added a
// padding +0.0), so the final +0.0 maps the one possible difference (-0.0 for +0.0) back.
template <int N, int OFF = 0, int STRIDE = 1, bool NZ = false, typename T, int M>
__device__ __forceinline__ T tree_sum_const(const T (&a)[M]) {
    constexpr int P = next_pow2(N);
    T w[P];
#pragma unroll
    for (int k = 0; k < P; ++k) w[k] = k < N ? a[OFF + k * STRIDE] : T(0);
    int n = N;   // w[n..) hold padding zeros (compile-time after unrolling)
#pragma unroll
    for (int s = P / 2; s >= 1; s >>= 1) {
#pragma unroll
        for (int k = 0; k < s; ++k)
            if (!NZ || k + s < n) w[k] = w[k] + w[k + s];
        n = n < s ? n : s;
    }
    if constexpr (NZ && N < P) return w[0] + T(0);
    return w[0];
}

}  // namespace acs
