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

// M = 2^k + 1 entries (the d + 1 entries of a d-regular receiver, d = 8 / 16 / 32): Batcher's
// network on entries 1..M-1, then entry 0 inserted by a compare-exchange chain (0,1), (1,2), ...
// For the t = 5 trimmed window of 33 entries: 218 compare-exchanges after pruning instead of 239
// for the pruned 64-wire Batcher network (full sort: 223 against 246).
#ifndef ACS_SORTNET_INSERT
#define ACS_SORTNET_INSERT 1
#endif
constexpr bool insert_net_applies(int M) { return ACS_SORTNET_INSERT && M >= 5 && ((M - 1) & (M - 2)) == 0; }

template <int P, int M, int LO, int HI>
constexpr CEList<ce_cap(P)> pruned_net() {
    CEList<ce_cap(P)> tmp{};
    tmp.n = 0;
    if constexpr (insert_net_applies(M)) {
        const auto all = batcher_all<M - 1>();
        for (int q = 0; q < all.n; ++q) {
            tmp.c[tmp.n].a = (int16_t)(all.c[q].a + 1);
            tmp.c[tmp.n].b = (int16_t)(all.c[q].b + 1);
            ++tmp.n;
        }
        for (int i = 0; i + 1 < M; ++i) {
            tmp.c[tmp.n].a = (int16_t)i;
            tmp.c[tmp.n].b = (int16_t)(i + 1);
            ++tmp.n;
        }
    } else {
        const auto all = batcher_all<P>();
        for (int q = 0; q < all.n; ++q)
            if (all.c[q].b < M) tmp.c[tmp.n++] = all.c[q];
    }
    bool need[P] = {};
    for (int w = 0; w < P; ++w) need[w] = (w >= LO && w < HI);
    bool keep[ce_cap(P)] = {};
    for (int q = tmp.n - 1; q >= 0; --q) {
        const int a = tmp.c[q].a, b = tmp.c[q].b;
        if (need[a] || need[b]) {
            keep[q] = true;
            need[a] = need[b] = true;
        }
    }
    CEList<ce_cap(P)> out{};
    out.n = 0;
    for (int q = 0; q < tmp.n; ++q)
        if (keep[q]) out.c[out.n++] = tmp.c[q];
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
    static constexpr auto list = pruned_net<P, M, LO, HI>();
    static constexpr int count = list.n;
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

// Sort v[0..M) so that positions [LO, HI) hold the ascending order statistics LO..HI-1.
template <int M, int LO = 0, int HI = M, typename T>
__device__ __forceinline__ void select_sort(T (&v)[M]) {
    using Net = SelectNet<M, LO, HI>;
    run_net<Net>(v, std::make_index_sequence<Net::count>{});
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
