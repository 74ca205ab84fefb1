// Host check of csrc/sortnet.hpp (compiled with g++ by tests/test_sortnet_host.py):
//  1. every selection network the register kernels instantiate (M = d + 1 entries, window [t, M - t))
//     puts the window's order statistics where std::sort does, on random multisets with ties, and
//     passes the 0-1 principle (exhaustively: every 0-1 vector, 2^33 at d = 32);
//  2. the NZ tree sum (padding adds skipped, one final +0.0) equals the spec's tree bit for bit,
//     signed zeros and denormals included.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

#define __device__
#define __forceinline__ inline
#include "sortnet.hpp"

using namespace acs;

static uint64_t bits(double x) {
    uint64_t u;
    memcpy(&u, &x, 8);
    return u;
}

template <int M, int LO, int HI>
static long check_net(std::mt19937_64& g, int iters) {
    long bad = 0;
    for (int it = 0; it < iters; ++it) {
        double v[M], ref[M];
        for (int k = 0; k < M; ++k) v[k] = ref[k] = (double)(int)(g() % 9) * 0.125 + (g() % 4 ? 0.0 : 1e-3 * (g() % 7));
        select_sort<M, LO, HI>(v);
        std::sort(ref, ref + M);
        for (int k = LO; k < HI; ++k) bad += bits(v[k]) != bits(ref[k]);
    }
    return bad;
}

// 0-1 principle, 64 inputs per word: every 0-1 vector (M <= 20) or `samples` random words of them
// (with every density of ones) through the pruned network and its output permutation; the
// window must hold the sorted vector's ones and zeros.
template <int M, int LO, int HI>
static long check_01(std::mt19937_64& g, long samples) {
    using Net = SelectNet<M, LO, HI>;
    const bool all = M <= 20;
    const long words = all ? ((1L << M) + 63) / 64 : samples;
    long bad = 0;
    for (long w = 0; w < words; ++w) {
        uint64_t x[M];
        if (all) {
            for (int k = 0; k < M; ++k) {
                uint64_t m = 0;
                for (int j = 0; j < 64; ++j) m |= (uint64_t)(((w * 64 + j) >> k) & 1) << j;
                x[k] = m;
            }
        } else {
            const int dens = (int)(w % (M + 1));   // P(one) = dens / M
            for (int k = 0; k < M; ++k) {
                uint64_t m = 0;
                for (int j = 0; j < 64; ++j) m |= (uint64_t)((int)(g() % M) < dens) << j;
                x[k] = m;
            }
        }
        int ones[64] = {};
        for (int k = 0; k < M; ++k)
            for (int j = 0; j < 64; ++j) ones[j] += (int)((x[k] >> j) & 1);
        for (int q = 0; q < Net::count; ++q) {
            const int a = Net::list.c[q].a, b = Net::list.c[q].b;
            const uint64_t lo = x[a] & x[b], hi = x[a] | x[b];
            x[a] = lo;
            x[b] = hi;
        }
        for (int k = LO; k < HI; ++k) {
            const uint64_t got = x[Net::net.perm[k]];
            for (int j = 0; j < 64; ++j)
                bad += (int)((got >> j) & 1) != (k >= M - ones[j] ? 1 : 0);
        }
    }
    return bad;
}

// 0-1 principle, EXHAUSTIVE for any M <= 40 (the 33-entry networks were only sampled):
// the low 6 wires carry the lane index (64 inputs per word) and the other M - 6 wires are constant
// in a word (all ones or all zeros, from the word index w), so an input's count of ones is
// popcount(lane) + popcount(w) and the sorted value of window position k is one exactly for the
// lanes with popcount(lane) >= M - k - popcount(w): one precomputed lane mask per threshold.
// 2^(M-6) words (2^27 at M = 33), split over OpenMP threads.
template <int M, int LO, int HI>
static long check_01_all() {
    static_assert(M > 6 && M <= 40, "lanes carry 6 wires");
    using Net = SelectNet<M, LO, HI>;
    uint64_t lanes[6], ge[8];   // ge[t]: lanes with popcount >= t (t = 0..7)
    for (int k = 0; k < 6; ++k) {
        lanes[k] = 0;
        for (int j = 0; j < 64; ++j) lanes[k] |= (uint64_t)((j >> k) & 1) << j;
    }
    for (int t = 0; t < 8; ++t) {
        ge[t] = 0;
        for (int j = 0; j < 64; ++j) ge[t] |= (uint64_t)(__builtin_popcount(j) >= t) << j;
    }
    const long words = 1L << (M - 6);
    long bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
    for (long w = 0; w < words; ++w) {
        uint64_t x[M];
        for (int k = 0; k < 6; ++k) x[k] = lanes[k];
        for (int k = 6; k < M; ++k) x[k] = ((w >> (k - 6)) & 1) ? ~0ull : 0ull;
        const int pw = __builtin_popcountl((unsigned long)w);
        for (int q = 0; q < Net::count; ++q) {
            const int a = Net::list.c[q].a, b = Net::list.c[q].b;
            const uint64_t lo = x[a] & x[b], hi = x[a] | x[b];
            x[a] = lo;
            x[b] = hi;
        }
        for (int k = LO; k < HI; ++k) {
            const int t = M - k - pw;   // lanes whose popcount reaches t hold a one at rank k
            const uint64_t want = t <= 0 ? ~0ull : t > 6 ? 0ull : ge[t];
            bad += __builtin_popcountll(x[Net::net.perm[k]] ^ want);
        }
    }
    return bad;
}

template <int N, int OFF, int STRIDE, int M>
static long check_tree(const double (&a)[M]) {
    return bits(tree_sum_const<N, OFF, STRIDE, false>(a)) != bits(tree_sum_const<N, OFF, STRIDE, true>(a));
}

int main() {
    std::mt19937_64 g(7);
    long bad = 0;
    bad += check_net<33, 5, 28>(g, 200000);   // cfg4: d = 32, t = 5
    bad += check_net<33, 0, 33>(g, 100000);   // d = 32, t = 0 (full sort)
    bad += check_net<17, 5, 12>(g, 200000);   // cfg5: d = 16, t = 5
    bad += check_net<17, 0, 17>(g, 100000);
    bad += check_net<9, 2, 7>(g, 100000);     // d = 8, t = 2
    bad += check_net<5, 1, 4>(g, 100000);     // d = 4, t = 1
    bad += check_01<17, 0, 17>(g, 0);         // every 0-1 vector: Green's network + insertion
    bad += check_01<17, 5, 12>(g, 0);
    bad += check_01<9, 2, 7>(g, 0);
    bad += check_01<33, 5, 28>(g, 60000);     // 3.8 M random 0-1 vectors, all densities
    bad += check_01<33, 0, 33>(g, 60000);
    bad += check_01_all<33, 5, 28>();          // every one of the 2^33 0-1 vectors (cfg4's network)
    bad += check_01_all<33, 0, 33>();
    bad += check_01_all<17, 5, 12>();          // (the same checker on the exhaustively checked 17)
    long nbad_net = bad;
    const double pool[] = {0.0, -0.0, 5e-324, -5e-324, 1.0, -1.0, 0.5, -0.5, 1e-310, -1e-310, 3.0, -3.0};
    long ntree = 0;
    for (int it = 0; it < 300000; ++it) {
        double a[33];
        for (int k = 0; k < 33; ++k) {
            const int c = (int)(g() % 14);
            a[k] = c < 12 ? pool[c] : (double)((int64_t)(g() % 2001) - 1000) * 0.25;
        }
        bad += check_tree<23, 5, 1>(a);    // TRIMMED t = 5 of 33
        bad += check_tree<5, 5, 5>(a);     // DLPSW t = 5
        bad += check_tree<33, 0, 1>(a);    // AVERAGE over 33 entries
        bad += check_tree<7, 5, 1>(a);     // TRIMMED t = 5 of 17
        bad += check_tree<16, 0, 1>(a);    // a power of two: nothing skipped
        ntree += 5;
    }
    printf("networks: %ld mismatches; trees: %ld checked, %ld mismatches\n", nbad_net, ntree, bad - nbad_net);
    return bad != 0;
}
