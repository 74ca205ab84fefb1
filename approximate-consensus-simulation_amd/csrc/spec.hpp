// spec.hpp — deterministic per-message functions of the round engine (SURVEY.md §A.1–§A.7),
// usable on host and device.  This is the PRODUCT's implementation; the CPU oracle
// (oracle/acs_oracle.c) restates the same rules independently and is never linked here.
//
// Upstream reference: none (the mount holds only README.md:1); each function cites the frozen
// spec rule it implements.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define ACS_HD __host__ __device__ __forceinline__

namespace acs {

constexpr uint32_t kHonest = 0xFFFFFFFFu;     // §A.4 status word: honest
constexpr uint32_t kByz = 0xFFFFFFFEu;        // §A.4 status word: Byzantine (else: crash round)
constexpr uint32_t kStreamDelay = 7;   // bounded-delay rounds
constexpr uint32_t kStreamInit = 0, kStreamDrop = 1, kStreamFaultset = 2, kStreamCrashRound = 3,
                   kStreamCrashPartial = 4, kStreamByz = 5, kStreamGraph = 6;

struct Key {
    uint32_t k0, k1;
};

ACS_HD Key key_of(uint64_t seed) { return Key{(uint32_t)(seed & 0xFFFFFFFFu), (uint32_t)(seed >> 32)}; }

struct U4 {
    uint32_t v[4];
};

ACS_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
#endif
}

// §A.1 Philox4x32-10 (Random123 constants; PHILOX_H:62-65, round PHILOX_H:286-296,
// key bump PHILOX_H:298-302).
ACS_HD U4 philox10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, Key key) {
    uint32_t k0 = key.k0, k1 = key.k1;
#pragma unroll
    for (int rnd = 0; rnd < 10; ++rnd) {
        if (rnd) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
#if defined(ACS_PHILOX_SPLIT_MUL)
        const uint32_t hi0 = mulhi32(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        const uint32_t hi1 = mulhi32(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
#else
        // one full 32x32->64 product per multiplier (v_mad_u64_u32) instead of mul_hi + mul_lo
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
#endif
#if defined(__HIP_DEVICE_COMPILE__)
        // gfx950 v_bitop3_b32 with the XOR3 truth table (0x96): one VALU op per output word
        // instead of two v_xor_b32 (gfx950 has no v_xor3_b32); 20 fewer per call
        const uint32_t n0 = __builtin_amdgcn_bitop3_b32(hi1, c1, k0, 0x96);
        const uint32_t n2 = __builtin_amdgcn_bitop3_b32(hi0, c3, k1, 0x96);
#else
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
#endif
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
    }
    U4 o;
    o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
    return o;
}

ACS_HD uint32_t pick(const U4& w, uint32_t sel) {
    // branch-free select of word sel (0..3) without dynamic register indexing
    const uint32_t a = (sel & 1u) ? w.v[1] : w.v[0];
    const uint32_t b = (sel & 1u) ? w.v[3] : w.v[2];
    return (sel & 2u) ? b : a;
}

// §A.1 draw(stream, b, r, s) = philox((s>>2, r, b, stream), key)[s & 3]
ACS_HD uint32_t draw(Key key, uint32_t stream, uint32_t b, uint32_t r, uint64_t s) {
    const U4 w = philox10((uint32_t)(s >> 2), r, b, stream, key);
    return pick(w, (uint32_t)(s & 3u));
}

// §A.5 drop mask of receiver `row` of a complete-graph instance with N = 4*nq <= 64 nodes:
// bit j set when the message on slot row*N + j is dropped (draw < thr), one Philox call per 4
// slots.  Each bit is shifted in from the right (m = 2m + (w < thr): a compare and two cheap ops
// per draw instead of a 64-bit shift, select and or), so draw j of a 32-draw half lands at bit
// (n - 1 - j); one bit reverse per half restores bit j.
// m = 2m + (w < thr) as v_cmp (borrow into vcc) + v_addc (m + m + vcc).  Written out: the compiler
// turns the add into an or of disjoint bits and spends a v_cndmask plus a share of a v_or3 per draw.
// (The s_nop covers the VALU vcc write -> VALU vcc read distance; thr is uniform, an SGPR.)
__device__ __forceinline__ uint32_t shift_in_lt(uint32_t m, uint32_t w, uint32_t thr) {
    uint32_t out;
    asm("v_cmp_gt_u32 vcc, %2, %1\n\ts_nop 1\n\tv_addc_co_u32 %0, vcc, %3, %3, vcc"
        : "=v"(out)
        : "v"(w), "s"(thr), "v"(m)
        : "vcc");
    return out;
}

__device__ __forceinline__ uint64_t drop_mask_n4(uint32_t row, uint32_t nq, uint32_t r, uint32_t bG, Key key,
                                                 uint32_t thr) {
    const uint32_t n0 = nq < 8u ? nq : 8u;
    uint32_t m0 = 0, m1 = 0;
    for (uint32_t g = 0; g < n0; ++g) {
        const U4 w = philox10(row * nq + g, r, bG, kStreamDrop, key);
#pragma unroll
        for (int e = 0; e < 4; ++e) m0 = shift_in_lt(m0, w.v[e], thr);
    }
    for (uint32_t g = 8; g < nq; ++g) {
        const U4 w = philox10(row * nq + g, r, bG, kStreamDrop, key);
#pragma unroll
        for (int e = 0; e < 4; ++e) m1 = shift_in_lt(m1, w.v[e], thr);
    }
    const uint32_t b0 = __builtin_bitreverse32(m0) >> (32u - 4u * n0);
    const uint32_t b1 = nq > 8u ? __builtin_bitreverse32(m1) >> (32u - 4u * (nq - 8u)) : 0u;
    return (uint64_t)b1 << 32 | b0;
}

// §A.1 u53(w0, w1) = ((w0>>5)·2^26 + (w1>>6)) · 2^-53  (exact)
ACS_HD double u53(uint32_t w0, uint32_t w1) {
    const uint64_t m = ((uint64_t)(w0 >> 5) << 26) | (uint64_t)(w1 >> 6);
    return (double)m * 0x1p-53;
}

// §A.3 Feistel permutation π_k of [0, n) and its inverse (4 rounds, cycle walking).
struct Feistel {
    uint32_t n;      // domain size N (< 2^31)
    uint32_t h;      // half width
    uint32_t mask;   // 2^h - 1
    Key key;         // key(graph_seed)
};

inline Feistel make_feistel(uint64_t n, uint64_t graph_seed) {
    int mb = 0;
    for (uint64_t v = n - 1; v; v >>= 1) ++mb;
    if (mb < 2) mb = 2;
    if (mb & 1) mb += 1;
    Feistel f;
    f.n = (uint32_t)n;
    f.h = (uint32_t)(mb / 2);
    f.mask = (uint32_t)((1ull << f.h) - 1ull);
    f.key = key_of(graph_seed);
    return f;
}

ACS_HD uint32_t feistel_fwd(const Feistel& f, uint32_t k, uint32_t v) {
    do {
        uint32_t L = v >> f.h, R = v & f.mask;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
            const uint32_t F = philox10(R, j, k, kStreamGraph, f.key).v[0] & f.mask;
            const uint32_t nl = R, nr = L ^ F;
            L = nl;
            R = nr;
        }
        v = (uint32_t)(((uint64_t)L << f.h) | R);
    } while (v >= f.n);
    return v;
}

ACS_HD uint32_t feistel_inv(const Feistel& f, uint32_t k, uint32_t v) {
    do {
        uint32_t L = v >> f.h, R = v & f.mask;
#pragma unroll
        for (int j = 3; j >= 0; --j) {
            const uint32_t F = philox10(L, (uint32_t)j, k, kStreamGraph, f.key).v[0] & f.mask;
            const uint32_t nl = R ^ F, nr = L;
            L = nl;
            R = nr;
        }
        v = (uint32_t)(((uint64_t)L << f.h) | R);
    } while (v >= f.n);
    return v;
}

// Per-round message-resolution parameters (§A.4–§A.6), uniform over a launch.
struct MsgParams {
    Key key;              // key(seed)
    uint32_t thr;         // §A.5 drop threshold (0: no loss)
    uint32_t fault;       // ACS_FAULT_*
    uint32_t byz;         // ACS_BYZ_*
    uint32_t mask_group;  // G
    uint64_t inst_offset; // global id of local instance 0
    double delta;         // Δ
    double bconst;        // c
    uint32_t omit;        // missing_policy = OMIT: missing entries leave S_i
};

// §A.4 Byzantine value on slot s for receiver i in round r (lo, hi = honest min/max of x^r).
ACS_HD double byz_value(const MsgParams& p, uint32_t b, uint32_t r, uint32_t i, uint64_t s, double lo,
                        double hi) {
    if (p.byz == 0) return (i & 1u) == 0 ? hi + p.delta : lo - p.delta;  // SPLIT
    if (p.byz == 2) return p.bconst;                                      // CONSTANT
    // RANDOM: words 2s and 2s+1 share one Philox call (ctr (2s)>>2 = s>>1)
    const U4 w = philox10((uint32_t)(s >> 1), r, b, kStreamByz, p.key);
    const uint32_t lo_word = (uint32_t)((s & 1u) << 1);
    const double u = u53(pick(w, lo_word), pick(w, lo_word + 1));
    const double width = (hi - lo) + 2.0 * p.delta;
    return (lo - p.delta) + u * width;
}

// DESIGN.md §9 fp32 mode: Δ and c rounded to binary32 once; RANDOM uses u24 = (draw(BYZ, b, r,
// 2s) >> 8) * 2^-24; every step is a binary32 operation in the order written (no FMA).
ACS_HD float byz_value_f32(const MsgParams& p, uint32_t b, uint32_t r, uint32_t i, uint64_t s, float lo,
                           float hi) {
    const float dl = (float)p.delta;
    if (p.byz == 0) return (i & 1u) == 0 ? hi + dl : lo - dl;   // SPLIT
    if (p.byz == 2) return (float)p.bconst + 0.0f;               // CONSTANT (canonical +0)
    const float u = (float)(draw(p.key, kStreamByz, b, r, 2 * s) >> 8) * 0x1p-24f;
    const float width = (hi - lo) + 2.0f * dl;
    return (lo - dl) + u * width;
}
ACS_HD double byz_value_t(const MsgParams& p, uint32_t b, uint32_t r, uint32_t i, uint64_t s, double lo,
                          double hi) {
    return byz_value(p, b, r, i, s, lo, hi);
}
ACS_HD float byz_value_t(const MsgParams& p, uint32_t b, uint32_t r, uint32_t i, uint64_t s, float lo, float hi) {
    return byz_value_f32(p, b, r, i, s, lo, hi);
}

// §A.4 crash semantics of a sender with status word st in round r: true = message missing.
ACS_HD bool crash_missing(const MsgParams& p, uint32_t st, uint32_t b, uint32_t r, uint64_t s) {
    if (st >= kByz) return false;  // honest or Byzantine
    if (r > st) return true;
    if (r == st) return draw(p.key, kStreamCrashPartial, b, st, s) >= 0x80000000u;
    return false;
}

// §A.6 active receiver in round r: honest, or crash-faulty with r < r_v
ACS_HD bool is_active(uint32_t st, uint32_t r) { return st == kHonest || (st != kByz && r < st); }

}  // namespace acs
