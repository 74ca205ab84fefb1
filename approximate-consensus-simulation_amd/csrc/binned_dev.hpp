// binned_dev.hpp — device pieces of the binned exchange (round_binned.hip): cache-policy switches,
// the phase-A index stream, the LDS-DMA run copies and the NP-pass image bound.  SURVEY §8(a) a5 / a7.
#pragma once

#include "finalize.hpp"
#include "resolve.hpp"
#include "rules.hpp"

namespace acs {

constexpr uint32_t kBinA = 512;        // phase-A / phase-M workgroup: 8 waves
constexpr uint32_t kBinMCap = 19456;   // phase-M LDS image capacity (elements, 152 KiB)
// cache-policy switches of the exchange (launch argument `pol`; ACSIM_BIN_POL overrides the default)
// (Retired in round 6, measured slower in the driver's shape and in 200-round A/Bs, DESIGN.md §5.11;
// their bits are ignored now: 1 nontemporal phase-B run copies, 4 plain instead of nontemporal
// invpos loads — the nontemporal load is unconditional —, 8 RevB (each XCD walking its receiver
// blocks downwards), 16 NoPf (per-part descriptor loads instead of the prefetch).  In git history.)
constexpr uint32_t kPolNtStore = 2;    // phase A: nontemporal stage stores (two-level plans' default)
constexpr uint32_t kPolBfPick = 32;     // phase B (NP > 1): branch-free pick-up (clamped read + select)
constexpr uint32_t kPolSc1Store = 64;   // phase A: write-through (sc1) stage stores instead of nt: no
                                        // dirty stage lines left in L2 for the kernel boundary to write back
constexpr uint32_t kPolNtStoreM = 128;  // phase M (two-level plans): nontemporal stage-2 stores
constexpr uint32_t kPolSc1StoreM = 256; // phase M: write-through (sc1) stage-2 stores
constexpr uint32_t kPolSc1X = 512;      // phase B: write-through (sc1) stores of x^{r+1}
constexpr uint32_t kPolClampPick = 1024; // phase B (NP = 2): pick-up by clamped index into a zero slot, OR-merged
// (2048: a scalar-descriptor buffer LDS-DMA form of phase B's run copies, measured slower in round 5
// and removed)
constexpr uint32_t kPolBytePick = 4096;  // phase B (clamped pick-up, clean plans): packed 16-bit pick-up, add-merged
constexpr uint32_t kPolAsmDma = 8192;    // phase B (clamped pick-up): run copies by asm saddr LDS-DMA (bin_dma_runs_asm)
constexpr uint32_t kPolAsmDmaT = 16384;  // phase M and one-pass phase B: run copies by asm saddr LDS-DMA (bin_dma_runs_asm_tb)
constexpr uint32_t kPolMask = 32767;     // every switch (ACSIM_BIN_POL)
// Default switches (the stage-store bits are chosen per plan).  Until round 4 the
// stream's store flavour was a runtime argument, and the compiler merged the nontemporal and the
// plain store of its two branches into one plain store: every "nontemporal stage store" measured
// in rounds 1-3 was a plain store.  Made explicit (bin_stream_t<SMODE>), real nontemporal stage
// stores cost cfg4 about 25 us per round (phase A), so one-level plans store plain.
// stage stores by plan (DESIGN.md §5.8, A/B inside one build): one level (cfg4) write-through phase-A
// stores, 118 against 122 us per round for plain ones (no dirty stage lines for the kernel boundary
// to write back; nontemporal ones 137 us); two levels (cfg5) nontemporal phase-A and phase-M stores,
// 7.60 against 7.86 ms per round for plain ones (the 16 GiB of stages far exceed the MALL)
constexpr uint32_t kPolOneLevelStores = kPolSc1Store;
constexpr uint32_t kPolTwoLevelStores = kPolNtStore | kPolNtStoreM;
constexpr uint32_t kPolDefault = kPolBfPick | kPolClampPick | kPolBytePick | kPolAsmDma | kPolAsmDmaT;
// measured (cfg4): phase B 80 -> 71 (nt invpos) -> 63.2 us (pick-up); the clamped pick-up: round 117.2-118.8 ->
// 112.3-112.9 us; the packed 16-bit pick-up: 112.2-113.0 -> 110.2-111.0 us; the asm run copies:
// a further -0.4 us, and cfg4 fp32 (one-pass phase B) 79.0 -> 76.8 us (§5.11)

// ------------------------------------------------------------------------------ shared pieces
// Stream [p0, p1) of an index stream: out[p] = lds[idx[p]].  Super-steps of 512 positions per
// wave; instruction q of a lane covers positions q*128 + 2*lane, +1 (one u32 of two indices, one
// 16-byte store), so every wave-instruction reads 256 B and writes 1 KiB contiguously.
// Software-pipelined by batches of SB super-steps: the index loads of batch k+1 are issued before
// batch k's gathers and stores.  (gfx9 counts loads and stores in one in-order vmcnt: the plain
// loop's wait for its index loads also waited for the previous batch's store completions, so each
// batch paid a full store round trip.)
__device__ __forceinline__ double2 bin_pair(double a, double b) { return make_double2(a, b); }
__device__ __forceinline__ float2 bin_pair(float a, float b) { return make_float2(a, b); }

// Write-through (sc1) 16- or 8-byte store through a buffer descriptor (MI355X guide, Guideline 16
// R1 store form): the line leaves L2 with the store instead of staying dirty there.
template <typename V2>
__device__ __forceinline__ void bin_store_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off, const V2& v) {
    if constexpr (sizeof(V2) == 16) {
        using UV = unsigned int __attribute__((ext_vector_type(4)));
        UV bits;
        __builtin_memcpy(&bits, &v, 16);
        __builtin_amdgcn_raw_buffer_store_b128(bits, rs, off, 0, 16);
    } else {
        using UV = unsigned int __attribute__((ext_vector_type(2)));
        UV bits;
        __builtin_memcpy(&bits, &v, 8);
        __builtin_amdgcn_raw_buffer_store_b64(bits, rs, off, 0, 16);
    }
}

template <typename V2>
__device__ __forceinline__ void bin_store(V2* dst, const V2& v, bool nt) {
    if (nt) {   // as an integer vector of V2's size (the builtin takes native vector types)
        using UV = unsigned int __attribute__((ext_vector_type(sizeof(V2) / 4)));
        UV bits;
        __builtin_memcpy(&bits, &v, sizeof(V2));
        __builtin_nontemporal_store(bits, reinterpret_cast<UV*>(dst));
    } else {
        *dst = v;
    }
}

// VT = double, or float for fp32 plans (the instruction's store is then 8 bytes)
// SMODE: 0 plain stores, 1 nontemporal, 2 write-through (sc1) — a template parameter, so the stream
// loop carries no per-store branch and no buffer descriptor unless it writes through (round 3 had
// it as a runtime argument: cfg5's phase M and round measured 2-5 % slower)
template <uint32_t SMODE, typename VT = double>
__device__ __forceinline__ void bin_stream_t(const VT* lx, const uint16_t* __restrict__ idx, VT* __restrict__ out,
                                             uint64_t p0, uint64_t p1) {
    using V2 = decltype(bin_pair(VT(0), VT(0)));
    constexpr bool nt_store = SMODE == 1;
    constexpr uint32_t smode = SMODE;
    constexpr uint32_t SUP = kBinA / 64 * 512, SUPW = SUP / 2;
    constexpr uint32_t SB = 1;   // super-steps per pipelined batch
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t p = p0;
    if ((p0 & 1) == 0) {
        const uint64_t nsup = (p1 - p0) / SUP;
        const uint64_t nb = nsup / SB;
        const uint32_t* ip = reinterpret_cast<const uint32_t*>(idx + p0) + w * 256 + lane;
        V2* op = reinterpret_cast<V2*>(out + p0) + w * 256 + lane;
        uint32_t c[SB][4];
        if (nb) {
#pragma unroll
            for (uint32_t u = 0; u < SB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) c[u][q] = __builtin_nontemporal_load(ip + u * SUPW + q * 64);
        }
        // (measured on cfg4: SB = 1 59-61 us, SB = 2 62, SB = 4 64; keeping the previous
        // super-step's stores in flight across the loop head — first indices consumed before the
        // loop — 67 us; the loop kept rolled 62 us)
        // write-through stores go through a descriptor based at this range (offsets < 4 GiB)
        // (unused, and dropped by the compiler, unless SMODE == 2)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                out + p0, 0, (int)((p1 - p0) * sizeof(VT) < 0x7FFFFFF0ull ? (p1 - p0) * sizeof(VT) : 0x7FFFFFF0ull),
                0x00020000);
        const uint32_t ob = (w * 256 + lane) * (uint32_t)sizeof(V2);   // this lane's byte offset in a super-step
        // (rolled: with the store flavour a template parameter the body got small enough for the
        // compiler to unroll it, which measured like SB = 2..4 below: ~10 us slower on cfg4)
#pragma unroll 1
        for (uint64_t bi = 0; bi < nb; ++bi) {
            // next batch's indices (the last batch re-reads itself: no branch around the loads)
            const uint64_t bn = bi + 1 < nb ? bi + 1 : bi;
            uint32_t cn[SB][4];
#pragma unroll
            for (uint32_t u = 0; u < SB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) cn[u][q] = __builtin_nontemporal_load(ip + (bn * SB + u) * SUPW + q * 64);
#pragma unroll
            for (uint32_t u = 0; u < SB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const V2 v = bin_pair(lx[c[u][q] & 0xFFFFu], lx[c[u][q] >> 16]);
                    if constexpr (smode == 2)
                        bin_store_sc1(rs, ob + (uint32_t)(((bi * SB + u) * SUPW + q * 64) * sizeof(V2)), v);
                    else
                        bin_store(op + (bi * SB + u) * SUPW + q * 64, v, nt_store);
                }
#pragma unroll
            for (uint32_t u = 0; u < SB; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) c[u][q] = cn[u][q];
        }
        for (uint64_t k = nb * SB; k < nsup; ++k) {   // the last < SB super-steps
            uint32_t cc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) cc[q] = __builtin_nontemporal_load(ip + k * SUPW + q * 64);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                bin_store(op + k * SUPW + q * 64, bin_pair(lx[cc[q] & 0xFFFFu], lx[cc[q] >> 16]), nt_store);
        }
        p = p0 + nsup * SUP;
    }
    for (uint64_t q = p + threadIdx.x; q < p1; q += blockDim.x) out[q] = lx[idx[q]];
}

// runtime store policy -> the matching instantiation (the branch is taken once per workgroup)
template <typename VT = double>
__device__ __forceinline__ void bin_stream(const VT* lx, const uint16_t* __restrict__ idx, VT* __restrict__ out,
                                           uint64_t p0, uint64_t p1, uint32_t smode = 0) {
    if (smode == 1)
        bin_stream_t<1>(lx, idx, out, p0, p1);
    else if (smode == 2)
        bin_stream_t<2>(lx, idx, out, p0, p1);
    else
        bin_stream_t<0>(lx, idx, out, p0, p1);
}

// ------------------------------------------------------------------------------ packed phase-A indices
// 14-bit packed idxA (source blocks of at most 16384 senders; fp64 and fp32 plans): the
// stream is cut into blocks of 512 positions (one wave's super-step); block m holds lane l's eight
// indices — positions 512m + 2(64q + l) + e, index k = 2q + e at bits [14k, 14k + 14) of a 112-bit
// word — in three u32 planes (words m*224 + 64j + l, j = 0..2: bits 0-95) and one u16 plane
// (u16 element m*448 + 384 + l: bits 96-111).  896 B per 512 positions instead of 1024.
constexpr uint32_t kPk14Words = 224;   // u32 words per 512-position block

__device__ __forceinline__ uint32_t pk14_extract(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t h, int k) {
    switch (k) {   // k is a compile-time constant at every call site: one or two VALU each
        case 0: return w0 & 0x3FFFu;
        case 1: return (w0 >> 14) & 0x3FFFu;
        case 2: return __builtin_amdgcn_alignbit(w1, w0, 28) & 0x3FFFu;
        case 3: return (w1 >> 10) & 0x3FFFu;
        case 4: return __builtin_amdgcn_alignbit(w2, w1, 24) & 0x3FFFu;
        case 5: return (w2 >> 6) & 0x3FFFu;
        case 6: return __builtin_amdgcn_alignbit(h, w2, 20) & 0x3FFFu;
        default: return (h >> 2) & 0x3FFFu;
    }
}

// random access (head / tail positions of a range)
__device__ __forceinline__ uint32_t pk14_at(const uint32_t* __restrict__ pk, uint64_t p) {
    const uint64_t m = p >> 9;
    const uint32_t j = (uint32_t)p & 511u, q = j >> 7, l = (j & 127u) >> 1, e = j & 1u;
    const uint32_t* b = pk + m * kPk14Words;
    const uint32_t w0 = b[l], w1 = b[64 + l], w2 = b[128 + l];
    const uint32_t h = reinterpret_cast<const uint16_t*>(pk)[m * (2 * kPk14Words) + 384 + l];
    const uint32_t k = 2 * q + e;
    const uint32_t bit = 14 * k, wi = bit >> 5, sh = bit & 31;
    const uint32_t ws[4] = {w0, w1, w2, h};
    const uint64_t two = (uint64_t)ws[wi] | (wi < 3 ? (uint64_t)ws[wi + 1] << 32 : 0ull);
    return (uint32_t)(two >> sh) & 0x3FFFu;
}

// Stream [p0, p1) with packed indices: out[p] = lx[idx(p)].  Whole 512-position blocks go to the
// waves in turn (wave w takes blocks mb + w, mb + w + NW, ...), software-pipelined like
// bin_stream_t (the next block's four index loads are issued before this block's gathers and
// stores); the partial blocks at the ends go position by position.
// NAR (narrow stage, fp64 plans): out holds u32 entries, the low word of each
// value's bits minus the low word of the round's base (nar_lo); only the low word is read from LDS.
template <uint32_t SMODE, typename VT = double, bool NAR = false>
__device__ __forceinline__ void bin_stream_pk14_t(const VT* lx, const uint32_t* __restrict__ pk,
                                                  std::conditional_t<NAR, uint32_t, VT>* __restrict__ out,
                                                  uint64_t p0, uint64_t p1, uint32_t nar_lo = 0) {
    static_assert(!NAR || sizeof(VT) == 8, "the narrow stage encodes fp64 values");
    using V2 = std::conditional_t<NAR, uint2, decltype(bin_pair(VT(0), VT(0)))>;
    const uint32_t* l32 = reinterpret_cast<const uint32_t*>(lx);   // (NAR: the low words)
    auto one = [&](uint32_t k) {
        if constexpr (NAR)
            return l32[2 * k] - nar_lo;
        else
            return lx[k];
    };
    auto pair = [&](uint32_t k0, uint32_t k1) -> V2 {
        if constexpr (NAR)
            return make_uint2(one(k0), one(k1));
        else
            return bin_pair(lx[k0], lx[k1]);
    };
    // V2 units per 1 GiB window: the descriptor's num_records (0x7FFFFFF0) must cover the whole window
    // plus one V2 (with 2 GiB windows the last pair of each window sat at offset 0x7FFFFFF0 and its
    // store failed the range check silently; stages above 2 GiB are two-level, cfg5-sized plans)
    constexpr uint32_t kRebaseBits = sizeof(V2) == 16 ? 26 : 27;
    constexpr uint32_t NW = kBinA / 64;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t mb = (p0 + 511) >> 9, me = p1 >> 9;
    if (mb < me) {
        const uint64_t nbw = (me - mb > w) ? (me - mb - w + NW - 1) / NW : 0;   // this wave's blocks
        const uint16_t* pk16 = reinterpret_cast<const uint16_t*>(pk);
        V2* o2 = reinterpret_cast<V2*>(out);
        uint64_t m = mb + w;
        uint32_t c0 = 0, c1 = 0, c2 = 0, ch = 0;
        if (nbw) {
            const uint32_t* b = pk + m * kPk14Words + lane;
            c0 = __builtin_nontemporal_load(b);
            c1 = __builtin_nontemporal_load(b + 64);
            c2 = __builtin_nontemporal_load(b + 128);
            ch = __builtin_nontemporal_load(pk16 + m * (2 * kPk14Words) + 384 + lane);
        }
#pragma unroll 1
        for (uint64_t i = 0; i < nbw; ++i, m += NW) {
            const uint64_t mn = i + 1 < nbw ? m + NW : m;   // the last block re-reads itself
            const uint32_t* bn = pk + mn * kPk14Words + lane;
            const uint32_t n0 = __builtin_nontemporal_load(bn);
            const uint32_t n1 = __builtin_nontemporal_load(bn + 64);
            const uint32_t n2 = __builtin_nontemporal_load(bn + 128);
            const uint32_t nh = __builtin_nontemporal_load(pk16 + mn * (2 * kPk14Words) + 384 + lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
#if defined(ACS_DIAG_A) && ACS_DIAG_A == 1
                // diagnostic (variant builds only, wrong values): the same extracts, kept live, but
                // bank-conflict-free LDS reads (consecutive 8-byte words across the wave)
                const uint32_t x0 = pk14_extract(c0, c1, c2, ch, 2 * q), x1 = pk14_extract(c0, c1, c2, ch, 2 * q + 1);
                asm volatile("" ::"v"(x0), "v"(x1));
                const V2 v = pair((q * 128u + lane) & 16383u, (q * 128u + 64u + lane) & 16383u);
#else
                const V2 v = pair(pk14_extract(c0, c1, c2, ch, 2 * q), pk14_extract(c0, c1, c2, ch, 2 * q + 1));
#endif
                const uint64_t vi = m * 256 + q * 64 + lane;   // pair index of positions 2vi, 2vi + 1
                if constexpr (SMODE == 2) {
                    // (buffer offsets are 32-bit: the descriptor is re-based per 1 GiB of stage)
                    constexpr uint64_t kMask = (1ull << kRebaseBits) - 1;
                    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
                        o2 + (vi & ~kMask), 0, 0x7FFFFFF0, 0x00020000);
                    bin_store_sc1(rb, (uint32_t)(vi & kMask) * (uint32_t)sizeof(V2), v);
                } else {
                    bin_store(o2 + vi, v, SMODE == 1);
                }
            }
            c0 = n0;
            c1 = n1;
            c2 = n2;
            ch = nh;
        }
    }
    // partial blocks at both ends (or the whole range when it holds no full block)
    const uint64_t h1 = mb < me ? (mb << 9) : p1;
    for (uint64_t q = p0 + threadIdx.x; q < h1; q += blockDim.x) out[q] = one(pk14_at(pk, q));
    if (mb < me)
        for (uint64_t q = (me << 9) + threadIdx.x; q < p1; q += blockDim.x) out[q] = one(pk14_at(pk, q));
}

template <typename VT>
__device__ __forceinline__ void bin_stream_pk14(const VT* lx, const uint32_t* __restrict__ pk, VT* __restrict__ out,
                                                uint64_t p0, uint64_t p1, uint32_t smode) {
    if (smode == 1)
        bin_stream_pk14_t<1, VT>(lx, pk, out, p0, p1);
    else if (smode == 2)
        bin_stream_pk14_t<2, VT>(lx, pk, out, p0, p1);
    else
        bin_stream_pk14_t<0, VT>(lx, pk, out, p0, p1);
}

// the narrow stage's stream (u32 entries; fp64 plans)
__device__ __forceinline__ void bin_stream_pk14_narrow(const double* lx, const uint32_t* __restrict__ pk,
                                                       uint32_t* __restrict__ out, uint64_t p0, uint64_t p1,
                                                       uint32_t smode, uint32_t nar_lo) {
    if (smode == 1)
        bin_stream_pk14_t<1, double, true>(lx, pk, out, p0, p1, nar_lo);
    else if (smode == 2)
        bin_stream_pk14_t<2, double, true>(lx, pk, out, p0, p1, nar_lo);
    else
        bin_stream_pk14_t<0, double, true>(lx, pk, out, p0, p1, nar_lo);
}

// Narrow stage: the stage entry width of a round from the exact (min, max) of
// x^r the previous phase B published (omin = ord(min), omax = ord(max); resolve.hpp ord_of).  When
// every value lies strictly on one side of zero, bit patterns are monotone in value, so every x^r
// is base + k with 0 <= k <= omax - omin (base: the smaller pattern, i.e. the min for positive
// values and the max for negative ones); with that span below 2^32, a u32 offset carries each
// value exactly.  w = 8: full width (nothing published, a zero or mixed signs, or a wider span).
__device__ __forceinline__ void narrow_choose(unsigned long long omin, unsigned long long omax, uint32_t& w,
                                              unsigned long long& base) {
    constexpr unsigned long long kOrdPos0 = 1ull << 63;      // ord(+0.0)
    constexpr unsigned long long kOrdNeg0 = ~(1ull << 63);   // ord(-0.0)
    w = 8;
    base = 0;
    if (omin > omax) return;   // nothing published (the pair's identity decodes to NaNs)
    const bool pos = omin > kOrdPos0, neg = omax < kOrdNeg0;
    if (!(pos || neg) || omax - omin > 0xFFFFFFFFull) return;
    w = 4;
    base = pos ? (omin & ~kOrdPos0) : ~omax;
}

// Copy runs [r0, r1) of a run table (start in `src` elements, element offset `pre` in the LDS
// image; run k ends where run k+1's image begins) into LDS by 16-byte LDS-DMA.  Every run is
// padded to an even length, so starts are 16-byte aligned on both sides.  Descriptors are fetched
// one per lane, 64 at a time, and broadcast with readlane: no run waits on a dependent load.
// Runs are padded to EPU = 16 / sizeof(VT) elements (2 for fp64, 4 for fp32).
template <typename VT = double>
__device__ __forceinline__ void bin_dma_runs(const uint2* __restrict__ tb, uint32_t r0, uint32_t r1,
                                             const VT* __restrict__ src, VT* dst,
                                             uint32_t base = 0) {   // base: image offset of dst[0]
    constexpr uint32_t EPU = 16 / sizeof(VT);
    const uint32_t lane = threadIdx.x & 63;
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(dst);
    for (uint32_t g = r0; g < r1; g += 64) {
        const uint32_t ng = r1 - g < 64 ? r1 - g : 64;
        uint2 dsc = make_uint2(0u, 0u);
        uint32_t nxt = 0;
        if (lane < ng) {
            dsc = tb[g + lane];
            nxt = tb[g + lane + 1].y;
        }
        for (uint32_t k = 0; k < ng; ++k) {
            const uint32_t so = __builtin_amdgcn_readlane(dsc.x, k);
            const uint32_t pre = __builtin_amdgcn_readlane(dsc.y, k);
            const uint32_t n16 = (__builtin_amdgcn_readlane(nxt, k) - pre) / EPU;   // 16-byte units
            const uint4* sp = s16 + so / EPU + lane;
            uint4* dp = d16 + (pre - base) / EPU;
            for (uint32_t o = 0; o < n16; o += 64)
                if (o + lane < n16) __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 0);
        }
    }
}

// The same copy for runs [r0, r1) of a block of at most 64 runs whose descriptors the wave already
// holds one per lane (dsc = tb[lane], nxt = tb[lane + 1].y): no load before the first DMA.
template <typename VT = double>
__device__ __forceinline__ void bin_dma_runs_pf(uint2 dsc, uint32_t nxt, uint32_t r0, uint32_t r1,
                                                const VT* __restrict__ src, VT* dst, uint32_t base) {
    constexpr uint32_t EPU = 16 / sizeof(VT);
    const uint32_t lane = threadIdx.x & 63;
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    uint4* d16 = reinterpret_cast<uint4*>(dst);
    for (uint32_t k = r0; k < r1; ++k) {
        const uint32_t so = __builtin_amdgcn_readlane(dsc.x, k);
        const uint32_t pre = __builtin_amdgcn_readlane(dsc.y, k);
#if defined(ACS_DIAG_B) && ACS_DIAG_B == 3   // diagnostic: phase B without its stage transfer
        const uint32_t n16 = (__builtin_amdgcn_readlane(nxt, k) - pre) / EPU > 0u ? 1u : 0u;
#else
        const uint32_t n16 = (__builtin_amdgcn_readlane(nxt, k) - pre) / EPU;
#endif
        const uint4* sp = s16 + so / EPU + lane;
        uint4* dp = d16 + (pre - base) / EPU;
        for (uint32_t o = 0; o < n16; o += 64)
            if (o + lane < n16) __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 0);
    }
}

// One `global_load_lds_dwordx4 voffset, sbase` with its LDS destination in M0.  The compiler treats
// M0 as a reserved register and does not model an asm write to it (a clobber entry is "undefined
// behaviour" to LLVM), so the statement saves the compiler's M0 into a scratch SGPR first and
// restores it after the issue: whatever M0 value the compiler's own LDS-DMA or M0-indexed code
// holds across the statement is preserved by construction.  (The instruction reads M0 at issue,
// so rewriting it right after is safe: consecutive copies already rewrite it back to back.)
__device__ __forceinline__ void bin_lds_dma16(uint32_t voff, uint64_t sbase, uint32_t m0) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved) : "v"(voff), "s"(sbase), "s"(m0) : "memory");
#endif
}

// bin_dma_runs_pf with the copies issued as asm `global_load_lds_dwordx4 voffset, sbase` (kPolAsmDma,
// DESIGN.md §5.11): the run's stage address is an SGPR pair (stage + start, SALU) and the per-lane
// offset the fixed lane * 16, and the LDS destination goes to M0 in the same statement, so a run
// costs two readlanes (its start, and its image offset and length packed as pre | n16 << 16 by the
// caller, one u32 per lane) and one tail compare per 64-unit column — against ≈ 9 VALU with the
// compiler's 64-bit per-lane addresses.  The compiler does not count these loads: the caller waits
// `vmcnt(0)` itself before the barrier that publishes the part (bin_dma_wait).
template <typename VT = double>
__device__ __forceinline__ void bin_dma_runs_asm(uint32_t so_l, uint32_t pk_l, uint32_t r0, uint32_t r1,
                                                 const VT* __restrict__ src, VT* dst, uint32_t base) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lane = threadIdx.x & 63, voff = lane * 16u;
    const uint32_t lb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)dst;
    for (uint32_t k = r0; k < r1; ++k) {
        const uint32_t so = __builtin_amdgcn_readlane(so_l, k), pq = __builtin_amdgcn_readlane(pk_l, k);
        const uint32_t pre = pq & 0xFFFFu, n16 = pq >> 16;
        // the start's low bits carry the run's pad count (round_binned.hip tiles): mask them off
        const uint64_t sb = (uint64_t)(uintptr_t)src + (uint64_t)(so & ~(16u / sizeof(VT) - 1u)) * sizeof(VT);
        const uint32_t m0 = lb + (pre - base) * (uint32_t)sizeof(VT);
        for (uint32_t o = 0; o < n16; o += 64)
            if (lane < n16 - o) bin_lds_dma16(voff, sb + o * 16u, m0 + o * 16u);
    }
#endif
}
// bin_dma_runs with asm copies (kPolAsmDmaT): descriptors fetched one per lane, 64 at a time, as
// there; each run's stage address in an SGPR pair and its LDS destination in M0 (bin_dma_runs_asm).
// The caller waits with bin_dma_wait before the barrier that publishes the image.
template <typename VT = double>
__device__ __forceinline__ void bin_dma_runs_asm_tb(const uint2* __restrict__ tb, uint32_t r0, uint32_t r1,
                                                    const VT* __restrict__ src, VT* dst, uint32_t base = 0) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr uint32_t EPU = 16 / sizeof(VT);
    const uint32_t lane = threadIdx.x & 63, voff = lane * 16u;
    const uint32_t lb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)dst;
    for (uint32_t g = r0; g < r1; g += 64) {
        const uint32_t ng = r1 - g < 64 ? r1 - g : 64;
        uint2 dsc = make_uint2(0u, 0u);
        uint32_t nxt = 0;
        if (lane < ng) {
            dsc = tb[g + lane];
            nxt = tb[g + lane + 1].y;
        }
        // the descriptors' wait, here: left to the compiler it sits in the run loop's header, where
        // (blind to the asm copies) it waits for every copy issued so far, once per run
        asm volatile("" : "+v"(dsc.x), "+v"(dsc.y), "+v"(nxt));
        for (uint32_t k = 0; k < ng; ++k) {
            const uint32_t so = __builtin_amdgcn_readlane(dsc.x, k) & ~(EPU - 1u);   // low bits: pad count
            const uint32_t pre = __builtin_amdgcn_readlane(dsc.y, k);
            const uint32_t n16 = (__builtin_amdgcn_readlane(nxt, k) - pre) / EPU;
            const uint64_t sb = (uint64_t)(uintptr_t)src + (uint64_t)so * sizeof(VT);
            const uint32_t m0 = lb + (pre - base) * (uint32_t)sizeof(VT);
            for (uint32_t o = 0; o < n16; o += 64)
                if (lane < n16 - o) bin_lds_dma16(voff, sb + o * 16u, m0 + o * 16u);
        }
    }
#endif
}
__device__ __forceinline__ void bin_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// diagnostic (ACSIM_BIN_TS): workgroup entry, end of its staging wait, end, in 100 MHz ticks
__device__ __forceinline__ void bin_ts(uint64_t* ts, uint64_t t0, uint64_t t1) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t t2 = __builtin_amdgcn_s_memrealtime();
        ts[3 * blockIdx.x] = t0;
        ts[3 * blockIdx.x + 1] = t1;
        ts[3 * blockIdx.x + 2] = t2;
    }
}

// NP-pass phase B (NP > 1, ACSIM_BIN_SPLIT=NP): block b's image is copied in NP parts (runs
// [k*nrun/NP, (k+1)*nrun/NP)) through an LDS buffer of kBinPartCap<D, NP> elements; after each
// part's DMA every lane picks up the values whose invpos falls in that part.  1/NP of the LDS per
// workgroup: more resident workgroups per CU.  The plan enables it only when every part fits.
template <int D, int NP, int SB = (int)kBinSB>
constexpr uint32_t kBinPartCap = D * SB / NP + D * SB / 16;   // + 1/16 of the image: run-length variation and padding

}  // namespace acs
