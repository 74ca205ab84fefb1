// round_binned.hip — the headline round (SURVEY §8(a) a5+a7+a8+a9, cfg4) as a binned exchange.
//
// Why: the per-lane kernel (round_regular.hip) issues N·d random 8-byte gathers per round.  On
// MI355X each one moves a whole cache line from L2 (or MALL, when x outgrows one XCD's 4 MiB L2)
// into L1, so the round is bound by line traffic, not by the 400 algorithmic bytes per node
// (DESIGN.md §5).  Here every HBM access is a coalesced stream and the only random accesses
// are 8-byte LDS accesses:
//
//   phase A  k_bin_scatter   workgroup = (source block a of SA senders, segment of its deliveries)
//            x[a·SA, (a+1)·SA) -> LDS (one coalesced read), then a pure stream over the block's
//            deliveries in A order: stage[p] = lds[idxA[p]].           2 B read + 8 B write / delivery
//   phase B  k_bin_gather    workgroup = receiver block b of kBinSB receivers (one lane each)
//            its P tile runs (a, b) of stage -> LDS by LDS-DMA, then per lane: own x_i, its d
//            values at invpos (LDS), the §A.7 rule in registers (rules.hpp), one store, block
//            (min, max) partial.                                       8 B + 2 B read / delivery
//
// Only clean configs with an order-independent rule (TRIMMED / MIDPOINT / DLPSW) take this path:
// the rule depends on the multiset of received values only, so the slot a value lands in does
// not matter and the result is bit-identical to the spec (same sorted sequence, same §A.7 sum).
#include <hipcub/hipcub.hpp>

#include <vector>

#include "resolve.hpp"
#include "rules.hpp"

namespace acs {

// ------------------------------------------------------------------------------ phase A
// aoffc[a][c] (C+1 per a): A-order start of tile (a, first receiver block of chunk c); the
// launch for chunk c covers [aoffc[a][c], aoffc[a][c+1]) of every source block a.
constexpr uint32_t kBinA = 512;   // phase-A workgroup: 8 waves streaming one LDS-resident source block

__global__ __launch_bounds__(kBinA) void k_bin_scatter(const double* __restrict__ x, const uint16_t* __restrict__ idxA,
                                                     const uint64_t* __restrict__ aoffc, double* __restrict__ stage,
                                                     const InstState* __restrict__ st, uint64_t N, uint32_t SA,
                                                     uint32_t segs, uint32_t chunk, uint32_t C, uint32_t c) {
    extern __shared__ double lx[];
    if (st->done) return;
    const uint32_t a = blockIdx.x / segs, sg = blockIdx.x % segs;
    const uint64_t pa1 = aoffc[(uint64_t)a * (C + 1) + c + 1];
    const uint64_t p0 = aoffc[(uint64_t)a * (C + 1) + c] + (uint64_t)sg * chunk;
    if (p0 >= pa1) return;
    const uint64_t p1 = p0 + chunk < pa1 ? p0 + chunk : pa1;
    const uint64_t base = (uint64_t)a * SA;
    const uint32_t n = (uint32_t)(N - base < SA ? N - base : SA);
    {   // x block -> LDS by LDS-DMA, 16 B per lane (x is allocated with one spare element, so the
        // last odd element's pair never reads past the buffer)
        const uint32_t n16 = (n + 1) / 2;
        const uint4* xs = reinterpret_cast<const uint4*>(x + base) + threadIdx.x;
        uint4* ld = reinterpret_cast<uint4*>(lx) + (threadIdx.x & ~63u);
        for (uint32_t o = 0; o < n16; o += kBinA)
            if (o + threadIdx.x < n16) __builtin_amdgcn_global_load_lds(xs + o, ld + o, 16, 0, 0);
    }
    __syncthreads();

    // super-steps of 512 positions per wave: wave w takes [w*512, w*512+512); instruction q of a
    // lane covers positions q*128 + 2*lane, +1 (one u32 of two indices, one 16-byte store)
    constexpr uint32_t SUP = kBinA / 64 * 512, SUPW = SUP / 2;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t p = p0;
    if ((p0 & 1) == 0) {
        const uint64_t nsup = (p1 - p0) / SUP;
        const uint32_t* ip = reinterpret_cast<const uint32_t*>(idxA + p0) + w * 256 + lane;
        double2* op = reinterpret_cast<double2*>(stage + p0) + w * 256 + lane;
#pragma unroll 4
        for (uint64_t k = 0; k < nsup; ++k) {
            uint32_t c[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) c[q] = __builtin_nontemporal_load(ip + k * SUPW + q * 64);
#pragma unroll
            for (int q = 0; q < 4; ++q) op[k * SUPW + q * 64] = make_double2(lx[c[q] & 0xFFFFu], lx[c[q] >> 16]);
        }
        p = p0 + nsup * SUP;
    }
    for (uint64_t q = p + threadIdx.x; q < p1; q += kBinA) stage[q] = lx[idxA[q]];
}

// ------------------------------------------------------------------------------ phase B
// The P tile runs of block b are copied global -> LDS by LDS-DMA (global_load_lds, no VGPR
// staging, so a wave keeps all its runs in flight), concatenated in a order: run a lands at
// element pre(a, b).  Lane i_local then reads its D values at invpos[b][t][i_local].
template <int D, int T>
__global__ __launch_bounds__(kBinSB) void k_bin_gather(const RoundArgs a, const double* __restrict__ stage,
                                                       const uint16_t* __restrict__ invpos,
                                                       const uint2* __restrict__ tiles, uint32_t P, uint32_t b0,
                                                       uint32_t b1, uint32_t Qc) {
    static_assert(D % 8 == 0, "invpos is read 8 slots at a time");
    // runs are padded to even lengths; P <= D*kBinSB/16 (binned_supported's mean-run bound)
    __shared__ __attribute__((aligned(16))) double raw[D * kBinSB + D * kBinSB / 16];
    InstState* S = a.st;
    if (S->done) return;
    // XCD-aware order: consecutive receiver blocks (which share the lines at their tile-run
    // seams) run on the same XCD (dispatch is round-robin over the 8 XCDs by blockIdx)
    const uint32_t b = b0 + (blockIdx.x & 7u) * Qc + (blockIdx.x >> 3);
    if (b >= b1) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t i = (uint64_t)b * kBinSB + threadIdx.x;
    const bool live = i < a.N;
    // ordinary loads first (their wait is the barrier's vmcnt(0) anyway)
    const double xi = live ? a.xin[i] : 0.0;
    uint4 ip[D / 8];
    const uint4* ipp = reinterpret_cast<const uint4*>(invpos) + (uint64_t)b * (D / 8) * kBinSB + threadIdx.x;
#pragma unroll
    for (int q = 0; q < D / 8; ++q) ip[q] = ipp[q * kBinSB];
    // wave w copies runs [r0, r1); their descriptors are fetched once, one per lane (64 at a
    // time), and broadcast with readlane, so no run waits on a dependent scalar load
    const uint2* tb = tiles + (uint64_t)b * (P + 1);
    const uint4* src = reinterpret_cast<const uint4*>(stage);
    uint4* dst = reinterpret_cast<uint4*>(raw);
    constexpr uint32_t NW = kBinSB / 64;
    const uint32_t r0 = w * P / NW, r1 = (w + 1) * P / NW;
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
            const uint32_t n16 = (__builtin_amdgcn_readlane(nxt, k) - pre) >> 1;   // 16-byte units (padded run)
            const uint4* sp = src + (so >> 1) + lane;
            uint4* dp = dst + (pre >> 1);
            for (uint32_t o = 0; o < n16; o += 64)
                if (o + lane < n16) __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 0);
        }
    }
    __syncthreads();

    double mn = kInf, mx = -kInf;
    if (live) {
        double v[D + 1];
        v[0] = xi;
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            const uint32_t wd[4] = {ip[q].x, ip[q].y, ip[q].z, ip[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[1 + 8 * q + 2 * e] = raw[wd[e] & 0xFFFFu];
                v[2 + 8 * q + 2 * e] = raw[wd[e] >> 16];
            }
        }
        const double res = apply_rule_reg<D, T>(a.rule, v);
        a.xout[i] = res;
        mn = res;
        mx = res;
    }
    block_minmax_store<kBinSB>(mn, mx, a.partial + b);
}

// ------------------------------------------------------------------------------ plan build
__device__ __forceinline__ uint32_t ell_at(const uint32_t* ell, uint64_t i, uint32_t t, uint32_t dp) {
    return ell[(((i >> 6) * (dp >> 2) + (t >> 2)) * 64 + (i & 63)) * 4 + (t & 3)];
}

__global__ __launch_bounds__(256) void k_bin_keys(const uint32_t* __restrict__ ell, uint64_t E, uint32_t D,
                                                  uint32_t dp, uint32_t SA, uint32_t Q, uint32_t* __restrict__ keys,
                                                  uint32_t* __restrict__ vals) {
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const uint64_t i = e / D;
    const uint32_t t = (uint32_t)(e % D);
    const uint32_t j = ell_at(ell, i, t, dp);
    keys[e] = (j / SA) * Q + (uint32_t)(i / kBinSB);
    vals[e] = (uint32_t)e;
}

// tile boundaries in the sorted keys: tl[key] = (first, last+1) unpadded A-order positions
__global__ __launch_bounds__(256) void k_bin_bounds(uint64_t E, const uint32_t* __restrict__ ks, uint2* __restrict__ tl) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t key = ks[p];
    if (p == 0 || ks[p - 1] != key) tl[key].x = (uint32_t)p;
    if (p == E - 1 || ks[p + 1] != key) tl[key].y = (uint32_t)(p + 1);
}

// padded tile lengths (even, so every run starts 16-byte aligned in stage and in LDS)
__global__ __launch_bounds__(256) void k_bin_plen(const uint2* __restrict__ tl, uint64_t nt, uint32_t* __restrict__ plen) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= nt) return;
    const uint2 t = tl[k];
    plen[k] = t.y ? (t.y - t.x + 1u) & ~1u : 0u;
}

__global__ __launch_bounds__(256) void k_bin_fill(const uint32_t* __restrict__ ell, uint64_t E, uint32_t D,
                                                  uint32_t dp, uint32_t SA, const uint32_t* __restrict__ ks,
                                                  const uint32_t* __restrict__ vs, const uint2* __restrict__ tl,
                                                  const uint32_t* __restrict__ pstart, uint16_t* __restrict__ idxA) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t e = vs[p], key = ks[p];
    const uint64_t i = e / D;
    const uint32_t t = e % D;
    idxA[pstart[key] + (p - tl[key].x)] = (uint16_t)(ell_at(ell, i, t, dp) % SA);
}

// per receiver block b: tiles[b][a] = (padded A-order start, element offset of run a inside the
// block's concatenated padded runs), tiles[b][P] = (0, total)
__global__ __launch_bounds__(256) void k_bin_prefix(const uint32_t* __restrict__ pstart, const uint32_t* __restrict__ plen,
                                                    uint2* __restrict__ tiles, uint32_t P, uint32_t Q) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= Q) return;
    uint32_t pre = 0;
    for (uint32_t a = 0; a < P; ++a) {
        const uint64_t key = (uint64_t)a * Q + b;
        tiles[(uint64_t)b * (P + 1) + a] = make_uint2(pstart[key], pre);
        pre += plen[key];
    }
    tiles[(uint64_t)b * (P + 1) + P] = make_uint2(0u, pre);
}

// invpos[b][t/8][i_local][t%8] = element position of (receiver i_local, slot t) in block b's runs
__global__ __launch_bounds__(256) void k_bin_inv(uint64_t E, uint32_t D, uint32_t P, uint32_t Q,
                                                 const uint32_t* __restrict__ ks, const uint32_t* __restrict__ vs,
                                                 const uint2* __restrict__ tl, const uint2* __restrict__ tiles,
                                                 uint16_t* __restrict__ invpos) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t e = vs[p];
    const uint64_t i = e / D;
    const uint32_t t = e % D;
    const uint32_t key = ks[p], a = key / Q, b = key % Q;
    const uint32_t pos = tiles[(uint64_t)b * (P + 1) + a].y + (uint32_t)(p - tl[key].x);
    const uint32_t il = (uint32_t)(i % kBinSB);
    invpos[(((uint64_t)b * (D / 8) + t / 8) * kBinSB + il) * 8 + (t & 7)] = (uint16_t)pos;
}

// aoffc[a][c] = padded A-order start of tile (a, first receiver block of chunk c)
__global__ __launch_bounds__(256) void k_bin_aoffc(const uint32_t* __restrict__ pstart, uint32_t P, uint32_t Q,
                                                   uint32_t C, uint64_t Ep, uint64_t* __restrict__ aoffc) {
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= P * (C + 1)) return;
    const uint32_t a = k / (C + 1), c = k % (C + 1);
    const uint64_t key = (uint64_t)a * Q + (uint64_t)c * Q / C;
    aoffc[k] = key < (uint64_t)P * Q ? pstart[key] : Ep;
}

__global__ __launch_bounds__(256) void k_fill_u64(uint64_t* p, uint64_t n, uint64_t v) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < n) p[k] = v;
}

// ------------------------------------------------------------------------------ host side
#define ACS_BINNED_VARIANTS(X) X(16, 5) X(32, 5) X(16, 0) X(32, 0) X(8, 2) X(8, 0)

bool binned_supported(uint32_t d, uint32_t t, uint32_t rule) {
    if (rule != 1 && rule != 2 && rule != 3) return false;   // sort-based rules only
    if (rule == 3 && t < 1) return false;
#define X(DD, TT) if (d == DD && t == TT) return true;
    ACS_BINNED_VARIANTS(X)
#undef X
    return false;
}

void binned_free(BinnedPlan& p) {
    (void)hipFree(p.idxA);
    (void)hipFree(p.invpos);
    (void)hipFree(p.tiles);
    (void)hipFree(p.aoffc);
    (void)hipFree(p.stage);
    p = BinnedPlan{};
}

hipError_t binned_build(BinnedPlan& p, const uint32_t* ell, uint64_t N, uint32_t d, uint32_t dp, uint32_t sa,
                        uint32_t chunks, hipStream_t s) {
    hipError_t e;
    p.D = d;
    p.SA = sa;
    p.E = N * d;
    p.P = (uint32_t)((N + sa - 1) / sa);
    p.Q = (uint32_t)((N + kBinSB - 1) / kBinSB);
    p.C = chunks < 1 ? 1 : chunks > p.Q ? p.Q : chunks;
    // deliveries per phase-A workgroup (a multiple of the 4096-position super-step): about 512
    // workgroups per launch (two generations per CU measured faster than one), few x-block refills
    {
        const uint64_t per_a = ((uint64_t)sa * d + p.C - 1) / p.C;
        const uint64_t want = (512 + p.P - 1) / p.P;
        uint64_t ch = (per_a + want - 1) / want;
        ch = ch < 8192 ? 8192 : ch;
        p.chunk = (uint32_t)((ch + 4095) / 4096 * 4096);
    }
    p.segs = 1;   // set from the real per-(a, c) range lengths once aoffc is built
    const uint64_t E = p.E, nt = (uint64_t)p.P * p.Q;
    if (E >= (1ull << 31) || nt >= (1ull << 32)) return hipErrorNotSupported;
    const uint64_t Qp = (uint64_t)p.Q * kBinSB;   // receiver slots incl. the ragged last block's padding
    if ((e = hipMalloc(&p.invpos, Qp * d * 2)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(p.invpos, 0, Qp * d * 2, s)) != hipSuccess) return e;
    if ((e = hipMalloc(&p.tiles, ((uint64_t)p.P + 1) * p.Q * sizeof(uint2))) != hipSuccess) return e;
    if ((e = hipMalloc(&p.aoffc, (uint64_t)p.P * (p.C + 1) * sizeof(uint64_t))) != hipSuccess) return e;

    uint32_t *keys = nullptr, *vals = nullptr, *ks = nullptr, *vs = nullptr, *plen = nullptr, *pstart = nullptr;
    uint2* tl = nullptr;
    void* temp = nullptr;
    size_t tb = 0, tb2 = 0;
    int bits = 1;
    while (bits < 32 && (1ull << bits) < nt) ++bits;
    const unsigned grid = (unsigned)((E + 255) / 256), gridt = (unsigned)((nt + 255) / 256);
    e = hipMalloc(&keys, E * 4);
    if (e == hipSuccess) e = hipMalloc(&vals, E * 4);
    if (e == hipSuccess) e = hipMalloc(&ks, E * 4);
    if (e == hipSuccess) e = hipMalloc(&vs, E * 4);
    if (e == hipSuccess) e = hipMalloc(&tl, nt * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&plen, nt * 4);
    if (e == hipSuccess) e = hipMalloc(&pstart, nt * 4);
    if (e == hipSuccess) e = hipMemsetAsync(tl, 0, nt * sizeof(uint2), s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_keys, dim3(grid), dim3(256), 0, s, ell, E, d, dp, sa, p.Q, keys, vals);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, ks, vals, vs, (int)E, 0, bits, s);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, plen, pstart, (int)nt, s);
    if (tb2 > tb) tb = tb2;
    if (e == hipSuccess) e = hipMalloc(&temp, tb ? tb : 16);
    if (e == hipSuccess)   // LSD radix sort is stable: (a, b, then i, slot) order
        e = hipcub::DeviceRadixSort::SortPairs(temp, tb, keys, ks, vals, vs, (int)E, 0, bits, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_bounds, dim3(grid), dim3(256), 0, s, E, ks, tl);
        hipLaunchKernelGGL(k_bin_plen, dim3(gridt), dim3(256), 0, s, tl, nt, plen);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(temp, tb, plen, pstart, (int)nt, s);
    uint32_t last[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(&last[0], pstart + nt - 1, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&last[1], plen + nt - 1, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    p.Ep = (uint64_t)last[0] + last[1];
    if (e == hipSuccess) e = hipMalloc(&p.idxA, p.Ep * 2);
    if (e == hipSuccess) e = hipMemsetAsync(p.idxA, 0, p.Ep * 2, s);
    if (e == hipSuccess) e = hipMalloc(&p.stage, p.Ep * sizeof(double));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_fill, dim3(grid), dim3(256), 0, s, ell, E, d, dp, sa, ks, vs, tl, pstart, p.idxA);
        hipLaunchKernelGGL(k_bin_prefix, dim3((p.Q + 255) / 256), dim3(256), 0, s, pstart, plen, p.tiles, p.P, p.Q);
        hipLaunchKernelGGL(k_bin_inv, dim3(grid), dim3(256), 0, s, E, d, p.P, p.Q, ks, vs, tl, p.tiles, p.invpos);
        const uint32_t n = p.P * (p.C + 1);
        hipLaunchKernelGGL(k_bin_aoffc, dim3((n + 255) / 256), dim3(256), 0, s, pstart, p.P, p.Q, p.C, p.Ep, p.aoffc);
        e = hipGetLastError();
    }
    hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess) {   // every (a, c) range must be covered by segs workgroups of `chunk`
        std::vector<uint64_t> h((uint64_t)p.P * (p.C + 1));
        e = hipMemcpy(h.data(), p.aoffc, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
        uint64_t mx = 0;
        for (uint32_t a = 0; a < p.P; ++a)
            for (uint32_t c = 0; c < p.C; ++c) {
                const uint64_t len = h[(uint64_t)a * (p.C + 1) + c + 1] - h[(uint64_t)a * (p.C + 1) + c];
                if (len > mx) mx = len;
            }
        p.segs = (uint32_t)((mx + p.chunk - 1) / p.chunk);
        if (p.segs == 0) p.segs = 1;
    }
    (void)hipFree(temp);
    (void)hipFree(keys);
    (void)hipFree(vals);
    (void)hipFree(ks);
    (void)hipFree(vs);
    (void)hipFree(tl);
    (void)hipFree(plen);
    (void)hipFree(pstart);
    return e;
}

hipError_t launch_round_binned(const BinnedPlan& p, const RoundArgs& a, hipStream_t s) {
    static bool attr = false;   // source blocks above 8192 senders need more than 64 KiB of LDS
    if (!attr) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_scatter),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 16384 * sizeof(double));
        if (e != hipSuccess) return e;
        attr = true;
    }
    for (uint32_t c = 0; c < p.C; ++c) {
        hipLaunchKernelGGL(k_bin_scatter, dim3(p.P * p.segs), dim3(kBinA), p.SA * sizeof(double), s, a.xin, p.idxA,
                           p.aoffc, p.stage, a.st, a.N, p.SA, p.segs, p.chunk, p.C, c);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        const uint32_t b0 = (uint32_t)((uint64_t)c * p.Q / p.C), b1 = (uint32_t)((uint64_t)(c + 1) * p.Q / p.C);
        const uint32_t Qc = (b1 - b0 + 7) / 8;
        const dim3 grid(8 * Qc);
        bool ok = false;
#define X(DD, TT)                                                                                   \
        if (!ok && p.D == DD && a.trim == TT) {                                                     \
            hipLaunchKernelGGL((k_bin_gather<DD, TT>), grid, dim3(kBinSB), 0, s, a, p.stage, p.invpos, \
                               p.tiles, p.P, b0, b1, Qc);                                           \
            ok = true;                                                                              \
        }
        ACS_BINNED_VARIANTS(X)
#undef X
        if (!ok) return hipErrorNotSupported;
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace acs
