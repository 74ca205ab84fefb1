// round_persist.hip — the cfg4 round (SURVEY §8(a) a5+a7+a8+a9, §8(d) headline) as ONE persistent
// launch over k rounds: the binned exchange of round_binned.hip with its two kernels per round
// replaced by concurrent roles inside one grid.
//
// Why: each round of the two-kernel exchange pays ≈14 µs that moves no bytes — the dispatch ramp
// and tail of both kernels, phase A's imbalance tail, two kernel boundaries and the write-back of
// the L2 lines the stage stores leave dirty.  Here nothing separates the
// phases: receiver blocks are gathered as soon as every source block's stream has passed them,
// and a source block's next round starts as soon as the receiver blocks of its own rows are done.
//
// Grid: one 1024-thread workgroup per CU (cooperative launch: all resident, so every wait below
// is on a workgroup that runs).
//   A-workers  w < NA = P·S: source block a = w % P, segment s = w / P (receiver blocks
//              [s·Qs, (s+1)·Qs), a contiguous range of a's stream).  Per round: wait until the
//              receiver blocks of a's rows finished the previous round, stage x^r of the block in
//              LDS (LDS-DMA), stream stage[r&1][p] = lds[idxA[p]] with write-through (sc1) stores,
//              publishing the stream position every super-step.
//   B-workers  four 256-thread sub-groups each (one lane per receiver, 36 KiB of LDS each, as the
//              4-workgroups-per-CU phase B of round_binned.hip): receiver blocks in segment-
//              interleaved order; a block waits until every source block's stream passed its
//              tile, copies its runs by sc1 LDS-DMA in NP parts, runs the §A.7 rule in registers,
//              stores x^{r+1} write-through, and counts itself done; the last block of a round
//              folds the block partials (§A.8) and records the verdict.
// Hand-offs follow the MI355X guide's write-through form (cdna_hip_programming.md Guideline 16,
// MI355X_MICROARCH.md visibility table row 1): every handed-off byte is stored sc1 and drained by
// every storing wave (s_waitcnt vmcnt) before the signal, every signal is an agent-scope atomic,
// and every load of handed-off bytes is an sc1 load (stage runs and x blocks by sc1 LDS-DMA, x_i,
// partials and control words by sc1 loads).  Every wait is bounded (ctl abort word + watchdog).
#include <mutex>
#include <vector>

#include "binned_dev.hpp"

namespace acs {

namespace {

constexpr uint32_t kPT = 1024;           // threads per workgroup (16 waves, one workgroup per CU)
constexpr uint32_t kPW = kPT / 64;       // waves
constexpr uint32_t kAPos = 512 * kPW;    // stream positions per super-step (each wave 512)
constexpr uint32_t kNch = kPersistNch;   // readiness chunks per segment (receiver-block ranges)

// ctl layout: [0, S*kNch) streams done per (segment, chunk) — every source block's A-worker adds 1
// when its stream has written and drained a chunk's tiles; then [P) receiver blocks done per
// source block, blocks done, folds done, abort.  One word per wait: B-workers poll the chunk word
// of their block (polling a progress word per source block — 64 sc1 loads per block and poll —
// cost more fabric bandwidth than the round itself moved).
struct Ctl {
    uint64_t* chunk;
    uint64_t* cntb;
    uint64_t* cntr;
    uint64_t* vcnt;
    uint64_t* abort;
};
__device__ __forceinline__ Ctl ctl_of(const PersistArgs& a) {
    Ctl c;
    c.chunk = a.ctl;
    c.cntb = a.ctl + (uint64_t)a.S * kNch;
    c.cntr = c.cntb + a.P;
    c.vcnt = c.cntr + 1;
    c.abort = c.cntr + 2;
    return c;
}
// receiver blocks per chunk of a segment of Qs blocks
__device__ __forceinline__ uint32_t chunk_blocks(uint32_t Qs) { return (Qs + kNch - 1) / kNch; }

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), (uint64_t)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double((long long)ld_sc1(reinterpret_cast<const uint64_t*>(p)));
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// A waiting lane gives up when anyone has aborted or this wait outlived the watchdog (it then
// raises the abort word, so every other wait ends too and the grid drains).
__device__ __forceinline__ bool give_up(const Ctl& c, uint64_t t0, uint64_t tmo) {
    if (ld_sc1(c.abort)) return true;
    if (now_ticks() - t0 > tmo) {
        st_sc1(c.abort, 1ull);
        return true;
    }
    return false;
}

// verdict of the previous round known and not final (B-workers, before writing x^{r+1})
__device__ __forceinline__ bool instance_done(const InstState* st) {
    return ld_sc1(&st->done) != 0;
}

// ------------------------------------------------------------------------------ A-worker
// Stream [p0, p1) of idxA into `out` (write-through), 16 waves.  A wave records in lprog[w] how
// many super-steps of its slices are drained; wave 0 turns the minimum over the waves into a stream
// position and, for every chunk whose tiles end at or below it (lane q of wave 0 holds chunk q's
// end position cend, nch chunks), adds 1 to that chunk's counter.
__device__ void persist_stream(const double* lx, const uint16_t* __restrict__ idx, double* __restrict__ out,
                               uint64_t p0, uint64_t p1, uint64_t* chunkc, uint64_t cend, uint32_t nch,
                               volatile uint32_t* lprog, uint32_t diag) {
    constexpr uint32_t SUPW = kAPos / 2;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t nsup = (p1 - p0) / kAPos;
    const uint32_t* ip = reinterpret_cast<const uint32_t*>(idx + p0) + w * 256 + lane;
    const uint64_t bytes = (p1 - p0) * sizeof(double);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(out + p0, 0, (int)(bytes < 0x7FFFFFF0ull ? bytes : 0x7FFFFFF0ull), 0x00020000);
    const uint32_t ob = (w * 256 + lane) * 16u;
    uint32_t pub = 0, pubc = 0;   // super-steps / chunks published (wave 0)
    // wave 0: publish the chunks whose tiles end at or below position pos
    auto publish = [&](uint64_t pos) {
        const uint32_t n = (uint32_t)__builtin_popcountll(__ballot(lane < nch && cend <= pos));
        if (n > pubc) {
            if (lane >= pubc && lane < n)
                __hip_atomic_fetch_add(chunkc + lane, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pubc = n;
        }
    };
    if (w == 0) publish(p0);   // chunks with no tiles in this stream
    uint32_t c[4];
    if (nsup) {
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = __builtin_nontemporal_load(ip + q * 64);
    }
#pragma unroll 1
    for (uint64_t bi = 0; bi < nsup; ++bi) {
        const uint64_t bn = bi + 1 < nsup ? bi + 1 : bi;
        uint32_t cn[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) cn[q] = __builtin_nontemporal_load(ip + bn * SUPW + q * 64);
        // Issue order per super-step j: index loads of j + 1, then the stores of j.  Leaving the 12
        // youngest operations (loads of bi and bi + 1, stores of bi - 1) in flight completes the
        // stores of super-steps < bi - 1: the same wait the gathers of bi need anyway for their
        // index loads, so up to two super-steps of stores stay in flight.  (Waiting for the stores
        // of bi - 1 here — one super-step in flight — halved the stream: 170 µs per half block.)
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        lprog[w] = bi ? (uint32_t)bi - 1u : 0u;
        if (w == 0) {
            uint32_t m = lane < kPW ? lprog[lane] : 0xFFFFFFFFu;
#pragma unroll
            for (int o = 8; o >= 1; o >>= 1) {
                const uint32_t t = __shfl_xor(m, o, 64);
                m = t < m ? t : m;
            }
            m = __builtin_amdgcn_readfirstlane(m);
            if (m > pub) {
                pub = m;
                publish(p0 + (uint64_t)m * kAPos);
            }
        }
        if (diag & 1) {   // timing diagnostic only: nontemporal stores carry no publication guarantee
            double2* op = reinterpret_cast<double2*>(out + p0) + w * 256 + lane;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                bin_store(op + bi * SUPW + q * 64, make_double2(lx[c[q] & 0xFFFFu], lx[c[q] >> 16]), true);
        } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
                bin_store_sc1(rs, ob + (uint32_t)((bi * SUPW + q * 64) * 16),
                              make_double2(lx[c[q] & 0xFFFFu], lx[c[q] >> 16]));
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) c[q] = cn[q];
    }
    for (uint64_t q = p0 + nsup * kAPos + threadIdx.x; q < p1; q += kPT) st_sc1(out + q, lx[idx[q]]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w == 0) publish(p1);
}

__device__ void persist_a(const PersistArgs& a, unsigned char* smem) {
    double* lx = reinterpret_cast<double*>(smem);
    volatile uint32_t* lprog = reinterpret_cast<volatile uint32_t*>(smem + (size_t)a.SA * sizeof(double));
    volatile uint32_t* lstop = lprog + kPW;
    const Ctl c = ctl_of(a);
    const uint32_t w = blockIdx.x;
    const uint32_t src = w % a.P, seg = w / a.P;
    const uint64_t p0 = a.aseg[src * a.S + seg], p1 = a.aseg[src * a.S + seg + 1];
    const uint64_t base = (uint64_t)src * a.SA;
    const uint32_t n = (uint32_t)(a.N - base < a.SA ? a.N - base : a.SA);
    const uint32_t nbA = (uint32_t)((base + n + kBinSB - 1) / kBinSB - base / kBinSB);   // receiver blocks of a's rows
    // chunk q of this segment: receiver blocks [b0 + q*QC, b0 + (q+1)*QC); lane q of wave 0 holds the
    // stream position where the chunk's tiles end (the start of the next block's tile of source src)
    const uint32_t Qs = (a.Q + a.S - 1) / a.S, QC = chunk_blocks(Qs);
    const uint32_t b0 = seg * Qs, b1 = b0 + Qs < a.Q ? b0 + Qs : a.Q;
    const uint32_t nch = b1 > b0 ? (b1 - b0 + QC - 1) / QC : 0;
    uint64_t cend = p1;
    {
        const uint32_t q = threadIdx.x & 63, e = b0 + (q + 1) * QC;
        if (threadIdx.x < 64 && q < nch && e < b1) cend = a.tiles[(uint64_t)e * (a.P + 1) + src].x & ~1u;
    }
    uint64_t* chunkc = c.chunk + (uint64_t)seg * kNch;
    for (uint32_t rr = 0; rr < a.k; ++rr) {
        const uint32_t r = a.r0 + rr;
        uint64_t* tsa = a.ts ? a.ts + ((uint64_t)rr * a.NA + w) * 3 : nullptr;
        if (tsa && threadIdx.x == 0) tsa[0] = now_ticks();
        if (threadIdx.x < kPW) lprog[threadIdx.x] = 0;
        if (threadIdx.x == 0) {
            uint32_t stop = 0;
            if (rr) {   // x^r of this source block: its receiver blocks finished round r - 1
                const uint64_t need = (uint64_t)nbA * rr, t0 = now_ticks();
                while (ld_sc1(c.cntb + src) < need) {
                    if (instance_done(a.st) || give_up(c, t0, a.tmo)) {
                        stop = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            *lstop = stop;
        }
        __syncthreads();
        if (*lstop) return;
        {   // x^r block -> LDS by write-through-coherent (sc1) LDS-DMA, 16 B per lane
            const uint32_t n16 = (n + 1) / 2;
            const uint4* xs = reinterpret_cast<const uint4*>(a.x[r & 1] + base) + threadIdx.x;
            uint4* ld = reinterpret_cast<uint4*>(lx) + (threadIdx.x & ~63u);
            for (uint32_t o = 0; o < n16; o += kPT)
                if (o + threadIdx.x < n16) __builtin_amdgcn_global_load_lds(xs + o, ld + o, 16, 0, 16);
        }
        __syncthreads();
        if (tsa && threadIdx.x == 0) tsa[1] = now_ticks();
        persist_stream(lx, a.idxA, a.stage[r & 1], p0, p1, chunkc, cend, nch, lprog, a.diag);
        if (tsa && threadIdx.x == 0) tsa[2] = now_ticks();
    }
}

// ------------------------------------------------------------------------------ B-worker
// Barrier of one 4-wave sub-group (s_barrier is workgroup-wide): every wave drains its memory
// operations (LDS-DMA included), arrives on an LDS counter, and waits for the 4 arrivals of this
// epoch.
__device__ __forceinline__ void sg_sync(uint32_t* cnt, uint32_t& epoch) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    ++epoch;
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t target = 4 * epoch;
    while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
}

constexpr uint32_t kSubBytes = 36864;                  // one sub-group's LDS part buffer (kBinPartCap<32, 2>)
constexpr uint32_t kSubCtl = 4 * kSubBytes;            // sub-group control words after the 4 buffers
constexpr uint32_t kSubCtlStride = 32;                 // u32 words of control per sub-group (128 B)
constexpr uint32_t kPersistLds = kSubCtl + 4 * kSubCtlStride * 4;   // B-worker LDS; the A-worker needs SA*8 + 128

// One receiver block b of round rr.  Returns false when the worker must stop (the run ended, or
// the watchdog fired).
template <int D, int T, bool WMSR, int NP>
__device__ bool persist_block(const PersistArgs& a, const Ctl& c, unsigned char* smem, uint32_t& epoch, uint32_t b,
                              uint32_t rr) {
    const uint32_t r = a.r0 + rr;
    // the thread id re-read opaquely per block: otherwise every lane-dependent address of the body
    // is hoisted out of the worker's loops and held live across them (spills)
    uint32_t tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const uint32_t tl = tid & 255, wv = tl >> 6, lane = tid & 63;
    const uint32_t g = __builtin_amdgcn_readfirstlane(tid >> 8);   // sub-group (wave-uniform)
    double* raw = reinterpret_cast<double*>(smem + g * kSubBytes);
    uint32_t* sbar = reinterpret_cast<uint32_t*>(smem + kSubCtl) + g * kSubCtlStride;
    volatile uint32_t* sflag = sbar + 1;
    double2* red = reinterpret_cast<double2*>(sbar + 4);
    const uint32_t P = a.P;
    const uint32_t Qs = (a.Q + a.S - 1) / a.S;
    const uint32_t seg = b / Qs;
    const uint2* tb = a.tiles + (uint64_t)b * (P + 1);
    uint2 pdsc = make_uint2(0u, 0u);
    uint32_t pnxt = 0;
    if (lane < P) {
        pdsc = tb[lane];
        pnxt = tb[lane + 1].y;
    }
    uint64_t* tsb = a.ts ? a.ts + (uint64_t)a.k * a.NA * 3 + ((uint64_t)rr * a.Q + b) * 5 : nullptr;
    if (tsb && tl == 0) tsb[0] = now_ticks();
    // wave 0 waits for the previous round's verdict and for every source block's stream to pass
    // this block's tile; the sub-group learns the outcome through sflag
    if (wv == 0) {
        uint32_t go = 1;
        const uint64_t t0 = now_ticks();
        if (rr) {
            while (ld_sc1(c.vcnt) < rr) {
                if (give_up(c, t0, a.tmo)) {
                    go = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            if (go && instance_done(a.st)) go = 0;
        }
        if (go) {   // every source block's stream has drained this block's chunk
            const uint64_t need = (uint64_t)P * (rr + 1);
            const uint64_t* cw = c.chunk + (uint64_t)seg * kNch + (b - seg * Qs) / chunk_blocks(Qs);
            while (__builtin_amdgcn_readfirstlane((uint32_t)(ld_sc1(cw) >= need)) == 0u) {
                if (give_up(c, t0, a.tmo)) {
                    go = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
        }
        if (lane == 0) *sflag = go;
    }
    sg_sync(sbar, epoch);
    if (!*sflag) return false;
    if (tsb && tl == 0) tsb[1] = now_ticks();

    const uint32_t nrun = P;
    const uint64_t li = (uint64_t)b * kBinSB + tl;   // receiver
    const bool live = li < a.N;
    // part 0's runs first (sc1 LDS-DMA), then the ordinary loads
    const uint32_t j1p = nrun / NP;
    {
        const uint32_t r0 = wv * j1p / 4, r1 = (wv + 1) * j1p / 4;
        const uint4* s16 = reinterpret_cast<const uint4*>(a.stage[r & 1]);
        uint4* d16 = reinterpret_cast<uint4*>(raw);
        for (uint32_t k = r0; k < r1; ++k) {
            const uint32_t so = __builtin_amdgcn_readlane(pdsc.x, k) & ~1u;
            const uint32_t pre = __builtin_amdgcn_readlane(pdsc.y, k);
            const uint32_t n16 = (__builtin_amdgcn_readlane(pnxt, k) - pre) / 2;
            const uint4* sp = s16 + so / 2 + lane;
            uint4* dp = d16 + pre / 2;
            for (uint32_t o = 0; o < n16; o += 64)
                if (o + lane < n16) {
                    if (a.diag & 2) __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 0);
                    else __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 16);
                }
        }
    }
    const double xi = live ? ld_sc1(a.x[r & 1] + li) : 0.0;
    uint4 ip[D / 8];
    {
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const u32x4* ipn = reinterpret_cast<const u32x4*>(a.invpos) + (uint64_t)b * (D / 8) * kBinSB + tl;
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            const u32x4 t4 = __builtin_nontemporal_load(ipn + q * kBinSB);
            ip[q] = make_uint4(t4.x, t4.y, t4.z, t4.w);
        }
    }
    double v[D + 1];
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NP; ++k) {
        const uint32_t j0 = k * nrun / NP, j1 = (k + 1) * nrun / NP;
        const uint32_t lo = __builtin_amdgcn_readlane(pdsc.y, j0);
        const uint32_t hi = j1 < nrun ? __builtin_amdgcn_readlane(pdsc.y, j1) : __builtin_amdgcn_readlane(pnxt, nrun - 1);
        if (k) {
            sg_sync(sbar, epoch);   // every lane has read the previous part
            const uint32_t r0 = j0 + wv * (j1 - j0) / 4, r1 = j0 + (wv + 1) * (j1 - j0) / 4;
            const uint4* s16 = reinterpret_cast<const uint4*>(a.stage[r & 1]);
            uint4* d16 = reinterpret_cast<uint4*>(raw);
            for (uint32_t q = r0; q < r1; ++q) {
                const uint32_t so = __builtin_amdgcn_readlane(pdsc.x, q) & ~1u;
                const uint32_t pre = __builtin_amdgcn_readlane(pdsc.y, q);
                const uint32_t n16 = (__builtin_amdgcn_readlane(pnxt, q) - pre) / 2;
                const uint4* sp = s16 + so / 2 + lane;
                uint4* dp = d16 + (pre - lo) / 2;
                for (uint32_t o = 0; o < n16; o += 64)
                    if (o + lane < n16) {
                    if (a.diag & 2) __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 0);
                    else __builtin_amdgcn_global_load_lds(sp + o, dp + o, 16, 0, 16);
                }
            }
        }
        sg_sync(sbar, epoch);   // this part's runs are in LDS
        if (tsb && tl == 0) tsb[k == 0 ? 2 : 3] = now_ticks();
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            const uint32_t wd[4] = {ip[q].x, ip[q].y, ip[q].z, ip[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const uint32_t q0 = wd[e] & 0xFFFFu, q1 = wd[e] >> 16;
                if constexpr (NP == 1) {
                    v[1 + 8 * q + 2 * e] = raw[q0];
                    v[2 + 8 * q + 2 * e] = raw[q1];
                } else {
                    const bool in0 = (k == 0 || q0 >= lo) && (k + 1 == (uint32_t)NP || q0 < hi);
                    const bool in1 = (k == 0 || q1 >= lo) && (k + 1 == (uint32_t)NP || q1 < hi);
                    // exec-masked reads straight into v (the branch-free clamped read + select of
                    // round_binned.hip holds old and new values together here: 128+ VGPRs, spills)
                    if (in0) v[1 + 8 * q + 2 * e] = raw[q0 - lo];
                    if (in1) v[2 + 8 * q + 2 * e] = raw[q1 - lo];
                }
            }
        }
    }
    double mn = kInf, mx = -kInf, res = 0.0;
    if (live) {
        v[0] = xi;
        res = apply_rule_reg<D, T, WMSR>(a.rule, v);
        mn = res;
        mx = res;
    }
    // x^{r+1} write-through, two receivers per 16-byte store (even lanes)
    {
        const double nb = __shfl_down(res, 1, 64);
        double* xo = a.x[(r + 1) & 1];
        if (live && (lane & 1) == 0) {
            if (li + 1 < a.N) {
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(xo + (uint64_t)b * kBinSB, 0,
                                                                                    kBinSB * 8, 0x00020000);
                bin_store_sc1(rs, tl * 8u, make_double2(res, nb));
            } else {
                st_sc1(xo + li, res);
            }
        }
    }
    // block (min, max) partial: waves -> LDS -> wave 0; the barrier also drains every wave's x stores
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) red[wv] = make_double2(mn, mx);
    sg_sync(sbar, epoch);
    if (tsb && tl == 0) tsb[4] = now_ticks();
    if (wv == 0) {
        uint32_t last = 0;
        if (lane == 0) {
            double p = red[0].x, q = red[0].y;
#pragma unroll
            for (int k = 1; k < 4; ++k) {
                p = __builtin_fmin(p, red[k].x);
                q = __builtin_fmax(q, red[k].y);
            }
            store_partial_sc1(a.partial[r & 1] + b, make_double2(p, q));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the partial, before the signals
            __hip_atomic_fetch_add(c.cntb + (uint32_t)(((uint64_t)b * kBinSB) / a.SA), 1ull, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t old = __hip_atomic_fetch_add(c.cntr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = old + 1 == (uint64_t)a.Q * (rr + 1) ? 1u : 0u;
        }
        last = __builtin_amdgcn_readfirstlane(last);
        if (last) {   // §A.8 fold of round r by this wave: partials -> lo, hi, spread, verdict, trace
            const double2* pp = a.partial[r & 1];
            double fmn = kInf, fmx = -kInf;
            uint32_t k = lane;
            for (; k + 7 * 64 < a.Q; k += 8 * 64) {
                double2 t[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) t[u] = load_partial<true>(pp + k + u * 64);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    fmn = __builtin_fmin(fmn, t[u].x);
                    fmx = __builtin_fmax(fmx, t[u].y);
                }
            }
            for (; k < a.Q; k += 64) {
                const double2 t = load_partial<true>(pp + k);
                fmn = __builtin_fmin(fmn, t.x);
                fmx = __builtin_fmax(fmx, t.y);
            }
            fmn = wave_min(fmn);
            fmx = wave_max(fmx);
            const double spread = fmx - fmn;
            const bool conv = spread <= a.eps;
            const uint32_t r_next = r + 1;
            const bool done = (a.term_eps && conv) || r_next >= a.max_rounds;
            if (lane == 0) {
                InstState* S = a.st;
                st_sc1(&S->lo, fmn);
                st_sc1(&S->hi, fmx);
                st_sc1(&S->spread, spread);
                st_sc1(&S->rounds, r_next);
                st_sc1(&S->converged, conv ? 1u : 0u);
                st_sc1(&S->done, done ? 1u : 0u);
                if (a.trace) st_sc1(a.trace + r_next, spread);
                if (done) __hip_atomic_fetch_add(a.n_done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_fetch_add(c.vcnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    return true;
}

template <int D, int T, bool WMSR, int NP>
__device__ void persist_b(const PersistArgs& a, unsigned char* smem) {
    const uint32_t g = threadIdx.x >> 8;                       // sub-group
    // per sub-group control words: [0] barrier count, [1] go flag, [4..19] the 4 waves' (min, max)
    static_assert(4 + 4 * 4 <= kSubCtlStride, "a sub-group's control words");
    if ((threadIdx.x & 255) == 0) reinterpret_cast<uint32_t*>(smem + kSubCtl)[g * kSubCtlStride] = 0;
    __syncthreads();
    uint32_t epoch = 0;
    const Ctl c = ctl_of(a);
    const uint32_t wb = blockIdx.x - a.NA;
    const uint32_t NG = 4 * a.NB, gg = g * a.NB + wb;
    const uint32_t Qs = (a.Q + a.S - 1) / a.S;
    const uint32_t nlist = Qs * a.S;
    for (uint32_t rr = 0; rr < a.k; ++rr) {
        for (uint32_t j = gg; j < nlist; j += NG) {
            const uint32_t b = (j % a.S) * Qs + j / a.S;   // segment-interleaved: every stream's front
            if (b >= a.Q) continue;
            if (!persist_block<D, T, WMSR, NP>(a, c, smem, epoch, b, rr)) return;
        }
    }
}

template <int D, int T, bool WMSR, int NP>
__global__ __launch_bounds__(kPT, 1) void k_bin_persist(const PersistArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char psmem[];
    if (blockIdx.x < a.NA)
        persist_a(a, psmem);
    else
        persist_b<D, T, WMSR, NP>(a, psmem);
}

}  // namespace

// ------------------------------------------------------------------------------ host side
void persist_free(PersistPlan& pp) {
    (void)hipFree(pp.ts);
    (void)hipFree(pp.aseg);
    (void)hipFree(pp.stage2);
    (void)hipFree(pp.partial2);
    (void)hipFree(pp.ctl);
    pp = PersistPlan{};
}

// (d, t, phase-B passes).  Not here, and so on the two-kernel round: d = 32 with t = 0 and W-MSR
// at d = 32 (full 33-value sorts: 160 VGPRs in round_binned.hip, above the 128 a 16-wave
// workgroup allows, measured as 100-270 B/lane of scratch here).
#define ACS_PERSIST_VARIANTS(X) X(32, 5, 2) X(16, 5, 1) X(16, 0, 1)

static bool persist_variant(uint32_t d, uint32_t t, uint32_t rule) {
    if (d == 32 && rule == 4) return false;
#define X(DD, TT, NPP) if (d == DD && t == TT) return true;
    ACS_PERSIST_VARIANTS(X)
#undef X
    return false;
}

hipError_t persist_build(PersistPlan& pp, const BinnedPlan& p, uint64_t N, uint32_t d, uint32_t trim, uint32_t rule,
                         hipStream_t s) {
    pp = PersistPlan{};
    if (p.f32 || p.levels != 1 || p.var || p.ofree || p.SA != 16384 || !persist_variant(d, trim, rule))
        return hipErrorNotSupported;
    const uint32_t NP = d == 32 ? 2u : 1u;
    if (p.split != NP && !(NP == 1 && p.split == 1)) return hipErrorNotSupported;
    if (p.P > 64 || p.P == 0) return hipErrorNotSupported;   // descriptors: one per lane
    int dev = 0, ncu = 0, coop = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev);
    if (e != hipSuccess) return e;
    if (!coop) return hipErrorNotSupported;
    // segments per source block: about half of the CUs stream phase A (its bytes ≈ phase B's)
    uint32_t S = (uint32_t)((ncu / 2) / p.P);
    if (const char* v = getenv("ACSIM_PERSIST_S")) S = (uint32_t)strtoul(v, nullptr, 10);
    if (S == 0 || p.P * S >= (uint32_t)ncu || S > p.Q) return hipErrorNotSupported;
    pp.S = S;
    pp.NA = p.P * S;
    pp.NB = (uint32_t)ncu - pp.NA;
    pp.NP = NP;
    // stream starts of (a, s): tile (a, s*Qs) of the one-level A order (key a*Q + b)
    std::vector<uint2> h(((uint64_t)p.nrun + 1) * p.Q);
    e = hipMemcpy(h.data(), p.tiles, h.size() * sizeof(uint2), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    const uint32_t Qs = (p.Q + S - 1) / S;
    std::vector<uint64_t> as((uint64_t)p.P * S + 1);
    for (uint32_t a = 0; a < p.P; ++a)
        for (uint32_t sg = 0; sg < S; ++sg) {
            const uint32_t b = sg * Qs;
            as[(uint64_t)a * S + sg] = b < p.Q ? (uint64_t)(h[(uint64_t)b * (p.nrun + 1) + a].x & ~1u)
                                     : (a + 1 < p.P ? (uint64_t)(h[a + 1].x & ~1u) : p.Ep1);
        }
    as[(uint64_t)p.P * S] = p.Ep1;
    for (uint64_t k = 0; k + 1 < as.size(); ++k)
        if (as[k] > as[k + 1] || (as[k] & 1)) return hipErrorNotSupported;   // A order, even starts
    pp.nctl = (uint32_t)((persist_ctl_abort(pp, p.P) + 1 + 1) & ~1ull);   // through the abort word, even
    e = hipMalloc(&pp.aseg, as.size() * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMemcpy(pp.aseg, as.data(), as.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&pp.stage2, p.Ep1 * sizeof(double));
    if (e == hipSuccess) e = hipMalloc(&pp.partial2, (uint64_t)p.Q * sizeof(double2));
    if (e == hipSuccess) e = hipMalloc(&pp.ctl, (uint64_t)pp.nctl * sizeof(uint64_t));
    double tmo_s = 2.0;   // per wait: far above any round (≈ 0.1 ms), far below the job limits
    if (const char* v = getenv("ACSIM_PERSIST_TMO")) tmo_s = strtod(v, nullptr);
    pp.tmo = (uint64_t)(tmo_s * 1e8);
    if (e == hipSuccess) {
        static std::once_flag once[64];
        static hipError_t st[64];
        if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
        std::call_once(once[dev], [dev] {
            hipError_t r = hipSuccess;
#define X(DD, TT, NPP)                                                                                            \
    if (r == hipSuccess)                                                                                         \
        r = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_persist<DD, TT, false, NPP>),               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, kPersistLds);                       \
    if (r == hipSuccess && DD != 32)                                                                             \
        r = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_persist<DD, TT, DD != 32, NPP>),            \
                                hipFuncAttributeMaxDynamicSharedMemorySize, kPersistLds);
            ACS_PERSIST_VARIANTS(X)
#undef X
            st[dev] = r;
        });
        e = st[dev];
    }
    if (e != hipSuccess) {
        persist_free(pp);
        return e;
    }
    (void)s;
    pp.on = true;
    return hipSuccess;
}

hipError_t launch_round_persist(const PersistPlan& pp, const BinnedPlan& p, const PersistArgs& a, uint32_t d,
                                uint32_t trim, hipStream_t s) {
    static_assert(kPersistLds >= 16384 * sizeof(double) + 128, "the A-worker's x block and progress words");
    static_assert(kBinPartCap<32, 2> * sizeof(double) <= kSubBytes && kBinPartCap<16, 1> * sizeof(double) <= kSubBytes,
                  "a sub-group's part buffer");
    if (!pp.on) return hipErrorNotSupported;
    hipError_t e = hipMemsetAsync(pp.ctl, 0, (uint64_t)pp.nctl * sizeof(uint64_t), s);
    if (e != hipSuccess) return e;
    PersistArgs aa = a;
    if (const char* dv = getenv("ACSIM_PERSIST_DIAG")) aa.diag = (uint32_t)strtoul(dv, nullptr, 0);
    const char* tsf = getenv("ACSIM_PERSIST_TS");
    const uint64_t nts = 3ull * a.k * pp.NA + 5ull * a.k * a.Q;
    if (tsf && a.k) {   // diagnostic timeline of this launch (the last launch's is left in the file)
        PersistPlan& mp = const_cast<PersistPlan&>(pp);
        if (mp.ts_k < a.k) {
            (void)hipFree(mp.ts);
            mp.ts = nullptr;
            if ((e = hipMalloc(&mp.ts, nts * sizeof(uint64_t))) != hipSuccess) return e;
            mp.ts_k = a.k;
        }
        if ((e = hipMemsetAsync(mp.ts, 0, nts * sizeof(uint64_t), s)) != hipSuccess) return e;
        aa.ts = mp.ts;
    } else {
        aa.ts = nullptr;
    }
    void* args[] = {&aa};
    const dim3 grid(pp.NA + pp.NB), block(kPT);
    const bool w = a.rule == 4;
    if (aa.ts) {   // launch, wait, dump: kind,round,index,t0,t1,t2
        hipError_t le = hipErrorNotSupported;
#define X(DD, TT, NPP)                                                                                             \
        if (d == DD && trim == TT)                                                                                 \
            le = hipLaunchCooperativeKernel(w ? reinterpret_cast<const void*>(k_bin_persist<DD, TT, DD != 32, NPP>) \
                                              : reinterpret_cast<const void*>(k_bin_persist<DD, TT, false, NPP>), \
                                            grid, block, args, kPersistLds, s);
        ACS_PERSIST_VARIANTS(X)
#undef X
        if (le != hipSuccess) return le;
        std::vector<uint64_t> h(nts);
        if ((e = hipMemcpyAsync(h.data(), aa.ts, nts * 8, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
        if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
        if (FILE* f = fopen(tsf, "w")) {
            for (uint32_t rr = 0; rr < a.k; ++rr)
                for (uint32_t q = 0; q < pp.NA; ++q) {
                    const uint64_t* t = h.data() + ((uint64_t)rr * pp.NA + q) * 3;
                    fprintf(f, "A,%u,%u,%llu,%llu,%llu\n", rr, q, (unsigned long long)t[0], (unsigned long long)t[1],
                            (unsigned long long)t[2]);
                }
            for (uint32_t rr = 0; rr < a.k; ++rr)
                for (uint32_t q = 0; q < a.Q; ++q) {
                    const uint64_t* t = h.data() + (uint64_t)a.k * pp.NA * 3 + ((uint64_t)rr * a.Q + q) * 5;
                    fprintf(f, "B,%u,%u,%llu,%llu,%llu,%llu,%llu\n", rr, q, (unsigned long long)t[0],
                            (unsigned long long)t[1], (unsigned long long)t[4], (unsigned long long)t[2],
                            (unsigned long long)t[3]);
                }
            fclose(f);
        }
        return hipSuccess;
    }
#define X(DD, TT, NPP)                                                                                             \
    if (d == DD && trim == TT)                                                                                     \
        return hipLaunchCooperativeKernel(w ? reinterpret_cast<const void*>(k_bin_persist<DD, TT, DD != 32, NPP>)   \
                                            : reinterpret_cast<const void*>(k_bin_persist<DD, TT, false, NPP>),     \
                                          grid, block, args, kPersistLds, s);
    ACS_PERSIST_VARIANTS(X)
#undef X
    (void)p;
    return hipErrorNotSupported;
}

}  // namespace acs
