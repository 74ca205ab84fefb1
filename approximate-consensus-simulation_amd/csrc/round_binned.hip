// round_binned.hip — the sparse round (SURVEY §8(a) a5+a7+a8+a9: cfg4, cfg5) as a binned exchange.
//
// Why: the per-lane kernel (round_regular.hip) issues N·d random 8-byte gathers per round.  On
// MI355X each one moves a whole cache line into L1 (from L2 / MALL at cfg4, from HBM at cfg5), so
// the round is bound by line traffic, not by the algorithmic bytes per node.  Here
// every HBM access is a coalesced stream or a ≥ 1 KiB run, and the only random accesses are
// 8-byte LDS accesses.  A "delivery" is one (receiver i <- sender j, slot t) entry.
//
//   phase A  k_bin_scatter   workgroup = (source block a of SA senders, segment of its deliveries)
//            x[a·SA, (a+1)·SA) -> LDS by LDS-DMA, then a pure stream over the block's deliveries:
//            stage1[p] = lds[idxA[p]]                                  2 B read + 8 B write / delivery
//   phase M  k_bin_regroup   (two-level plans only: cfg5-sized graphs, where a (source block,
//            receiver block) tile would hold about one delivery)  workgroup = (receiver
//            super-block r, source-block chunk k): its PK runs of stage1 -> LDS by LDS-DMA, then
//            stage2[p] = lds[idxM[p]] grouped by receiver block         8 B + 2 B read + 8 B write
//   phase B  k_bin_gather    workgroup = receiver block b of kBinSB receivers (one lane each)
//            its runs of the last stage -> LDS by LDS-DMA, then per lane: own x_i, its d values at
//            invpos (LDS), the §A.7 rule in registers (rules.hpp), one store, block (min, max)
//            partial.                                                  8 B + 2 B read / delivery
//
// invpos is indexed by ELL slot t, so phase B sees receiver i's values in slot order: with the
// ELL in spec order (every config but the clean sort-based ones, whose rows are stored sorted)
// slot t is the spec slot s = i·d + t and the §A.5 drop draws, §A.4 crash draws and AVERAGE's
// entry-order sum all follow the spec exactly.
//
// Fault schedules (§A.4): phase B needs each delivered value's sender status.  Instead of a
// second exchange of status words, k_bin_tag rewrites x into xtag once per round: a sender that
// is Byzantine, crashing this round (partial) or crashed earlier (silent) is replaced by a quiet
// NaN whose payload holds that mode (x is never NaN, validated); phase A streams xtag instead of
// x, and phase B decodes the tag to the sender's §A.6 resolution.  A partial sender's message
// still delivers x_j when its per-slot draw passes, so its tag also carries j and phase B
// fetches x_j itself (n_faulty / crash_window senders per round at most).  +12 B read, +8 B
// written per node per round, against the 8·d B of random gathers the per-lane kernel spends.
#include <hipcub/hipcub.hpp>

#include <mutex>
#include <vector>

// ACS_DIAG_B (variant builds only, tools/build_variant.sh; wrong values): the clean two-pass phase B
// without 1 its selection network, 2 its position-dependent pick-up, 3 its stage DMA, 4 its invpos
// stream (in-range synthetic positions)
#ifndef ACS_DIAG_B
#define ACS_DIAG_B 0
#endif

#include "binned_dev.hpp"

namespace acs {

// ------------------------------------------------------------------------------ phase A
template <typename VT = double>
__global__ __launch_bounds__(kBinA) void k_bin_scatter(const VT* __restrict__ x, const uint16_t* __restrict__ idxA,
                                                     const uint64_t* __restrict__ aoff, VT* __restrict__ stage,
                                                     const InstState* __restrict__ st, uint64_t N, uint32_t SA,
                                                     uint32_t segs, uint32_t chunk, uint32_t pol,
                                                     const FinalizeArgs fin, uint32_t fin_on, const SrcSel sel,
                                                     uint64_t* __restrict__ ts, unsigned long long* __restrict__ ereset,
                                                     const uint32_t* __restrict__ pkA, uint4* __restrict__ nhdr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lx_raw[];
    VT* lx = reinterpret_cast<VT*>(lx_raw);
    if (st->done) return;
    // this round's phase B publishes its verdict into ereset (the pair the previous phase B filled is
    // fin.eacc, read below; the next phase A reads this one)
    if (ereset && blockIdx.x == 0 && threadIdx.x < kEaccSlots) {
        unsigned long long* e = ereset + threadIdx.x * kEaccStride;
        __hip_atomic_store(e, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(e + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint64_t t0 = ts ? __builtin_amdgcn_s_memrealtime() : 0;
    // XCD-aware order (dispatch deals blocks round-robin over the 8 XCDs): every segment of source
    // block a runs on the XCD of blockIdx % 8 = a % 8, so its x block is fetched into one L2 once
    // instead of once per XCD.  The grid is 8 * ceil(P / 8) * segs.
    const uint32_t slot = blockIdx.x >> 3;
    const uint32_t u = (slot / segs) * 8 + (blockIdx.x & 7u), sg = slot % segs;
    // selected source blocks (chunked partitioned rounds): launch-local block u -> global block a
    const uint32_t a = sel.n ? (u < sel.n ? (u / sel.bpc) * sel.bpr + sel.k0 + u % sel.bpc : 0xFFFFFFFFu) : u;
    // padding past the last source block, or a segment past its block's deliveries: idle (but
    // workgroup 0 still records a deferred finalize)
    const bool noblk = a == 0xFFFFFFFFu || (uint64_t)a * SA >= N;
    uint64_t p0 = 0, p1 = 0;
    if (!noblk) {
        const uint64_t s0 = aoff[a], s1 = aoff[a + 1];
        if (pkA) {
            // packed stream: the block's deliveries in `segs` equal parts cut at 512-position
            // boundaries (the stream's block grid), so no segment is short and no interior cut
            // needs the position-by-position head / tail decode
            auto cut = [&](uint32_t k) -> uint64_t {
                if (k == 0) return s0;
                if (k >= segs) return s1;
                const uint64_t c = (s0 + (s1 - s0) * k / segs + 256) & ~511ull;
                return c < s0 ? s0 : c > s1 ? s1 : c;
            };
            p0 = cut(sg);
            p1 = cut(sg + 1);
        } else {
            p0 = s0 + (uint64_t)sg * chunk;
            p1 = p0 + chunk < s1 ? p0 + chunk : s1;
        }
    }
    const bool idle = noblk || p0 >= p1;
    // (workgroup 0 always records the deferred finalize and, on narrow plans, the round's width)
    if (idle && !(blockIdx.x == 0 && (fin_on || nhdr))) return;
    const uint64_t base = (uint64_t)a * SA;
    const uint32_t n = idle ? 0u : (uint32_t)(N - base < SA ? N - base : SA);
    {   // x block -> LDS by LDS-DMA, 16 B per lane (x is allocated with spare elements, so the
        // last odd element's pair never reads past the buffer)
        constexpr uint32_t EPU = 16 / sizeof(VT);
        const uint32_t n16 = (n + EPU - 1) / EPU;
        const uint4* xs = reinterpret_cast<const uint4*>(x + base) + threadIdx.x;
        uint4* ld = reinterpret_cast<uint4*>(lx) + (threadIdx.x & ~63u);
        for (uint32_t o = 0; o < n16; o += kBinA)
            if (o + threadIdx.x < n16) __builtin_amdgcn_global_load_lds(xs + o, ld + o, 16, 0, 0);
    }
    // The (min, max) of x^r the previous phase B published (fin.eacc; plain loads: its atomics
    // completed before this launch began, and the kernel boundary makes them visible here as it
    // does x^r itself): the EPS verdict of workgroups other than 0, and on narrow plans (nhdr) the
    // round's stage entry width, which workgroup 0 records for phase B.  Every
    // workgroup reads the same pair, so all of them choose the same width.
    __shared__ uint32_t pub_done, nar_w;
    __shared__ unsigned long long nar_base;
    const bool pub_in = fin_on && fin.eacc;
    if (fin_on || nhdr) {
        if (threadIdx.x < 64) {
            unsigned long long lo = 0, hi = 0;
            if (pub_in && threadIdx.x < kEaccSlots) {
                lo = fin.eacc[threadIdx.x * kEaccStride];
                hi = fin.eacc[threadIdx.x * kEaccStride + 1];
            }
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const unsigned long long l2 = __shfl_xor(lo, o, 64), h2 = __shfl_xor(hi, o, 64);
                lo = l2 > lo ? l2 : lo;
                hi = h2 > hi ? h2 : hi;
            }
            if (threadIdx.x == 0) {
                const double mn = ord_inv(~lo), mx = ord_inv(hi);
                const double spread = fin.f32 ? (double)(float)(mx - mn) : mx - mn;
                pub_done = pub_in && fin.term_eps && spread <= fin.eps ? 1u : 0u;
                uint32_t w = 8;
                unsigned long long base = 0;
                if (nhdr && pub_in) narrow_choose(~lo, hi, w, base);
                nar_w = w;
                nar_base = base;
                if (nhdr && blockIdx.x == 0) *nhdr = make_uint4((uint32_t)base, (uint32_t)(base >> 32), w, 0u);
            }
        }
    }
    if (fin_on) {
        // deferred finalize of the previous round.  Only workgroup 0 folds the
        // partials and records the verdict (the loads overlap the x staging above; the fold's
        // barrier drains both).  The other workgroups take the verdict the previous phase B
        // published (fin.eacc: the same exact min / max, so the same ε test), or without one stream
        // unconditionally unless the round cap is reached: if the EPS test has just ended the run,
        // their stage is never read, because phase B (the next launch) sees the done flag
        // workgroup 0 set and exits, and every later launch exits at its first line.  A finished
        // instance stops here.  (Every writer of the partials publishes: see the invariant where
        // api.hip enqueue_round chooses `pub`.)
        bool done;
        if (blockIdx.x == 0) {
            done = fold_partials<false, kBinA>(fin, 0, true);
        } else {
            __syncthreads();
            done = pub_done != 0u || fin.r_next >= fin.max_rounds;
        }
        if (done || idle) return;
    } else {
        __syncthreads();
    }
    const uint64_t t1 = ts ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t smode = (pol & kPolSc1Store) ? 2u : (pol & kPolNtStore) ? 1u : 0u;
    if (pkA) {   // 14-bit packed indices
        if constexpr (sizeof(VT) == 8) {
            if (nhdr && nar_w == 4u) {   // narrow stage: u32 offsets from the round's base
                bin_stream_pk14_narrow(lx, pkA, reinterpret_cast<uint32_t*>(stage), p0, p1, smode, (uint32_t)nar_base);
                if (ts) bin_ts(ts, t0, t1);
                return;
            }
        }
        bin_stream_pk14(lx, pkA, stage, p0, p1, smode);
        if (ts) bin_ts(ts, t0, t1);
        return;
    }
    bin_stream(lx, idxA, stage, p0, p1, smode);
    if (ts) bin_ts(ts, t0, t1);
}

// ------------------------------------------------------------------------------ phase M
// mt[g][0..PK] (g = r*K + k): (stage1 start, image offset) of run (a = k*PK + j, r); entry PK holds
// the image size.  moff[g] .. moff[g+1]: the group's output range in stage2.
// VT = float for fp32 plans (runs padded to 4 elements, the image holds floats)
template <typename VT = double>
__global__ __launch_bounds__(kBinA) void k_bin_regroup(const VT* __restrict__ stage1, const uint2* __restrict__ mt,
                                                     const uint64_t* __restrict__ moff, const uint16_t* __restrict__ idxM,
                                                     VT* __restrict__ stage2, const InstState* __restrict__ st,
                                                     uint32_t PK, uint32_t pol, uint64_t* __restrict__ ts) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lm_raw[];
    VT* lm = reinterpret_cast<VT*>(lm_raw);
    if (st->done) return;
    const uint64_t t0 = ts ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t g = blockIdx.x;
    constexpr uint32_t NW = kBinA / 64;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (pol & kPolAsmDmaT) {
        bin_dma_runs_asm_tb(mt + (uint64_t)g * (PK + 1), w * PK / NW, (w + 1) * PK / NW, stage1, lm);
        bin_dma_wait();
    } else {
        bin_dma_runs(mt + (uint64_t)g * (PK + 1), w * PK / NW, (w + 1) * PK / NW, stage1, lm);
    }
    __syncthreads();
    const uint64_t t1 = ts ? __builtin_amdgcn_s_memrealtime() : 0;
    bin_stream(lm, idxM, stage2, moff[g], moff[g + 1], (pol & kPolSc1StoreM) ? 2u : (pol & kPolNtStoreM) ? 1u : 0u);
    if (ts) bin_ts(ts, t0, t1);
}

// ------------------------------------------------------------------------------ phase B
// The runs of block b (run j of a table row of nrun + 1 descriptors) are copied into LDS,
// concatenated; lane i_local then reads its D values at invpos[b][t][i_local].
// quiet-NaN tag of a non-normal sender: payload bits 0-1 = 1 Byzantine, 2 crashing this round,
// 3 silent; bits 2-33 = the sender id (read back for mode 2; binned plans hold one instance, N < 2^32)
constexpr uint64_t kTagBase = 0x7FF8000000000000ull;

// fp32 plans use the binary32 quiet NaN 0x7FC00000 with the same payload layout in
// its 22 payload bits: bits 0-1 mode, bits 2-21 the sender id (N <= 2^20), or above 2^20 nodes the
// sender's rank among the round's crashing senders (RoundArgs::crank / clist; only mode 2 reads it)
constexpr uint32_t kTagBase32 = 0x7FC00000u;

__device__ __forceinline__ double bin_tag_value(uint64_t j, uint64_t mode, double) {
    return __longlong_as_double((long long)(kTagBase | j << 2 | mode));
}
__device__ __forceinline__ float bin_tag_value(uint64_t j, uint64_t mode, float) {   // 20-bit id field
    return __uint_as_float(kTagBase32 | (uint32_t)((j & 0xFFFFFu) << 2 | mode));
}

template <typename VT = double>
__global__ __launch_bounds__(256) void k_bin_tag(const VT* __restrict__ x, const uint32_t* __restrict__ status,
                                                 VT* __restrict__ xt, uint64_t N, uint32_t r,
                                                 const InstState* __restrict__ st, const uint32_t* __restrict__ crank) {
    if (st->done) return;
    const uint64_t j = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 2;
    if (j >= N) return;
    const uint32_t n = N - j >= 2 ? 2u : 1u;
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
        if (k >= n) break;
        const uint32_t sj = status[j + k];
        const uint64_t mode = sj == kHonest ? 0 : sj == kByz ? 1 : r < sj ? 0 : r == sj ? 2 : 3;
        // (crank: fp32 above 2^20 nodes, the id field holds the rank among round r's crashing senders)
        const uint64_t id = crank && mode == 2 ? crank[j + k] : j + k;
        xt[j + k] = mode ? bin_tag_value(id, mode, VT(0)) : x[j + k];
    }
}

// Fault fix-up: fix[k] = (stage position, local receiver row, slot t, sender j) for
// every delivery from a sender that is not honest.  Each round it writes the §A.4 / §A.6 resolution
// of that delivery into the last stage (Byzantine value, x_j, or a quiet NaN for a missing
// message); drops are phase B's.  The stream of phase A carried plain x there.
template <typename VT = double>
__global__ __launch_bounds__(256) void k_bin_fixup(const uint4* __restrict__ fix, uint32_t nfix, const RoundArgs a,
                                                   VT* __restrict__ stage, uint32_t D) {
    const InstState* S = a.st;
    if (S->done) return;
    const uint32_t k = blockIdx.x * 256 + threadIdx.x;
    if (k >= nfix) return;
    const uint4 f = fix[k];
    const uint64_t i = a.row0 + f.y;
    const uint32_t stj = a.status[f.w];
    const uint64_t slot = a.rowptr ? a.rowptr[i] + f.z : i * D + f.z;
    const VT xj = reinterpret_cast<const VT*>(a.xin)[f.w];
    bool miss;
    const VT v = resolve_entry_m(a.mp, stj, xj, xj, false, (uint32_t)a.mp.inst_offset, a.r, (uint32_t)i, slot,
                                 (VT)S->lo, (VT)S->hi, miss);
    if constexpr (sizeof(VT) == 8)
        stage[f.x] = miss ? __longlong_as_double((long long)(kTagBase | 3u)) : v;
    else
        stage[f.x] = miss ? __uint_as_float(kTagBase32 | 3u) : v;
}


// VAR: a CSR graph padded to D (§8(f) row 1): slots t >= deg(i) are absent entries, slot numbers
// are rowptr[i] + t (one drop draw each); single pass only.
// Faulty NP > 1: the parts' LDS buffers admit 4 workgroups per CU, but the faulty bodies need more
// than the 128 VGPRs of 4 waves per SIMD (bounded to 4 they spilled 148-312 B/lane of scratch).
// The cfg4_byz shape (t = 5, not W-MSR) needs 163 with the drop mask drawn up front: 3 waves per
// SIMD (168 VGPRs), no scratch.  W-MSR and t = 0 (full 33-value sorts) need up to 203: 2.
// ACS_FAULTY_WPE overrides (variant builds).
#ifdef ACS_FAULTY_WPE
#define ACS_FAULTY_WPE_OF(T, W) ACS_FAULTY_WPE
#else
#define ACS_FAULTY_WPE_OF(T, W) ((T) == 5 && !(W) ? 3 : 2)
#endif
// FIX (fault fix-up plans): the stage already holds every faulty sender's resolved
// delivery (k_bin_fixup), a missing one as a quiet NaN; phase B draws the §A.5 drop mask, turns
// dropped and NaN entries into missing ones and applies the receiver's own status — no tag
// decoding, no Byzantine draws, clean-kernel registers.
// x^{r+1}_i, plain or write-through (kPolSc1X: no dirty x lines left in L2 at the kernel boundary)
template <int SB, typename VT>
__device__ __forceinline__ void bin_store_x(const RoundArgs& a, uint64_t i, VT res, uint32_t pol) {
    if (pol & kPolSc1X) {
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<VT*>(a.xout) + (i - threadIdx.x), 0, (int)(SB * sizeof(VT)), 0x00020000);
        if constexpr (sizeof(VT) == 8) {
            using UV = unsigned int __attribute__((ext_vector_type(2)));
            UV bits;
            __builtin_memcpy(&bits, &res, 8);
            __builtin_amdgcn_raw_buffer_store_b64(bits, rx, threadIdx.x * 8u, 0, 16);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, res), rx, threadIdx.x * 4u, 0, 16);
        }
    } else {
        reinterpret_cast<VT*>(a.xout)[i] = res;
    }
}

// The narrow header as a scalar load (constant address space: phase A wrote it before this launch
// and nothing writes it during one, so the scalar cache may serve it; as a vector load the compiler
// made every workgroup wait for it alone before its first copies)
__device__ __forceinline__ uint4 bin_nhdr_load(const uint4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __attribute__((address_space(4))) uint32_t* q = (const __attribute__((address_space(4))) uint32_t*)p;
    return make_uint4(q[0], q[1], q[2], q[3]);
#else
    return *p;
#endif
}

// NAR (narrow plans; clean fp64 only): each round reads the stage entry width
// phase A chose (a.nhdr); in a 4-byte round the whole image of u32 offsets is copied in one pass
// into the same LDS and every pick-up adds the round's base to recover the value's bits.
template <int D, int T, bool WMSR = false, bool FAULTY = false, typename VT = double, int NP = 1, bool VAR = false,
          bool FIX = false, int SB = (int)kBinSB, bool NAR = false>
__global__ __launch_bounds__(SB, FAULTY && NP > 1 ? ACS_FAULTY_WPE_OF(T, WMSR) : (FIX || NAR) && NP > 1 && (T || WMSR) ? 4 : 1) void k_bin_gather(const RoundArgs a, const VT* __restrict__ stage,
                                                       const uint16_t* __restrict__ invpos,
                                                       const uint2* __restrict__ tiles, uint32_t nrun, uint32_t Q,
                                                       uint32_t Qc, uint32_t pol) {
    static_assert(D % 8 == 0, "invpos is read 8 slots at a time");
    static_assert(!(FIX && FAULTY), "FIX replaces the tagged resolution");
    static_assert(!NAR || (sizeof(VT) == 8 && !FAULTY && !FIX && !VAR), "narrow stages: clean fp64 plans");
    constexpr bool FLT = FAULTY || FIX;   // a fault schedule or loss: receiver status and drop mask
    // runs are padded to 16-byte multiples; nrun <= D*SB/16 (checked when the plan is built)
    __shared__ __attribute__((aligned(16)))
    VT raw[NP > 1 ? kBinPartCap<D, NP, SB> + 16 / sizeof(VT) : D * SB + D * SB / 16 * (16 / sizeof(VT) - 1)];
    InstState* S = a.st;
    if (S->done) return;
    const uint64_t t0 = a.ts ? __builtin_amdgcn_s_memrealtime() : 0;
    uint64_t t1 = 0;
    // XCD-aware order: consecutive receiver blocks (which share the lines at their tile-run
    // seams) run on the same XCD (dispatch is round-robin over the 8 XCDs by blockIdx)
    const uint32_t b = a.qlo + (blockIdx.x & 7u) * Qc + (blockIdx.x >> 3);
    if (b >= a.qhi) return;   // past this launch's block range
    if (b >= Q) {   // partial slots past this partition's blocks: neutral (the finalize folds a.nblk)
        if (b < a.nblk && threadIdx.x == 0) a.partial[b] = make_double2(kInf, -kInf);
        return;
    }
    constexpr uint32_t NW = SB / 64;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t li = (uint64_t)b * SB + threadIdx.x;   // local row
    const uint64_t i = a.row0 + li;                              // global receiver
    bool live = li < a.nrows;
    if constexpr (VAR) {   // CSR hub rows (no deliveries in the plan): the generic kernel serves them
        if (live && a.deg[i] == kDegHub) live = false;
    }
    const uint2* tb = tiles + (uint64_t)b * (nrun + 1);
    // narrow plans: this round's stage entry width (4: u32 offsets from the base in .x/.y), read
    // after the first loads this workgroup needs anyway, so that one wait covers both (read first,
    // it was waited for alone ahead of them: phase B +4-5 us in 8-byte rounds)
    uint4 nh = make_uint4(0u, 0u, 8u, 0u);
    bool nar = false;
    // NP-pass blocks of at most 64 runs: every wave fetches all descriptors first (one per lane)
    // and issues part 0's DMA before anything else is in flight, so the only wait ahead of the
    // first transfer is the descriptor load itself; later parts issue from registers.
    const bool pf = NP > 1 && nrun <= 64;
    // Clamped pick-up (kPolClampPick; two passes, prefetched descriptors, not the tagged kernels):
    // part 0 lies END-aligned in the buffer (image position p at raw[p + cap - hi0]) and part 1
    // start-aligned (p at raw[p - lo1]); raw[cap] holds zeros.  A slot's index, clamped to cap, then
    // reads its value in its own part and +0 bits in the other, and the two reads are OR-merged: no
    // compare or select per slot and part.
    uint2 pdsc = make_uint2(0u, 0u);
    uint32_t pnxt = 0;
    constexpr uint32_t cap = kBinPartCap<D, NP, SB>;
    const bool clampm = NP == 2 && sizeof(VT) == 8 && !FAULTY && pf && (pol & kPolClampPick);
    uint32_t hi0 = 0;
    const bool adma = clampm && (pol & kPolAsmDma);   // asm saddr LDS-DMA (binned_dev.hpp)
    uint32_t ppk = 0;                                   // this lane's run: image offset | 16-B units << 16
    if (pf) {
        const uint32_t lane = threadIdx.x & 63;
        if (lane < nrun) {
            pdsc = tb[lane];
            pnxt = tb[lane + 1].y;
        }
        if constexpr (NAR) {
            asm volatile("" ::: "memory");   // (issued after the descriptor loads)
            nh = bin_nhdr_load(a.nhdr);
            nar = nh.z == 4u;
        }
        const uint32_t j1 = nrun / NP;
        hi0 = __builtin_amdgcn_readlane(pdsc.y, j1);
        if (adma) ppk = pdsc.y | ((pnxt - pdsc.y) / (16 / sizeof(VT))) << 16;
        if (!nar) {   // (a narrow round copies its whole u32 image below)
            if (adma)
                bin_dma_runs_asm(pdsc.x, ppk, w * j1 / NW, (w + 1) * j1 / NW, stage, raw, hi0 - cap);
            else
                bin_dma_runs_pf(pdsc, pnxt, w * j1 / NW, (w + 1) * j1 / NW, stage, raw, clampm ? hi0 - cap : 0u);
        }
    }
    if constexpr (NP > 1) {
        if (clampm && !nar && threadIdx.x < 16 / sizeof(VT)) raw[cap + threadIdx.x] = VT(0);   // +0 bits
    }
    // ordinary loads next (their wait is the barrier's vmcnt(0) anyway)
    const VT xi = live ? reinterpret_cast<const VT*>(a.xin)[i] : VT(0);
    uint32_t si = kHonest;
    if constexpr (FLT) {
        if (a.status && live) si = a.status[i];
    }
    uint32_t dg = D;
    uint64_t rp = 0;
    if constexpr (VAR) {
        if (live) {
            dg = a.deg[i];
            if constexpr (FLT) rp = a.rowptr[i];
        }
    }
    // §A.5 drop decisions of the lane's D slots as a bit mask, drawn before the values arrive: the
    // Philox state is then dead while the D + 1 values are live (drawn inside the resolution loop
    // below, the faulty two-pass kernels spilled 36-49 VGPRs at their 128-VGPR bound, and the CSR
    // slot loop — one draw per slot — was too large to unroll, so v[] went to scratch)
    uint32_t dmask = 0;
    if constexpr (FLT) {
        static_assert(D <= 32, "one drop bit per slot in a 32-bit mask");
        const MsgParams& mp = a.mp;
        if (mp.thr && live) {
            const uint32_t bI = (uint32_t)mp.inst_offset, bG = bI - bI % mp.mask_group;
            if constexpr (!VAR) {
#pragma unroll
                for (int q = 0; q < D / 4; ++q) {
                    const U4 w = philox10((uint32_t)i * (uint32_t)(D / 4) + q, a.r, bG, kStreamDrop, mp.key);
#pragma unroll
                    for (int e = 0; e < 4; ++e) dmask |= (uint32_t)(w.v[e] < mp.thr) << (4 * q + e);
                }
            } else if (dg) {   // slots rowptr[i] .. + deg(i) - 1: one call per 4 consecutive slots
                const uint64_t c1 = (rp + dg + 3) >> 2;
                for (uint64_t c = rp >> 2; c < c1; ++c) {
                    const U4 w = philox10((uint32_t)c, a.r, bG, kStreamDrop, mp.key);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint64_t t = 4 * c + e - rp;   // wraps past 2^64 below rp: out of range
                        if (t < dg) dmask |= (uint32_t)(w.v[e] < mp.thr) << t;
                    }
                }
            }
        }
    }
    uint4 ip[D / 8];
    // position of slot t (compile-time t)
    auto pos_of = [&](int t) -> uint32_t {
        const uint4& u = ip[t / 8];
        const uint32_t wd = (t & 6) == 0 ? u.x : (t & 6) == 2 ? u.y : (t & 6) == 4 ? u.z : u.w;
        return (t & 1) ? wd >> 16 : wd & 0xFFFFu;
    };
    const uint4* ipp = reinterpret_cast<const uint4*>(invpos) + (uint64_t)b * (D / 8) * SB + threadIdx.x;
#if ACS_DIAG_B == 4   // diagnostic: no invpos stream; in-range synthetic positions (wrong values)
    if (true) {
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            uint32_t w4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e)
                w4[e] = ((8 * q + 2 * e) * SB + threadIdx.x) | ((8 * q + 2 * e + 1) * SB + threadIdx.x) << 16;
            ip[q] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
    } else
#endif
    {   // once-read stream: nontemporal loads (phase B 80 -> 71 us on cfg4)
        using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
        const u32x4* ipn = reinterpret_cast<const u32x4*>(ipp);
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            const u32x4 t4 = __builtin_nontemporal_load(ipn + q * SB);
            ip[q] = make_uint4(t4.x, t4.y, t4.z, t4.w);
        }
    }
    if constexpr (NAR) {
        if (!pf) {   // (one-pass kernels: after the x_i and invpos loads)
            asm volatile("" ::: "memory");
            nh = bin_nhdr_load(a.nhdr);
            nar = nh.z == 4u;
        }
    }
    VT v[D + 1];
    bool picked = false;
    if constexpr (NAR) {
        if (nar) {   // narrow round: the block's u32 image in one pass, values = base + offset
            uint32_t* r32 = reinterpret_cast<uint32_t*>(raw);
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(stage);
            if (pf) {
                const uint32_t pk32 = pdsc.y | ((pnxt - pdsc.y) / 4u) << 16;
                bin_dma_runs_asm(pdsc.x, pk32, w * nrun / NW, (w + 1) * nrun / NW, s32, r32, 0u);
            } else {
                bin_dma_runs_asm_tb(tb, w * nrun / NW, (w + 1) * nrun / NW, s32, r32);
            }
            bin_dma_wait();
            __syncthreads();
            if (a.ts) t1 = __builtin_amdgcn_s_memrealtime();
            const uint64_t base = (uint64_t)nh.x | (uint64_t)nh.y << 32;
#pragma unroll
            for (int t = 0; t < D; ++t) v[1 + t] = __longlong_as_double((long long)(base + r32[pos_of(t)]));
            picked = true;
            // (the rule, store and partial below are shared with the 8-byte path; a separate copy
            // here measured slower in both kinds of round: narrow 44.5 against 42.5 us)
        }
    }
    if (picked) {
    } else if constexpr (NP == 1) {
        if (pol & kPolAsmDmaT) {
            bin_dma_runs_asm_tb(tb, w * nrun / NW, (w + 1) * nrun / NW, stage, raw);
            bin_dma_wait();
        } else {
            bin_dma_runs(tb, w * nrun / NW, (w + 1) * nrun / NW, stage, raw);
        }
        __syncthreads();
        if (a.ts) t1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
        for (int t = 0; t < D; ++t) v[1 + t] = raw[pos_of(t)];
    } else if (sizeof(VT) == 8 && clampm && !FLT && (pol & kPolBytePick)) {
        // Packed 16-bit pick-up (kPolBytePick, clean plans).  A u32 of invpos holds
        // two slots' positions: one v_pk_add_u16 shifts both into the part's buffer frame, one
        // v_pk_min_u16 clamps both to the zero slot at cap, and each becomes a byte offset by one
        // shift (the low half by an SDWA shift of its WORD_0; the high half by >> 13, exact because
        // both clamped halves are < cap < 2^13, so the low half's bits 13-15 are zero).  Part 1's
        // value is merged by one fp64 add: +0.0 is the identity for every value a clean round
        // carries (finite, never -0.0).  2 VALU per slot and part + 1 per slot for the merge,
        // against 3 + 3 + 2.  Positions p + (cap - hi0) stay below 2^16 (p < 2^14, cap < 2^13), and
        // p - lo1 for a part-0 slot wraps to at least 2^16 - 2^14 > cap.
        static_assert(cap < 8192, "two clamped positions per u32: each below 2^13");
        using us2 = unsigned short __attribute__((ext_vector_type(2)));
        const us2 cap2 = {(unsigned short)cap, (unsigned short)cap};
        const unsigned char* rb = reinterpret_cast<const unsigned char*>(raw);
        auto pick = [&](uint32_t word, const us2 sh, bool sub, VT& lo, VT& hi) {
            us2 q = __builtin_bit_cast(us2, word);
            q = sub ? q - sh : q + sh;
            q = __builtin_elementwise_min(q, cap2);
            const uint32_t qw = __builtin_bit_cast(uint32_t, q);
            uint32_t blo;
            asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                : "=v"(blo) : "v"(qw));
            lo = *reinterpret_cast<const VT*>(rb + blo);
            hi = *reinterpret_cast<const VT*>(rb + (qw >> 13));
        };
        if (adma) bin_dma_wait();   // (the asm copies are not in the compiler's count)
        __syncthreads();
        if (a.ts) t1 = __builtin_amdgcn_s_memrealtime();
        uint32_t sh0 = cap - hi0;
        asm volatile("" : "+s"(sh0));   // (opaque: see the clamped branch below)
        const us2 s0 = {(unsigned short)sh0, (unsigned short)sh0};
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            pick(ip[q].x, s0, false, v[1 + 8 * q], v[2 + 8 * q]);
            pick(ip[q].y, s0, false, v[3 + 8 * q], v[4 + 8 * q]);
            pick(ip[q].z, s0, false, v[5 + 8 * q], v[6 + 8 * q]);
            pick(ip[q].w, s0, false, v[7 + 8 * q], v[8 + 8 * q]);
        }
        __syncthreads();   // every lane has read part 0 before part 1 overwrites the buffer's front
        const uint32_t lo1 = hi0, j1 = nrun / NP;
        if (adma) {
            bin_dma_runs_asm(pdsc.x, ppk, j1 + w * (nrun - j1) / NW, j1 + (w + 1) * (nrun - j1) / NW, stage, raw, lo1);
            bin_dma_wait();
        } else {
            bin_dma_runs_pf(pdsc, pnxt, j1 + w * (nrun - j1) / NW, j1 + (w + 1) * (nrun - j1) / NW, stage, raw, lo1);
        }
        __syncthreads();
        uint32_t l1 = lo1;
        asm volatile("" : "+s"(l1));
        const us2 s1 = {(unsigned short)l1, (unsigned short)l1};
#pragma unroll
        for (int q = 0; q < D / 8; ++q) {
            const uint32_t wd[4] = {ip[q].x, ip[q].y, ip[q].z, ip[q].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                VT u0, u1;
                pick(wd[e], s1, true, u0, u1);
                v[1 + 8 * q + 2 * e] = v[1 + 8 * q + 2 * e] + u0;
                v[2 + 8 * q + 2 * e] = v[2 + 8 * q + 2 * e] + u1;
            }
        }
    } else if (sizeof(VT) == 8 && clampm) {
        const uint32_t lo1 = hi0;
        // part 0
        if (adma) bin_dma_wait();
        __syncthreads();
        if (a.ts) t1 = __builtin_amdgcn_s_memrealtime();
        uint32_t sh0 = cap - hi0;
        // opaque to the compiler: it otherwise computes (p - lo1) once for both parts, p - lo1 + cap
        // for part 0 (two VALU instead of one SDWA add) and keeps the 32 differences live across
        asm volatile("" : "+s"(sh0));
#pragma unroll
        for (int t = 0; t < D; ++t) {
#if ACS_DIAG_B == 2   // diagnostic: conflict-free reads that ignore the positions (kept live)
            asm volatile("" ::"v"(pos_of(t)));
            v[1 + t] = raw[(t * SB + threadIdx.x) % cap];
#else
            const uint32_t q = pos_of(t) + sh0;
            v[1 + t] = raw[q < cap ? q : cap];
#endif
        }
        __syncthreads();   // every lane has read part 0 before part 1 overwrites the buffer's front
        if (adma) {
            bin_dma_runs_asm(pdsc.x, ppk, nrun / NP + w * (nrun - nrun / NP) / NW,
                             nrun / NP + (w + 1) * (nrun - nrun / NP) / NW, stage, raw, lo1);
            bin_dma_wait();
        } else {
            bin_dma_runs_pf(pdsc, pnxt, nrun / NP + w * (nrun - nrun / NP) / NW,
                            nrun / NP + (w + 1) * (nrun - nrun / NP) / NW, stage, raw, lo1);
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < D; ++t) {
#if ACS_DIAG_B == 2
            const VT u = raw[(t * SB + threadIdx.x + 7) % cap];
#else
            const uint32_t q = pos_of(t) - lo1;   // wraps above cap below lo1
            const VT u = raw[q < cap ? q : cap];
#endif
            using UB = std::conditional_t<sizeof(VT) == 8, uint64_t, uint32_t>;
            v[1 + t] = __builtin_bit_cast(VT, (UB)(__builtin_bit_cast(UB, v[1 + t]) | __builtin_bit_cast(UB, u)));
        }
    } else {
#pragma unroll
        // Unrolled: the first part skips the p >= lo test and the last part the p < hi test.  This
        // relies on two invariants of the plan (binned_build checks both on the host): tb[0].y == 0
        // (lo of part 0), and every lane's invpos — live lanes and the zero-filled padding lanes of
        // a ragged last block alike — is below tb[nrun].y (hi of the last part).
        for (uint32_t k = 0; k < (uint32_t)NP; ++k) {
            const uint32_t j0 = k * nrun / NP, j1 = (k + 1) * nrun / NP;
            uint32_t lo, hi;   // image range of this part (pad-unit aligned)
            if (pf) {
                lo = __builtin_amdgcn_readlane(pdsc.y, j0);
                hi = j1 < nrun ? __builtin_amdgcn_readlane(pdsc.y, j1) : __builtin_amdgcn_readlane(pnxt, nrun - 1);
            } else {
                lo = tb[j0].y;
                hi = tb[j1].y;
            }
            if (k) __syncthreads();   // every lane has read the previous part before it is overwritten
            if (pf) {
                if (k) bin_dma_runs_pf(pdsc, pnxt, j0 + w * (j1 - j0) / NW, j0 + (w + 1) * (j1 - j0) / NW, stage, raw, lo);
            } else {
                bin_dma_runs(tb, j0 + w * (j1 - j0) / NW, j0 + (w + 1) * (j1 - j0) / NW, stage, raw, lo);
            }
            __syncthreads();
            if (k == 0 && a.ts) t1 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
            for (int q = 0; q < D / 8; ++q) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t p0 = pos_of(8 * q + 2 * e), p1 = pos_of(8 * q + 2 * e + 1);
                    const bool in0 = (k == 0 || p0 >= lo) && (k + 1 == (uint32_t)NP || p0 < hi);
                    const bool in1 = (k == 0 || p1 >= lo) && (k + 1 == (uint32_t)NP || p1 < hi);
                    // (faulty kernels: exec-masked reads straight into v; the clamped read + select
                    // holds the old and the new values together: 148-312 B/lane of scratch at their
                    // 128-VGPR bound)
                    if (!FAULTY && (pol & kPolBfPick)) {   // every lane reads (offset 0 when out of this part), then selects
                        const VT t0 = raw[in0 ? p0 - lo : 0u], t1 = raw[in1 ? p1 - lo : 0u];
                        v[1 + 8 * q + 2 * e] = in0 ? t0 : v[1 + 8 * q + 2 * e];
                        v[2 + 8 * q + 2 * e] = in1 ? t1 : v[2 + 8 * q + 2 * e];
                    } else {
                        if (in0) v[1 + 8 * q + 2 * e] = raw[p0 - lo];
                        if (in1) v[2 + 8 * q + 2 * e] = raw[p1 - lo];
                    }
                }
            }
        }
    }

    double mn = kInf, mx = -kInf;
    if (live) {
        VT res = xi;
        if (!FLT || is_active(si, a.r)) {
            v[0] = xi;
            uint32_t nmiss = 0;   // entries left out under missing_policy = OMIT
            if constexpr (VAR && !FAULTY && !FIX) {   // absent CSR entries
#pragma unroll
                for (int t = 0; t < D; ++t)
                    if ((uint32_t)t >= dg) {
                        v[1 + t] = omit_fill<VT>(a.rule);
                        ++nmiss;
                    }
            }
            if constexpr (FAULTY) {   // §A.5 drops, §A.4 / §A.6 sender resolution (round_regular.hip order)
                const MsgParams& mp = a.mp;
                const uint32_t bI = (uint32_t)mp.inst_offset;
                const uint32_t r = a.r, iu = (uint32_t)i;
                const VT lo = (VT)S->lo, hi = (VT)S->hi;
#pragma unroll
                for (int q = 0; q < D / 4; ++q) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int t = 4 * q + e;
                        if (VAR && (uint32_t)t >= dg) {   // absent CSR entry
                            v[1 + t] = omit_fill<VT>(a.rule);
                            ++nmiss;
                            continue;
                        }
                        const uint64_t slot = VAR ? rp + t : (uint64_t)iu * D + t;
                        const bool dropped = (dmask >> t) & 1u;
                        VT u = v[1 + t];
                        uint32_t stj = kHonest;
                        if constexpr (sizeof(VT) == 8) {
                            const uint64_t bits = (uint64_t)__double_as_longlong(u);
                            if ((bits >> 51) == 0xFFFull) {
                                const uint32_t md = (uint32_t)(bits & 3u);
                                stj = md == 1 ? kByz : md == 2 ? r : r - 1;   // silent implies r >= 1
                                if (md == 2) u = reinterpret_cast<const VT*>(a.xin)[(bits >> 2) & 0xFFFFFFFFull];
                            }
                        } else {
                            const uint32_t bits = __float_as_uint(u);
                            if ((bits >> 22) == 0x1FFu) {
                                const uint32_t md = bits & 3u;
                                stj = md == 1 ? kByz : md == 2 ? r : r - 1;
                                if (md == 2) {
                                    const uint32_t f = (bits >> 2) & 0xFFFFFu;
                                    u = reinterpret_cast<const VT*>(a.xin)[a.clist ? a.clist[a.coff + f] : f];
                                }
                            }
                        }
                        bool miss;
                        const VT rv = resolve_entry_m(mp, stj, u, xi, dropped, bI, r, iu, slot, lo, hi, miss);
                        const bool out = mp.omit && miss;
                        v[1 + t] = out ? omit_fill<VT>(a.rule) : rv;
                        nmiss += out;
                    }
                }
            }
            if constexpr (FIX) {   // drops and the fix-up's missing entries (NaN) -> x_i (missing_policy
                                   // = SUBSTITUTE: OMIT configs keep the tagged path); absent CSR entries
#pragma unroll
                for (int t = 0; t < D; ++t) {
                    if (VAR && (uint32_t)t >= dg) {
                        v[1 + t] = omit_fill<VT>(a.rule);
                        ++nmiss;
                        continue;
                    }
                    const VT u = v[1 + t];
                    v[1 + t] = (((dmask >> t) & 1u) || u != u) ? xi : u;
                }
            }
            if (VAR || (FAULTY && a.mp.omit))
                res = apply_rule_reg_omit<D, T, WMSR>(a.rule, v, nmiss);
#if ACS_DIAG_B == 1   // diagnostic: the plain sum instead of the selection network (wrong values)
            else if (NP == 2 && !FLT)
                res = tree_sum_const<D + 1>(v) / (VT)(D + 1);
#endif
            else if constexpr (!FLT)   // padding adds skipped, exact for every input (sortnet.hpp)
                res = apply_rule_reg<D, T, WMSR, true>(a.rule, v);
            else
                res = apply_rule_reg<D, T, WMSR>(a.rule, v);
        }
        bin_store_x<SB>(a, i, res, pol);
        if (si == kHonest) {
            mn = res;
            mx = res;
        }
    }
    block_minmax_store<SB>(mn, mx, a.partial + b, a.eacc);
    if (a.ts) bin_ts(a.ts, t0, t1);
}

// ------------------------------------------------------------------------------ plan build
// Geometry shared by the setup kernels.  Local receiver rows li in [0, NR) (a node partition's
// rows, or all N); global sender ids j in [0, N).
//   one level:  key1 = a*Q + b                         (phase B reads stage1)
//   two levels: key1 = a*R + r, key2 = (r*K + k)*QR + bl  with r = li / SR, k = a / PK,
//               bl = (li % SR) / SB                    (phase B reads stage2)
struct BinGeom {
    uint32_t D, dp, SA, P, Q, levels, SR, R, K, PK, QR;
    uint32_t SB;    // receivers per phase-B block (BinnedPlan::SB)
    uint32_t pad;   // tile lengths padded to 16 bytes: 2 (fp64) or 4 (fp32, narrow fp64) elements
    uint32_t npad_or;   // 1: tiles' starts carry the run's pad count in their low bits (not on narrow
                        // plans, whose 8-byte rounds address the starts in units of 2 entries)
    uint32_t none1, none2;   // tile count of level 1 / 2: the key of an absent CSR column (kEllNone),
                             // which sorts past every tile and is skipped by every fill kernel
};

__device__ __forceinline__ uint32_t ell_at(const uint32_t* ell, uint64_t i, uint32_t t, uint32_t dp) {
    return ell[(((i >> 6) * (dp >> 2) + (t >> 2)) * 64 + (i & 63)) * 4 + (t & 3)];
}

__global__ __launch_bounds__(256) void k_bin_keys(const uint32_t* __restrict__ ell, uint64_t E, BinGeom G, int level,
                                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const uint64_t li = e / G.D;
    const uint32_t t = (uint32_t)(e % G.D);
    const uint32_t col = ell_at(ell, li, t, G.dp);
    const uint32_t a = col / G.SA;
    uint32_t key;
    if (col == kEllNone)
        key = level == 1 ? G.none1 : G.none2;
    else if (G.levels == 1)
        key = a * G.Q + (uint32_t)(li / G.SB);
    else if (level == 1)
        key = a * G.R + (uint32_t)(li / G.SR);
    else
        key = ((uint32_t)(li / G.SR) * G.K + a / G.PK) * G.QR + (uint32_t)((li % G.SR) / G.SB);
    keys[e] = key;
    vals[e] = (uint32_t)e;
}

// tile boundaries in the sorted keys: tl[key] = (first, last+1) unpadded sorted positions
__global__ __launch_bounds__(256) void k_bin_bounds(uint64_t E, const uint32_t* __restrict__ ks, uint2* __restrict__ tl,
                                                    uint64_t nt) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t key = ks[p];
    if (key >= nt) return;   // absent CSR columns
    if (p == 0 || ks[p - 1] != key) tl[key].x = (uint32_t)p;
    if (p == E - 1 || ks[p + 1] != key) tl[key].y = (uint32_t)(p + 1);
}

// padded tile lengths (even, so every run starts 16-byte aligned in the stage and in LDS)
__global__ __launch_bounds__(256) void k_bin_plen(const uint2* __restrict__ tl, uint64_t nt, uint32_t pad,
                                                  uint32_t* __restrict__ plen) {
    const uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= nt) return;
    const uint2 t = tl[k];
    plen[k] = t.y ? (t.y - t.x + pad - 1u) & ~(pad - 1u) : 0u;
}

// idxA[padded position] = sender index inside its source block (level-1 order)
__global__ __launch_bounds__(256) void k_bin_fill_a(const uint32_t* __restrict__ ell, uint64_t E, BinGeom G,
                                                    const uint32_t* __restrict__ ks, const uint32_t* __restrict__ vs,
                                                    const uint2* __restrict__ tl, const uint32_t* __restrict__ pstart,
                                                    uint16_t* __restrict__ idxA) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t e = vs[p], key = ks[p];
    if (key >= G.none1) return;
    idxA[pstart[key] + (p - tl[key].x)] = (uint16_t)(ell_at(ell, e / G.D, e % G.D, G.dp) % G.SA);
}

// idxA -> 14-bit packed blocks (binned_dev.hpp pk14): one thread per (512-position block m, lane l)
__global__ __launch_bounds__(256) void k_bin_pack14(const uint16_t* __restrict__ idx, uint64_t n, uint32_t* __restrict__ pk) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t m = t >> 6;
    const uint32_t l = (uint32_t)t & 63u;
    if (m * 512 >= n) return;
    uint64_t acc[2] = {0ull, 0ull};   // bits 0-63, 64-127
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint64_t pos = m * 512 + 2 * (64 * (uint64_t)(k >> 1) + l) + (k & 1);
        const uint64_t v = pos < n ? (uint64_t)(idx[pos] & 0x3FFFu) : 0ull;
        const int bit = 14 * k;
        if (bit < 64) {
            acc[0] |= v << bit;
            if (bit + 14 > 64) acc[1] |= v >> (64 - bit);
        } else {
            acc[1] |= v << (bit - 64);
        }
    }
    uint32_t* b = pk + m * kPk14Words + l;
    b[0] = (uint32_t)acc[0];
    b[64] = (uint32_t)(acc[0] >> 32);
    b[128] = (uint32_t)acc[1];
    reinterpret_cast<uint16_t*>(pk)[m * (2 * kPk14Words) + 384 + l] = (uint16_t)(acc[1] >> 32);
}


// phase-A ranges: aoff[a] = padded start of source block a's deliveries (aoff[P] = Ep)
__global__ __launch_bounds__(256) void k_bin_aoff(const uint32_t* __restrict__ pstart, uint32_t P, uint32_t G1,
                                                  uint64_t Ep, uint64_t* __restrict__ aoff) {
    const uint32_t a = blockIdx.x * 256 + threadIdx.x;
    if (a > P) return;
    aoff[a] = a < P ? pstart[(uint64_t)a * G1] : Ep;
}

// phase-M run tables: mt[g][j] for group g = r*K + k, run a = k*PK + j; total image size in cap[g]
__global__ __launch_bounds__(256) void k_bin_mtiles(const uint32_t* __restrict__ pstart1, const uint32_t* __restrict__ plen1,
                                                    BinGeom G, uint2* __restrict__ mt, uint32_t* __restrict__ cap) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= G.R * G.K) return;
    const uint32_t r = g / G.K, k = g % G.K;
    uint32_t pre = 0;
    for (uint32_t j = 0; j < G.PK; ++j) {
        const uint32_t a = k * G.PK + j;
        if (a < G.P) {
            const uint64_t key = (uint64_t)a * G.R + r;
            mt[(uint64_t)g * (G.PK + 1) + j] = make_uint2(pstart1[key], pre);
            pre += plen1[key];
        } else {
            mt[(uint64_t)g * (G.PK + 1) + j] = make_uint2(0u, pre);
        }
    }
    mt[(uint64_t)g * (G.PK + 1) + G.PK] = make_uint2(0u, pre);
    cap[g] = pre;
}

// lpos[e] = position of delivery e inside its phase-M LDS image
__global__ __launch_bounds__(256) void k_bin_lpos(uint64_t E, BinGeom G, const uint32_t* __restrict__ ks1,
                                                  const uint32_t* __restrict__ vs1, const uint2* __restrict__ tl1,
                                                  const uint2* __restrict__ mt, uint16_t* __restrict__ lpos) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t key = ks1[p], a = key / G.R, r = key % G.R;
    if (key >= G.none1) return;
    const uint32_t g = r * G.K + a / G.PK;
    lpos[vs1[p]] = (uint16_t)(mt[(uint64_t)g * (G.PK + 1) + a % G.PK].y + (p - tl1[key].x));
}

// idxM[padded level-2 position] = lpos of that delivery
__global__ __launch_bounds__(256) void k_bin_fill_m(uint64_t E, const uint32_t* __restrict__ ks2,
                                                    const uint32_t* __restrict__ vs2, const uint2* __restrict__ tl2,
                                                    const uint32_t* __restrict__ pstart2, const uint16_t* __restrict__ lpos,
                                                    uint16_t* __restrict__ idxM, uint32_t none2) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t key = ks2[p];
    if (key >= none2) return;
    idxM[pstart2[key] + (p - tl2[key].x)] = lpos[vs2[p]];
}

// phase-M output ranges: moff[g] = padded level-2 start of group g (moff[R*K] = Ep2)
__global__ __launch_bounds__(256) void k_bin_moff(const uint32_t* __restrict__ pstart2, BinGeom G, uint64_t Ep2,
                                                  uint64_t* __restrict__ moff) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    const uint32_t ng = G.R * G.K;
    if (g > ng) return;
    moff[g] = g < ng ? pstart2[(uint64_t)g * G.QR] : Ep2;
}

// Runs read by phase B for block b: one level: keys j*Q + b (j = source block, nrun = P); two
// levels: keys (r*K + j)*QR + bl (j = chunk, nrun = K).
__device__ __forceinline__ uint64_t bin_run_key(const BinGeom& G, uint32_t b, uint32_t j) {
    if (G.levels == 1) return (uint64_t)j * G.Q + b;
    return ((uint64_t)(b / G.QR) * G.K + j) * G.QR + b % G.QR;
}

// tiles[b][j] = (padded start | pad count, element offset inside block b's concatenated runs);
// tiles[b][nrun] = (0, total).  Starts are multiples of the pad unit, so the low bits carry the
// number of padding entries at the run's end.
__global__ __launch_bounds__(256) void k_bin_prefix(const uint32_t* __restrict__ pstart, const uint32_t* __restrict__ plen,
                                                    const uint2* __restrict__ tl, BinGeom G, uint32_t nrun,
                                                    uint2* __restrict__ tiles) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= G.Q) return;
    uint32_t pre = 0;
    for (uint32_t j = 0; j < nrun; ++j) {
        const uint64_t key = bin_run_key(G, b, j);
        const uint32_t npad = plen[key] - (tl[key].y - tl[key].x);
        tiles[(uint64_t)b * (nrun + 1) + j] = make_uint2(pstart[key] | (G.npad_or ? npad : 0u), pre);
        pre += plen[key];
    }
    tiles[(uint64_t)b * (nrun + 1) + nrun] = make_uint2(0u, pre);
}

// invpos[b][t/8][i_local][t%8] = element position of (receiver i_local, slot t) in block b's runs
__global__ __launch_bounds__(256) void k_bin_inv(uint64_t E, BinGeom G, uint32_t nrun, const uint32_t* __restrict__ ks,
                                                 const uint32_t* __restrict__ vs, const uint2* __restrict__ tl,
                                                 const uint2* __restrict__ tiles, uint16_t* __restrict__ invpos) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t e = vs[p], key = ks[p];
    if (key >= (G.levels == 1 ? G.none1 : G.none2)) return;
    const uint64_t li = e / G.D;
    const uint32_t t = e % G.D;
    const uint32_t b = (uint32_t)(li / G.SB);
    const uint32_t j = G.levels == 1 ? key / G.Q : (key / G.QR) % G.K;
    const uint32_t pos = tiles[(uint64_t)b * (nrun + 1) + j].y + (uint32_t)(p - tl[key].x);
    invpos[(((uint64_t)b * (G.D / 8) + t / 8) * G.SB + (li % G.SB)) * 8 + (t & 7)] = (uint16_t)pos;
}

// fix-up list: every sorted position p of the last level whose sender is not honest
__global__ __launch_bounds__(256) void k_bin_fixlist(const uint32_t* __restrict__ ell, uint64_t E, uint32_t D,
                                                     uint32_t dp, uint32_t none, const uint32_t* __restrict__ ks,
                                                     const uint32_t* __restrict__ vs, const uint2* __restrict__ tl,
                                                     const uint32_t* __restrict__ pstart,
                                                     const uint32_t* __restrict__ status,
                                                     uint4* __restrict__ fix, uint32_t cap, uint32_t* __restrict__ cnt) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= E) return;
    const uint32_t key = ks[p];
    if (key >= none) return;
    const uint32_t e = vs[p];
    const uint64_t li = e / D;
    const uint32_t t = e % D;
    const uint32_t j = ell_at(ell, li, t, dp);
    if (status[j] == kHonest) return;
    const uint32_t k = atomicAdd(cnt, 1u);
    if (k < cap) fix[k] = make_uint4(pstart[key] + (uint32_t)(p - tl[key].x), (uint32_t)li, t, j);
}

// ------------------------------------------------------------------------------ host side
#define ACS_BINNED_VARIANTS(X) X(16, 5) X(32, 5) X(16, 0) X(32, 0) X(8, 2) X(8, 0)

bool binned_supported(uint32_t d, uint32_t t, uint32_t rule) {
    if (rule > 4) return false;
    if (rule == 0 && t != 0) return false;   // AVERAGE: entry order (the rows must be in spec order)
    if (rule == 3 && t < 1) return false;
#define X(DD, TT) if (d == DD && t == TT) return true;
    ACS_BINNED_VARIANTS(X)
#undef X
    return false;
}

uint32_t binned_levels(uint64_t N, uint64_t NR, uint32_t d, uint32_t sa, uint32_t sb, uint32_t* sr_out) {
    if (d == 0 || sa == 0 || NR == 0 || sb == 0) return 0;
    const uint64_t P = (N + sa - 1) / sa;
    const uint64_t Q = (NR + sb - 1) / sb;
    // (the one- / two-level choice is the default block's, so a plan's level count and its
    // phase A / M do not change with the receiver block)
    const uint64_t Q0 = (NR + kBinSB - 1) / kBinSB;
    const double run1 = (double)NR * d / ((double)P * (double)Q0);
    if (run1 >= 64.0) {
        if (sr_out) *sr_out = sb;
        return (uint64_t)P <= (uint64_t)d * sb / 16 && Q >= 1 ? 1u : 0u;   // phase-B LDS bound
    }
    // level-1 runs (a, r) average NR*d / (P * R) with R = NR / SR: about 128 at SR = 128 * P / d
    // (SR a multiple of both the default block and sb: powers of two)
    const uint64_t unit = sb > kBinSB ? sb : kBinSB;
    uint64_t sr = (128ull * P / d + unit - 1) / unit * unit;
    if (sr < 4 * kBinSB) sr = 4 * kBinSB;
    if (sr % sb) return 0;
    if (sr > 65536) return 0;
    if (sr_out) *sr_out = (uint32_t)sr;
    return 2;
}

void binned_free(BinnedPlan& p) {
    if (p.ts) {   // diagnostic dump: phase,workgroup,t_entry,t_staged,t_end (100 MHz ticks)
        std::vector<uint64_t> h(3ull * (p.ts_a + p.ts_b + p.ts_m));
        const char* fn = getenv("ACSIM_BIN_TS");
        if (fn && hipMemcpy(h.data(), p.ts, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
            if (FILE* f = fopen(fn, "w")) {
                for (uint64_t k = 0; k < p.ts_a + p.ts_b + p.ts_m; ++k)
                    fprintf(f, "%c,%llu,%llu,%llu,%llu\n", k < p.ts_a ? 'A' : k < p.ts_a + p.ts_b ? 'B' : 'M',
                            (unsigned long long)(k < p.ts_a ? k : k < p.ts_a + p.ts_b ? k - p.ts_a : k - p.ts_a - p.ts_b),
                            (unsigned long long)h[3 * k],
                            (unsigned long long)h[3 * k + 1], (unsigned long long)h[3 * k + 2]);
                fclose(f);
            }
        }
        (void)hipFree(p.ts);
    }
    (void)hipFree(p.idxA);
    (void)hipFree(p.pkA);
    (void)hipFree(p.idxM);
    (void)hipFree(p.invpos);
    (void)hipFree(p.tiles);
    (void)hipFree(p.mt);
    (void)hipFree(p.aoff);
    (void)hipFree(p.moff);
    (void)hipFree(p.stage1);
    (void)hipFree(p.stage2);
    (void)hipFree(p.xtag);
    (void)hipFree(p.fix);
    (void)hipFree(p.nhdr);
    p = BinnedPlan{};
}

namespace {

// Deliveries sorted by a tile key (stable LSD radix sort: ties stay in (row, slot) order) and the
// tiles padded to even lengths.  Owns its arrays.
struct TileSort {
    uint32_t *ks = nullptr, *vs = nullptr, *plen = nullptr, *pstart = nullptr;
    uint2* tl = nullptr;
    uint64_t nt = 0, Ep = 0;
    void release() {
        (void)hipFree(ks);
        (void)hipFree(vs);
        (void)hipFree(plen);
        (void)hipFree(pstart);
        (void)hipFree(tl);
        ks = vs = plen = pstart = nullptr;
        tl = nullptr;
    }
};

hipError_t tile_sort(const uint32_t* ell, uint64_t E, const BinGeom& G, int level, uint64_t nt, TileSort& T,
                     hipStream_t s) {
    hipError_t e;
    T.nt = nt;
    uint32_t *keys = nullptr, *vals = nullptr;
    void* temp = nullptr;
    size_t tb = 0, tb2 = 0;
    int bits = 1;
    while (bits < 32 && (1ull << bits) <= nt) ++bits;   // keys 0..nt (nt: absent CSR columns)
    const unsigned grid = (unsigned)((E + 255) / 256), gridt = (unsigned)((nt + 255) / 256);
    e = hipMalloc(&keys, E * 4);
    if (e == hipSuccess) e = hipMalloc(&vals, E * 4);
    if (e == hipSuccess) e = hipMalloc(&T.ks, E * 4);
    if (e == hipSuccess) e = hipMalloc(&T.vs, E * 4);
    if (e == hipSuccess) e = hipMalloc(&T.tl, nt * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&T.plen, nt * 4);
    if (e == hipSuccess) e = hipMalloc(&T.pstart, nt * 4);
    if (e == hipSuccess) e = hipMemsetAsync(T.tl, 0, nt * sizeof(uint2), s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_keys, dim3(grid), dim3(256), 0, s, ell, E, G, level, keys, vals);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, T.ks, vals, T.vs, (int)E, 0, bits, s);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, T.plen, T.pstart, (int)nt, s);
    if (tb2 > tb) tb = tb2;
    if (e == hipSuccess) e = hipMalloc(&temp, tb ? tb : 16);
    if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortPairs(temp, tb, keys, T.ks, vals, T.vs, (int)E, 0, bits, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_bounds, dim3(grid), dim3(256), 0, s, E, T.ks, T.tl, nt);
        hipLaunchKernelGGL(k_bin_plen, dim3(gridt), dim3(256), 0, s, T.tl, nt, G.pad, T.plen);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(temp, tb, T.plen, T.pstart, (int)nt, s);
    uint32_t last[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(&last[0], T.pstart + nt - 1, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(&last[1], T.plen + nt - 1, 4, hipMemcpyDeviceToHost, s);
    hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    T.Ep = (uint64_t)last[0] + last[1];
    (void)hipFree(temp);
    (void)hipFree(keys);
    (void)hipFree(vals);
    return e;
}

}  // namespace

hipError_t binned_build(BinnedPlan& p, const uint32_t* ell, uint64_t N, uint64_t NR, uint32_t d, uint32_t dp,
                        uint32_t sa, uint32_t sb, bool tagged, bool f32, hipStream_t s, bool var,
                        const uint32_t* status, bool clean, bool narrow) {
    if (var && f32) return hipErrorNotSupported;   // CSR plans: fp64
    // receiver blocks other than kBinSB: clean plans of a compiled (d, sb) pair only
    if (sb != kBinSB && (var || tagged || !clean)) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    uint32_t sr = 0;
    const uint32_t levels = binned_levels(N, NR, d, sa, sb, &sr);
    if (!levels) return hipErrorNotSupported;
    // ACSIM_BIN_PACK: bit 0 (default 1; 0: u16 phase-A index stream), read below
    const char* pack_env = getenv("ACSIM_BIN_PACK");
    const uint32_t pack = pack_env ? (uint32_t)strtoul(pack_env, nullptr, 10) : 1u;
    // narrow stage: clean one-level fp64 plans of d = 16 / 32 at the default
    // receiver block with the packed phase-A stream; confirmed at the end (phase-B LDS bound, passes)
    const bool nar_req = narrow && !f32 && !tagged && !var && clean && sb == kBinSB && levels == 1 && sa <= 16384 &&
                         (pack & 1u) && (d == 16 || d == 32);
    BinGeom G{};
    G.D = d;
    G.dp = dp;
    G.pad = f32 || nar_req ? 4u : 2u;
    G.npad_or = nar_req ? 0u : 1u;
    G.SA = sa;
    G.P = (uint32_t)((N + sa - 1) / sa);
    G.SB = sb;
    G.Q = (uint32_t)((NR + sb - 1) / sb);
    G.levels = levels;
    G.SR = sr;
    G.R = levels == 1 ? G.Q : (uint32_t)((NR + sr - 1) / sr);
    G.QR = sr / sb;
    G.PK = 1;
    if (levels == 2) {   // chunks of PK source blocks: an LDS image of about 16 Ki deliveries
        const double run1 = (double)NR * d / ((double)G.P * G.R);
        double img = 16384.0;   // ACSIM_BIN_MIMG: target deliveries per phase-M image (sweeps)
        if (const char* v = getenv("ACSIM_BIN_MIMG")) img = strtod(v, nullptr) > 0 ? strtod(v, nullptr) : img;
        const uint32_t pk = (uint32_t)(img / run1);
        G.PK = pk < 1 ? 1 : pk > G.P ? G.P : pk;
    }
    G.K = (G.P + G.PK - 1) / G.PK;
    G.none1 = G.P * G.R;
    G.none2 = levels == 2 ? G.R * G.K * G.QR : 0;
    p.var = var;
    p.D = d;
    p.SA = sa;
    p.SB = sb;
    p.f32 = f32;
    p.P = G.P;
    p.Q = G.Q;
    p.levels = levels;
    p.E = NR * d;
    p.PK = G.PK;
    p.ngroups = levels == 2 ? G.R * G.K : 0;
    p.nrun = levels == 1 ? G.P : G.K;
    const uint64_t E = p.E;
    const uint64_t nt1 = (uint64_t)G.P * G.R;
    const uint64_t nt2 = levels == 2 ? (uint64_t)G.R * G.K * G.QR : 0;
    if (E >= (1ull << 32) || nt1 >= (1ull << 32) || nt2 >= (1ull << 32)) return hipErrorNotSupported;
    if ((uint64_t)p.nrun > (uint64_t)d * sb / 16) return hipErrorNotSupported;   // phase-B LDS bound
    const unsigned grid = (unsigned)((E + 255) / 256);

    // ---- level 1 (phase A): key (a, b) or (a, r)
    TileSort T1, T2;
    e = tile_sort(ell, E, G, 1, nt1, T1, s);
    p.Ep1 = T1.Ep;
    if (e == hipSuccess) e = hipMalloc(&p.idxA, p.Ep1 * 2);
    if (e == hipSuccess) e = hipMemsetAsync(p.idxA, 0, p.Ep1 * 2, s);
    if (e == hipSuccess) e = hipMalloc(&p.stage1, p.Ep1 * (f32 ? sizeof(float) : sizeof(double)));
    if (e == hipSuccess) e = hipMalloc(&p.aoff, ((uint64_t)G.P + 1) * sizeof(uint64_t));
    if (e == hipSuccess && tagged) e = hipMalloc(&p.xtag, (N + 2) * sizeof(double));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_fill_a, dim3(grid), dim3(256), 0, s, ell, E, G, T1.ks, T1.vs, T1.tl, T1.pstart, p.idxA);
        hipLaunchKernelGGL(k_bin_aoff, dim3((G.P + 256) / 256), dim3(256), 0, s, T1.pstart, G.P, G.R, p.Ep1, p.aoff);
        e = hipGetLastError();
    }
    // 14-bit packed phase-A indices (fp64 plans with source blocks of at most 2^14 senders).
    // ACSIM_BIN_PACK bit 0.  Measured per kernel (rocprofv3, cfg4,
    // profiles/r04_s8_pack_kernel_stats.csv): packed idxA 59.4 -> 53-54 us.  Packed phase-B
    // positions measured slower (62.5-63.0 against 61.7-61.8 us: the decode sits on phase B's
    // critical path) and were removed in round 5 (history: d8efbd1).
    if (e == hipSuccess && sa <= 16384) {   // fp64 and fp32 (bit 2 of ACSIM_BIN_PACK: no longer needed)
        if (pack & 1u) {
            const uint64_t nb = (p.Ep1 + 511) / 512;
            e = hipMalloc(&p.pkA, nb * kPk14Words * 4);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_bin_pack14, dim3((unsigned)((nb * 64 + 255) / 256)), dim3(256), 0, s, p.idxA, p.Ep1,
                                   p.pkA);
                e = hipGetLastError();
            }
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e == hipSuccess) {
                (void)hipFree(p.idxA);
                p.idxA = nullptr;
            }
        }
    }
    TileSort* last = &T1;
    if (e == hipSuccess && levels == 2) {
        // ---- level 2 (phase M): PK-run images per (r, k), regrouped by receiver block
        uint16_t* lpos = nullptr;
        uint32_t* cap = nullptr;
        const uint32_t ng = p.ngroups;
        e = hipMalloc(&p.mt, (uint64_t)ng * (G.PK + 1) * sizeof(uint2));
        if (e == hipSuccess) e = hipMalloc(&cap, (uint64_t)ng * 4);
        if (e == hipSuccess) e = hipMalloc(&lpos, E * 2);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_bin_mtiles, dim3((ng + 255) / 256), dim3(256), 0, s, T1.pstart, T1.plen, G, p.mt, cap);
            hipLaunchKernelGGL(k_bin_lpos, dim3(grid), dim3(256), 0, s, E, G, T1.ks, T1.vs, T1.tl, p.mt, lpos);
            e = hipGetLastError();
        }
        if (e == hipSuccess) {   // every image must fit the phase-M LDS
            std::vector<uint32_t> h(ng);
            e = hipMemcpyAsync(h.data(), cap, (uint64_t)ng * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            uint32_t mx = 0;
            for (uint32_t v : h) mx = v > mx ? v : mx;
            p.mcap = mx;
            if (e == hipSuccess && mx > kBinMCap) e = hipErrorNotSupported;
        }
        if (e == hipSuccess) e = tile_sort(ell, E, G, 2, nt2, T2, s);
        p.Ep2 = T2.Ep;
        if (e == hipSuccess) e = hipMalloc(&p.idxM, p.Ep2 * 2);
        if (e == hipSuccess) e = hipMemsetAsync(p.idxM, 0, p.Ep2 * 2, s);
        if (e == hipSuccess) e = hipMalloc(&p.stage2, p.Ep2 * (f32 ? sizeof(float) : sizeof(double)));
        if (e == hipSuccess) e = hipMalloc(&p.moff, ((uint64_t)ng + 1) * sizeof(uint64_t));
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_bin_fill_m, dim3(grid), dim3(256), 0, s, E, T2.ks, T2.vs, T2.tl, T2.pstart, lpos, p.idxM,
                               G.none2);
            hipLaunchKernelGGL(k_bin_moff, dim3((ng + 256) / 256), dim3(256), 0, s, T2.pstart, G, p.Ep2, p.moff);
            e = hipGetLastError();
        }
        hipError_t e2 = hipStreamSynchronize(s);
        if (e == hipSuccess) e = e2;
        (void)hipFree(lpos);
        (void)hipFree(cap);
        last = &T2;
    }
    // ---- phase B tables over the last stage
    const uint64_t Qp = (uint64_t)G.Q * sb;   // receiver slots incl. the ragged last block's padding
    if (e == hipSuccess) e = hipMalloc(&p.tiles, ((uint64_t)p.nrun + 1) * G.Q * sizeof(uint2));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_prefix, dim3((G.Q + 255) / 256), dim3(256), 0, s, last->pstart, last->plen, last->tl, G,
                           p.nrun, p.tiles);
        e = hipGetLastError();
    }
    {
        const char* v = getenv("ACSIM_BIN_POL");
        p.pol = v ? (uint32_t)strtoul(v, nullptr, 0) & kPolMask
                  : kPolDefault | (G.levels == 2 ? kPolTwoLevelStores : kPolOneLevelStores);
    }
    if (e == hipSuccess) e = hipMalloc(&p.invpos, Qp * d * 2);
    if (e == hipSuccess) e = hipMemsetAsync(p.invpos, 0, Qp * d * 2, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_bin_inv, dim3(grid), dim3(256), 0, s, E, G, p.nrun, last->ks, last->vs, last->tl,
                           p.tiles, p.invpos);
        e = hipGetLastError();
    }
    // fault fix-up list: when the faulty senders' deliveries are few (at most an
    // eighth of all), their resolutions are written into the stage instead of tagging every sender
    if (e == hipSuccess && tagged && status && !getenv("ACSIM_BIN_NOFIX")) {
        // two passes: count (cap 0), then fill a list of exactly that size
        uint32_t* cnt = nullptr;
        uint32_t n = 0;
        e = hipMalloc(&cnt, sizeof(uint32_t));
        for (int pass = 0; pass < 2 && e == hipSuccess; ++pass) {
            if (pass == 1 && (n == 0 || (uint64_t)n > E / 8)) break;   // none, or too many to list
            if (pass == 1) e = hipMalloc(&p.fix, (uint64_t)n * sizeof(uint4));
            if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, sizeof(uint32_t), s);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_bin_fixlist, dim3(grid), dim3(256), 0, s, ell, E, G.D, G.dp,
                                   levels == 1 ? G.none1 : G.none2, last->ks, last->vs, last->tl, last->pstart,
                                   status, p.fix, pass ? n : 0u, cnt);
                e = hipGetLastError();
            }
            uint32_t c = 0;
            if (e == hipSuccess) e = hipMemcpyAsync(&c, cnt, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (pass == 0) n = c;
            else if (e == hipSuccess && c == n) p.nfix = n;
        }
        (void)hipFree(cnt);
        if (!p.nfix) {
            (void)hipFree(p.fix);
            p.fix = nullptr;
        }
    }
    hipError_t e2 = hipStreamSynchronize(s);
    if (e == hipSuccess) e = e2;
    // NP-pass phase B: 2 passes by default where the whole image limits phase B to 2 workgroups
    // per CU (fp64, d = 32: 68 KiB of LDS; measured 72.7 -> 65.0 us on cfg4; fp32 images already
    // allow 4 and a second pass only costs: 39.3 -> 43.8 us), and only when every part of every
    // block's image fits.  ACSIM_BIN_SPLIT=1..4 overrides (1: one pass).
    p.split = 1;
    if (e == hipSuccess) {
        const char* v = getenv("ACSIM_BIN_SPLIT");
        uint32_t np = v ? (uint32_t)strtoul(v, nullptr, 10) : (!f32 && G.D == 32 ? 2u : 1u);
        if (np < 1 || np > 4 || var) np = 1;   // CSR plans: single pass (the VAR kernels)
        if (f32 && tagged && np > 1) np = 1;   // tagged fp32 phase B: one pass (no split instantiation)
        if (tagged && np > 2) np = 2;          // tagged fp64 phase B: two passes at most
        if (np > 1) {
            const uint32_t D = G.D;
            const uint32_t cap = D * sb / np + D * sb / 16;   // kBinPartCap<D, np, sb>
            std::vector<uint2> h(((uint64_t)p.nrun + 1) * G.Q);
            e = hipMemcpy(h.data(), p.tiles, h.size() * sizeof(uint2), hipMemcpyDeviceToHost);
            bool fits = e == hipSuccess && p.nrun >= np;
            for (uint32_t b = 0; fits && b < G.Q; ++b) {
                const uint2* row = h.data() + (uint64_t)b * (p.nrun + 1);
                // the NP-pass kernel's skipped bound tests: part 0 starts at image offset 0, and the
                // image is non-empty (padding lanes read invpos 0, which must lie in the last part)
                fits = row[0].y == 0 && row[p.nrun].y > 0;
                for (uint32_t k = 0; fits && k < np; ++k)
                    fits = row[(k + 1) * p.nrun / np].y - row[k * p.nrun / np].y <= cap;
            }
            if (fits) p.split = np;
        }
    }
    // phase-A segmentation: for few source blocks one generation of workgroups per launch, a
    // multiple of the 4096-position super-step, covering the longest block.  A generation is 256
    // workgroups times the x images that fit a CU's 160 KiB of LDS together, at most 2: fp64
    // source blocks (128 KiB) take one per CU, each x block staged once per CU (measured 66-68 ->
    // 64 us against 512 workgroups on cfg4); fp32 ones (64 KiB) two, so that one stages its x block
    // while the other streams (round 6, profiles/r06_fp32_awg_ab.json: phase A 40.0 -> 33.7 us on
    // cfg4_f32 at 512 workgroups; 384 and 768 slower, as round 1 had measured 512 before the
    // packed stream)
    if (e == hipSuccess) {
        std::vector<uint64_t> h((uint64_t)G.P + 1);
        e = hipMemcpy(h.data(), p.aoff, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
        uint64_t mx = 0;
        for (uint32_t a = 0; a < G.P; ++a) mx = h[a + 1] - h[a] > mx ? h[a + 1] - h[a] : mx;
        // With more source blocks than CUs (cfg5-sized graphs: several generations anyway), shorter
        // workgroups of about 48 Ki deliveries measured faster: cfg5 phase A 2525 -> 2085 us at 6
        // segments per block (profiles/r01_s38_cfg5_awg.txt).
        const uint64_t fit = (160ull * 1024) / ((uint64_t)sa * (f32 ? 4 : 8) + 1024);
        const uint64_t gen = 256 * (fit >= 2 ? 2 : 1);
        uint64_t want = (gen + G.P - 1) / G.P;
        if (G.P > 256) want = (mx + 49151) / 49152;
        if (const char* v = getenv("ACSIM_BIN_AWG")) {   // phase-A workgroups per launch (sweeps)
            const uint64_t awg = strtoull(v, nullptr, 10);
            if (awg) want = (awg + G.P - 1) / G.P;
        }
        if (want == 0) want = 1;
        uint64_t ch = (mx + want - 1) / want;
        ch = ch < 8192 ? 8192 : ch;
        p.chunk = (uint32_t)((ch + 4095) / 4096 * 4096);
        p.segs = (uint32_t)((mx + p.chunk - 1) / p.chunk);
        if (p.segs == 0) p.segs = 1;
    }
    // narrow plans: every block's u32 image must fit the phase-B LDS of its instantiation (the
    // one- or two-pass kernel's buffer, in u32 entries), and the 8-byte rounds take one or two passes
    if (e == hipSuccess && nar_req && p.pkA && p.split <= 2) {
        const uint32_t raw_u32 = p.split == 2 ? 2u * (d * sb / 2 + d * sb / 16 + 2u) : 2u * (d * sb + d * sb / 16);
        std::vector<uint2> h(((uint64_t)p.nrun + 1) * G.Q);
        e = hipMemcpy(h.data(), p.tiles, h.size() * sizeof(uint2), hipMemcpyDeviceToHost);
        bool fits = e == hipSuccess;
        for (uint32_t b = 0; fits && b < G.Q; ++b) fits = h[(uint64_t)b * (p.nrun + 1) + p.nrun].y <= raw_u32;
        if (fits) e = hipMalloc(&p.nhdr, sizeof(uint4));
        if (fits && e == hipSuccess) e = hipMemset(p.nhdr, 0, sizeof(uint4));   // width 0: an 8-byte round
        p.narrow = fits && e == hipSuccess;
    }
    if (e == hipSuccess && getenv("ACSIM_BIN_TS")) {   // diagnostic workgroup timestamps
        p.ts_a = (p.P + 7) / 8 * 8 * p.segs;
        p.ts_b = (p.Q + 7) / 8 * 8;
        p.ts_m = p.ngroups;
        e = hipMalloc(&p.ts, 3ull * (p.ts_a + p.ts_b + p.ts_m) * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMemset(p.ts, 0, 3ull * (p.ts_a + p.ts_b + p.ts_m) * sizeof(uint64_t));
    }
    T1.release();
    T2.release();
    return e;
}

// Source blocks above 8192 senders and phase-M images need more than 64 KiB of dynamic LDS.  The
// attribute belongs to the current device, so it is set once per device ordinal (a process may
// drive several devices from several threads).
static hipError_t binned_set_lds_attributes() {
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static hipError_t status[kMaxDev];
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    std::call_once(once[dev], [dev] {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_scatter<double>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 16384 * sizeof(double));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_scatter<float>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 16384 * sizeof(double));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_regroup<double>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (kBinMCap + 2) * sizeof(double));
        if (e == hipSuccess)
            e = hipFuncSetAttribute(reinterpret_cast<const void*>(k_bin_regroup<float>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (kBinMCap + 4) * sizeof(float));
        status[dev] = e;
    });
    return status[dev];
}

// clean phase B in p.split (2..4) passes
#define ACS_BIN_NP_LAUNCH(DD, TT, W, VT_, SRC)                                                         \
    {                                                                                                  \
        if (p.split == 2)                                                                              \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, W, false, VT_, 2>), grid, dim3(kBinSB), 0, s, a, SRC, \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                  \
        else if (p.split == 3)                                                                         \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, W, false, VT_, 3>), grid, dim3(kBinSB), 0, s, a, SRC, \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                  \
        else                                                                                           \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, W, false, VT_, 4>), grid, dim3(kBinSB), 0, s, a, SRC, \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                  \
    }

// ---- receiver blocks other than kBinSB (BinnedPlan::SB): clean plans, t = 5 sort-based rules
// other than W-MSR, d = 32 at 128 receivers and d = 16 at 128 / 512 (fp64 one or two passes, fp32
// one pass).  Each (d, SB) is one more phase-B instantiation, so the set stays small.
bool binned_sb_supported(uint32_t d, uint32_t t, uint32_t rule, uint32_t sb, bool clean_fast) {
    if (sb == kBinSB) return true;
    if (!clean_fast || t != 5 || rule == 4 || rule == 0) return false;
    return (sb == 128 && (d == 16 || d == 32)) || (sb == 512 && d == 16);
}

uint32_t binned_block_size(uint32_t d, uint32_t t, uint32_t rule, bool clean_fast) {
    uint32_t sb = kBinSB;
    if (const char* v = getenv("ACSIM_BIN_SB")) sb = (uint32_t)strtoul(v, nullptr, 10);
    return binned_sb_supported(d, t, rule, sb, clean_fast) ? sb : kBinSB;
}

template <int D, int T, typename VT>
static hipError_t launch_gather_sb(const BinnedPlan& p, const RoundArgs& a, const VT* src, dim3 grid, uint32_t Qc,
                                   uint32_t pol, hipStream_t s) {
    if constexpr (T == 5 && (D == 16 || D == 32)) {
        if (a.rule == 4 || a.rule == 0) return hipErrorNotSupported;
        const uint32_t np = sizeof(VT) == 8 ? p.split : 1u;   // (fp32: one pass, as at kBinSB)
#define ACS_SB_LAUNCH(SB_, NP_)                                                                          \
    hipLaunchKernelGGL((k_bin_gather<D, T, false, false, VT, NP_, false, false, SB_>), grid, dim3(SB_), 0, s, a, \
                       src, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol)
        if (p.SB == 128 && np == 1) {
            ACS_SB_LAUNCH(128, 1);
            return hipGetLastError();
        }
        if constexpr (sizeof(VT) == 8) {
            if (p.SB == 128 && np == 2) {
                ACS_SB_LAUNCH(128, 2);
                return hipGetLastError();
            }
        }
        if constexpr (D == 16) {
            if (p.SB == 512 && np == 1) {
                ACS_SB_LAUNCH(512, 1);
                return hipGetLastError();
            }
            if constexpr (sizeof(VT) == 8) {
                if (p.SB == 512 && np == 2) {
                    ACS_SB_LAUNCH(512, 2);
                    return hipGetLastError();
                }
            }
        }
#undef ACS_SB_LAUNCH
    }
    return hipErrorNotSupported;
}

// Narrow plans: clean, default receiver block, d = 16 / 32, one or two passes
// in the 8-byte rounds (the 4-byte rounds take one).
template <int D, int T>
static hipError_t launch_gather_narrow(const BinnedPlan& p, const RoundArgs& a, const double* src, dim3 grid,
                                       uint32_t Qc, uint32_t pol, hipStream_t s) {
    if constexpr (D == 16 || D == 32) {
        const bool w_ = a.rule == 4;
#define ACS_NAR_LAUNCH(W_, NP_)                                                                                  \
    hipLaunchKernelGGL((k_bin_gather<D, T, W_, false, double, NP_, false, false, (int)kBinSB, true>), grid,         \
                       dim3(kBinSB), 0, s, a, src, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol)
        if (p.split == 1) {
            if (w_)
                ACS_NAR_LAUNCH(true, 1);
            else
                ACS_NAR_LAUNCH(false, 1);
            return hipGetLastError();
        }
        if (p.split == 2) {
            if (w_)
                ACS_NAR_LAUNCH(true, 2);
            else
                ACS_NAR_LAUNCH(false, 2);
            return hipGetLastError();
        }
#undef ACS_NAR_LAUNCH
    }
    return hipErrorNotSupported;
}

hipError_t launch_round_binned(const BinnedPlan& p, const RoundArgs& a0, bool clean, hipStream_t s,
                               const FinalizeArgs* fin, uint32_t phases, SrcSel sel) {
    const FinalizeArgs fa = fin ? *fin : FinalizeArgs{};
    const uint32_t fin_on = fin ? 1u : 0u;
    const uint32_t pol = p.pol;
    if (hipError_t e = binned_set_lds_attributes(); e != hipSuccess) return e;
    const uint32_t nsrc = sel.n ? sel.n : p.P;
    // phase B block range: every partial slot by default (blocks past the plan's Q write neutral
    // partials), or the caller's [qlo, qhi)
    RoundArgs a = a0;
    a.ts = p.ts ? p.ts + 3ull * p.ts_a : nullptr;
    // narrow plans: clean whole rounds only (the chunked partitioned sequence never builds one)
    const bool nar = p.narrow && p.nhdr && clean && !p.var && sel.n == 0 && p.SB == kBinSB;
    if (p.narrow && !nar) return hipErrorInvalidValue;
    a.nhdr = nar ? p.nhdr : nullptr;
    // phase B writes a.partial[b] for each of its receiver blocks b < p.Q (and neutral pairs up to
    // a.nblk): partials sized for fewer blocks would be written past their slice
    if ((phases & 4u) && a.nblk < p.Q) return hipErrorInvalidValue;
    if (p.SB != kBinSB && (!clean || p.var)) return hipErrorInvalidValue;
    const uint32_t nslot_all = a.nblk > p.Q ? a.nblk : p.Q;
    if (a.qhi > nslot_all) a.qhi = nslot_all;
    if (a.qlo >= a.qhi) phases &= ~4u;
    // fault fix-up on whole rounds; chunked partitioned rounds keep the tagged senders
    const bool fixp = !clean && a.status && p.fix && phases == 7 && sel.n == 0 && !a.mp.omit;
    if (p.f32) {   // fp32 plans: one or two levels; tagged senders need N <= 2^20
        float* st1 = reinterpret_cast<float*>(p.stage1);
        const float* fsrc = reinterpret_cast<const float*>(a.xin);
        if (!clean && a.status && !fixp) {
            // the 20-bit id field holds a sender id up to 2^20 nodes, beyond that a crash rank
            if (!p.xtag || (a.N > (1ull << 20) && a.mp.fault == 1 && !a.crank)) return hipErrorInvalidValue;
            float* xt = reinterpret_cast<float*>(p.xtag);
            if (phases & 1)
                hipLaunchKernelGGL(k_bin_tag<float>, dim3((unsigned)((a.N + 511) / 512)), dim3(256), 0, s, fsrc, a.status,
                                   xt, a.N, a.r, a.st, a.crank);
            fsrc = xt;
        }
        if (phases & 1)
            hipLaunchKernelGGL(k_bin_scatter<float>, dim3((nsrc + 7) / 8 * 8 * p.segs), dim3(kBinA), p.SA * sizeof(float), s,
                               fsrc, p.idxA, p.aoff, st1, a.st, a.N, p.SA, p.segs, p.chunk, pol, fa, fin_on, sel, p.ts, a.eacc,
                               p.pkA, nullptr);
        if (p.levels == 2) {
            float* st2 = reinterpret_cast<float*>(p.stage2);
            if (phases & 2)
                hipLaunchKernelGGL(k_bin_regroup<float>, dim3(p.ngroups), dim3(kBinA), (p.mcap + 4) * sizeof(float), s, st1,
                                   p.mt, p.moff, p.idxM, st2, a.st, p.PK, pol,
                                   p.ts ? p.ts + 3ull * (p.ts_a + p.ts_b) : nullptr);
            st1 = st2;   // phase B reads the regrouped stage
        }
        if (fixp)
            hipLaunchKernelGGL(k_bin_fixup<float>, dim3((p.nfix + 255) / 256), dim3(256), 0, s, p.fix, p.nfix, a, st1, p.D);
        if (!(phases & 4)) return hipGetLastError();
        const uint32_t Qc = (a.qhi - a.qlo + 7) / 8;
        const dim3 grid(8 * Qc);
#define X(DD, TT)                                                                                        \
    if (p.D == DD && a.trim == TT) {                                                                     \
        if (p.SB != kBinSB) return launch_gather_sb<DD, TT, float>(p, a, st1, grid, Qc, pol, s);          \
        if (fixp && a.rule == 4)                                                                         \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, false, float, 1, false, true>), grid, dim3(kBinSB), 0, \
                               s, a, st1, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                           \
        else if (fixp)                                                                                   \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, false, float, 1, false, true>), grid, dim3(kBinSB), 0, \
                               s, a, st1, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                           \
        else if (!clean && a.rule == 4)                                                                  \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, true, float>), grid, dim3(kBinSB), 0, s, a, st1,  \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                      \
        else if (!clean)                                                                                 \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, true, float>), grid, dim3(kBinSB), 0, s, a, st1, \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                      \
        else if (p.split > 1 && a.rule == 4)                                                             \
            ACS_BIN_NP_LAUNCH(DD, TT, true, float, st1)                                                  \
        else if (p.split > 1)                                                                            \
            ACS_BIN_NP_LAUNCH(DD, TT, false, float, st1)                                                 \
        else if (a.rule == 4)                                                                            \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, false, float>), grid, dim3(kBinSB), 0, s, a, st1, \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                      \
        else                                                                                             \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, false, float>), grid, dim3(kBinSB), 0, s, a, st1, \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                      \
        return hipGetLastError();                                                                        \
    }
        ACS_BINNED_VARIANTS(X)
#undef X
        return hipErrorNotSupported;
    }
    const double* src = a.xin;
    if (!clean && a.status && !fixp) {
        if (!p.xtag) return hipErrorInvalidValue;
        if (phases & 1)
            hipLaunchKernelGGL(k_bin_tag<double>, dim3((unsigned)((a.N + 511) / 512)), dim3(256), 0, s, a.xin, a.status,
                               p.xtag, a.N, a.r, a.st, nullptr);
        src = p.xtag;
    }
    if (phases & 1)
        hipLaunchKernelGGL(k_bin_scatter<double>, dim3((nsrc + 7) / 8 * 8 * p.segs), dim3(kBinA), p.SA * sizeof(double), s, src,
                           p.idxA, p.aoff, p.stage1, a.st, a.N, p.SA, p.segs, p.chunk, pol, fa, fin_on, sel, p.ts, a.eacc,
                           p.pkA, nar ? p.nhdr : nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const double* last = p.stage1;
    if (p.levels == 2) {
        if (phases & 2)
            hipLaunchKernelGGL(k_bin_regroup<double>, dim3(p.ngroups), dim3(kBinA), (p.mcap + 2) * sizeof(double), s,
                               p.stage1, p.mt, p.moff, p.idxM, p.stage2, a.st, p.PK, pol,
                               p.ts ? p.ts + 3ull * (p.ts_a + p.ts_b) : nullptr);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        last = p.stage2;
    }
    if (fixp)
        hipLaunchKernelGGL(k_bin_fixup<double>, dim3((p.nfix + 255) / 256), dim3(256), 0, s, p.fix, p.nfix, a,
                           const_cast<double*>(last), p.D);
    if (!(phases & 4)) return hipGetLastError();
    const uint32_t Qc = (a.qhi - a.qlo + 7) / 8;
    const dim3 grid(8 * Qc);
#define X(DD, TT)                                                                                        \
    if (p.D == DD && a.trim == TT) {                                                                     \
        if (nar) return launch_gather_narrow<DD, TT>(p, a, last, grid, Qc, pol, s);                      \
        if (p.SB != kBinSB) return launch_gather_sb<DD, TT, double>(p, a, last, grid, Qc, pol, s);       \
        const bool w_ = a.rule == 4;                                                                     \
        if (p.var && clean && w_)                                                                        \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, false, double, 1, true>), grid, dim3(kBinSB), 0, s, \
                               a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                             \
        else if (p.var && clean)                                                                         \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, false, double, 1, true>), grid, dim3(kBinSB), 0, s, \
                               a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                             \
        else if (fixp && p.var && w_)                                                                    \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, false, double, 1, true, true>), grid, dim3(kBinSB), 0, \
                               s, a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                          \
        else if (fixp && p.var)                                                                          \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, false, double, 1, true, true>), grid, dim3(kBinSB), 0, \
                               s, a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                          \
        else if (fixp && p.split == 2 && w_)                                                             \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, false, double, 2, false, true>), grid, dim3(kBinSB), 0, \
                               s, a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                          \
        else if (fixp && p.split == 2)                                                                   \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, false, double, 2, false, true>), grid, dim3(kBinSB), 0, \
                               s, a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                          \
        else if (fixp && w_)                                                                             \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, false, double, 1, false, true>), grid, dim3(kBinSB), 0, \
                               s, a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                          \
        else if (fixp)                                                                                   \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, false, double, 1, false, true>), grid, dim3(kBinSB), 0, \
                               s, a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                          \
        else if (p.var && w_)                                                                            \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, true, double, 1, true>), grid, dim3(kBinSB), 0, s, \
                               a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                             \
        else if (p.var)                                                                                  \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, true, double, 1, true>), grid, dim3(kBinSB), 0, s, \
                               a, last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                             \
        else if (clean && p.split > 1 && w_)                                                             \
            ACS_BIN_NP_LAUNCH(DD, TT, true, double, last)                                                \
        else if (clean && p.split > 1)                                                                   \
            ACS_BIN_NP_LAUNCH(DD, TT, false, double, last)                                               \
        else if (clean && w_)                                                                            \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true>), grid, dim3(kBinSB), 0, s, a, last, p.invpos,   \
                               p.tiles, p.nrun, p.Q, Qc, pol);                                                \
        else if (clean)                                                                                  \
            hipLaunchKernelGGL((k_bin_gather<DD, TT>), grid, dim3(kBinSB), 0, s, a, last, p.invpos, p.tiles, \
                               p.nrun, p.Q, Qc, pol);                                                         \
        else if (p.split == 2 && w_)   /* faulty: two passes only */                                     \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, true, double, 2>), grid, dim3(kBinSB), 0, s, a,  \
                               last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                \
        else if (p.split == 2)                                                                           \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, true, double, 2>), grid, dim3(kBinSB), 0, s, a, \
                               last, p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                \
        else if (w_)                                                                                     \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, true, true>), grid, dim3(kBinSB), 0, s, a, last,       \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                      \
        else                                                                                             \
            hipLaunchKernelGGL((k_bin_gather<DD, TT, false, true>), grid, dim3(kBinSB), 0, s, a, last,      \
                               p.invpos, p.tiles, p.nrun, p.Q, Qc, pol);                                      \
        return hipGetLastError();                                                                        \
    }
    ACS_BINNED_VARIANTS(X)
#undef X
    return hipErrorNotSupported;
}

}  // namespace acs
