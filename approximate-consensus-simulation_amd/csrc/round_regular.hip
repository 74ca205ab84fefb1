// round_regular.hip — the headline hot-path kernel (SURVEY §8(a) a5+a7+a8+a9, cfg4/cfg5).
//
// One lane = one receiver i of a RANDOM_REGULAR graph with a compile-time degree D and trim T.
// Per lane and round:
//   - D/4 coalesced 16-byte loads of neighbour ids (the wave reads 1 KiB contiguous per group);
//   - D random 8-byte gathers of x_j (issued together: D loads in flight per lane);
//   - [faults/loss only] status gathers, one Philox call per 4 slots for the drop mask (§A.5),
//     crash / Byzantine resolution (§A.4, §A.6);
//   - a compile-time selection network over the m = D+1 entries kept in VGPRs (§A.7; only the
//     comparators that reach the window [T, m-T) survive pruning);
//   - the rule (tree sum in the §A.7 order + IEEE divide, or the midpoint), one 8-byte store;
//   - honest (min, max) of x^{r+1} reduced per block -> one partial (§A.8 epilogue).
// Algorithmic traffic (no faults, no loss): 4D + 8D + 8 + 8 bytes per node-round (400 B at
// D = 32).  Everything is bit-exact with the spec: no FMA (-ffp-contract=off), IEEE division.
#include "resolve.hpp"
#include "rules.hpp"

namespace acs {

// VT = double, or float in fp32 mode (4-byte gathers, binary32 rule arithmetic).
// VAR: a CSR graph (§8(f) row 1) padded to D (SELL-64: column groups past the slice's widest row
// are not loaded; columns past deg(i) are absent entries; slot s = rowptr[i] + t, one draw per
// slot).  VAR kernels always take the resolving (non-CLEAN) body.
template <int D, int T, bool CLEAN, bool WMSR = false, typename VT = double, bool VAR = false>
__global__ __launch_bounds__(kRegularBlock) void k_round_regular(const RoundArgs a) {
    static_assert(D % 4 == 0, "compiled degrees are multiples of 4");
    constexpr int M = D + 1;
    constexpr int NQ = D / 4;
    const uint32_t lb = blockIdx.y;
    InstState* S = a.st + lb;
    if (S->done) return;  // device-side early exit (uniform per block)

    const uint64_t N = a.N;
    const VT* __restrict__ x = reinterpret_cast<const VT*>(a.xin) + lb * N;
    VT* __restrict__ xo = reinterpret_cast<VT*>(a.xout) + lb * N;
    const uint32_t li = blockIdx.x * kRegularBlock + threadIdx.x;   // local row (ELL row)
    const uint32_t i = (uint32_t)a.row0 + li;                        // global receiver id

    double mn = kInf, mx = -kInf;   // exact for binary32 values too
    if (li < a.nrows && i < N && !(VAR && a.deg[i] == kDegHub)) {   // (CSR hub rows: the generic kernel)
        const VT xi = x[i];
        VT res = xi;
        bool honest = true, active = true;
        const uint32_t* stv = nullptr;   // null: loss only, no fault schedule
        if constexpr (!CLEAN) {
            if (a.status) {
                stv = a.status + lb * N;
                const uint32_t si = stv[i];
                honest = si == kHonest;
                active = is_active(si, a.r);
            }
        }
        if (active) {
            const uint4* cp = reinterpret_cast<const uint4*>(a.ell) +
                              (uint64_t)(li >> 6) * (NQ * 64) + (li & 63);
            uint32_t col[D];
            uint32_t nqs = NQ, dg = D;
            uint64_t rp = 0;
            if constexpr (VAR) {
                nqs = a.sw[li >> 6];   // uniform over the wave (one 64-row slice)
                dg = a.deg[i];
                rp = a.rowptr[i];
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const uint4 c = (!VAR || (uint32_t)q < nqs) ? cp[q * 64] : make_uint4(kEllNone, kEllNone, kEllNone, kEllNone);
                col[4 * q + 0] = c.x;
                col[4 * q + 1] = c.y;
                col[4 * q + 2] = c.z;
                col[4 * q + 3] = c.w;
            }
            VT v[M];
            v[0] = xi;
            uint32_t nmiss = 0;   // entries left out under missing_policy = OMIT
            if constexpr (CLEAN) {
#pragma unroll
                for (int t = 0; t < D; ++t) v[1 + t] = x[col[t]];
            } else {
                const MsgParams& mp = a.mp;
                const uint32_t b = (uint32_t)(mp.inst_offset + lb);
                const uint32_t bG = b - b % mp.mask_group;
                const VT lo = (VT)S->lo, hi = (VT)S->hi;
                const uint32_t r = a.r;
                VT xj[D];
                uint32_t sj[D];
                // all gathers first, unconditionally (the branch is uniform and hoisted)
                if constexpr (VAR) {   // CSR: absent columns load nothing (their entries are filled below)
#pragma unroll
                    for (int t = 0; t < D; ++t) {
                        const bool ok = (uint32_t)t < dg;
                        const uint32_t j = ok ? col[t] : i;
                        if (a.delay)
                            xj[t] = ok ? delayed_x<VT>(a, lb, r, draw(mp.key, kStreamDelay, b, r, rp + t), j) : xi;
                        else
                            xj[t] = ok ? x[j] : xi;
                        sj[t] = (ok && stv) ? stv[j] : kHonest;
                    }
                } else if (a.delay) {   // bounded delay: one DELAY Philox call per 4 slots, history gathers
#pragma unroll
                    for (int q = 0; q < NQ; ++q) {
                        const U4 wd = philox10(i * (uint32_t)NQ + q, r, b, kStreamDelay, mp.key);
#pragma unroll
                        for (int e = 0; e < 4; ++e) {
                            const int t = 4 * q + e;
                            xj[t] = delayed_x<VT>(a, lb, r, wd.v[e], col[t]);
                            sj[t] = stv ? stv[col[t]] : kHonest;
                        }
                    }
                } else if (stv) {
#pragma unroll
                    for (int t = 0; t < D; ++t) {
                        xj[t] = x[col[t]];
                        sj[t] = stv[col[t]];
                    }
                } else {
#pragma unroll
                    for (int t = 0; t < D; ++t) {
                        xj[t] = x[col[t]];
                        sj[t] = kHonest;
                    }
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    // slots s = i*D + 4q .. +3 share Philox counter s>>2 = i*(D/4) + q (§A.5); CSR
                    // slots rowptr[i] + t are not 4-aligned: one draw each
                    U4 w;
                    w.v[0] = w.v[1] = w.v[2] = w.v[3] = 0xFFFFFFFFu;
                    if (!VAR && mp.thr) w = philox10(i * (uint32_t)NQ + q, r, bG, kStreamDrop, mp.key);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int t = 4 * q + e;
                        const uint64_t s = VAR ? rp + t : (uint64_t)i * D + t;
                        if (VAR && (uint32_t)t >= dg) {   // absent entry (not in S_i at all)
                            v[1 + t] = omit_fill<VT>(a.rule);
                            ++nmiss;
                            continue;
                        }
                        const bool dropped = VAR ? (mp.thr && draw(mp.key, kStreamDrop, bG, r, s) < mp.thr)
                                                 : w.v[e] < mp.thr;
                        bool miss;
                        const VT u = resolve_entry_m(mp, sj[t], xj[t], xi, dropped, b, r, i, s, lo, hi, miss);
                        const bool out = mp.omit && miss;
                        v[1 + t] = out ? omit_fill<VT>(a.rule) : u;
                        nmiss += out;
                    }
                }
            }
            if (!CLEAN && (VAR || a.mp.omit))
                res = apply_rule_reg_omit<D, T, WMSR>(a.rule, v, nmiss);
            else
                res = apply_rule_reg<D, T, WMSR>(a.rule, v);
        }
        xo[i] = res;
        if (honest) {
            mn = res;
            mx = res;
        }
    }
    block_minmax_store<kRegularBlock>(mn, mx, a.partial + (uint64_t)lb * a.nblk + blockIdx.x);
}

template <int D, int T, typename VT>
static void launch_regular_t(const RoundArgs& a, dim3 grid, dim3 block, bool clean, hipStream_t s) {
    const bool w = a.rule == 4;
    if (a.deg && w)
        hipLaunchKernelGGL((k_round_regular<D, T, false, true, VT, true>), grid, block, 0, s, a);
    else if (a.deg)
        hipLaunchKernelGGL((k_round_regular<D, T, false, false, VT, true>), grid, block, 0, s, a);
    else if (clean && w)
        hipLaunchKernelGGL((k_round_regular<D, T, true, true, VT>), grid, block, 0, s, a);
    else if (clean)
        hipLaunchKernelGGL((k_round_regular<D, T, true, false, VT>), grid, block, 0, s, a);
    else if (w)
        hipLaunchKernelGGL((k_round_regular<D, T, false, true, VT>), grid, block, 0, s, a);
    else
        hipLaunchKernelGGL((k_round_regular<D, T, false, false, VT>), grid, block, 0, s, a);
}

// ---------------------------------------------------------------------------- dispatch
// (D, T) pairs compiled into the register path; anything else uses the generic kernel.
#define ACS_REGULAR_VARIANTS(X) \
    X(4, 0) X(4, 1) X(8, 0) X(8, 2) X(16, 0) X(16, 5) X(32, 0) X(32, 5)

static bool rule_ok(uint32_t t, uint32_t rule) {
    if (rule == 0) return t == 0;     // AVERAGE
    if (rule == 3) return t >= 1;     // DLPSW
    if (rule == 4) return true;       // W-MSR
    return rule == 1 || rule == 2;
}

bool regular_fast_supported(uint32_t d, uint32_t t, uint32_t rule) {
#define X(DD, TT) if (d == DD && t == TT) return rule_ok(t, rule);
    ACS_REGULAR_VARIANTS(X)
#undef X
    return false;
}

const char* regular_fast_name(uint32_t d, uint32_t t, bool clean) {
#define X(DD, TT)                                                                          \
    if (d == DD && t == TT)                                                                \
        return clean ? "k_round_regular<" #DD "," #TT ",clean>" : "k_round_regular<" #DD "," #TT ",faulty>";
    ACS_REGULAR_VARIANTS(X)
#undef X
    return "k_round_regular<?>";
}

hipError_t launch_round_regular(const RoundArgs& a, uint64_t B, bool clean, hipStream_t s) {
    // one block per partial slot: blocks past nrows only write neutral (+inf, -inf) partials, so
    // the finalize can fold every slot of every partition
    const dim3 grid((unsigned)a.nblk, (unsigned)B);
    const dim3 block(kRegularBlock);
#define X(DD, TT)                                                                         \
    if (a.d == DD && a.trim == TT) {                                                      \
        if (a.f32)                                                                        \
            launch_regular_t<DD, TT, float>(a, grid, block, clean, s);                     \
        else                                                                              \
            launch_regular_t<DD, TT, double>(a, grid, block, clean, s);                    \
        return hipGetLastError();                                                         \
    }
    ACS_REGULAR_VARIANTS(X)
#undef X
    return hipErrorNotSupported;
}

}  // namespace acs
