// round_generic.hip — general-purpose round kernel: one 256-thread workgroup per receiver.
//
// Covers every (topology, m <= 8192, rule, t, fault, loss) combination the register kernels do
// not (receivers with more entries take the big-m path at the end of this file): the workgroup resolves the m entries (§A.6) into LDS, bitonic-sorts them in LDS padded to
// a power of two with +inf (§A.7; a sort network, so the sorted sequence — and therefore the
// tree sum — is the spec's), then applies the rule with an LDS stride-halving tree sum.
// Used for the dense cfg2 shape (N = 1024 complete, t = 341) and any odd (d, t).
#include <cstdlib>
#include <mutex>

#include "resolve.hpp"
#include "sortnet.hpp"

namespace acs {

constexpr int kGenericBlock = 256;

template <int BLK, typename VT>
__device__ __forceinline__ VT block_tree_sum(VT* w, uint32_t P) {
    for (uint32_t s = P >> 1; s >= 1; s >>= 1) {
        for (uint32_t k = threadIdx.x; k < s; k += BLK) w[k] = w[k] + w[k + s];
        __syncthreads();
    }
    return w[0];
}

template <int BLK, typename VT>
__device__ __forceinline__ void block_bitonic_sort(VT* v, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t idx = threadIdx.x; idx < P; idx += BLK) {
                const uint32_t ixj = idx ^ j;
                if (ixj > idx) {
                    const VT p = v[idx], q = v[ixj];
                    const bool up = (idx & k) == 0;
                    if (up ? (q < p) : (p < q)) {
                        v[idx] = q;
                        v[ixj] = p;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// Merge sort of v[0, P) in LDS for 256 <= P <= 8 * BLK (a power of two): runs of 8 sorted in
// registers (19-comparator network), then log2(P / 8) merge-path passes between v and tmp, one
// barrier each (a bitonic network needs log2(P)·(log2(P)+1)/2 barriered passes).  Returns the
// buffer that holds the sorted sequence.  Values are never -0.0 or NaN, so equal values are
// bit-identical and the result is the sorted sequence whatever the tie order.
template <int BLK, typename VT>
__device__ VT* block_merge_sort(VT* v, VT* tmp, uint32_t P) {
    const uint32_t nt = P >> 3, t = threadIdx.x;
    if (t < nt) {
        VT r[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = v[t * 8 + q];
        select_sort<8>(r);
#pragma unroll
        for (int q = 0; q < 8; ++q) v[t * 8 + q] = r[q];
    }
    __syncthreads();
    VT* src = v;
    VT* dst = tmp;
    for (uint32_t w = 8; w < P; w <<= 1) {
        if (t < nt) {
            const uint32_t o0 = t * 8, s0 = o0 & ~(2 * w - 1), d = o0 - s0;
            const VT* A = src + s0;
            const VT* Bv = src + s0 + w;
            // co-rank: the number i of A elements among the pair's first d outputs
            uint32_t lo = d > w ? d - w : 0, hi = d < w ? d : w;
            while (lo < hi) {
                const uint32_t i = (lo + hi) >> 1;
                if (A[i] <= Bv[d - i - 1]) lo = i + 1;
                else hi = i;
            }
            uint32_t i = lo, j = d - lo;
            VT* out = dst + o0;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const bool ta = j >= w || (i < w && A[i] <= Bv[j]);
                out[q] = ta ? A[i] : Bv[j];
                i += ta;
                j += !ta;
            }
        }
        __syncthreads();
        VT* sw = src;
        src = dst;
        dst = sw;
    }
    return src;
}

// Entry e of receiver i (§A.3 topology order, §A.5 drop, §A.4 / §A.6 resolution, bounded delay):
// the value that goes into S_i, or omit_fill with out = true when missing_policy = OMIT leaves it out.
template <typename VT>
__device__ __forceinline__ VT generic_entry(const RoundArgs& a, uint32_t lb, uint32_t b, uint32_t bG, uint32_t i,
                                            uint64_t rp, uint32_t e, const VT* __restrict__ x,
                                            const uint32_t* __restrict__ stv, VT xi, VT lo, VT hi, bool& out) {
    const MsgParams& mp = a.mp;
    const uint64_t N = a.N;
    const uint32_t r = a.r;
    out = false;
    uint32_t j;
    uint64_t slot;
    bool self;
    if (a.topology == 0) {   // COMPLETE: entry j from node j, slot i*N + j
        j = e;
        slot = (uint64_t)i * N + j;
        self = j == i;
    } else if (a.topology == 2) {   // CSR: entry 0 self, entry 1+t from colidx[rp+t]
        self = e == 0;
        j = self ? i : a.colidx[rp + e - 1];
        slot = rp + e - 1;
    } else {                 // RANDOM_REGULAR: entry 0 self, entry 1+t from nbr(i,t)
        self = e == 0;
        const uint32_t t = e - 1;
        j = self ? i : a.ell[(((uint64_t)(i >> 6) * (a.dp >> 2) + (t >> 2)) * 64 + (i & 63)) * 4 + (t & 3)];
        slot = (uint64_t)i * a.d + t;
    }
    if (self) return xi;
    const uint32_t stj = stv ? stv[j] : kHonest;
    const bool dropped = mp.thr && draw(mp.key, kStreamDrop, bG, r, slot) < mp.thr;
    const VT xj = a.delay ? delayed_x<VT>(a, lb, r, draw(mp.key, kStreamDelay, b, r, slot), j) : x[j];
    bool miss;
    const VT v = resolve_entry_m(mp, stj, xj, xi, dropped, b, r, i, slot, lo, hi, miss);
    if (mp.omit && miss) {
        out = true;
        return omit_fill<VT>(a.rule);
    }
    return v;
}

// VT = double, or float in fp32 mode
// BLK threads per workgroup: 64 for receivers of at most 512 entries (one wave), 1024 above 2048
// entries (the serial sort passes of one receiver are the kernel's tail), 256 otherwise.
template <int BLK, typename VT>
__global__ __launch_bounds__(BLK) void k_round_generic(const RoundArgs a, uint32_t Pmax) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sh_raw[];
    VT* sh = reinterpret_cast<VT*>(sh_raw);   // [Pmax] entries + [Pmax] scratch
    const uint32_t lb = blockIdx.y, i = a.rid ? a.rid[blockIdx.x] : blockIdx.x;
    InstState* S = a.st + lb;
    if (S->done) return;
    const uint64_t N = a.N;
    const VT* __restrict__ x = reinterpret_cast<const VT*>(a.xin) + lb * N;
    VT* __restrict__ xo = reinterpret_cast<VT*>(a.xout) + lb * N;
    const uint32_t* stv = a.status ? a.status + lb * N : nullptr;
    const VT xi = x[i];
    const uint32_t si = stv ? stv[i] : kHonest;
    const bool honest = si == kHonest;
    double2* part = a.partial + (uint64_t)lb * a.nblk + (a.rid ? a.pbase + blockIdx.x : i);
    if (!is_active(si, a.r)) {   // Byzantine or crashed: value frozen (§A.6); never honest
        if (threadIdx.x == 0) {
            xo[i] = xi;
            *part = make_double2(kInf, -kInf);
        }
        return;
    }
    const MsgParams& mp = a.mp;
    const uint32_t b = (uint32_t)(mp.inst_offset + lb);
    const uint32_t bG = b - b % mp.mask_group;
    uint32_t m = a.m;
    uint64_t rp = 0;
    if (a.topology == 2) {   // CSR: m_i = deg(i) + 1 (a.m is the maximum, which sized P)
        rp = a.rowptr[i];
        m = (uint32_t)(a.rowptr[i + 1] - rp) + 1;
    }
    if (m > Pmax) return;   // above kGenericMaxM: the big-m path (below) handles this receiver
    // this receiver's power of two (CSR rows differ; the sort is a sort and the +0.0 / +inf padding
    // leaves the tree sum unchanged, so any P >= m gives the spec's result)
    uint32_t P = 1;
    while (P < m) P <<= 1;
    const VT lo = (VT)S->lo, hi = (VT)S->hi;
    const bool avg = a.rule == 0;
    __shared__ uint32_t nmiss_s;   // entries left out under missing_policy = OMIT
    if (threadIdx.x == 0) nmiss_s = 0;
    __syncthreads();
    uint32_t nmiss = 0;
    for (uint32_t e = threadIdx.x; e < P; e += BLK) {
        VT v;
        if (e >= m) {
            v = avg ? VT(0) : (VT)kInf;
        } else {
            bool out;
            v = generic_entry<VT>(a, lb, b, bG, i, rp, e, x, stv, xi, lo, hi, out);
            nmiss += out;
        }
        sh[e] = v;
    }
    if (nmiss) atomicAdd(&nmiss_s, nmiss);
    __syncthreads();
    m -= nmiss_s;   // m' = present entries (OMIT); the fillers sort past them (+inf) or add +0.0
    VT res;
    if (avg) {
        res = block_tree_sum<BLK>(sh, P) / (VT)m;
    } else if (a.rule != 4 && m <= 2 * a.trim) {   // OMIT: too few entries to trim, keep x_i
        res = xi;
    } else {
        // sorted sequence in srt, the other half of the LDS buffer is the window's scratch
        VT* srt = sh;
        if (P >= 256 && P <= 8u * BLK)
            srt = block_merge_sort<BLK>(sh, sh + P, P);
        else
            block_bitonic_sort<BLK>(sh, P);
        VT* wbuf = srt == sh ? sh + P : sh;
        const uint32_t t = a.trim, nr = m - 2 * t;
        if (a.rule == 4) {   // W-MSR: window [min(t, #below), m - min(t, #above))
            uint32_t nl = 0, nle = 0;   // #entries < xi, #entries <= xi (srt is sorted)
            {
                uint32_t lo_ = 0, hi_ = m;
                while (lo_ < hi_) { const uint32_t md = (lo_ + hi_) >> 1; if (srt[md] < xi) lo_ = md + 1; else hi_ = md; }
                nl = lo_;
                hi_ = m;
                while (lo_ < hi_) { const uint32_t md = (lo_ + hi_) >> 1; if (srt[md] <= xi) lo_ = md + 1; else hi_ = md; }
                nle = lo_;
            }
            const uint32_t ng = m - nle;
            const uint32_t wlo = nl < t ? nl : t, whi = ng < t ? ng : t, cnt = m - wlo - whi;
            uint32_t P2 = 1;
            while (P2 < cnt) P2 <<= 1;
            VT* w = wbuf;
            for (uint32_t k = threadIdx.x; k < P2; k += BLK) w[k] = k < cnt ? srt[wlo + k] : VT(0);
            __syncthreads();
            res = block_tree_sum<BLK>(w, P2) / (VT)cnt;
        } else if (a.rule == 2) {
            res = (srt[t] + srt[m - t - 1]) * VT(0.5);
        } else {
            const uint32_t step = a.rule == 3 ? t : 1;
            const uint32_t cnt = a.rule == 3 ? (nr + t - 1) / t : nr;
            uint32_t P2 = 1;
            while (P2 < cnt) P2 <<= 1;
            VT* w = wbuf;
            for (uint32_t k = threadIdx.x; k < P2; k += BLK) w[k] = k < cnt ? srt[t + k * step] : VT(0);
            __syncthreads();
            res = block_tree_sum<BLK>(w, P2) / (VT)cnt;
        }
    }
    if (threadIdx.x == 0) {
        xo[i] = res;
        *part = honest ? make_double2((double)res, (double)res) : make_double2(kInf, -kInf);
    }
}


// ------------------------------------------------------------------------------ big m
// Receivers with m_i > kGenericMaxM (complete graphs above 8192 nodes, CSR hubs; m_i <=
// kGenericBigMaxM): the entries go to global scratch, k_big_sort orders each receiver's segment
// (sort-based rules; LDS merge sorts of 8192-entry chunks, then merge-path passes in global
// memory), and one workgroup per receiver applies the rule with the same stride-halving sums in
// global memory.  Receivers are processed in batches of at most
// GenericBig::cap entries; g.ids lists them, g.eoff[k] is the scratch offset of ids[k]'s segment.
template <typename VT>
__device__ __forceinline__ VT big_inst_ptrs(const RoundArgs& a, uint32_t lb, uint32_t i, const VT*& x, VT*& xo,
                                            const uint32_t*& stv, uint32_t& si) {
    x = reinterpret_cast<const VT*>(a.xin) + (uint64_t)lb * a.N;
    xo = reinterpret_cast<VT*>(a.xout) + (uint64_t)lb * a.N;
    stv = a.status ? a.status + (uint64_t)lb * a.N : nullptr;
    si = stv ? stv[i] : kHonest;
    return x[i];
}

template <typename VT>
__global__ __launch_bounds__(kGenericBlock) void k_big_resolve(const RoundArgs a, uint32_t lb,
                                                               const uint32_t* __restrict__ ids,
                                                               const uint64_t* __restrict__ eoff, uint64_t k0,
                                                               VT* __restrict__ ent, uint32_t* __restrict__ nmiss_out) {
    const InstState* S = a.st + lb;
    if (S->done) return;
    const uint64_t k = k0 + blockIdx.x;
    const uint32_t i = ids[k];
    const uint64_t o = eoff[k] - eoff[k0];
    const uint32_t m = (uint32_t)(eoff[k + 1] - eoff[k]);
    const VT* x;
    VT* xo;
    const uint32_t* stv;
    uint32_t si;
    const VT xi = big_inst_ptrs<VT>(a, lb, i, x, xo, stv, si);
    if (!is_active(si, a.r)) return;   // frozen value; the rule kernel writes it
    const uint32_t b = (uint32_t)(a.mp.inst_offset + lb);
    const uint32_t bG = b - b % a.mp.mask_group;
    const uint64_t rp = a.topology == 2 ? a.rowptr[i] : 0;
    const VT lo = (VT)S->lo, hi = (VT)S->hi;
    uint32_t nmiss = 0;
    for (uint32_t e = threadIdx.x; e < m; e += kGenericBlock) {
        bool out;
        ent[o + e] = generic_entry<VT>(a, lb, b, bG, i, rp, e, x, stv, xi, lo, hi, out);
        nmiss += out;
    }
    __shared__ uint32_t nm_s;
    if (threadIdx.x == 0) nm_s = 0;
    __syncthreads();
    if (nmiss) atomicAdd(&nm_s, nmiss);
    __syncthreads();
    if (threadIdx.x == 0) nmiss_out[blockIdx.x] = nm_s;
}

// §A.7 tree_sum of v(q) = q < cnt ? src[off + q*step] : 0 over q < P2 (the next power of two), in
// w (which may alias src when off = 0 and step = 1): the first pass reads src, later passes run in
// place; every pass is the stride-halving pass of the LDS kernels.
template <typename VT>
__device__ VT big_tree_sum(const VT* src, VT* w, uint64_t off, uint64_t step, uint64_t cnt) {
    uint64_t P2 = 1;
    while (P2 < cnt) P2 <<= 1;
    if (P2 == 1) return src[off];
    uint64_t s = P2 >> 1;
    for (uint64_t k = threadIdx.x; k < s; k += kGenericBlock) {
        const VT u = src[off + k * step];
        const VT v = k + s < cnt ? src[off + (k + s) * step] : VT(0);
        w[k] = u + v;
    }
    __syncthreads();
    for (s >>= 1; s >= 1; s >>= 1) {
        for (uint64_t k = threadIdx.x; k < s; k += kGenericBlock) w[k] = w[k] + w[k + s];
        __syncthreads();
    }
    return w[0];
}

template <typename VT>
__global__ __launch_bounds__(kGenericBlock) void k_big_rule(const RoundArgs a, uint32_t lb, const uint32_t* __restrict__ ids,
                                                            const uint64_t* __restrict__ eoff, uint64_t k0,
                                                            const VT* srt, VT* wsp, const uint32_t* __restrict__ nmiss_in,
                                                            uint64_t pbase) {
    const InstState* S = a.st + lb;
    if (S->done) return;
    const uint64_t k = k0 + blockIdx.x;
    const uint32_t i = ids[k];
    const uint64_t o = eoff[k] - eoff[k0];
    const VT* x;
    VT* xo;
    const uint32_t* stv;
    uint32_t si;
    const VT xi = big_inst_ptrs<VT>(a, lb, i, x, xo, stv, si);
    double2* part = a.partial + (uint64_t)lb * a.nblk + (pbase == ~0ull ? (uint64_t)i : pbase + k);
    if (!is_active(si, a.r)) {   // Byzantine or crashed: value frozen (§A.6); never honest
        if (threadIdx.x == 0) {
            xo[i] = xi;
            *part = make_double2(kInf, -kInf);
        }
        return;
    }
    const uint32_t m = (uint32_t)(eoff[k + 1] - eoff[k]) - nmiss_in[blockIdx.x];   // m' (OMIT)
    const VT* v = srt + o;
    VT* w = wsp + o;
    const uint32_t t = a.trim;
    VT res;
    if (a.rule == 0) {
        res = big_tree_sum<VT>(v, w, 0, 1, (uint64_t)(eoff[k + 1] - eoff[k])) / (VT)m;   // fillers add +0.0
    } else if (a.rule != 4 && m <= 2 * t) {   // OMIT: too few entries to trim, keep x_i
        res = xi;
    } else if (a.rule == 4) {   // W-MSR
        uint32_t lo_ = 0, hi_ = m;
        while (lo_ < hi_) { const uint32_t md = (lo_ + hi_) >> 1; if (v[md] < xi) lo_ = md + 1; else hi_ = md; }
        const uint32_t nl = lo_;
        hi_ = m;
        while (lo_ < hi_) { const uint32_t md = (lo_ + hi_) >> 1; if (v[md] <= xi) lo_ = md + 1; else hi_ = md; }
        const uint32_t ng = m - lo_;
        const uint32_t wlo = nl < t ? nl : t, whi = ng < t ? ng : t, cnt = m - wlo - whi;
        res = big_tree_sum<VT>(v, w, wlo, 1, cnt) / (VT)cnt;
    } else if (a.rule == 2) {
        res = (v[t] + v[m - t - 1]) * VT(0.5);
    } else {
        const uint32_t nr = m - 2 * t;
        const uint32_t step = a.rule == 3 ? t : 1;
        const uint32_t cnt = a.rule == 3 ? (nr + t - 1) / t : nr;
        res = big_tree_sum<VT>(v, w, t, step, cnt) / (VT)cnt;
    }
    if (threadIdx.x == 0) {
        xo[i] = res;
        *part = si == kHonest ? make_double2((double)res, (double)res) : make_double2(kInf, -kInf);
    }
}

// Sort of each receiver's segment (one 1024-thread workgroup per receiver): chunks of kBigChunk
// entries merge-sorted in LDS (+inf pads drop off the end), then merge-path passes over the
// segment in global memory, ping-ponging between ent and srt so the result lands in srt.
constexpr uint32_t kBigChunk = 8192;
constexpr int kBigSortBlk = 1024;

template <typename VT>
__global__ __launch_bounds__(kBigSortBlk) void k_big_sort(const RoundArgs a, uint32_t lb,
                                                          const uint64_t* __restrict__ eoff, uint64_t k0,
                                                          VT* ent, VT* srt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char bs_raw[];
    VT* lv = reinterpret_cast<VT*>(bs_raw);   // [2 * kBigChunk]
    if (a.st[lb].done) return;
    const uint64_t k = k0 + blockIdx.x;
    const uint64_t o = eoff[k] - eoff[k0], m = eoff[k + 1] - eoff[k];
    const uint64_t nch = (m + kBigChunk - 1) / kBigChunk;
    int np = 0;
    while ((1ull << np) < nch) ++np;
    VT* const bufs[2] = {ent + o, srt + o};
    // chunk sorts write buffer (np & 1) ? ent : srt, so that np passes end in srt
    VT* dst = bufs[(np & 1) ? 0 : 1];
    for (uint64_t c = 0; c < nch; ++c) {
        const uint64_t c0 = c * kBigChunk, L = m - c0 < kBigChunk ? m - c0 : kBigChunk;
        uint32_t P = 256;
        while (P < L) P <<= 1;
        for (uint32_t e = threadIdx.x; e < P; e += kBigSortBlk) lv[e] = e < L ? ent[o + c0 + e] : (VT)kInf;
        __syncthreads();
        const VT* sorted = block_merge_sort<kBigSortBlk>(lv, lv + P, P);
        for (uint32_t e = threadIdx.x; e < L; e += kBigSortBlk) dst[c0 + e] = sorted[e];
        __syncthreads();
    }
    // merge passes: runs of w -> 2w over [0, m)
    VT* src = dst;
    dst = src == bufs[0] ? bufs[1] : bufs[0];
    constexpr uint32_t E = 8;
    for (uint64_t w = kBigChunk; w < m; w <<= 1) {
        for (uint64_t o0 = (uint64_t)threadIdx.x * E; o0 < m; o0 += (uint64_t)kBigSortBlk * E) {
            const uint64_t s0 = o0 / (2 * w) * (2 * w), d = o0 - s0;
            const uint64_t la = m - s0 < w ? m - s0 : w;
            const uint64_t lbn = m - s0 > w ? (m - s0 - w < w ? m - s0 - w : w) : 0;
            const VT* A = src + s0;
            const VT* Bv = src + s0 + la;
            uint64_t lo = d > lbn ? d - lbn : 0, hi = d < la ? d : la;
            while (lo < hi) {
                const uint64_t i = (lo + hi) >> 1;
                if (A[i] <= Bv[d - i - 1]) lo = i + 1;
                else hi = i;
            }
            uint64_t i = lo, j = d - lo;
            const uint64_t n = la + lbn - d < E ? la + lbn - d : E;
            for (uint64_t q = 0; q < n; ++q) {
                const bool ta = j >= lbn || (i < la && A[i] <= Bv[j]);
                dst[o0 + q] = ta ? A[i] : Bv[j];
                i += ta;
                j += !ta;
            }
        }
        __syncthreads();
        VT* sw = src;
        src = dst;
        dst = sw;
    }
}


hipError_t generic_big_build(GenericBig& g, const std::vector<uint32_t>& ids, const std::vector<uint64_t>& m_of,
                             bool f32, hipStream_t s) {
    g = GenericBig{};
    if (ids.empty()) return hipSuccess;
    const uint64_t es = f32 ? 4 : 8;
    g.h_eoff.resize(ids.size() + 1);
    g.h_eoff[0] = 0;
    uint64_t mx = 0;
    for (size_t k = 0; k < ids.size(); ++k) {
        g.h_eoff[k + 1] = g.h_eoff[k] + m_of[k];
        mx = m_of[k] > mx ? m_of[k] : mx;
    }
    if (mx > kGenericBigMaxM) return hipErrorNotSupported;
    g.cap = g.h_eoff.back() < kGenericBigCap ? g.h_eoff.back() : kGenericBigCap;
    if (g.cap < mx) g.cap = mx;
    if (const char* v = getenv("ACSIM_BIG_CAP")) {   // tests: several batches on small configs
        const uint64_t c = strtoull(v, nullptr, 10);
        if (c >= mx && c < g.cap) g.cap = c;
    }
    // batches: consecutive receivers whose segments fit cap
    uint64_t maxseg = 0;
    for (uint64_t k0 = 0; k0 < ids.size();) {
        uint64_t k1 = k0 + 1;
        while (k1 < ids.size() && g.h_eoff[k1 + 1] - g.h_eoff[k0] <= g.cap) ++k1;
        g.batches.push_back({k0, k1});
        maxseg = k1 - k0 > maxseg ? k1 - k0 : maxseg;
        k0 = k1;
    }
    g.f32 = f32;
    g.n = ids.size();
    hipError_t e = hipMalloc(&g.ids, ids.size() * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&g.eoff, g.h_eoff.size() * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&g.ent, g.cap * es);
    if (e == hipSuccess) e = hipMalloc(&g.srt, g.cap * es);
    if (e == hipSuccess) e = hipMalloc(&g.nmiss, maxseg * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemcpy(g.ids, ids.data(), ids.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(g.eoff, g.h_eoff.data(), g.h_eoff.size() * sizeof(uint64_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) generic_big_free(g);
    return e;
}

void generic_big_free(GenericBig& g) {
    (void)hipFree(g.ids);
    (void)hipFree(g.eoff);
    (void)hipFree(g.ent);
    (void)hipFree(g.srt);
    (void)hipFree(g.nmiss);
    g = GenericBig{};
}

template <typename VT>
static hipError_t big_round(const GenericBig& g, const RoundArgs& a, uint64_t B, hipStream_t s) {
    VT* ent = reinterpret_cast<VT*>(g.ent);
    VT* srt = reinterpret_cast<VT*>(g.srt);
    const bool sorted = a.rule != 0;
    for (uint64_t lb = 0; lb < B; ++lb) {
        for (const auto& bt : g.batches) {
            const uint64_t k0 = bt.first, nk = bt.second - bt.first;
            hipLaunchKernelGGL(k_big_resolve<VT>, dim3((unsigned)nk), dim3(kGenericBlock), 0, s, a, (uint32_t)lb, g.ids,
                               g.eoff, k0, ent, g.nmiss);
            if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
            if (sorted) {
                hipLaunchKernelGGL(k_big_sort<VT>, dim3((unsigned)nk), dim3(kBigSortBlk), 2 * kBigChunk * sizeof(VT), s, a,
                                   (uint32_t)lb, g.eoff, k0, ent, srt);
                if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
            }
            hipLaunchKernelGGL(k_big_rule<VT>, dim3((unsigned)nk), dim3(kGenericBlock), 0, s, a, (uint32_t)lb, g.ids,
                               g.eoff, k0, sorted ? (const VT*)srt : (const VT*)ent, ent, g.nmiss, g.pbase);
            if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
        }
    }
    return hipSuccess;
}

hipError_t launch_round_generic_big(const GenericBig& g, const RoundArgs& a, uint64_t B, hipStream_t s) {
    if (!g.n) return hipSuccess;
    {   // 128 KiB of dynamic LDS for k_big_sort: the attribute is per device, set once per device ordinal
        constexpr int kMaxDev = 64;
        static std::once_flag once[kMaxDev];
        static hipError_t status[kMaxDev];
        int dev = 0;
        if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
        std::call_once(once[dev], [dev] {
            status[dev] = hipFuncSetAttribute((const void*)k_big_sort<double>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)(2 * kBigChunk * sizeof(double)));
        });
        if (status[dev] != hipSuccess) return status[dev];
    }
    return g.f32 ? big_round<float>(g, a, B, s) : big_round<double>(g, a, B, s);
}

hipError_t launch_round_generic(const RoundArgs& a, uint64_t B, hipStream_t s, uint64_t nrecv, uint32_t Pcls) {
    // receivers above kGenericMaxM entries return at once (the big-m path serves them); Pcls: the
    // size class of a receiver list (every m_i <= Pcls; smaller LDS, more workgroups per CU)
    uint32_t P = 1;
    while (P < a.m && P < kGenericMaxM) P <<= 1;
    if (Pcls && Pcls < P) P = Pcls;
    const size_t lds = 2 * (size_t)P * (a.f32 ? sizeof(float) : sizeof(double));
    {   // > 64 KiB of dynamic LDS: the attribute is per device, set once per device ordinal
        constexpr int kMaxDev = 64;
        static std::once_flag once[kMaxDev];
        static hipError_t status[kMaxDev];
        int dev = 0;
        if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
        std::call_once(once[dev], [dev] {
            const int bytes = (int)(2 * kGenericMaxM * sizeof(double));
            hipError_t e = hipFuncSetAttribute((const void*)k_round_generic<256, double>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void*)k_round_generic<1024, double>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
            status[dev] = e;
        });
        if (status[dev] != hipSuccess) return status[dev];
    }
    const dim3 grid((unsigned)(nrecv ? nrecv : a.N), (unsigned)B);
    const int blk = P <= 512 ? 64 : P <= 2048 ? 256 : 1024;   // (merge sort: P / 8 threads per pass)
#define ACS_GEN_LAUNCH(BB)                                                                                         \
    {                                                                                                              \
        if (a.f32)                                                                                                 \
            hipLaunchKernelGGL((k_round_generic<BB, float>), grid, dim3(BB), lds, s, a, P);                        \
        else                                                                                                       \
            hipLaunchKernelGGL((k_round_generic<BB, double>), grid, dim3(BB), lds, s, a, P);                       \
    }
    if (blk == 64)
        ACS_GEN_LAUNCH(64)
    else if (blk == 1024)
        ACS_GEN_LAUNCH(1024)
    else
        ACS_GEN_LAUNCH(256)
#undef ACS_GEN_LAUNCH
    return hipGetLastError();
}

}  // namespace acs
