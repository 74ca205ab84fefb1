// round_generic.hip — general-purpose round kernel: one 256-thread workgroup per receiver.
//
// Covers every (topology, m <= 8192, rule, t, fault, loss) combination the register kernels do
// not: the workgroup resolves the m entries (§A.6) into LDS, bitonic-sorts them in LDS padded to
// a power of two with +inf (§A.7; a sort network, so the sorted sequence — and therefore the
// tree sum — is the spec's), then applies the rule with an LDS stride-halving tree sum.
// Used for the dense cfg2 shape (N = 1024 complete, t = 341) and any odd (d, t).
#include <mutex>

#include "resolve.hpp"

namespace acs {

constexpr int kGenericBlock = 256;

template <typename VT>
__device__ __forceinline__ VT block_tree_sum(VT* w, uint32_t P) {
    for (uint32_t s = P >> 1; s >= 1; s >>= 1) {
        for (uint32_t k = threadIdx.x; k < s; k += kGenericBlock) w[k] = w[k] + w[k + s];
        __syncthreads();
    }
    return w[0];
}

template <typename VT>
__device__ __forceinline__ void block_bitonic_sort(VT* v, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t idx = threadIdx.x; idx < P; idx += kGenericBlock) {
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

// VT = double, or float in fp32 mode
template <typename VT>
__global__ __launch_bounds__(kGenericBlock) void k_round_generic(const RoundArgs a, uint32_t P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char sh_raw[];
    VT* sh = reinterpret_cast<VT*>(sh_raw);   // [P] entries + [P] scratch
    const uint32_t lb = blockIdx.y, i = blockIdx.x;
    InstState* S = a.st + lb;
    if (S->done) return;
    const uint64_t N = a.N;
    const VT* __restrict__ x = reinterpret_cast<const VT*>(a.xin) + lb * N;
    VT* __restrict__ xo = reinterpret_cast<VT*>(a.xout) + lb * N;
    const uint32_t* stv = a.status ? a.status + lb * N : nullptr;
    const VT xi = x[i];
    const uint32_t si = stv ? stv[i] : kHonest;
    const bool honest = si == kHonest;
    double2* part = a.partial + (uint64_t)lb * a.nblk + i;
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
    const uint32_t r = a.r;
    uint32_t m = a.m;
    uint64_t rp = 0;
    if (a.topology == 2) {   // CSR: m_i = deg(i) + 1 (a.m is the maximum, which sized P)
        rp = a.rowptr[i];
        m = (uint32_t)(a.rowptr[i + 1] - rp) + 1;
    }
    const VT lo = (VT)S->lo, hi = (VT)S->hi;
    const bool avg = a.rule == 0;
    __shared__ uint32_t nmiss_s;   // entries left out under missing_policy = OMIT
    if (threadIdx.x == 0) nmiss_s = 0;
    __syncthreads();
    uint32_t nmiss = 0;
    for (uint32_t e = threadIdx.x; e < P; e += kGenericBlock) {
        VT v;
        if (e >= m) {
            v = avg ? VT(0) : (VT)kInf;
        } else {
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
            if (self) {
                v = xi;
            } else {
                const uint32_t stj = stv ? stv[j] : kHonest;
                const bool dropped = mp.thr && draw(mp.key, kStreamDrop, bG, r, slot) < mp.thr;
                const VT xj = a.delay ? delayed_x<VT>(a, lb, r, draw(mp.key, kStreamDelay, b, r, slot), j) : x[j];
                bool miss;
                v = resolve_entry_m(mp, stj, xj, xi, dropped, b, r, i, slot, lo, hi, miss);
                if (mp.omit && miss) {
                    v = omit_fill<VT>(a.rule);
                    ++nmiss;
                }
            }
        }
        sh[e] = v;
    }
    if (nmiss) atomicAdd(&nmiss_s, nmiss);
    __syncthreads();
    m -= nmiss_s;   // m' = present entries (OMIT); the fillers sort past them (+inf) or add +0.0
    VT res;
    if (avg) {
        res = block_tree_sum(sh, P) / (VT)m;
    } else if (a.rule != 4 && m <= 2 * a.trim) {   // OMIT: too few entries to trim, keep x_i
        res = xi;
    } else {
        block_bitonic_sort(sh, P);
        const uint32_t t = a.trim, nr = m - 2 * t;
        if (a.rule == 4) {   // W-MSR: window [min(t, #below), m - min(t, #above))
            uint32_t nl = 0, nle = 0;   // #entries < xi, #entries <= xi (sh is sorted)
            {
                uint32_t lo_ = 0, hi_ = m;
                while (lo_ < hi_) { const uint32_t md = (lo_ + hi_) >> 1; if (sh[md] < xi) lo_ = md + 1; else hi_ = md; }
                nl = lo_;
                hi_ = m;
                while (lo_ < hi_) { const uint32_t md = (lo_ + hi_) >> 1; if (sh[md] <= xi) lo_ = md + 1; else hi_ = md; }
                nle = lo_;
            }
            const uint32_t ng = m - nle;
            const uint32_t wlo = nl < t ? nl : t, whi = ng < t ? ng : t, cnt = m - wlo - whi;
            uint32_t P2 = 1;
            while (P2 < cnt) P2 <<= 1;
            VT* w = sh + P;
            for (uint32_t k = threadIdx.x; k < P2; k += kGenericBlock) w[k] = k < cnt ? sh[wlo + k] : VT(0);
            __syncthreads();
            res = block_tree_sum(w, P2) / (VT)cnt;
        } else if (a.rule == 2) {
            res = (sh[t] + sh[m - t - 1]) * VT(0.5);
        } else {
            const uint32_t step = a.rule == 3 ? t : 1;
            const uint32_t cnt = a.rule == 3 ? (nr + t - 1) / t : nr;
            uint32_t P2 = 1;
            while (P2 < cnt) P2 <<= 1;
            VT* w = sh + P;
            for (uint32_t k = threadIdx.x; k < P2; k += kGenericBlock) w[k] = k < cnt ? sh[t + k * step] : VT(0);
            __syncthreads();
            res = block_tree_sum(w, P2) / (VT)cnt;
        }
    }
    if (threadIdx.x == 0) {
        xo[i] = res;
        *part = honest ? make_double2((double)res, (double)res) : make_double2(kInf, -kInf);
    }
}

hipError_t launch_round_generic(const RoundArgs& a, uint64_t B, hipStream_t s) {
    uint32_t P = 1;
    while (P < a.m) P <<= 1;
    if (P > kGenericMaxM) return hipErrorNotSupported;
    const size_t lds = 2 * (size_t)P * (a.f32 ? sizeof(float) : sizeof(double));
    {   // > 64 KiB of dynamic LDS: the attribute is per device, set once per device ordinal
        constexpr int kMaxDev = 64;
        static std::once_flag once[kMaxDev];
        static hipError_t status[kMaxDev];
        int dev = 0;
        if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
        std::call_once(once[dev], [dev] {
            status[dev] = hipFuncSetAttribute((const void*)k_round_generic<double>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize,
                                              (int)(2 * kGenericMaxM * sizeof(double)));
        });
        if (status[dev] != hipSuccess) return status[dev];
    }
    const dim3 grid((unsigned)a.N, (unsigned)B);
    if (a.f32)
        hipLaunchKernelGGL(k_round_generic<float>, grid, dim3(kGenericBlock), lds, s, a, P);
    else
        hipLaunchKernelGGL(k_round_generic<double>, grid, dim3(kGenericBlock), lds, s, a, P);
    return hipGetLastError();
}

}  // namespace acs
