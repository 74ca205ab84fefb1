// batched_mfma.hip — cfg3's "batched W·X averaging on MFMA" (BASELINE.json north star; SURVEY
// §8(a) a12, §A.10 cfg3 G = 16 variant).
//
// When 16 consecutive instances share their drop masks (mask_group G a multiple of 16, §A.5:
// b_G = b − b mod G), one round of AVERAGE for the whole group is a single matrix product
//     Y = W · X,   X = [64 nodes × 16 instances],   W_ij = delivered(j -> i) for j != i,
//                  W_ii = 1 + #missing messages of i   (§A.6 self-substitution; rows sum to N)
// followed by x' = Y / N.  One wavefront per group: lane i builds row i's drop mask (16 Philox
// calls, shared by the 16 instances instead of recomputed per instance), the masks meet in LDS,
// and 4 row tiles × 16 k-steps of v_mfma_f64_16x16x4_f64 form Y.  The accumulator layout of
// tile m (row (lane>>4) + 4·reg, column lane&15) is exactly the B-operand layout of k-step
// 4m + reg, so the next round consumes the result in place: no LDS, no shuffles for X.
//
// Parity: the MFMA sums in hardware order, not §A.7's tree order, so this path matches the oracle
// to ≤ 1e-12 relative (BASELINE.json north star), not bit for bit; rounds-to-convergence must
// still match.  ACSIM_MFMA=0 selects the bit-exact VALU kernel (batched_small.hip) instead.
#include "resolve.hpp"

namespace acs {

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k_batched_mfma(const BatchArgs a, uint32_t kmax, uint32_t B) {
    __shared__ uint64_t miss_s[64];
    const uint32_t lane = threadIdx.x, h = lane >> 4, il = lane & 15;
    const uint32_t N = a.N;
    const MsgParams& mp = a.mp;
    const uint64_t lb = (uint64_t)blockIdx.x * 16 + il;   // this lane's instance (column)
    const bool inst_ok = lb < B;
    InstState* S = a.st + (inst_ok ? lb : 0);
    const uint32_t b0 = (uint32_t)(mp.inst_offset + (uint64_t)blockIdx.x * 16);
    const uint32_t bG = b0 - b0 % mp.mask_group;   // shared by the group (G % 16 == 0, offset % 16 == 0)

    uint32_t r = S->rounds;
    bool done = !inst_ok || S->done;
    double lo = S->lo, hi = S->hi, spread = S->spread;
    bool conv = S->converged != 0;
    // B operands: xb[s] = X[node 4s + h][instance il]
    double xb[16];
    {
        const double* xin = ((r & 1u) ? a.x1 : a.x0) + lb * N;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const uint32_t node = 4 * s + h;
            xb[s] = inst_ok && node < N ? xin[node] : 0.0;
        }
    }
    const double dN = (double)N;   // §A.7 divides by the entry count m = N
    for (uint32_t q = 0; q < kmax; ++q) {
        if (!__any(!done)) break;   // every instance of the group has terminated
        // round of the group's active instances (they advance together)
        uint32_t R = 0;
        {
            uint32_t v = done ? 0u : r;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
                const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
                v = u > v ? u : v;
            }
            R = v;
        }
        // drop mask of row `lane` (§A.5 slot s = i*N + j, counter s >> 2): bit j = message j -> i missing
        uint64_t miss = 0;
        if (mp.thr && lane < N) {
            if ((N & 3u) == 0) {
                miss = drop_mask_n4(lane, N >> 2, R, bG, mp.key, mp.thr);
            } else {
                for (uint32_t j = 0; j < N; ++j)
                    if (draw(mp.key, kStreamDrop, bG, R, (uint64_t)lane * N + j) < mp.thr) miss |= 1ull << j;
            }
            miss &= ~(1ull << lane);
        }
        miss_s[lane] = miss;
        __syncthreads();
        d4 acc[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m] = d4{0.0, 0.0, 0.0, 0.0};
        uint64_t mrow[4];
        double wdiag[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            mrow[m] = miss_s[16 * m + il];
            // §A.6: a missing message is x_i (diagonal weight 1 + #missing); OMIT:
            // it is left out (weight 1) and the row divides by its present count below
            wdiag[m] = mp.omit ? 1.0 : (double)(1 + __builtin_popcountll(mrow[m]));
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const uint32_t j = 4 * s + h;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t i = 16 * m + il;
                const double w = (i >= N || j >= N) ? 0.0 : i == j ? wdiag[m] : (((mrow[m] >> j) & 1ull) ? 0.0 : 1.0);
                acc[m] = __builtin_amdgcn_mfma_f64_16x16x4f64(w, xb[s], acc[m], 0, 0, 0);
            }
        }
        // accumulator (m, reg) holds node 16m + h + 4reg = 4(4m + reg) + h: the B operand of step 4m + reg
        double mn = kInf, mx = -kInf;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int s = 4 * m + g;
                const uint32_t node = 4 * s + h;
                const double cnt = mp.omit && node < N ? (double)(N - __builtin_popcountll(miss_s[node])) : dN;
                const double v = done ? xb[s] : (node < N ? acc[m][g] / cnt : 0.0);
                xb[s] = v;
                if (node < N) {
                    mn = __builtin_fmin(mn, v);
                    mx = __builtin_fmax(mx, v);
                }
            }
        }
        __syncthreads();   // miss_s is rewritten next round
        // per-instance (column) min / max over the 4 lanes holding its 64 nodes
        mn = __builtin_fmin(mn, __shfl_xor(mn, 16, 64));
        mn = __builtin_fmin(mn, __shfl_xor(mn, 32, 64));
        mx = __builtin_fmax(mx, __shfl_xor(mx, 16, 64));
        mx = __builtin_fmax(mx, __shfl_xor(mx, 32, 64));
        if (!done) {
            r += 1;
            lo = mn;
            hi = mx;
            spread = hi - lo;
            if (a.trace && h == 0) a.trace[lb * a.trace_stride + r] = spread;
            conv = spread <= a.eps;
            done = (a.term_eps && conv) || r >= a.max_rounds;
        }
    }
    if (!inst_ok) return;
    double* xout = ((r & 1u) ? a.x1 : a.x0) + lb * N;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const uint32_t node = 4 * s + h;
        if (node < N) xout[node] = xb[s];
    }
    if (h == 0) {
        S->lo = lo;
        S->hi = hi;
        S->spread = spread;
        S->rounds = r;
        S->converged = conv ? 1u : 0u;
        S->done = done ? 1u : 0u;
    }
}

bool batched_mfma_supported(uint32_t N, uint32_t rule, bool faults, uint32_t mask_group, uint64_t inst_offset) {
    return N >= 1 && N <= 64 && rule == 0 && !faults && mask_group % 16 == 0 && inst_offset % 16 == 0;
}

hipError_t launch_batched_mfma(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s) {
    if (a.N < 1 || a.N > 64 || a.rule != 0 || a.status || a.mp.mask_group % 16) return hipErrorNotSupported;
    hipLaunchKernelGGL(k_batched_mfma, dim3((unsigned)((B + 15) / 16)), dim3(64), 0, s, a, k, (uint32_t)B);
    return hipGetLastError();
}

}  // namespace acs
