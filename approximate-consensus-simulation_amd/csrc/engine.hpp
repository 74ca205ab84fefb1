// engine.hpp — device-resident state and kernel launch interface of the round engine.
//
// HBM layout (per handle, one GPU):
//   x[2]      : two fp64 buffers [B][N]; instance b at round r lives in x[r & 1] (Jacobi
//               double buffer, never read and written in the same launch)
//   ell       : RANDOM_REGULAR adjacency as column-major 64-row slices of 4-wide column
//               groups, u32 [ceil(N/64)][Dp/4][64][4] (Dp = d rounded up to 4): lane l of a
//               wave loads its 4 neighbour ids of group q with one 16-byte load, and the wave's
//               64 loads are one contiguous 1 KiB line run
//   status    : u32 [B][N] fault status (§A.4), absent when there are no faults
//   st        : InstState [B] — honest lo/hi/spread of the current round, rounds, done flags
//   partial   : double2 [B][nblk] per-block honest (min, max) partials of x^{r+1} (§A.8)
//   trace     : f64 [B][max_rounds+1] optional spread trace
#pragma once

#include <utility>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "spec.hpp"

namespace acs {

struct InstState {
    double lo, hi, spread;  // honest min / max / spread of the current x (§A.8)
    uint32_t rounds;        // rounds executed
    uint32_t done;          // terminated
    uint32_t converged;     // spread <= eps
    uint32_t pad;
};

struct RoundArgs {
    const double* xin;        // x^r, instance-major [B][N]
    double* xout;             // x^{r+1}
    const uint32_t* ell;      // RANDOM_REGULAR adjacency of rows [row0, row0+nrows) (see layout above)
    const uint32_t* status;   // [B][N] or nullptr when there are no faults
    InstState* st;            // [B]
    double2* partial;         // [B][nblk]
    uint64_t N;
    uint64_t row0, nrows;     // receivers handled by this launch (node partition; 0, N otherwise)
    const uint64_t* rowptr;   // CSR topology: [N+1] row offsets (slot of entry 1+t = rowptr[i]+t)
    const uint32_t* colidx;   // CSR topology: [rowptr[N]] sender ids
    uint32_t m;               // entries per receiver
    uint32_t d, dp;           // degree, degree rounded up to 4
    uint32_t topology, rule, trim;
    uint32_t r;               // round being produced: x^r -> x^{r+1}
    uint32_t nblk;            // partial blocks per instance
    MsgParams mp;
    // bounded-delay rounds: x^q lives at xh + (q % H) * xstride (instance-major)
    const double* xh;
    uint64_t xstride;
    uint32_t H, delay;        // delay = D (0: synchronous)
    uint32_t f32;             // ACS_F32: x buffers hold binary32 values
    // CSR graphs on the register / binned paths (§8(f) row 1): the ELL is padded to the compiled
    // degree d with kEllNone; deg[i] = deg(i) (< 256), sw[slice] = 4-wide column groups a 64-row
    // slice actually uses (SELL-64: groups past it are never loaded).  nullptr otherwise.
    const uint8_t* deg;
    const uint8_t* sw;
    // binned phase B: receiver-block range of this launch, [qlo, qhi) (chunked partitioned rounds
    // exchange finished chunks while later ones compute); 0, ~0u = every block
    uint32_t qlo, qhi;
    uint64_t* ts;             // diagnostic per-workgroup timestamps (ACSIM_BIN_TS; nullptr otherwise)
    // generic kernel over a receiver list (CSR hub rows beside a fast path): receiver rid[blockIdx.x],
    // block partial slot pbase + blockIdx.x; nullptr: receiver blockIdx.x, slot = receiver
    const uint32_t* rid;
    uint32_t pbase;
    // fp32 tagged binned plans above 2^20 nodes with crash faults: the binary32 tag of a sender
    // crashing this round carries crank[j], its rank among the round's crashing senders, and
    // phase B reads j = clist[coff + rank] (clist: faulty nodes by crash round; nullptr otherwise)
    const uint32_t* crank;
    const uint32_t* clist;
    uint32_t coff;
    // EPS verdict publication (binned phase B): non-null: every block also folds its
    // (min, max) into eacc[0] = max ~ord(min), eacc[1] = max ord(max) (ord: order-preserving bits,
    // identity 0), so the next phase A's workgroups can stop without the block partials
    unsigned long long* eacc;
    // narrow stage (binned phase B of narrow plans): {base lo, base hi, entry
    // width 4 or 8, 0}, written by this round's phase A (BinnedPlan::nhdr; launch_round_binned sets it)
    const uint4* nhdr;
};
constexpr uint32_t kEaccSlots = 32, kEaccStride = 16;       // eacc pairs, u64 words between pairs
constexpr uint32_t kEaccWords = kEaccSlots * kEaccStride;   // eacc words of one round parity

constexpr uint32_t kEllNone = 0xFFFFFFFFu;   // padding column of a CSR row below the compiled degree
constexpr uint8_t kDegHub = 0xFF;             // deg[] of a CSR hub row (above the compiled degree): the fast
                                              // kernels skip it, the generic kernel serves it

struct FinalizeArgs {
    InstState* st;
    const double2* partial;
    uint32_t nblk;
    uint32_t r_next;          // rounds value after this step (or the resumed round in init mode)
    uint32_t max_rounds;
    uint32_t term_eps;        // 1: EPS termination
    uint32_t f32;             // ACS_F32: spread = binary32(hi - lo)
    double eps;
    double* trace;            // nullptr if disabled
    uint64_t trace_stride;    // max_rounds + 1
    uint32_t* n_done;
    uint32_t init_mode;       // 1: (re)initialisation, ignores the done flag
    uint32_t negmin;          // 1: partial[k].x holds -min (after an all-reduce MAX of (-min, max))
    double2* fold_out;        // non-null: only fold the partials into (-min, max) here (node partition)
    const unsigned long long* eacc;   // binned phase A: the verdict the previous phase B published (or null)
};

struct BatchArgs {
    double* x0;               // buffer 0 [B][N]
    double* x1;               // buffer 1 [B][N]
    const uint32_t* status;   // [B][N] or nullptr
    InstState* st;
    double* trace;
    uint64_t trace_stride;
    uint32_t* n_done;
    uint32_t N, rule, trim, max_rounds, term_eps;
    double eps;
    MsgParams mp;
    uint32_t f32;             // values are binary32 (batched_small.hip only)
};

// ---- setup kernels (setup.hip)
hipError_t launch_init_values(double* x, uint64_t B, uint64_t N, Key key, uint64_t inst_offset, bool f32,
                              hipStream_t s);
hipError_t launch_build_ell(uint32_t* ell, uint64_t N, uint64_t row0, uint64_t nrows, uint32_t d, uint32_t dp,
                            const Feistel& f, hipStream_t s);
// Sort each ELL row ascending (clean configs with order-independent rules only; d in {4,8,16,32}).
hipError_t launch_sort_ell_rows(uint32_t* ell, uint64_t N, uint32_t d, hipStream_t s);
// CSR (§8(f) row 1) -> the padded ELL of width d (a multiple of 4 >= every degree, <= 252), the u8
// degree of every row and the SELL-64 slice widths (4-wide groups per 64-row slice).
hipError_t launch_csr_to_ell(const uint64_t* rowptr, const uint32_t* colidx, uint64_t N, uint32_t d, uint32_t* ell,
                             uint8_t* deg, uint8_t* sw, hipStream_t s);
hipError_t build_fault_status(uint32_t* status, uint64_t B, uint64_t N, uint32_t f,
                              uint32_t fault_model, uint32_t crash_window, Key key,
                              uint64_t inst_offset, hipStream_t s);

// ---- spread / termination (reduce.hip)
hipError_t launch_partials_from_x(const double* x, const uint32_t* status, uint64_t B, uint64_t N,
                                  double2* partial, uint32_t nblk, bool f32, hipStream_t s);
hipError_t launch_finalize(const FinalizeArgs& a, uint64_t B, hipStream_t s);
struct RunSummary {   // acs_run's result, folded on the device (40 bytes)
    unsigned int rounds_max, n_done;   // n_done: instances whose done flag is set
    unsigned long long n_converged, rounds_sum, spread_max_bits;
    unsigned long long seq;            // stored last (system-scope release): the launch's sequence number
};
// acs_run's summary in ONE launch with no copy: block partials, then the last block to arrive folds
// them and stores the summary (with the count of done instances) straight into host-mapped memory
// `out`.  scratch: a device buffer of kSummaryScratch bytes whose first word is zero (the last block
// re-zeroes it).  The summary's fields land before `seq` (a system-scope release store of the
// launch's sequence number), so the host may read them once it sees `seq` without waiting for the
// stream's completion signal.
constexpr uint32_t kSummaryScratch = 1024 * 48 + 64;
// Instance states read back through host-mapped memory (acs_round's info and the state getters on
// handles of at most kMappedStates instances): one small launch copies them and then releases a
// sequence number at system scope, and the host polls that number instead of a device-to-host copy
// and the stream's completion signal.
constexpr uint32_t kMappedStates = 16;
struct MappedStates {
    InstState st[kMappedStates];
    uint32_t n_done, pad;     // the device's count of done instances
    unsigned long long seq;   // stored last (system-scope release)
};
hipError_t launch_states_mapped(const InstState* st, const uint32_t* n_done, uint32_t B, MappedStates* out,
                                unsigned long long seq, hipStream_t s);
hipError_t launch_run_summary_mapped(const InstState* st, uint64_t B, void* scratch, RunSummary* out,
                                     unsigned long long seq, hipStream_t s);

// ---- round kernels
// Register-resident kernel for RANDOM_REGULAR with a compiled (d, t) pair; returns
// hipErrorNotSupported (without launching) when (d, t, rule) has no compiled variant.
bool regular_fast_supported(uint32_t d, uint32_t t, uint32_t rule);
const char* regular_fast_name(uint32_t d, uint32_t t, bool clean);
hipError_t launch_round_regular(const RoundArgs& a, uint64_t B, bool clean, hipStream_t s);
constexpr uint32_t kRegularBlock = 256;

// Binned exchange (round_binned.hip): the one-instance RANDOM_REGULAR round as streaming kernels
// instead of N·d random 8-byte gathers (clean, lossy and faulty configs; no delays).  Deliveries (i <- j) are grouped into
// tiles of (source block of SA senders, receiver group) and stored with tiles padded to even
// lengths.  Phase A (an LDS-resident source block per workgroup) streams stage1[p] = x[src(p)];
// for two-level plans phase M regroups stage1 by receiver block into stage2; phase B (one
// receiver block per workgroup) copies its runs into LDS by LDS-DMA, then every lane reads its d
// values through invpos and applies the rule in registers.
// Receivers per phase-B workgroup (one lane each) is a property of the plan (BinnedPlan::SB), not a
// build constant: the phase-B grid, invpos layout, tiles and the block-partial slots all follow
// it (one partial per receiver block, so a handle sizes its partials by the plan's SB).  kBinSB is
// the default; clean fp64 / fp32 plans of d = 16 / 32 also take 128 (and d = 16 512), by
// ACSIM_BIN_SB or the per-degree default (binned_block_size).
constexpr uint32_t kBinSB = 256;
bool binned_sb_supported(uint32_t d, uint32_t t, uint32_t rule, uint32_t sb, bool clean_fast);
// the phase-B receiver block a plan of degree d would use (ACSIM_BIN_SB, else the default for d)
uint32_t binned_block_size(uint32_t d, uint32_t t, uint32_t rule, bool clean_fast);
struct BinnedPlan {
    uint32_t D = 0, SA = 0, P = 0, Q = 0, levels = 0, PK = 0, ngroups = 0, nrun = 0, mcap = 0;
    uint32_t SB = kBinSB;               // receivers per phase-B workgroup (receiver block)
    bool f32 = false;                   // fp32 plan (float stage, runs padded to 4 elements)
    uint32_t segs = 0, chunk = 0;       // phase-A workgroups per source block, deliveries per workgroup
    uint64_t E = 0;                     // deliveries = local rows * D
    uint64_t Ep1 = 0, Ep2 = 0;          // padded stage lengths
    uint16_t* idxA = nullptr;           // [Ep1] sender index within its source block (0 in pads)
    uint32_t* pkA = nullptr;            // idxA packed to 14 bits (binned_dev.hpp pk14; fp64, SA <= 16384), idxA then freed
    uint16_t* idxM = nullptr;           // [Ep2] position inside the phase-M LDS image (two levels)
    uint16_t* invpos = nullptr;         // [Q][D/8][SB][8]: position of (receiver, slot) in block b's runs
    uint2* tiles = nullptr;             // [Q][nrun+1] (stage start | pad count, element offset in block b's runs)
    bool var = false;                   // CSR rows below the compiled degree (kEllNone columns)
    uint32_t split = 1;                 // phase-B passes over the image (ACSIM_BIN_SPLIT; 1 = whole image)
    uint32_t pol = 0;                   // cache-policy switches (round_binned.hip kPol*)
    uint2* mt = nullptr;                // [ngroups][PK+1] phase-M run tables (two levels)
    uint64_t* aoff = nullptr;           // [P+1] stage1 start of source block a
    uint64_t* moff = nullptr;           // [ngroups+1] stage2 start of phase-M group g
    double* stage1 = nullptr;           // [Ep1]
    double* stage2 = nullptr;           // [Ep2] (two levels)
    double* xtag = nullptr;             // [N+2] tagged sender values (fault schedules only)
    uint64_t* ts = nullptr;             // ACSIM_BIN_TS=<file>: [3 * (ts_a + ts_b + ts_m)] workgroup timestamps of the last round
    uint32_t ts_a = 0, ts_b = 0, ts_m = 0;   // phase-A / phase-B / phase-M workgroups recorded
    // fault fix-up: fix[k] = (last-stage position, local row, slot, sender) of every
    // delivery from a sender that is not honest; nullptr: tagged senders (k_bin_tag) instead
    uint4* fix = nullptr;
    uint32_t nfix = 0;
    // narrow stage (ACSIM_BIN_NARROW=1; clean one-level fp64 plans): a round whose
    // values all lie strictly on one side of zero within 2^32 ulps of each other stages u32 offsets
    // from their base instead of 8-byte values; runs are then padded to 4 entries
    bool narrow = false;
    uint4* nhdr = nullptr;              // the round's {base, width} (phase A writes, phase B reads)
};
bool binned_supported(uint32_t d, uint32_t t, uint32_t rule);
// 1 or 2 exchange levels for NR local receivers of an N-node graph (0: not supported); sb = receiver block.
uint32_t binned_levels(uint64_t N, uint64_t NR, uint32_t d, uint32_t sa, uint32_t sb, uint32_t* sr_out);
// Builds the plan from the ELL of the NR local rows (sorted or spec order; slot-dependent configs
// need spec order); sa = source block size; sb = receiver block (binned_block_size; must satisfy
// binned_sb_supported); tagged: the config has a fault schedule.
// narrow: build a narrow plan where the plan qualifies (p.narrow says whether it did).
hipError_t binned_build(BinnedPlan& p, const uint32_t* ell, uint64_t N, uint64_t NR, uint32_t d, uint32_t dp,
                        uint32_t sa, uint32_t sb, bool tagged, bool f32, hipStream_t s, bool var = false,
                        const uint32_t* status = nullptr, bool clean = false, bool narrow = false);
void binned_free(BinnedPlan& p);
// clean: no slot-dependent decision (selects the plain phase-B instantiation)
// fin: the previous round's finalize, deferred into this round's phase A (nullptr: none pending)
// Source-block selection of a phase-A launch (chunked partitioned rounds): with
// n > 0 only the n blocks a = (u / bpc) * bpr + k0 + u % bpc, u < n, run (chunk k of every rank:
// bpr blocks per rank, bpc per chunk, k0 = k * bpc); n = 0 runs every block.
struct SrcSel {
    uint32_t n, bpr, bpc, k0;
};
// Which phases one launch_round_binned call enqueues: 1 = [tag +] scatter (A), 2 = regroup (M),
// 4 = gather (B, over a.qlo .. a.qhi).  Phase B writes partial slot b of its receiver block b:
// a.nblk must be at least p.Q (hipErrorInvalidValue otherwise, before anything is launched).
hipError_t launch_round_binned(const BinnedPlan& p, const RoundArgs& a, bool clean, hipStream_t s,
                               const FinalizeArgs* fin = nullptr, uint32_t phases = 7, SrcSel sel = SrcSel{});


// Generic kernel: one workgroup per receiver, LDS bitonic sort (any topology, m <= 8192).
constexpr uint32_t kGenericMaxM = 8192;   // receivers with more entries take the big-m path
// nrecv: grid over a.rid's list (0: every receiver); Pcls: the list's size class (0: from a.m)
hipError_t launch_round_generic(const RoundArgs& a, uint64_t B, hipStream_t s, uint64_t nrecv = 0, uint32_t Pcls = 0);
// big-m path (round_generic.hip): receivers with kGenericMaxM < m_i <= kGenericBigMaxM, entries
// in global scratch (batches of at most kGenericBigCap entries), a per-receiver merge sort, rule.
// kGenericBigMaxM keeps every sum of admitted values (|x| <= 1e300) finite.
constexpr uint64_t kGenericBigMaxM = 1ull << 27;
constexpr uint64_t kGenericBigCap = 1ull << 27;
struct GenericBig {
    uint64_t n = 0, cap = 0;                 // receivers on the path, scratch entries per batch
    uint64_t pbase = ~0ull;                  // partial slot of ids[k]: pbase + k (~0: the receiver id)
    bool f32 = false;
    uint32_t* ids = nullptr;                 // [n] receiver ids
    uint64_t* eoff = nullptr;                // [n+1] segment offsets (device)
    std::vector<uint64_t> h_eoff;            // the same on the host (batch bases)
    std::vector<std::pair<uint64_t, uint64_t>> batches;   // [k0, k1) ranges of ids
    void* ent = nullptr;                     // [cap] resolved entries (then tree-sum scratch)
    void* srt = nullptr;                     // [cap] sorted entries
    uint32_t* nmiss = nullptr;               // [max batch] entries left out (OMIT)
};
hipError_t generic_big_build(GenericBig& g, const std::vector<uint32_t>& ids, const std::vector<uint64_t>& m_of,
                             bool f32, hipStream_t s);
void generic_big_free(GenericBig& g);
hipError_t launch_round_generic_big(const GenericBig& g, const RoundArgs& a, uint64_t B, hipStream_t s);

// Dense shared-sort kernels (round_dense.hip): COMPLETE topology, no loss, sort-based rule,
// no crash faults, Byzantine SPLIT/CONSTANT; one instance.
struct DenseArgs {
    const double* x;          // x^r
    double* xo;               // x^{r+1}
    const uint32_t* status;   // [N] or nullptr
    InstState* st;
    double2* partial;         // [dense_nblk(N)]
    double* sorted;           // [N] scratch: sorted base multiset
    uint32_t* counts;         // [3] scratch: |B|, #Byzantine, #crash-silent
    uint32_t N, P, r, rule, trim, byz;
    double delta, bconst;
    uint32_t f32;             // ACS_F32: x, xo and sorted hold binary32 values
};
bool dense_supported(uint32_t fault_model, uint32_t byz, uint32_t rule, uint32_t thr, uint64_t N);
uint32_t dense_nblk(uint64_t N);
hipError_t launch_round_dense(const DenseArgs& a, hipStream_t s);
// Persistent dense variant: one workgroup per instance, x in LDS, k rounds per launch (N <= 4096).
constexpr uint32_t kDensePersistMaxN = 4096;
hipError_t launch_dense_persist(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s);

// Persistent batched kernel: COMPLETE topology with N <= 64, one wavefront per instance,
// state in VGPRs across rounds.
constexpr uint32_t kBatchedMaxN = 64;
// MFMA variant (batched_mfma.hip): AVERAGE, no faults, 16-instance groups sharing drop masks
// (mask_group % 16 == 0); one wavefront per group, Y = W·X by v_mfma_f64_16x16x4_f64 (≤ 1e-12).
bool batched_mfma_supported(uint32_t N, uint32_t rule, bool faults, uint32_t mask_group, uint64_t inst_offset);
hipError_t launch_batched_mfma(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s);
hipError_t launch_batched_small(const BatchArgs& a, uint64_t B, uint32_t k, hipStream_t s);
const char* batched_small_name(uint32_t N, uint32_t rule, bool faults);
// lanes per receiver of the clean AVERAGE N = 64 batch (k_batched_split<F>; 1 = k_batched_small)
uint32_t batched_split_factor(uint32_t N, uint32_t rule, bool faults);

}  // namespace acs
