// api.hip — C ABI (include/acsim.h) over the HIP round engine: handle lifecycle, HBM buffer
// ownership, kernel-path selection, the round-chunk loop with device-side early exit, node
// partitioning with RCCL (cfg5), and the bench-time kernel event timing.  SURVEY §8(b), §8(e).
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <chrono>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../include/acsim.h"
#include "engine.hpp"

using namespace acs;

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(ACS_EDEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                              \
    } while (0)

#define NCCL_TRY(expr)                                                                    \
    do {                                                                                  \
        ncclResult_t r_ = (expr);                                                         \
        if (r_ != ncclSuccess)                                                            \
            return fail(ACS_ECOMM, "%s failed: %s (%s:%d)", #expr, ncclGetErrorString(r_), \
                        __FILE__, __LINE__);                                              \
    } while (0)

enum Path { PATH_REGULAR = 0, PATH_GENERIC = 1, PATH_BATCHED = 2, PATH_DENSE = 3 };

// CSR plans (and hub rows beside them) share one partial-slot numbering between the binned phase B
// and the per-lane / generic kernels: their receiver blocks must agree.
static_assert(kBinSB == kRegularBlock, "CSR binned plans index partials by kRegularBlock-row blocks");

struct Part {              // one node partition's private copy (virtual partitions only)
    double* x[2] = {nullptr, nullptr};
    uint32_t* ell = nullptr;
    BinnedPlan bin{};
};

struct acs_sim {
    acs_config c{};
    int device = 0;
    hipStream_t stream = nullptr;
    uint64_t N = 0, B = 0, m = 0;
    uint32_t d = 0, dp = 0;
    Path path = PATH_GENERIC;
    bool clean = true;
    bool ell_sorted = false;       // rows stored ascending (clean + order-independent rule)
    bool binned = false;           // PATH_REGULAR served by the binned exchange (round_binned.hip)
    bool defer_fin = false;        // binned, one instance, unpartitioned: a round's finalize runs inside
                                   // the next round's phase A (the last round of a chunk launches it)
    bool fin_pending = false;
    FinalizeArgs fin_args{};
    bool mfma = false;             // PATH_BATCHED served by the MFMA group kernel (batched_mfma.hip)
    bool dense_persist = false;    // PATH_DENSE served by the persistent LDS-resident kernel
    BinnedPlan bin{};
    GenericBig big{};              // PATH_GENERIC receivers above kGenericMaxM entries (round_generic.hip)
    bool generic_small = true;     // PATH_GENERIC: some receiver has at most kGenericMaxM entries
    MsgParams mp{};
    double* x[2] = {nullptr, nullptr};   // x[k] = xb(k): the synchronous double buffer
    double* xall = nullptr;        // H value buffers of B*Npad (+2) doubles, x^q in buffer q % H
    uint64_t xstride = 0;          // elements per buffer
    uint32_t es = 8;               // value bytes: 8 (ACS_F64) or 4 (ACS_F32)
    bool f32 = false;
    uint32_t H = 2;                // delay_max + 2: x^{r-D} .. x^r read, x^{r+1} written
    uint32_t* ell = nullptr;       // rows [row0, row0 + rows_per) of this rank
    uint32_t* status = nullptr;
    InstState* st = nullptr;
    double2* partial = nullptr;
    uint32_t nblk = 0, nblk_init = 0;
    uint32_t* n_done = nullptr;
    double* trace = nullptr;
    uint32_t* h_ndone = nullptr;   // pinned [2]
    RunSummary* h_sum = nullptr;   // pinned, host-mapped: the one-launch summary writes it directly
    RunSummary* h_sum_dev = nullptr;   // h_sum's device address
    void* sum_scratch = nullptr;       // launch_run_summary_mapped's partials and arrival counter
    unsigned long long* eacc = nullptr;   // [2][kEaccWords] published EPS verdicts (RoundArgs::eacc), by round parity
    bool want_summary = false;     // acs_run on a one-launch path: enqueue the summary before the sync
    bool summary_ready = false;    // h_sum holds the summary of the current state
    unsigned long long sum_seq = 0;    // sequence number of the last summary launch (h_sum->seq)
    MappedStates* h_ms = nullptr;      // pinned, host-mapped instance states (B <= kMappedStates), or null
    MappedStates* h_ms_dev = nullptr;  // its device address
    unsigned long long ms_seq = 0;     // sequence number of the last launch_states_mapped
    bool ms_fresh = false;             // h_ms holds the states advance() ended with (acs_round reuses them)
    uint32_t round = 0;            // round of every unfinished instance
    bool all_done = false;
    // node partitioning: rank owns rows [rank*rows_per, (rank+1)*rows_per) ∩ [0, N)
    int nranks = 1, rank = 0;
    bool partitioned = false;      // node partition mode (virtual, or RCCL with >= 1 rank)
    bool virt = false;             // all nranks partitions simulated on this device
    uint64_t rows_per = 0, Npad = 0;
    ncclComm_t comm = nullptr;
    double2* gpart = nullptr;      // (-min, max) exchanged by all-reduce
    // chunked exchange (binned partitions): the round's rows in xchunks row chunks;
    // chunk k is sent on cstream as soon as its phase B finishes, and the next round's phase A for
    // the source blocks of chunk k starts as soon as chunk k has arrived from every rank
    uint32_t xchunks = 0;          // 0: the unchunked sequence (all-gather after the round)
    uint32_t bin_sa = 0;           // source-block size of the binned plans (chunks align to it)
    hipStream_t cstream = nullptr;
    static constexpr uint32_t kMaxX = 8;
    hipEvent_t ev_b[kMaxX] = {}, ev_x[kMaxX] = {};
    hipEvent_t ev_fin = nullptr;
    uint64_t* rowptr = nullptr;    // CSR topology (device copies)
    uint32_t* colidx = nullptr;
    bool csr_var = false;          // CSR on the register / binned paths: padded ELL of a compiled degree
    uint8_t* deg = nullptr;        // [N] deg(i) (csr_var)
    uint8_t* sw = nullptr;         // [ceil(N/64)] SELL-64 slice widths in 4-wide groups (csr_var)
    // CSR hub rows (deg > d beside a fast path): the generic kernel over hub_ids (rows with at most
    // kGenericMaxM entries) and the big-m path (the rest); their partial slots follow the fast
    // path's nblk_fast block partials
    // CSR rows on the generic kernel go by size class (LDS per workgroup sized to the class):
    // gen_ids = the listed rows, class k = gen_ids[gcls[k].off, +n) with every m_i <= gcls[k].P;
    // row gen_ids[q]'s partial slot is gen_base + q
    struct GenClass {
        uint64_t off, n;
        uint32_t P;
    };
    uint32_t* crank = nullptr;     // fp32 tagged binned plans above 2^20 nodes with crash faults (RoundArgs::crank)
    uint32_t* clist = nullptr;
    std::vector<uint32_t> coff;    // [crash_window + 1] start of round r's crashing senders in clist
    uint32_t* gen_ids = nullptr;
    std::vector<GenClass> gcls;
    uint32_t gen_base = 0;
    uint64_t n_hub = 0;
    uint32_t nblk_fast = 0;
    double* dsorted = nullptr;     // dense path: sorted base multiset [N]
    uint32_t* dcounts = nullptr;   // dense path: |B|, #Byzantine, #crash-silent
    std::vector<Part> parts;       // virtual partitions 1..P-1 (partition 0 uses x / ell)
    // kernel timing (bench)
    uint32_t timing = 0;           // 0 off, else bracket every timing-th round (sampling)
    bool timing_runs = false;      // bracket runs of `timing` consecutive rounds instead (one pair each)
    hipEvent_t run_end = nullptr;  // the open run's end event (recorded after its last round)
    uint32_t run_rounds = 0;       // rounds in the open run
    std::vector<uint32_t> ev_w;    // rounds covered by each event pair
    uint64_t timing_ctr = 0;
    std::vector<hipEvent_t> ev;    // pairs (start, stop)
    size_t ev_used = 0;
    double timed_ms = 0.0;
    uint64_t timed_launches = 0;
    std::string kname;
};

// ------------------------------------------------------------------------- validation
// §A.8 constraints (restated here independently of the oracle's copy).
static int validate(const acs_config* c) {
    if (!c) return fail(ACS_EINVAL, "null config");
    if (c->struct_size != sizeof(acs_config))
        return fail(ACS_EINVAL, "struct_size %u != %zu", c->struct_size, sizeof(acs_config));
    if (c->n_nodes < 1 || c->n_nodes > 0x7FFFFFFFull) return fail(ACS_EINVAL, "n_nodes out of range");
    if (c->n_instances < 1) return fail(ACS_EINVAL, "n_instances must be >= 1");
    if (c->instance_offset + c->n_instances > 0x100000000ull)
        return fail(ACS_EINVAL, "global instance ids must fit in u32");
    uint64_t m, slots;
    if (c->topology == ACS_TOPO_COMPLETE) {
        m = c->n_nodes;
        slots = c->n_nodes * c->n_nodes;
    } else if (c->topology == ACS_TOPO_RANDOM_REGULAR) {
        if (c->degree < 2 || (c->degree & 1u) || c->degree > 4096)
            return fail(ACS_EINVAL, "degree must be even, in [2, 4096]");
        m = (uint64_t)c->degree + 1;
        slots = c->n_nodes * (uint64_t)c->degree;
    } else if (c->topology == ACS_TOPO_CSR) {
        m = 0;       // per receiver: checked against the arrays in acs_create_csr
        slots = 0;
    } else {
        return fail(ACS_EINVAL, "unknown topology %u", c->topology);
    }
    if (slots >= (1ull << 34)) return fail(ACS_EINVAL, "slot count must be < 2^34");
    if (c->topology == ACS_TOPO_CSR) {
        if (c->rule > ACS_RULE_WMSR) return fail(ACS_EINVAL, "unknown rule %u", c->rule);
        if (c->rule == ACS_RULE_AVERAGE && c->trim != 0) return fail(ACS_EINVAL, "AVERAGE requires trim == 0");
        if (c->rule == ACS_RULE_DLPSW_SELECT && c->trim < 1) return fail(ACS_EINVAL, "DLPSW needs t >= 1");
    } else
    switch (c->rule) {
        case ACS_RULE_AVERAGE:
            if (c->trim != 0) return fail(ACS_EINVAL, "AVERAGE requires trim == 0");
            break;
        case ACS_RULE_TRIMMED_MEAN:
        case ACS_RULE_MIDPOINT:
        case ACS_RULE_WMSR:
            if (m <= 2ull * c->trim) return fail(ACS_EINVAL, "need m > 2t");
            break;
        case ACS_RULE_DLPSW_SELECT:
            if (c->trim < 1 || m <= 2ull * c->trim) return fail(ACS_EINVAL, "DLPSW needs t >= 1, m > 2t");
            break;
        default:
            return fail(ACS_EINVAL, "unknown rule %u", c->rule);
    }
    if (c->fault_model == ACS_FAULT_NONE) {
        if (c->n_faulty != 0) return fail(ACS_EINVAL, "n_faulty must be 0 without a fault model");
    } else if (c->fault_model == ACS_FAULT_CRASH || c->fault_model == ACS_FAULT_BYZANTINE) {
        if ((uint64_t)c->n_faulty >= c->n_nodes) return fail(ACS_EINVAL, "n_faulty must be < n_nodes");
    } else {
        return fail(ACS_EINVAL, "unknown fault model %u", c->fault_model);
    }
    if (c->fault_model == ACS_FAULT_CRASH && (c->crash_window < 1 || c->crash_window > (1u << 30)))
        return fail(ACS_EINVAL, "crash_window must be in [1, 2^30]");
    if (c->fault_model == ACS_FAULT_BYZANTINE) {
        if (c->byz_strategy > ACS_BYZ_CONSTANT) return fail(ACS_EINVAL, "unknown byz strategy");
        if (!(fabs(c->byz_delta) <= 1e100) || !(fabs(c->byz_const) <= 1e100))
            return fail(ACS_EINVAL, "byz_delta / byz_const must be finite, |.| <= 1e100");
        if (c->byz_strategy == ACS_BYZ_RANDOM && slots > (1ull << 33))
            return fail(ACS_EINVAL, "BYZ RANDOM needs slot count <= 2^33");
    }
    if (!(c->loss_p >= 0.0 && c->loss_p < 1.0)) return fail(ACS_EINVAL, "loss_p must be in [0,1)");
    if (c->mask_group < 1) return fail(ACS_EINVAL, "mask_group must be >= 1");
    if (!(c->eps >= 0.0 && c->eps <= 1e300)) return fail(ACS_EINVAL, "eps must be finite, >= 0");
    if (c->termination > ACS_TERM_FIXED) return fail(ACS_EINVAL, "unknown termination");
    if (c->dtype != ACS_F64 && c->dtype != ACS_F32) return fail(ACS_EINVAL, "unknown dtype %u", c->dtype);
    if (c->dtype == ACS_F32 && c->fault_model == ACS_FAULT_BYZANTINE &&
        !(fabs(c->byz_delta) <= 1e30 && fabs(c->byz_const) <= 1e30))
        return fail(ACS_EINVAL, "fp32: byz_delta / byz_const must satisfy |.| <= 1e30");
    if (c->delay_max > 64) return fail(ACS_EINVAL, "delay_max must be <= 64");
    if (c->missing_policy > ACS_MISSING_OMIT) return fail(ACS_EINVAL, "unknown missing_policy %u", c->missing_policy);
    if (c->trace_spread && c->n_instances * ((uint64_t)c->max_rounds + 1) > (1ull << 28))
        return fail(ACS_EINVAL, "spread trace too large (B*(max_rounds+1) > 2^28)");
    return ACS_OK;
}

// Tuning / cross-check switches: ACSIM_<NAME>=0 turns an optional fast path off.
static bool env_off(const char* name) {
    const char* v = getenv(name);
    return v && v[0] == '0';
}

static uint32_t drop_threshold(double p) {
    const double t = floor(p * 4294967296.0);   // §A.5, in fp64
    if (t <= 0.0) return 0u;
    if (t >= 4294967295.0) return 0xFFFFFFFFu;
    return (uint32_t)t;
}

// ------------------------------------------------------------------------- internals
static void release(acs_sim* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->cstream) (void)hipStreamSynchronize(s->cstream);
    if (s->comm) (void)ncclCommDestroy(s->comm);
    for (uint32_t k = 0; k < acs_sim::kMaxX; ++k) {
        if (s->ev_b[k]) (void)hipEventDestroy(s->ev_b[k]);
        if (s->ev_x[k]) (void)hipEventDestroy(s->ev_x[k]);
    }
    if (s->ev_fin) (void)hipEventDestroy(s->ev_fin);
    if (s->cstream) (void)hipStreamDestroy(s->cstream);
    for (hipEvent_t e : s->ev) (void)hipEventDestroy(e);
    for (Part& p : s->parts) {
        (void)hipFree(p.x[0]);
        (void)hipFree(p.x[1]);
        (void)hipFree(p.ell);
        binned_free(p.bin);
    }
    (void)hipFree(s->xall);
    (void)hipFree(s->ell);
    binned_free(s->bin);
    generic_big_free(s->big);
    (void)hipFree(s->status);
    (void)hipFree(s->st);
    (void)hipFree(s->partial);
    (void)hipFree(s->gpart);
    (void)hipFree(s->rowptr);
    (void)hipFree(s->colidx);
    (void)hipFree(s->deg);
    (void)hipFree(s->sw);
    (void)hipFree(s->gen_ids);
    (void)hipFree(s->crank);
    (void)hipFree(s->clist);
    (void)hipFree(s->dsorted);
    (void)hipFree(s->dcounts);
    (void)hipFree(s->n_done);
    (void)hipFree(s->trace);
    if (s->h_ndone) (void)hipHostFree(s->h_ndone);
    (void)hipFree(s->sum_scratch);
    if (s->h_sum) (void)hipHostFree(s->h_sum);
    if (s->h_ms) (void)hipHostFree(s->h_ms);
    if (s->eacc) (void)hipFree(s->eacc);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

// value buffer holding x^q
// value buffer q % H (typed double* for the kernels' argument structs; f32 kernels reinterpret)
static double* xb(const acs_sim* s, uint32_t q) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(s->xall) + (uint64_t)(q % s->H) * s->xstride * s->es);
}
// element k of a value buffer (byte arithmetic on the config's value size)
static void* xat(const acs_sim* s, const void* base, uint64_t k) {
    return const_cast<char*>(static_cast<const char*>(base)) + k * s->es;
}

static FinalizeArgs make_finalize(acs_sim* s, uint32_t r_next, const double2* partial, uint32_t nblk,
                                  bool init) {
    FinalizeArgs f{};
    f.st = s->st;
    f.partial = partial;
    f.nblk = nblk;
    f.r_next = r_next;
    f.max_rounds = s->c.max_rounds;
    f.term_eps = s->c.termination == ACS_TERM_EPS;
    f.eps = s->c.eps;
    f.trace = s->trace;
    f.trace_stride = (uint64_t)s->c.max_rounds + 1;
    f.n_done = s->n_done;
    f.init_mode = init ? 1u : 0u;
    f.f32 = s->f32 ? 1u : 0u;
    return f;
}

static uint64_t part_row0(const acs_sim* s, int p) { return (uint64_t)p * s->rows_per; }
static uint64_t part_rows(const acs_sim* s, int p) {
    const uint64_t r0 = part_row0(s, p);
    if (r0 >= s->N) return 0;
    return s->N - r0 < s->rows_per ? s->N - r0 : s->rows_per;
}

// (Re)initialise the per-instance state from x[round & 1] (create and set_state).  Every rank
// holds the full x, so the initial honest min/max needs no exchange.
static int init_state(acs_sim* s, uint32_t round) {
    HIP_TRY(hipMemsetAsync(s->n_done, 0, sizeof(uint32_t), s->stream));
    HIP_TRY(launch_partials_from_x(xb(s, round), s->status, s->B, s->N, s->partial, s->nblk_init, s->f32, s->stream));
    const FinalizeArgs f = make_finalize(s, round, s->partial, s->nblk_init, true);
    HIP_TRY(launch_finalize(f, s->B, s->stream));
    HIP_TRY(hipMemcpyAsync(s->h_ndone, s->n_done, sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    s->round = round;
    s->all_done = s->h_ndone[0] == s->B;
    return ACS_OK;
}

static hipEvent_t next_event(acs_sim* s) {
    if (s->ev_used == s->ev.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        s->ev.push_back(e);
    }
    return s->ev[s->ev_used++];
}

static int harvest_timing(acs_sim* s) {
    if (s->ev_used == 0) return ACS_OK;
    HIP_TRY(hipStreamSynchronize(s->stream));
    for (size_t k = 0; k + 1 < s->ev_used; k += 2) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev[k], s->ev[k + 1]));
        s->timed_ms += ms;
        s->timed_launches += k / 2 < s->ev_w.size() ? s->ev_w[k / 2] : 1u;
    }
    s->ev_used = 0;
    return ACS_OK;
}

// one bracketed launch (the binned pair of a round, one partition round, or one batched / dense
// launch covering a whole round(k) call: acs_get_kernel_timing counts launches, not rounds)
static int timing_begin(acs_sim* s, hipEvent_t* e1) {
    *e1 = nullptr;
    if (s->timing && s->timing_runs) {   // runs of `timing` consecutive rounds, one pair per run
        const uint64_t pos = s->timing_ctr++ % s->timing;
        if (pos == 0 && !s->run_end) {
            if (s->ev_used + 2 > 4096) {
                int rc = harvest_timing(s);
                if (rc) return rc;
            }
            if (s->ev_w.size() < s->ev_used / 2 + 1) s->ev_w.resize(s->ev_used / 2 + 1);
            s->ev_w[s->ev_used / 2] = 0;
            hipEvent_t e0 = next_event(s);
            s->run_end = next_event(s);
            if (!e0 || !s->run_end) return fail(ACS_EDEVICE, "hipEventCreate failed");
            HIP_TRY(hipEventRecord(e0, s->stream));
            s->run_rounds = 0;
        }
        s->run_rounds++;
        if (pos + 1 == s->timing) {   // the run's last round: the caller records the end event
            *e1 = s->run_end;
            s->ev_w[s->ev_used / 2 - 1] = s->run_rounds;
            s->run_end = nullptr;
        }
        return ACS_OK;
    }
    if (!s->timing || s->timing_ctr++ % s->timing != 0) return ACS_OK;
    if (s->ev_used + 2 > 4096) {
        int rc = harvest_timing(s);
        if (rc) return rc;
    }
    if (s->ev_w.size() < s->ev_used / 2 + 1) s->ev_w.resize(s->ev_used / 2 + 1);
    s->ev_w[s->ev_used / 2] = 1;
    hipEvent_t e0 = next_event(s);
    *e1 = next_event(s);
    if (!e0 || !*e1) return fail(ACS_EDEVICE, "hipEventCreate failed");
    HIP_TRY(hipEventRecord(e0, s->stream));
    return ACS_OK;
}

// Close a timing run still open at the end of an advance() call (run mode: a run never spans
// two calls, so host time between calls is never bracketed).
static int timing_close(acs_sim* s) {
    if (!s->run_end) return ACS_OK;
    HIP_TRY(hipEventRecord(s->run_end, s->stream));
    s->ev_w[s->ev_used / 2 - 1] = s->run_rounds;
    s->run_end = nullptr;
    s->timing_ctr = 0;
    return ACS_OK;
}

static RoundArgs round_args(acs_sim* s, uint32_t r) {
    RoundArgs a{};
    a.xin = xb(s, r);
    a.xout = xb(s, r + 1);
    a.xh = s->xall;
    a.xstride = s->xstride;
    a.H = s->H;
    a.delay = s->c.delay_max;
    a.ell = s->ell;
    a.status = s->status;
    a.st = s->st;
    a.partial = s->partial;
    a.N = s->N;
    a.row0 = 0;
    a.nrows = s->N;
    a.rowptr = s->rowptr;
    a.colidx = s->colidx;
    a.m = (uint32_t)s->m;
    a.d = s->d;
    a.dp = s->dp;
    a.topology = s->c.topology;
    a.rule = s->c.rule;
    a.trim = s->c.trim;
    a.r = r;
    a.nblk = s->nblk;
    a.mp = s->mp;
    a.f32 = s->f32 ? 1u : 0u;
    a.deg = s->deg;
    a.sw = s->sw;
    a.qlo = 0;
    a.qhi = 0xFFFFFFFFu;
    a.crank = s->crank;
    a.clist = s->clist;
    a.coff = s->clist && r < s->coff.size() ? s->coff[r] : 0u;
    return a;
}

static uint64_t chunk_rows(const acs_sim* s, int p, uint32_t k) {
    const uint64_t cs = s->rows_per / s->xchunks, n = part_rows(s, p), lo = (uint64_t)k * cs;
    return n > lo ? (n - lo < cs ? n - lo : cs) : 0;
}

// Chunked node-partitioned round on the binned path.  Compute stream: phase A by
// source-block chunk (chunk k of every rank, after round r-1's exchange of chunk k), phase M, then
// phase B by receiver-block chunk (after round r-1's verdict, so a finished run's phase B exits).
// Comm stream: each chunk's exchange as soon as its phase B is done (RCCL grouped send / recv to
// every peer over xGMI, or device copies between virtual partitions), then the spread fold,
// all-reduce and verdict.  Phase A / M of round r+1 may run before round r's verdict: they only
// write the stage, and phase B (the only writer of x) waits for the verdict.
static int enqueue_round_xchunked(acs_sim* s, uint32_t r) {
    const RoundArgs a = round_args(s, r);
    const uint32_t K = s->xchunks;
    const uint64_t cs = s->rows_per / K;
    const uint32_t SA = s->bin_sa;
    const uint32_t bpr = (uint32_t)(s->rows_per / SA), bpc = (uint32_t)(cs / SA);
    const uint32_t qpc = (uint32_t)(cs / s->bin.SB);   // phase-B receiver blocks per chunk
    const int nparts = s->virt ? s->nranks : 1;
    auto pargs = [&](int p) {
        RoundArgs ap = a;
        const int g = s->virt ? p : s->rank;
        if (s->virt && p > 0) {
            ap.xin = s->parts[p - 1].x[r & 1u];
            ap.xout = s->parts[p - 1].x[(r + 1) & 1u];
        }
        ap.row0 = part_row0(s, g);
        ap.nrows = part_rows(s, g);
        if (s->virt) ap.partial = s->partial + (uint64_t)p * s->nblk;
        return ap;
    };
    auto plan = [&](int p) -> const BinnedPlan& { return (s->virt && p > 0) ? s->parts[p - 1].bin : s->bin; };
    hipEvent_t e1;
    int rc = timing_begin(s, &e1);
    if (rc) return rc;
    for (uint32_t k = 0; k < K; ++k) {
        HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_x[k], 0));
        for (int p = 0; p < nparts; ++p)
            if (pargs(p).nrows)
                HIP_TRY(launch_round_binned(plan(p), pargs(p), s->clean, s->stream, nullptr, 1u,
                                            SrcSel{(uint32_t)s->nranks * bpc, bpr, bpc, k * bpc}));
    }
    for (int p = 0; p < nparts; ++p)
        if (pargs(p).nrows) HIP_TRY(launch_round_binned(plan(p), pargs(p), s->clean, s->stream, nullptr, 2u));
    HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_fin, 0));
    const ncclDataType_t dt = s->f32 ? ncclFloat32 : ncclFloat64;
    for (uint32_t k = 0; k < K; ++k) {
        for (int p = 0; p < nparts; ++p) {
            RoundArgs ap = pargs(p);
            if (!ap.nrows) continue;
            ap.qlo = k * qpc;
            ap.qhi = k + 1 == K ? 0xFFFFFFFFu : (k + 1) * qpc;
            HIP_TRY(launch_round_binned(plan(p), ap, s->clean, s->stream, nullptr, 4u));
        }
        HIP_TRY(hipEventRecord(s->ev_b[k], s->stream));
        HIP_TRY(hipStreamWaitEvent(s->cstream, s->ev_b[k], 0));
        if (s->virt) {   // chunk k of every partition into every other partition's copy
            const uint32_t o = (r + 1) & 1u;
            for (int p = 0; p < s->nranks; ++p) {
                const uint64_t n = chunk_rows(s, p, k), off = part_row0(s, p) + (uint64_t)k * cs;
                if (!n) continue;
                const double* src = p == 0 ? s->x[o] : s->parts[p - 1].x[o];
                for (int q = 0; q < s->nranks; ++q) {
                    if (q == p) continue;
                    double* dst = q == 0 ? s->x[o] : s->parts[q - 1].x[o];
                    HIP_TRY(hipMemcpyAsync(xat(s, dst, off), xat(s, src, off), n * s->es, hipMemcpyDeviceToDevice,
                                           s->cstream));
                }
            }
        } else if (s->nranks > 1) {
            double* xo = s->x[(r + 1) & 1u];
            NCCL_TRY(ncclGroupStart());
            for (int q = 0; q < s->nranks; ++q) {
                if (q == s->rank) continue;
                const uint64_t mine = chunk_rows(s, s->rank, k), theirs = chunk_rows(s, q, k);
                if (mine)
                    NCCL_TRY(ncclSend(xat(s, xo, part_row0(s, s->rank) + (uint64_t)k * cs), mine, dt, q, s->comm,
                                      s->cstream));
                if (theirs)
                    NCCL_TRY(ncclRecv(xat(s, xo, part_row0(s, q) + (uint64_t)k * cs), theirs, dt, q, s->comm,
                                      s->cstream));
            }
            NCCL_TRY(ncclGroupEnd());
        }
        HIP_TRY(hipEventRecord(s->ev_x[k], s->cstream));
    }
    if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
    // verdict of round r on the comm stream (it has waited for every phase-B chunk)
    if (s->virt) {
        uint32_t nblk_live = 0;
        for (int p = 0; p < s->nranks; ++p)
            if (part_rows(s, p)) nblk_live = (uint32_t)((p + 1) * s->nblk);
        HIP_TRY(launch_finalize(make_finalize(s, r + 1, s->partial, nblk_live, false), s->B, s->cstream));
    } else {
        FinalizeArgs fold = make_finalize(s, r + 1, s->partial, a.nrows ? s->nblk : 0, false);
        fold.fold_out = s->gpart;
        if (!part_rows(s, s->rank)) fold.nblk = 0;
        HIP_TRY(launch_finalize(fold, s->B, s->cstream));
        if (s->nranks > 1) NCCL_TRY(ncclAllReduce(s->gpart, s->gpart, 2, ncclFloat64, ncclMax, s->comm, s->cstream));
        FinalizeArgs fin = make_finalize(s, r + 1, s->gpart, 1, false);
        fin.negmin = 1;
        HIP_TRY(launch_finalize(fin, s->B, s->cstream));
    }
    HIP_TRY(hipEventRecord(s->ev_fin, s->cstream));
    return ACS_OK;
}

// One round x^r -> x^{r+1}: round kernel(s), [exchange], spread finalize.
static int enqueue_round(acs_sim* s, uint32_t r) {
    if (s->xchunks) return enqueue_round_xchunked(s, r);
    RoundArgs a = round_args(s, r);
    hipEvent_t e1;
    int rc = timing_begin(s, &e1);
    if (rc) return rc;
    // EPS verdict publication: phase B of round r folds its exact (min, max) into
    // eacc[(r + 1) & 1], so every workgroup of round r + 1's phase A can stop on convergence
    // (without it only workgroup 0 folds the partials and the others stream one last round).
    // Invariant: EVERY kernel that writes a.partial in such a round must also publish into ab.eacc
    // (block_minmax_store(..., a.eacc)): k_bin_gather in all its forms (NP = 1 / 2, VAR, FIX,
    // FAULTY) and k_bin_gather_of.  A writer that skipped it would not crash: phase A's other
    // workgroups would stop on a stale verdict while workgroup 0 streams.  Hub rows (generic
    // kernel partials) and partitioned rounds are therefore excluded here;
    // tests/test_gpu_binned.py::test_eps_publication_in_every_gather_variant covers each form.
    // (narrow plans publish in every round: the next phase A chooses its stage width from the pair)
    unsigned long long* pub = s->eacc && s->binned && s->defer_fin && !s->n_hub && !s->partitioned &&
                                      (s->c.termination == ACS_TERM_EPS || s->bin.narrow)
                                  ? s->eacc + kEaccWords * ((r + 1) & 1u)
                                  : nullptr;
    if (!s->partitioned) {
        if (s->binned) {
            RoundArgs ab = a;
            ab.eacc = pub;
            if (s->n_hub) ab.qhi = s->nblk_fast;   // the hub rows' partial slots are the generic kernel's
            HIP_TRY(launch_round_binned(s->bin, ab, s->clean, s->stream, s->fin_pending ? &s->fin_args : nullptr));
            s->fin_pending = false;
        } else if (s->path == PATH_REGULAR) {
            HIP_TRY(launch_round_regular(a, s->B, s->clean, s->stream));
        } else if (s->path == PATH_DENSE) {
            DenseArgs d{};
            d.x = a.xin;
            d.xo = a.xout;
            d.status = s->status;
            d.st = s->st;
            d.partial = s->partial;
            d.sorted = s->dsorted;
            d.counts = s->dcounts;
            d.N = (uint32_t)s->N;
            uint32_t P = 1;
            while (P < s->N) P <<= 1;
            d.P = P;
            d.r = r;
            d.rule = s->c.rule;
            d.trim = s->c.trim;
            d.byz = s->c.byz_strategy;
            d.delta = s->mp.delta;
            d.bconst = s->mp.bconst;
            d.f32 = s->f32 ? 1u : 0u;
            HIP_TRY(launch_round_dense(d, s->stream));
        } else if (s->c.topology != ACS_TOPO_CSR) {   // complete / regular graphs: one size for all
            if (s->generic_small) HIP_TRY(launch_round_generic(a, s->B, s->stream));
            HIP_TRY(launch_round_generic_big(s->big, a, s->B, s->stream));
        }
        if (s->c.topology == ACS_TOPO_CSR && (s->path == PATH_GENERIC || s->n_hub)) {
            // CSR rows on the generic kernels (every row, or the hub rows after the fast path):
            // by size class, then the rows above kGenericMaxM on the big-m path
            for (const auto& c : s->gcls) {
                RoundArgs ah = a;
                ah.rid = s->gen_ids + c.off;
                ah.pbase = s->gen_base + (uint32_t)c.off;
                HIP_TRY(launch_round_generic(ah, s->B, s->stream, c.n, c.P));
            }
            HIP_TRY(launch_round_generic_big(s->big, a, s->B, s->stream));
        }
        if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
        const FinalizeArgs fin = make_finalize(s, r + 1, s->partial, s->nblk, false);
        if (s->defer_fin) {   // folded by the next round's phase A, or by flush_finalize
            s->fin_args = fin;
            s->fin_args.eacc = pub;
            s->fin_pending = true;
            return ACS_OK;
        }
        HIP_TRY(launch_finalize(fin, s->B, s->stream));
        return ACS_OK;
    }
    if (s->virt) {
        // every partition p reads its own full copy, writes its own rows; block partials of
        // partition p land at partial[p * nblk]
        for (int p = 0; p < s->nranks; ++p) {
            RoundArgs ap = a;
            if (p > 0) {
                ap.xin = s->parts[p - 1].x[r & 1u];
                ap.xout = s->parts[p - 1].x[(r + 1) & 1u];
                ap.ell = s->parts[p - 1].ell;
            }
            ap.row0 = part_row0(s, p);
            ap.nrows = part_rows(s, p);
            ap.partial = s->partial + (uint64_t)p * s->nblk;
            if (ap.nrows == 0) continue;   // empty tail partition (its partials are not folded)
            if (s->binned)
                HIP_TRY(launch_round_binned(p == 0 ? s->bin : s->parts[p - 1].bin, ap, s->clean, s->stream));
            else
                HIP_TRY(launch_round_regular(ap, s->B, s->clean, s->stream));
        }
        if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
        // all-gather emulation: copy each partition's fresh rows into every other copy
        const uint32_t o = (r + 1) & 1u;
        for (int p = 0; p < s->nranks; ++p) {
            const uint64_t r0 = part_row0(s, p), nr = part_rows(s, p);
            if (!nr) continue;
            const double* src = p == 0 ? s->x[o] : s->parts[p - 1].x[o];
            for (int q = 0; q < s->nranks; ++q) {
                if (q == p) continue;
                double* dst = q == 0 ? s->x[o] : s->parts[q - 1].x[o];
                HIP_TRY(hipMemcpyAsync(xat(s, dst, r0), xat(s, src, r0), nr * s->es, hipMemcpyDeviceToDevice,
                                       s->stream));
            }
        }
        uint32_t nblk_live = 0;
        for (int p = 0; p < s->nranks; ++p)
            if (part_rows(s, p)) nblk_live = (uint32_t)((p + 1) * s->nblk);
        HIP_TRY(launch_finalize(make_finalize(s, r + 1, s->partial, nblk_live, false), s->B, s->stream));
        return ACS_OK;
    }
    // RCCL partition: own rows, then in-place all-gather of x^{r+1} and all-reduce of the spread
    a.row0 = part_row0(s, s->rank);
    a.nrows = part_rows(s, s->rank);
    if (a.nrows) {
        if (s->binned)
            HIP_TRY(launch_round_binned(s->bin, a, s->clean, s->stream));
        else
            HIP_TRY(launch_round_regular(a, s->B, s->clean, s->stream));
    }
    if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
    double* xo = s->x[(r + 1) & 1u];
    NCCL_TRY(ncclAllGather(xat(s, xo, a.row0), xo, s->rows_per, s->f32 ? ncclFloat32 : ncclFloat64, s->comm,
                           s->stream));
    FinalizeArgs fold = make_finalize(s, r + 1, s->partial, a.nrows ? s->nblk : 0, false);
    fold.fold_out = s->gpart;
    HIP_TRY(launch_finalize(fold, s->B, s->stream));
    NCCL_TRY(ncclAllReduce(s->gpart, s->gpart, 2, ncclFloat64, ncclMax, s->comm, s->stream));
    FinalizeArgs fin = make_finalize(s, r + 1, s->gpart, 1, false);
    fin.negmin = 1;
    HIP_TRY(launch_finalize(fin, s->B, s->stream));
    return ACS_OK;
}

// Host memory the device writes and the host polls (run summary, instance states): mapped into the
// device's address space and explicitly COHERENT, so the device's system-scope release of the
// sequence number (and the fields stored before it) reaches host memory without a cache flush at
// the end of the kernel; the polling protocol below depends on that and must not rest on the
// runtime's default or on HIP_HOST_COHERENT.  acs_runtime_info reports it.
static constexpr unsigned kPolledHostFlags = hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent;

// Poll a host-mapped sequence number a launch on s->stream releases at system scope.  The stream is
// queried every 256 spins, so a failed launch returns its error rather than spinning forever.
// patient: the wait may span a whole chunk of long rounds (EPS chunk verdicts of large graphs,
// milliseconds each): after 100 us of spinning the host yields the core between polls
// (sched_yield), so ranks and threads sharing the box's cores run meanwhile, without adding the
// wake-up latency of a sleep (a 20 us sleep_for, with the kernel's default timer slack, added
// ≈ 60 us to every cfg4 EPS run: profiles/r06_eps_yield_configs.jsonl).  The short call-end reads
// spin throughout (their wait is a few microseconds).
static int wait_mapped_seq(acs_sim* s, const unsigned long long* p, unsigned long long seq, const char* what,
                           bool patient = false) {
    const auto t0 = std::chrono::steady_clock::now();
    bool yielding = false;
    for (uint32_t it = 1;; ++it) {
        if (__atomic_load_n(p, __ATOMIC_ACQUIRE) == seq) return ACS_OK;
        if ((it & 255u) == 0) {
            const hipError_t q = hipStreamQuery(s->stream);
            if (q == hipSuccess) {
                if (__atomic_load_n(p, __ATOMIC_ACQUIRE) == seq) return ACS_OK;
                return fail(ACS_EDEVICE, "%s: stream idle without the sequence number", what);
            }
            if (q != hipErrorNotReady) return fail(ACS_EDEVICE, "%s: %s", what, hipGetErrorString(q));
            if (patient && !yielding && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(100))
                yielding = true;
        }
        if (yielding)
            std::this_thread::yield();
        else
            __builtin_ia32_pause();
    }
}

// The B instance states after everything enqueued so far.  Handles of at most kMappedStates
// instances take them through host-mapped memory (launch_states_mapped: no device-to-host copy,
// no wait on the stream's completion signal); the stream may still be retiring that small launch
// on return, and later work stays ordered behind it.
static int fetch_mapped_states(acs_sim* s, bool patient = false) {
    const unsigned long long seq = ++s->ms_seq;
    HIP_TRY(launch_states_mapped(s->st, s->n_done, (uint32_t)s->B, s->h_ms_dev, seq, s->stream));
    return wait_mapped_seq(s, &s->h_ms->seq, seq, "instance states", patient);
}

// The done count after everything enqueued so far (EPS chunks and call ends): through the mapped
// states where the handle has them (which then hold the states of that moment too).  patient: a
// chunk verdict behind a chunk of long rounds (wait_mapped_seq).
static int fetch_done_count(acs_sim* s, uint32_t& nd, bool patient = false) {
    if (s->h_ms) {
        if (int rc = fetch_mapped_states(s, patient)) return rc;
        nd = s->h_ms->n_done;
        return ACS_OK;
    }
    HIP_TRY(hipMemcpyAsync(s->h_ndone, s->n_done, sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    nd = s->h_ndone[0];
    return ACS_OK;
}

static int read_states(acs_sim* s, std::vector<InstState>& out, bool reuse_fresh = false) {
    out.resize(s->B);
    if (s->h_ms) {
        if (!(reuse_fresh && s->ms_fresh))
            if (int rc = fetch_mapped_states(s)) return rc;
        s->ms_fresh = false;
        memcpy(out.data(), s->h_ms->st, s->B * sizeof(InstState));
        return ACS_OK;
    }
    HIP_TRY(hipMemcpyAsync(out.data(), s->st, s->B * sizeof(InstState), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ACS_OK;
}

static constexpr uint32_t kChunk = 16;

// Enqueue the one-launch run summary and wait for it by polling its host-mapped sequence number
// instead of the stream's completion signal (the wake-up after that signal cost ≈ 6 µs per run on
// a 12 500-instance cfg3 shard).  The stream is queried every 256 spins, so a failed
// launch returns its error rather than spinning forever.  On return the summary's fields are
// valid; later stream work stays ordered behind the (finishing) summary kernel.
static int summary_and_wait(acs_sim* s) {
    const unsigned long long seq = ++s->sum_seq;
    HIP_TRY(launch_run_summary_mapped(s->st, s->B, s->sum_scratch, s->h_sum_dev, seq, s->stream));
    return wait_mapped_seq(s, &s->h_sum->seq, seq, "run summary");
}

// Launch a finalize still deferred (the last round enqueued has no next phase A to fold it).
static int flush_finalize(acs_sim* s) {
    if (!s->fin_pending) return ACS_OK;
    s->fin_pending = false;
    HIP_TRY(launch_finalize(s->fin_args, s->B, s->stream));
    return ACS_OK;
}

// roctx range for the rocprofv3 --marker-trace timeline: host-side enqueue spans of
// round chunks and the one-launch batched / dense paths.
struct RoctxRange {
    explicit RoctxRange(const char* m) { roctxRangePushA(m); }
    ~RoctxRange() { roctxRangePop(); }
};

// Advance every unfinished instance by at most k rounds.
static int advance(acs_sim* s, uint32_t k) {
    s->ms_fresh = false;
    if (s->all_done || k == 0) return ACS_OK;
    const uint32_t cap = s->c.max_rounds > s->round ? s->c.max_rounds - s->round : 0;
    if (k > cap) k = cap;
    if (k == 0) return ACS_OK;
    if (s->path == PATH_BATCHED || s->dense_persist) {
        BatchArgs a{};
        a.x0 = s->x[0];
        a.x1 = s->x[1];
        a.status = s->status;
        a.st = s->st;
        a.trace = s->trace;
        a.trace_stride = (uint64_t)s->c.max_rounds + 1;
        a.n_done = s->n_done;
        a.N = (uint32_t)s->N;
        a.rule = s->c.rule;
        a.trim = s->c.trim;
        a.max_rounds = s->c.max_rounds;
        a.term_eps = s->c.termination == ACS_TERM_EPS;
        a.eps = s->c.eps;
        a.mp = s->mp;
        a.f32 = s->f32 ? 1u : 0u;
        hipEvent_t e1;
        int rc = timing_begin(s, &e1);
        if (rc) return rc;
        RoctxRange range(s->dense_persist ? "acs: persistent dense rounds" : "acs: batched rounds");
        if (s->dense_persist)
            HIP_TRY(launch_dense_persist(a, s->B, k, s->stream));
        else if (s->mfma)
            HIP_TRY(launch_batched_mfma(a, s->B, k, s->stream));
        else
            HIP_TRY(launch_batched_small(a, s->B, k, s->stream));
        if (e1) HIP_TRY(hipEventRecord(e1, s->stream));
        if (int rc2 = timing_close(s)) return rc2;   // (run mode: one launch per call)
        // The done count (and, for acs_run, the result summary) ride on the same synchronisation,
        // folded from the instances' done flags in one launch that writes host memory: no copies
        // (each costs a DMA round trip) and no per-instance atomic on one counter (the batched
        // kernels' last generation finished together and serialised on it), DESIGN.md §6
        if (int rc2 = summary_and_wait(s)) return rc2;
        s->summary_ready = s->want_summary;
        s->round += k;
        s->h_ndone[0] = s->h_sum->n_done;
        s->all_done = s->h_ndone[0] == s->B;
        return ACS_OK;
    }
    const bool eps_mode = s->c.termination == ACS_TERM_EPS;
    // FIXED runs need no verdict between chunks: the deferred finalize of a chunk's last round is
    // folded by the next chunk's first phase A like any other, and one standalone finalize closes
    // the call (round 5: one 4.7 µs k_finalize per 16 rounds fewer)
    const bool chunk_flush = eps_mode || s->partitioned;
    // Long rounds (a chunk of them takes milliseconds): wait for each chunk's verdict before
    // enqueuing the next, so no chunk of no-op launches follows convergence (the host wake-up is
    // < 1 % of a chunk).  Short rounds keep one chunk in flight and poll the previous one.
    const bool sync_poll = eps_mode && s->N * (uint64_t)(s->d ? s->d : s->m) * s->B >= (1ull << 22);
    int slot = 0, prev = -1;
    hipEvent_t poll[2] = {nullptr, nullptr};
    while (k > 0 && !s->all_done) {
        const uint32_t chunk = k < kChunk ? k : kChunk;
        RoctxRange range("acs: round chunk (enqueue)");
        for (uint32_t q = 0; q < chunk; ++q) {
            int rc = enqueue_round(s, s->round + q);
            if (rc) return rc;
        }
        if (chunk_flush)
            if (int rc = flush_finalize(s)) return rc;
        if (s->xchunks) HIP_TRY(hipStreamWaitEvent(s->stream, s->ev_fin, 0));   // verdicts land on cstream
        s->round += chunk;
        k -= chunk;
        if (s->round >= s->c.max_rounds) break;
        if (sync_poll && k > 0) {
            uint32_t nd = 0;
            if (int rc = fetch_done_count(s, nd, true)) return rc;
            if (nd == s->B) s->all_done = true;
        } else if (eps_mode && !sync_poll) {
            // keep one chunk in flight: poll the previous chunk's done counter
            HIP_TRY(hipMemcpyAsync(s->h_ndone + slot, s->n_done, sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   s->stream));
            if (!poll[slot]) HIP_TRY(hipEventCreateWithFlags(&poll[slot], hipEventDisableTiming));
            HIP_TRY(hipEventRecord(poll[slot], s->stream));
            if (prev >= 0) {
                HIP_TRY(hipEventSynchronize(poll[prev]));
                if (s->h_ndone[prev] == s->B) s->all_done = true;
            }
            prev = slot;
            slot ^= 1;
        }
    }
    for (hipEvent_t e : poll)
        if (e) (void)hipEventDestroy(e);
    if (int rc = flush_finalize(s)) return rc;   // (FIXED: the call's last round)
    if (s->run_end)   // a timing run cut short by the end of this call
        if (int rc = timing_close(s)) return rc;
    if (!eps_mode) {
        // FIXED: every instance is done exactly at max_rounds, so no device round trip is needed
        // here (acs_round's state read and acs_run's summary synchronise the stream anyway)
        s->all_done = s->round >= s->c.max_rounds;
        return ACS_OK;
    }
    if (s->want_summary) {   // acs_run: the summary carries the done count (one round trip, not two)
        if (int rc = summary_and_wait(s)) return rc;
        s->summary_ready = true;
        s->all_done = s->h_sum->n_done == s->B;
        return ACS_OK;
    }
    uint32_t nd = 0;
    if (int rc = fetch_done_count(s, nd)) return rc;
    s->ms_fresh = s->h_ms != nullptr;   // nothing is enqueued after it: acs_round reuses these states
    s->all_done = nd == s->B;
    return ACS_OK;
}

// CSR on the register / binned paths (§8(f) row 1): the smallest compiled degree D >= the
// largest row with the config's (t, rule), 0 if none (the generic kernel then runs).
static uint32_t csr_fast_degree(uint64_t maxdeg, uint32_t t, uint32_t rule) {
    for (uint32_t d : {4u, 8u, 16u, 32u})
        if (d >= maxdeg && regular_fast_supported(d, t, rule)) return d;
    return 0;
}

// CSR graphs whose largest degree is above every compiled degree: the largest compiled degree d
// (for this t and rule) whose hub rows (deg > d) are at most a quarter of the rows; 0 if none.
// The hub rows go to the generic kernel, the rest to the register / binned path padded to d.
static uint32_t csr_hub_degree(const uint64_t* rowptr, uint64_t N, uint32_t t, uint32_t rule, uint64_t* nhub) {
    for (uint32_t d : {32u, 16u, 8u, 4u}) {
        if (!regular_fast_supported(d, t, rule)) continue;
        uint64_t h = 0;
        for (uint64_t i = 0; i < N; ++i) h += rowptr[i + 1] - rowptr[i] > d;
        if (h * 4 <= N) {
            *nhub = h;
            return d;
        }
        return 0;   // smaller compiled degrees would only leave more hubs
    }
    return 0;
}

// Build the adjacency rows of partition p into `ell` (sorted when the config allows it).
static hipError_t build_rows(acs_sim* s, uint32_t* ell, int p) {
    const uint64_t gseed = s->c.graph_seed ? s->c.graph_seed : s->c.seed;
    const uint64_t nr = !s->partitioned ? s->N : part_rows(s, p);
    if (nr == 0) return hipSuccess;
    hipError_t e = launch_build_ell(ell, s->N, !s->partitioned ? 0 : part_row0(s, p), nr, s->d, s->dp,
                                    make_feistel(s->N, gseed), s->stream);
    if (e == hipSuccess && s->ell_sorted) e = launch_sort_ell_rows(ell, nr, s->d, s->stream);
    return e;
}

static int create_impl(const acs_config* cfg, int device, int nranks, int rank, const void* comm_id,
                       uint64_t id_len, acs_sim** out, const uint64_t* h_rowptr = nullptr,
                       const uint32_t* h_colidx = nullptr) {
    if (!out) return fail(ACS_EINVAL, "null out");
    *out = nullptr;
    int rc = validate(cfg);
    if (rc) return rc;
    uint64_t csr_mmax = 0, csr_nnz = 0;
    if (cfg->topology == ACS_TOPO_CSR) {   // §8(f) row 1: check the arrays on the host
        if (!h_rowptr || !h_colidx) return fail(ACS_EINVAL, "CSR topology needs acs_create_csr(rowptr, colidx)");
        if (nranks != 1) return fail(ACS_EUNSUPPORTED, "node partitioning needs RANDOM_REGULAR");
        const uint64_t N = cfg->n_nodes;
        if (h_rowptr[0] != 0) return fail(ACS_EINVAL, "rowptr[0] must be 0");
        csr_mmax = 1;
        for (uint64_t i = 0; i < N; ++i) {
            if (h_rowptr[i + 1] < h_rowptr[i]) return fail(ACS_EINVAL, "rowptr must be non-decreasing");
            const uint64_t m = h_rowptr[i + 1] - h_rowptr[i] + 1;
            if (cfg->rule != ACS_RULE_AVERAGE && m <= 2ull * cfg->trim)
                return fail(ACS_EINVAL, "receiver %llu has m = %llu <= 2t", (unsigned long long)i,
                            (unsigned long long)m);
            if (m > csr_mmax) csr_mmax = m;
        }
        csr_nnz = h_rowptr[N];
        if (csr_nnz >= (1ull << 34)) return fail(ACS_EINVAL, "slot count must be < 2^34");
        if (cfg->fault_model == ACS_FAULT_BYZANTINE && cfg->byz_strategy == ACS_BYZ_RANDOM && csr_nnz > (1ull << 33))
            return fail(ACS_EINVAL, "BYZ RANDOM needs slot count <= 2^33");
        for (uint64_t k = 0; k < csr_nnz; ++k)
            if (h_colidx[k] >= N) return fail(ACS_EINVAL, "colidx[%llu] out of range", (unsigned long long)k);
    }
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(ACS_EINVAL, "bad rank / n_ranks");
    const bool partitioned = nranks > 1 || comm_id != nullptr;
    const bool virt = partitioned && !comm_id;
    if (virt && rank != 0) return fail(ACS_EINVAL, "virtual partitions live on one handle (rank 0)");
    if (comm_id && id_len != sizeof(ncclUniqueId))
        return fail(ACS_EINVAL, "comm id must be %zu bytes", sizeof(ncclUniqueId));
    if (partitioned && cfg->delay_max)
        return fail(ACS_EUNSUPPORTED, "node partitioning runs synchronous rounds only (delay_max = 0)");
    if (partitioned) {
        if (cfg->topology != ACS_TOPO_RANDOM_REGULAR || cfg->n_instances != 1 ||
            !regular_fast_supported(cfg->degree, cfg->trim, cfg->rule))
            return fail(ACS_EUNSUPPORTED, "node partitioning needs one RANDOM_REGULAR instance with a "
                                          "compiled (degree, trim) variant");
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(ACS_EDEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(ACS_EINVAL, "device %d out of range", device);

    RoctxRange range("acs: create (graph, plan, fault schedule, x0)");
    acs_sim* s = new acs_sim();
    s->c = *cfg;
    s->device = device;
    s->N = cfg->n_nodes;
    s->B = cfg->n_instances;
    s->m = cfg->topology == ACS_TOPO_COMPLETE ? s->N
         : cfg->topology == ACS_TOPO_CSR      ? csr_mmax
                                              : (uint64_t)cfg->degree + 1;
    s->d = cfg->topology == ACS_TOPO_CSR ? 0 : cfg->degree;
    s->dp = (cfg->degree + 3u) & ~3u;
    // "clean": no slot-dependent decision at all (no faults, no loss, no delays)
    s->clean = cfg->fault_model == ACS_FAULT_NONE && drop_threshold(cfg->loss_p) == 0 && cfg->delay_max == 0;
    s->mp.key = key_of(cfg->seed);
    s->mp.thr = drop_threshold(cfg->loss_p);
    s->mp.fault = cfg->fault_model;
    s->mp.byz = cfg->byz_strategy;
    s->mp.mask_group = cfg->mask_group;
    s->mp.inst_offset = cfg->instance_offset;
    s->mp.delta = cfg->byz_delta;
    s->mp.bconst = cfg->byz_const + 0.0;   // canonicalise -0.0 (no -0 ever enters a sort)
    s->mp.omit = cfg->missing_policy == ACS_MISSING_OMIT ? 1u : 0u;
    s->nranks = nranks;
    s->partitioned = partitioned;
    s->rank = rank;
    s->virt = virt;
    s->rows_per = partitioned ? ((s->N + nranks - 1) / nranks + 63) / 64 * 64 : s->N;
    s->Npad = partitioned ? s->rows_per * nranks : s->N;

    s->f32 = cfg->dtype == ACS_F32;
    s->es = s->f32 ? 4u : 8u;
    // fp32 runs on the register, generic, batched (N <= 64), dense (persistent up to
    // 4096 nodes, the two-kernel path up to 8192 since round 6) and binned kernels; the MFMA group
    // kernel is fp64-only (its hardware-ordered sums would not keep fp32 rounds-to-convergence)
    if (cfg->topology == ACS_TOPO_COMPLETE && s->N <= kBatchedMaxN && cfg->delay_max == 0) {
        s->path = PATH_BATCHED;
        s->kname = batched_small_name((uint32_t)s->N, cfg->rule, cfg->fault_model != ACS_FAULT_NONE);
        if (const uint32_t F = batched_split_factor((uint32_t)s->N, cfg->rule, cfg->fault_model != ACS_FAULT_NONE); F > 1)
            s->kname = "k_batched_split<" + std::to_string(F) + ">";
        const char* env = getenv("ACSIM_MFMA");
        s->mfma = !(env && env[0] == '0') && !s->f32 &&
                  batched_mfma_supported((uint32_t)s->N, cfg->rule, cfg->fault_model != ACS_FAULT_NONE, cfg->mask_group,
                                         cfg->instance_offset);
        if (s->mfma) s->kname = "k_batched_mfma<v_mfma_f64_16x16x4>";
    } else if (cfg->topology == ACS_TOPO_COMPLETE && !partitioned && cfg->delay_max == 0 &&
               (s->B == 1 || (s->N <= kDensePersistMaxN && !env_off("ACSIM_DENSE_PERSIST"))) &&
               dense_supported(cfg->fault_model, cfg->byz_strategy, cfg->rule, s->mp.thr, s->N)) {
        s->path = PATH_DENSE;
        s->dense_persist = s->N <= kDensePersistMaxN && !env_off("ACSIM_DENSE_PERSIST");
        s->kname = s->dense_persist ? "k_dense_persist" : "k_dense_sort+k_dense_recv";
    } else if (cfg->topology == ACS_TOPO_RANDOM_REGULAR && regular_fast_supported(s->d, cfg->trim, cfg->rule)) {
        s->path = PATH_REGULAR;
        s->kname = regular_fast_name(s->d, cfg->trim, s->clean);
    } else if (cfg->topology == ACS_TOPO_CSR && !env_off("ACSIM_CSR_FAST") &&
               ((s->d = csr_fast_degree(csr_mmax - 1, cfg->trim, cfg->rule)) != 0 ||
                (s->d = csr_hub_degree(h_rowptr, s->N, cfg->trim, cfg->rule, &s->n_hub)) != 0)) {
        // §8(f) row 1: rows padded to the smallest compiled degree >= max deg(i) with the same t, or
        // (power-law graphs) to the largest compiled degree with the rows above it as hub rows
        s->path = PATH_REGULAR;
        s->csr_var = true;
        s->dp = s->d;
        s->kname = std::string("k_round_regular<") + std::to_string(s->d) + "," + std::to_string(cfg->trim) + ",csr>";
    } else if (s->m <= kGenericBigMaxM) {
        s->path = PATH_GENERIC;
        s->generic_small = !(cfg->topology == ACS_TOPO_COMPLETE && s->m > kGenericMaxM);
        s->kname = s->m <= kGenericMaxM ? "k_round_generic"
                   : s->generic_small   ? "k_round_generic+k_big_resolve+sort+k_big_rule"
                                        : "k_big_resolve+sort+k_big_rule";
    } else {
        delete s;
        return fail(ACS_EUNSUPPORTED, "m = %llu entries per receiver exceeds the big-m generic path's %llu",
                    (unsigned long long)s->m, (unsigned long long)kGenericBigMaxM);
    }
    if (cfg->fault_model != ACS_FAULT_NONE && s->N >= (1ull << 31)) {   // (any B: setup.hip batches instances)
        delete s;
        return fail(ACS_EUNSUPPORTED, "fault schedules need N < 2^31");
    }
    s->ell_sorted = s->path == PATH_REGULAR && s->clean && cfg->rule != ACS_RULE_AVERAGE;
    const uint64_t rows_local = partitioned ? s->rows_per : s->N;
    // binned exchange (round_binned.hip): one instance, synchronous rounds, and a graph shape with
    // one or two exchange levels (faults and loss are resolved in phase B from tagged values and
    // slot-order draws); ACSIM_BINNED=0 forces the per-lane kernel and ACSIM_BIN_SA sets the
    // source block size (tests use small blocks on small graphs)
    // (128 KiB of LDS per phase-A source block: 16 Ki fp64 or 32 Ki fp32 senders).  Default 16 Ki for
    // fp32 too: 14-bit packed phase-A indices, and measured faster (cfg4_f32 82.2 -> 80.9 us per round,
    // cfg5_f32 4.69 -> 4.51 ms; profiles/r04_f32_sa_ab.jsonl); ACSIM_BIN_SA up to 32 Ki
    const uint32_t sa_max = s->f32 ? 32768u : 16384u;
    uint32_t bin_sa = 16384u;
    if (const char* v = getenv("ACSIM_BIN_SA")) bin_sa = (uint32_t)strtoul(v, nullptr, 10);
    if (bin_sa < 64 || bin_sa > sa_max || (bin_sa & (bin_sa - 1))) bin_sa = 16384u;
    // (the order-free phase B of rounds 1-5, ACSIM_BIN_OF=1, measured slower than the invpos phase
    // B and was removed in round 6: DESIGN.md §5.1, §5.13)
    std::string kname_lane;   // (set with the binned decision below)
    // phase-B receiver block (BinnedPlan::SB): the default, or ACSIM_BIN_SB where the clean (d, t)
    // pair has that instantiation; block partials follow it (one per receiver block)
    const uint32_t bin_sb = binned_block_size(s->d, cfg->trim, cfg->rule,
                                              s->clean && !s->csr_var && s->path == PATH_REGULAR);
    {
        const char* env = getenv("ACSIM_BINNED");
        const bool allow = !(env && env[0] == '0');
        const uint32_t lv =
            s->path == PATH_REGULAR && s->d ? binned_levels(s->N, rows_local, s->d, bin_sa, bin_sb, nullptr) : 0;
        // fp32 tags carry a 20-bit sender field: above 2^20 nodes a crash schedule stores crash ranks
        // there (at most 2^20 senders may crash in one round: n_faulty <= 2^20)
        const bool f32_tags_ok = !s->f32 || s->clean || s->N <= (1ull << 20) || cfg->fault_model != ACS_FAULT_CRASH ||
                                 cfg->n_faulty <= (1u << 20);
        s->binned = allow && f32_tags_ok && s->path == PATH_REGULAR && cfg->delay_max == 0 &&
                    !(s->csr_var && s->f32) &&
                    // (CSR hub rows own the partial slots after the fast path's blocks; CSR plans
                    // always take kBinSB = kRegularBlock receivers per block, so both paths agree:
                    // static_assert below)
                    s->B == 1 && lv != 0 &&
                    binned_supported(s->d, cfg->trim, cfg->rule) && rows_local * s->d < (1ull << 32);
        const char* df = getenv("ACSIM_DEFER_FIN");
        s->defer_fin = s->binned && !partitioned && s->B == 1 && !(df && df[0] == '0');
        kname_lane = s->kname;   // the per-lane kernel's name, should a binned plan not fit (below)
        if (s->binned) {
            char nm[96];
            snprintf(nm, sizeof nm, "k_bin_scatter+%sk_bin_gather<%u,%u%s%s>%s", lv == 2 ? "k_bin_regroup+" : "", s->d,
                     cfg->trim, s->clean ? "" : ",faulty", s->csr_var ? ",csr" : "",
                     cfg->fault_model != ACS_FAULT_NONE ? "+k_bin_tag" : "");
            s->kname = nm;
            if (bin_sb != kBinSB) s->kname += " sb" + std::to_string(bin_sb);
        }
    }
    if (s->n_hub) s->kname += "+k_round_generic(hubs)";
    if (s->f32) s->kname += " [f32]";
    // Block partials: one per receiver block of the round kernel.  The binned path's phase B writes
    // slot b of its bin_sb-row block b, the per-lane kernel slot b of its kRegularBlock-row block b;
    // a binned plan refused below falls back to the per-lane kernel, so the buffer holds the larger
    // count and nblk is reset to the per-lane count on that fallback (launch_round_binned refuses a
    // plan whose block count exceeds nblk).
    const uint32_t nblk_lane = (uint32_t)((rows_local + kRegularBlock - 1) / kRegularBlock);
    const uint32_t nblk_bin = (uint32_t)((rows_local + bin_sb - 1) / bin_sb);
    s->nblk = s->path == PATH_REGULAR ? (s->binned ? nblk_bin : nblk_lane)
            : s->path == PATH_GENERIC ? (uint32_t)s->N
            : s->path == PATH_DENSE   ? dense_nblk(s->N)
                                      : 0u;
    s->nblk_fast = s->nblk;
    s->nblk += (uint32_t)s->n_hub;   // hub rows: one partial slot each, after the fast path's
    s->nblk_init = (uint32_t)((s->N + 255) / 256);
    if (s->nblk_init > 1024) s->nblk_init = 1024;
    const uint32_t nblk_max = s->path == PATH_REGULAR ? (nblk_bin > nblk_lane ? nblk_bin : nblk_lane) + (uint32_t)s->n_hub
                                                      : s->nblk;
    // (virtual partitions: partition p's slice starts at p * nblk, with nblk the count in use)
    const uint64_t nround = (uint64_t)nblk_max * (virt ? nranks : 1);
    const uint64_t ncap = nround > s->nblk_init ? nround : s->nblk_init;

#define CREATE_TRY(expr)                                                                      \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            int code_ = (e_ == hipErrorOutOfMemory || e_ == hipErrorMemoryAllocation) ? ACS_ENOMEM \
                                                                                      : ACS_EDEVICE; \
            fail(code_, "%s failed: %s", #expr, hipGetErrorString(e_));                       \
            release(s);                                                                       \
            return code_;                                                                     \
        }                                                                                     \
    } while (0)

    CREATE_TRY(hipSetDevice(s->device));
    CREATE_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    const uint64_t xlen = s->B * s->Npad;
    s->H = cfg->delay_max + 2;
    s->xstride = xlen + 4;   // +4 elements: 16-byte tail reads (binned phase A staging)
    CREATE_TRY(hipMalloc(&s->xall, s->H * s->xstride * s->es));
    s->x[0] = xb(s, 0);
    s->x[1] = xb(s, 1);
    CREATE_TRY(hipMalloc(&s->st, s->B * sizeof(InstState)));
    CREATE_TRY(hipMemsetAsync(s->st, 0, s->B * sizeof(InstState), s->stream));
    CREATE_TRY(hipMalloc(&s->partial, s->B * ncap * sizeof(double2)));
    CREATE_TRY(hipMalloc(&s->gpart, sizeof(double2)));
    if (s->path == PATH_DENSE) {
        CREATE_TRY(hipMalloc(&s->dsorted, s->N * sizeof(double)));
        CREATE_TRY(hipMalloc(&s->dcounts, 4 * sizeof(uint32_t)));
    }
    CREATE_TRY(hipMalloc(&s->n_done, sizeof(uint32_t)));
    CREATE_TRY(hipHostMalloc(&s->h_ndone, 2 * sizeof(uint32_t), hipHostMallocDefault));
    CREATE_TRY(hipHostMalloc(&s->h_sum, sizeof(RunSummary), kPolledHostFlags));
    CREATE_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&s->h_sum_dev), s->h_sum, 0));
    memset(s->h_sum, 0, sizeof(RunSummary));
    if (s->B <= kMappedStates) {
        CREATE_TRY(hipHostMalloc(&s->h_ms, sizeof(MappedStates), kPolledHostFlags));
        CREATE_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&s->h_ms_dev), s->h_ms, 0));
        memset(s->h_ms, 0, sizeof(MappedStates));
    }
    CREATE_TRY(hipMalloc(&s->sum_scratch, kSummaryScratch));
    {
        const char* v = getenv("ACSIM_EPS_PUB");
        if (!(v && v[0] == '0')) {
            CREATE_TRY(hipMalloc(&s->eacc, 2 * kEaccWords * sizeof(unsigned long long)));
            CREATE_TRY(hipMemsetAsync(s->eacc, 0, 2 * kEaccWords * sizeof(unsigned long long), s->stream));
        }
    }
    CREATE_TRY(hipMemsetAsync(s->sum_scratch, 0, kSummaryScratch, s->stream));
    if (cfg->trace_spread) {
        const uint64_t nt = s->B * ((uint64_t)cfg->max_rounds + 1);
        CREATE_TRY(hipMalloc(&s->trace, nt * sizeof(double)));
        CREATE_TRY(hipMemsetAsync(s->trace, 0xFF, nt * sizeof(double), s->stream));   // NaN
    }
    const bool tagged = cfg->fault_model != ACS_FAULT_NONE;
    if (cfg->fault_model != ACS_FAULT_NONE) {
        CREATE_TRY(hipMalloc(&s->status, s->B * s->N * sizeof(uint32_t)));
        CREATE_TRY(build_fault_status(s->status, s->B, s->N, cfg->n_faulty, cfg->fault_model,
                                      cfg->crash_window, s->mp.key, cfg->instance_offset, s->stream));
        if (s->binned && s->f32 && cfg->fault_model == ACS_FAULT_CRASH && s->N > (1ull << 20)) {
            // crash ranks for the fp32 tags (RoundArgs::crank): faulty nodes grouped by crash round
            std::vector<uint32_t> st(s->N), rank(s->N, 0u), list;
            CREATE_TRY(hipMemcpy(st.data(), s->status, s->N * sizeof(uint32_t), hipMemcpyDeviceToHost));
            const uint32_t W = cfg->crash_window;
            s->coff.assign(W + 1, 0u);
            for (uint64_t i = 0; i < s->N; ++i)
                if (st[i] < W) ++s->coff[st[i] + 1];
            for (uint32_t w = 0; w < W; ++w) s->coff[w + 1] += s->coff[w];
            list.resize(s->coff[W] ? s->coff[W] : 1);
            std::vector<uint32_t> fill(s->coff.begin(), s->coff.end() - 1);
            for (uint64_t i = 0; i < s->N; ++i)
                if (st[i] < W) {
                    rank[i] = fill[st[i]] - s->coff[st[i]];
                    list[fill[st[i]]++] = (uint32_t)i;
                }
            CREATE_TRY(hipMalloc(&s->crank, s->N * sizeof(uint32_t)));
            CREATE_TRY(hipMalloc(&s->clist, list.size() * sizeof(uint32_t)));
            CREATE_TRY(hipMemcpy(s->crank, rank.data(), s->N * sizeof(uint32_t), hipMemcpyHostToDevice));
            CREATE_TRY(hipMemcpy(s->clist, list.data(), list.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
    }
    if (cfg->topology == ACS_TOPO_RANDOM_REGULAR) {
        const uint64_t words = ((rows_local + 63) / 64) * 64ull * s->dp;
        CREATE_TRY(hipMalloc(&s->ell, words * sizeof(uint32_t)));
        CREATE_TRY(hipMemsetAsync(s->ell, 0, words * sizeof(uint32_t), s->stream));
        CREATE_TRY(build_rows(s, s->ell, partitioned ? rank : 0));
        // The binned plans replace the ELLs in the round loop.  A plan can still be refused after
        // it is laid out (a two-level plan whose phase-M image outgrows the LDS, too many runs
        // per receiver block): then every partition keeps its ELL and runs the per-lane kernel,
        // which serves the same configs (binned_supported implies a compiled register variant).
        bool bin_refused = false;
        // narrow stage (ACSIM_BIN_NARROW=1, opt-in): whole unpartitioned rounds with
        // the deferred finalize, whose phase B publishes each round's (min, max) for the next phase A
        const char* nar_env = getenv("ACSIM_BIN_NARROW");
        const bool want_narrow = nar_env && nar_env[0] == '1' && !partitioned && s->defer_fin && s->eacc;
        auto try_plan = [&](BinnedPlan& plan, const uint32_t* ell, uint64_t nr) -> hipError_t {
            if (!s->binned || bin_refused || !nr) return hipSuccess;
            hipError_t e = binned_build(plan, ell, s->N, nr, s->d, s->dp, bin_sa, bin_sb, tagged, s->f32, s->stream,
                                        false, s->status, s->clean, want_narrow);
            if (e == hipErrorNotSupported) {
                bin_refused = true;
                return hipSuccess;
            }
            return e;
        };
        CREATE_TRY(try_plan(s->bin, s->ell, partitioned ? part_rows(s, rank) : s->N));
        if (virt) {
            s->parts.resize(nranks - 1);
            for (int p = 1; p < nranks; ++p) {
                Part& q = s->parts[p - 1];
                CREATE_TRY(hipMalloc(&q.x[0], (xlen + 4) * s->es));
                CREATE_TRY(hipMalloc(&q.x[1], (xlen + 4) * s->es));
                CREATE_TRY(hipMalloc(&q.ell, words * sizeof(uint32_t)));
                CREATE_TRY(hipMemsetAsync(q.ell, 0, words * sizeof(uint32_t), s->stream));
                CREATE_TRY(build_rows(s, q.ell, p));
                CREATE_TRY(try_plan(q.bin, q.ell, part_rows(s, p)));
            }
        }
        if (s->binned && bin_refused) {
            binned_free(s->bin);
            for (Part& q : s->parts) binned_free(q.bin);
            s->binned = false;
            s->defer_fin = false;
            s->kname = kname_lane + (s->f32 ? " [f32]" : "");
            s->nblk = s->nblk_fast = nblk_lane;   // the per-lane kernel's blocks (no hub rows here)
        }
        if (s->binned) {
            // NP-pass phase B (slot-dependent configs: fp64, two passes only; see launch_round_binned)
            if (s->bin.split > 1 && (s->clean || (!s->f32 && s->bin.split == 2)))
                s->kname += " split" + std::to_string(s->bin.split);
            if (s->bin.pkA)   // 14-bit packed phase-A index stream
                s->kname += " pk14A";
            if (s->bin.narrow)   // narrow stage
                s->kname += " narrow";
            if (s->bin.fix) {   // fault fix-up list instead of tagged senders
                const size_t pos = s->kname.find("+k_bin_tag");
                if (pos != std::string::npos) s->kname.replace(pos, 10, "+k_bin_fixup");
            }
            (void)hipFree(s->ell);
            s->ell = nullptr;
            for (Part& q : s->parts) {
                (void)hipFree(q.ell);
                q.ell = nullptr;
            }
        }
    }
    if (cfg->topology == ACS_TOPO_CSR) {
        CREATE_TRY(hipMalloc(&s->rowptr, (s->N + 1) * sizeof(uint64_t)));
        CREATE_TRY(hipMalloc(&s->colidx, (csr_nnz ? csr_nnz : 1) * sizeof(uint32_t)));
        CREATE_TRY(hipMemcpy(s->rowptr, h_rowptr, (s->N + 1) * sizeof(uint64_t), hipMemcpyHostToDevice));
        if (csr_nnz) CREATE_TRY(hipMemcpy(s->colidx, h_colidx, csr_nnz * sizeof(uint32_t), hipMemcpyHostToDevice));
        if (s->csr_var) {   // padded ELL (SELL-64 slice widths), sorted rows when order-independent, binned plan
            const uint64_t words = ((s->N + 63) / 64) * 64ull * s->dp;
            CREATE_TRY(hipMalloc(&s->ell, words * sizeof(uint32_t)));
            CREATE_TRY(hipMalloc(&s->deg, s->N));
            CREATE_TRY(hipMalloc(&s->sw, (s->N + 63) / 64));
            CREATE_TRY(hipMemsetAsync(s->ell, 0xFF, words * sizeof(uint32_t), s->stream));
            CREATE_TRY(launch_csr_to_ell(s->rowptr, s->colidx, s->N, s->d, s->ell, s->deg, s->sw, s->stream));
            if (s->ell_sorted) CREATE_TRY(launch_sort_ell_rows(s->ell, s->N, s->d, s->stream));
            if (s->binned) {
                const hipError_t be = binned_build(s->bin, s->ell, s->N, s->N, s->d, s->dp, bin_sa, kBinSB, tagged,
                                                   s->f32, s->stream, true, s->status);
                if (be == hipErrorNotSupported) {   // the plan does not fit: the per-lane kernel serves the rows
                    binned_free(s->bin);
                    s->binned = false;
                    s->defer_fin = false;
                    s->kname = kname_lane + (s->n_hub ? "+k_round_generic(hubs)" : "") + (s->f32 ? " [f32]" : "");
                    s->nblk_fast = nblk_lane;   // (equal to nblk_bin: CSR plans use kBinSB = kRegularBlock)
                    s->nblk = nblk_lane + (uint32_t)s->n_hub;
                } else {
                    CREATE_TRY(be);
                    (void)hipFree(s->ell);
                    s->ell = nullptr;
                }
            }
        }
    }
    if (s->n_hub || (s->path == PATH_GENERIC && cfg->topology == ACS_TOPO_CSR)) {
        // CSR rows for the generic kernels: the hub rows beside a fast path, or every row on the
        // generic path.  Rows up to kGenericMaxM entries by size class, the rest on the big-m path.
        constexpr uint32_t kCls[] = {64, 256, 1024, 4096, kGenericMaxM};
        std::vector<uint32_t> lists[5], big;
        std::vector<uint64_t> mv;
        for (uint64_t i = 0; i < s->N; ++i) {
            const uint64_t mi = h_rowptr[i + 1] - h_rowptr[i] + 1;
            if (s->n_hub && mi - 1 <= s->d) continue;   // a fast-path row
            if (mi > kGenericMaxM) {
                big.push_back((uint32_t)i);
                mv.push_back(mi);
                continue;
            }
            int k = 0;
            while (mi > kCls[k]) ++k;
            lists[k].push_back((uint32_t)i);
        }
        std::vector<uint32_t> all;
        for (int k = 0; k < 5; ++k) {
            if (lists[k].empty()) continue;
            s->gcls.push_back({all.size(), lists[k].size(), kCls[k]});
            all.insert(all.end(), lists[k].begin(), lists[k].end());
        }
        s->gen_base = s->n_hub ? s->nblk_fast : 0;
        if (!all.empty()) {
            CREATE_TRY(hipMalloc(&s->gen_ids, all.size() * sizeof(uint32_t)));
            CREATE_TRY(hipMemcpy(s->gen_ids, all.data(), all.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        }
        CREATE_TRY(generic_big_build(s->big, big, mv, s->f32, s->stream));
        s->big.pbase = s->gen_base + all.size();
    } else if (s->path == PATH_GENERIC && s->m > kGenericMaxM) {   // receivers for the big-m path
        std::vector<uint32_t> ids;
        std::vector<uint64_t> mv;
        for (uint64_t i = 0; i < s->N; ++i) {
            const uint64_t mi = cfg->topology == ACS_TOPO_CSR ? h_rowptr[i + 1] - h_rowptr[i] + 1 : s->m;
            if (mi > kGenericMaxM) {
                ids.push_back((uint32_t)i);
                mv.push_back(mi);
            }
        }
        CREATE_TRY(generic_big_build(s->big, ids, mv, s->f32, s->stream));
    }
    CREATE_TRY(launch_init_values(s->x[0], s->B, s->N, s->mp.key, cfg->instance_offset, s->f32, s->stream));
    for (Part& q : s->parts)
        CREATE_TRY(launch_init_values(q.x[0], s->B, s->N, s->mp.key, cfg->instance_offset, s->f32, s->stream));
#undef CREATE_TRY
    // chunked exchange: clean binned partitions whose row blocks split into
    // ACSIM_XCHUNKS chunks of whole source blocks AND of whole phase-B receiver blocks (chunk k's
    // exchange is recorded after phase B's blocks [k*qpc, (k+1)*qpc), which must cover exactly the
    // chunk's rows); 0 or 1 keeps the unchunked sequence.  Default: 4 for virtual partitions (GPU-
    // tested bit-exact), and the per-round all-gather for a real multi-rank communicator until a
    // multi-GPU run has matched the golden hash (the grouped send / receive path is opt-in there).
    if (partitioned && s->binned && s->clean) {
        uint32_t K = (comm_id && nranks > 1) ? 0u : 4u;
        if (const char* v = getenv("ACSIM_XCHUNKS")) K = (uint32_t)strtoul(v, nullptr, 10);
        if (K >= 2 && K <= acs_sim::kMaxX && s->rows_per % ((uint64_t)K * bin_sa) == 0 &&
            (s->rows_per / K) % s->bin.SB == 0)
            s->xchunks = K;
    }
    s->bin_sa = bin_sa;
    if (s->xchunks) {
        hipError_t e = hipStreamCreateWithFlags(&s->cstream, hipStreamNonBlocking);
        for (uint32_t k = 0; e == hipSuccess && k < s->xchunks; ++k) {
            e = hipEventCreateWithFlags(&s->ev_b[k], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_x[k], hipEventDisableTiming);
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&s->ev_fin, hipEventDisableTiming);
        if (e != hipSuccess) {
            fail(ACS_EDEVICE, "comm stream / events: %s", hipGetErrorString(e));
            release(s);
            return ACS_EDEVICE;
        }
        s->kname += " xchunks" + std::to_string(s->xchunks);
    }
    if (comm_id) {
        ncclUniqueId id;
        memcpy(&id, comm_id, sizeof id);
        ncclResult_t nr = ncclCommInitRank(&s->comm, nranks, id, rank);
        if (nr != ncclSuccess) {
            fail(ACS_ECOMM, "ncclCommInitRank(%d ranks, rank %d) failed: %s", nranks, rank, ncclGetErrorString(nr));
            release(s);
            return ACS_ECOMM;
        }
    }
    rc = init_state(s, 0);
    if (rc) {
        release(s);
        return rc;
    }
    *out = s;
    return ACS_OK;
}

// ------------------------------------------------------------------------- C ABI
extern "C" {

int acs_abi_version(void) { return ACS_ABI_VERSION; }

const char* acs_last_error(void) { return g_err.c_str(); }

int acs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return fail(ACS_EDEVICE, "hipGetDeviceCount failed");
    return n;
}

int acs_runtime_info(char* out, uint64_t cap) {
    if (!out || cap == 0) return fail(ACS_EINVAL, "acs_runtime_info: empty buffer");
    int hv = 0, nv = 0;
    if (hipRuntimeGetVersion(&hv) != hipSuccess) return fail(ACS_EDEVICE, "hipRuntimeGetVersion failed");
    if (ncclGetVersion(&nv) != ncclSuccess) return fail(ACS_ECOMM, "ncclGetVersion failed");
    snprintf(out, cap, "hip %d rccl %d polled-host-flags 0x%x", hv, nv, kPolledHostFlags);
    return ACS_OK;
}

int acs_create(const acs_config* cfg, int backend, const int* devices, int n_devices, acs_sim** out) {
    if (out) *out = nullptr;
    int rc = validate(cfg);
    if (rc) return rc;
    if (backend != ACS_HIP)
        return fail(ACS_EUNSUPPORTED, "libacsim implements ACS_HIP only (the CPU spec reference is the "
                                      "test oracle in oracle/, not a product backend)");
    if (n_devices != 1 || !devices)
        return fail(ACS_EINVAL, "exactly one device per handle (shard across processes, one rank per GPU)");
    if (cfg->topology == ACS_TOPO_CSR) return fail(ACS_EINVAL, "CSR topology: use acs_create_csr");
    return create_impl(cfg, devices[0], 1, 0, nullptr, 0, out);
}

int acs_create_csr(const acs_config* cfg, const uint64_t* rowptr, const uint32_t* colidx, int device,
                   acs_sim** out) {
    if (out) *out = nullptr;
    if (!cfg || cfg->topology != ACS_TOPO_CSR) return fail(ACS_EINVAL, "config topology must be ACS_TOPO_CSR");
    if (!rowptr || !colidx) return fail(ACS_EINVAL, "null CSR arrays");
    return create_impl(cfg, device, 1, 0, nullptr, 0, out, rowptr, colidx);
}

int acs_comm_id_size(void) { return (int)sizeof(ncclUniqueId); }

int acs_get_comm_id(void* out, uint64_t n) {
    if (!out || n < sizeof(ncclUniqueId)) return fail(ACS_EINVAL, "buffer must hold %zu bytes", sizeof(ncclUniqueId));
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof id);
    return ACS_OK;
}

int acs_create_partitioned(const acs_config* cfg, int device, int n_ranks, int rank, const void* comm_id,
                           uint64_t id_len, acs_sim** out) {
    return create_impl(cfg, device, n_ranks, rank, comm_id, id_len, out);
}

void acs_destroy(acs_sim* s) { release(s); }

static void fill_info(acs_sim* s, const std::vector<InstState>& v, acs_round_info* out) {
    (void)s;
    if (!out) return;
    memset(out, 0, sizeof *out);
    uint64_t nd = 0;
    double sp = -INFINITY;
    uint32_t rmax = 0;
    for (const InstState& e : v) {
        nd += e.done;
        if (e.spread > sp) sp = e.spread;
        if (e.rounds > rmax) rmax = e.rounds;
    }
    out->round = rmax;
    out->done = nd == v.size();
    out->spread = sp;
    out->lo = v[0].lo;
    out->hi = v[0].hi;
    out->instances_done = nd;
}

int acs_round(acs_sim* s, uint32_t k, acs_round_info* out) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    HIP_TRY(hipSetDevice(s->device));
    int rc = advance(s, k);
    if (rc) return rc;
    std::vector<InstState> v;
    rc = read_states(s, v, true);   // (EPS calls end with the states already fetched)
    if (rc) return rc;
    fill_info(s, v, out);
    return ACS_OK;
}

int acs_run(acs_sim* s, acs_result* out) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    HIP_TRY(hipSetDevice(s->device));
    const auto t0 = std::chrono::steady_clock::now();
    s->want_summary = out != nullptr;
    s->summary_ready = false;
    int rc = advance(s, s->c.max_rounds);
    s->want_summary = false;
    if (rc) return rc;
    if (!s->summary_ready) HIP_TRY(hipStreamSynchronize(s->stream));
    const auto t1 = std::chrono::steady_clock::now();
    if (out) {   // the summary is folded on the device: 32 bytes back instead of B states
        if (!s->summary_ready)
            if (int rc2 = summary_and_wait(s)) return rc2;
        s->summary_ready = false;
        const RunSummary& r = *s->h_sum;
        memset(out, 0, sizeof *out);
        out->n_instances = s->B;
        out->rounds_max = r.rounds_max;
        out->n_converged = (uint32_t)r.n_converged;
        out->node_rounds = s->N * r.rounds_sum;
        double sp;
        memcpy(&sp, &r.spread_max_bits, sizeof sp);
        out->final_spread_max = s->B ? sp : -INFINITY;
        out->wall_seconds = std::chrono::duration<double>(t1 - t0).count();
    }
    return ACS_OK;
}

int acs_sync(acs_sim* s) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ACS_OK;
}

int acs_get_values(acs_sim* s, uint64_t b, void* out, uint64_t n) {
    if (!s || !out || b >= s->B || n < s->N) return fail(ACS_EINVAL, "bad get_values arguments");
    HIP_TRY(hipSetDevice(s->device));
    InstState e;
    HIP_TRY(hipMemcpyAsync(&e, s->st + b, sizeof e, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    HIP_TRY(hipMemcpyAsync(out, xat(s, xb(s, e.rounds), b * s->Npad), s->N * s->es, hipMemcpyDeviceToHost,
                           s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ACS_OK;
}

int acs_get_all_values(acs_sim* s, void* out, uint64_t n) {
    if (!s || !out || n < s->B * s->N) return fail(ACS_EINVAL, "bad get_all_values arguments");
    HIP_TRY(hipSetDevice(s->device));
    std::vector<InstState> v;
    int rc = read_states(s, v);
    if (rc) return rc;
    // instances stop at different rounds: x_b lives in buffer rounds_b % H.  Copy the buffers
    // holding any instance whole (one transfer each), then pick every instance's row on the host.
    std::vector<unsigned char> used(s->H, 0);
    for (const InstState& e : v) used[e.rounds % s->H] = 1;
    const uint64_t row = s->N * s->es, buf = s->B * s->Npad * s->es;
    uint32_t only = s->H;
    for (uint32_t q = 0; q < s->H; ++q)
        if (used[q]) only = only == s->H ? q : s->H + 1;
    if (only < s->H && s->Npad == s->N) {   // every instance in one buffer: straight into `out`
        HIP_TRY(hipMemcpyAsync(out, xb(s, only), s->B * row, hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        return ACS_OK;
    }
    std::vector<unsigned char> h((size_t)buf);
    for (uint32_t q = 0; q < s->H; ++q) {
        if (!used[q]) continue;
        HIP_TRY(hipMemcpyAsync(h.data(), xb(s, q), buf, hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(hipStreamSynchronize(s->stream));
        for (uint64_t b = 0; b < s->B; ++b)
            if (v[b].rounds % s->H == q)
                memcpy(static_cast<unsigned char*>(out) + b * row, h.data() + b * s->Npad * s->es, row);
    }
    return ACS_OK;
}

int acs_get_partition_values(acs_sim* s, int partition, void* out, uint64_t n) {
    if (!s || !out || n < s->N) return fail(ACS_EINVAL, "bad arguments");
    if (partition < 0 || partition >= (s->virt ? s->nranks : 1)) return fail(ACS_EINVAL, "no such partition copy");
    HIP_TRY(hipSetDevice(s->device));
    InstState e;
    HIP_TRY(hipMemcpyAsync(&e, s->st, sizeof e, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    const double* src = partition == 0 ? s->x[e.rounds & 1u] : s->parts[partition - 1].x[e.rounds & 1u];
    HIP_TRY(hipMemcpyAsync(out, src, s->N * s->es, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ACS_OK;
}

int acs_get_instance_rounds(acs_sim* s, uint32_t* out, uint64_t n) {
    if (!s || !out || n < s->B) return fail(ACS_EINVAL, "bad arguments");
    std::vector<InstState> v;
    int rc = read_states(s, v);
    if (rc) return rc;
    for (uint64_t b = 0; b < s->B; ++b) out[b] = v[b].rounds;
    return ACS_OK;
}

int acs_get_instance_converged(acs_sim* s, uint8_t* out, uint64_t n) {
    if (!s || !out || n < s->B) return fail(ACS_EINVAL, "bad arguments");
    std::vector<InstState> v;
    int rc = read_states(s, v);
    if (rc) return rc;
    for (uint64_t b = 0; b < s->B; ++b) out[b] = (uint8_t)v[b].converged;
    return ACS_OK;
}

int acs_get_instance_spread(acs_sim* s, double* out, uint64_t n) {
    if (!s || !out || n < s->B) return fail(ACS_EINVAL, "bad arguments");
    std::vector<InstState> v;
    int rc = read_states(s, v);
    if (rc) return rc;
    for (uint64_t b = 0; b < s->B; ++b) out[b] = v[b].spread;
    return ACS_OK;
}

int acs_get_spread_trace(acs_sim* s, uint64_t b, double* out, uint64_t n, uint64_t* n_out) {
    if (!s || !out || b >= s->B) return fail(ACS_EINVAL, "bad arguments");
    if (!s->trace) return fail(ACS_EINVAL, "trace_spread was not enabled");
    InstState e;
    HIP_TRY(hipMemcpyAsync(&e, s->st + b, sizeof e, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    uint64_t cnt = (uint64_t)e.rounds + 1;
    if (cnt > n) cnt = n;
    HIP_TRY(hipMemcpyAsync(out, s->trace + b * ((uint64_t)s->c.max_rounds + 1), cnt * sizeof(double),
                           hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    if (n_out) *n_out = cnt;
    return ACS_OK;
}

int acs_set_state(acs_sim* s, uint32_t round, const void* x, uint64_t n) {
    if (!s || !x || n != s->B * s->N) return fail(ACS_EINVAL, "set_state needs B*N values");
    if (round > s->c.max_rounds) return fail(ACS_EINVAL, "round > max_rounds");
    // Values must be finite and bounded (sums of up to kGenericBigMaxM = 2^27 of them stay finite, so no
    // NaN can ever appear in x: the tagged binned phase B reads every quiet NaN as a sender tag),
    // and -0.0 is canonicalised to +0.0 (sorted value sequences stay unique).
    std::vector<unsigned char> canon(n * s->es);
    if (s->f32) {
        const float* xf = static_cast<const float*>(x);
        float* cf = reinterpret_cast<float*>(canon.data());
        for (uint64_t k = 0; k < n; ++k) {
            if (!(fabsf(xf[k]) <= 1e30f)) return fail(ACS_EINVAL, "set_state: value %llu is not finite or |x| > 1e30", (unsigned long long)k);
            cf[k] = xf[k] + 0.0f;
        }
    } else {
        const double* xd = static_cast<const double*>(x);
        double* cd = reinterpret_cast<double*>(canon.data());
        for (uint64_t k = 0; k < n; ++k) {
            if (!(fabs(xd[k]) <= 1e300)) return fail(ACS_EINVAL, "set_state: value %llu is not finite or |x| > 1e300", (unsigned long long)k);
            cd[k] = xd[k] + 0.0;
        }
    }
    x = canon.data();
    HIP_TRY(hipSetDevice(s->device));
    for (uint64_t b = 0; b < s->B; ++b) {
        const void* hb = xat(s, x, b * s->N);
        // every delay-history buffer restarts from x; one buffer when synchronous
        for (uint32_t q = 0; q < (s->c.delay_max ? s->H : 1u); ++q)
            HIP_TRY(hipMemcpyAsync(xat(s, s->c.delay_max ? xb(s, q) : xb(s, round), b * s->Npad), hb, s->N * s->es,
                                   hipMemcpyHostToDevice, s->stream));
        for (Part& q : s->parts)
            HIP_TRY(hipMemcpyAsync(xat(s, q.x[round & 1u], b * s->Npad), hb, s->N * s->es, hipMemcpyHostToDevice,
                                   s->stream));
    }
    return init_state(s, round);
}

int acs_get_fault_status(acs_sim* s, uint32_t* out, uint64_t n) {
    if (!s || !out || n < s->B * s->N) return fail(ACS_EINVAL, "bad arguments");
    HIP_TRY(hipSetDevice(s->device));
    if (!s->status) {
        for (uint64_t k = 0; k < s->B * s->N; ++k) out[k] = kHonest;
        return ACS_OK;
    }
    HIP_TRY(hipMemcpyAsync(out, s->status, s->B * s->N * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(hipStreamSynchronize(s->stream));
    return ACS_OK;
}

int acs_get_neighbors(acs_sim* s, uint32_t* out, uint64_t n) {
    if (!s || !out) return fail(ACS_EINVAL, "bad arguments");
    if (s->c.topology != ACS_TOPO_RANDOM_REGULAR) return fail(ACS_EINVAL, "not a RANDOM_REGULAR topology");
    if (n < s->N * s->d) return fail(ACS_EINVAL, "buffer too small");
    HIP_TRY(hipSetDevice(s->device));
    // always rebuild the full graph in spec (slot) order on the side: the handle's own ELL may be
    // sorted and may hold only this rank's rows
    const uint64_t words = ((s->N + 63) / 64) * 64ull * s->dp;
    std::vector<uint32_t> h(words);
    uint32_t* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, words * sizeof(uint32_t)));
    const uint64_t gseed = s->c.graph_seed ? s->c.graph_seed : s->c.seed;
    hipError_t e = launch_build_ell(tmp, s->N, 0, s->N, s->d, s->dp, make_feistel(s->N, gseed), s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), tmp, words * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(tmp);
    HIP_TRY(e);
    for (uint64_t i = 0; i < s->N; ++i)
        for (uint32_t t = 0; t < s->d; ++t)
            out[i * s->d + t] = h[(((i >> 6) * (s->dp >> 2) + (t >> 2)) * 64 + (i & 63)) * 4 + (t & 3)];
    return ACS_OK;
}

int acs_set_kernel_timing(acs_sim* s, int enable) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    HIP_TRY(hipSetDevice(s->device));
    int rc = harvest_timing(s);
    if (rc) return rc;
    s->timing = enable > 0 ? (uint32_t)enable : enable < 0 ? (uint32_t)(-(int64_t)enable) : 0u;
    s->timing_runs = enable < 0;
    s->run_end = nullptr;
    s->timing_ctr = 0;
    s->timed_ms = 0.0;
    s->timed_launches = 0;
    return ACS_OK;
}

int acs_get_kernel_timing(acs_sim* s, double* total_ms, uint64_t* launches, char* kernel_name,
                          uint64_t name_cap) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    HIP_TRY(hipSetDevice(s->device));
    int rc = harvest_timing(s);
    if (rc) return rc;
    if (total_ms) *total_ms = s->timed_ms;
    if (launches) *launches = s->timed_launches;
    if (kernel_name && name_cap) {
        strncpy(kernel_name, s->kname.c_str(), name_cap - 1);
        kernel_name[name_cap - 1] = 0;
    }
    return ACS_OK;
}

}  // extern "C"
