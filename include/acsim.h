/*
 * acsim.h — C ABI of the MI355X-native approximate-consensus round engine.
 *
 * Provenance.  The upstream reference (Dariusrussellkish/approximate-consensus-simulation,
 * mounted at /root/reference) holds exactly one file, README.md:1 ("# eventual-consensus-simulation"),
 * and no code.  There is therefore no upstream function this ABI can replace line for line; every
 * entry point below replaces the spec-level operation named in SURVEY.md §8(a)/(b), and the
 * semantics are those of SURVEY.md Appendix A (the frozen spec that stands in for the missing
 * reference).  Each declaration cites the §8 row / §A section it implements.
 *
 * Conventions.
 *  - Plain C, no C++ or torch types: pointers, sizes and POD structs only.
 *  - Every function returns 0 (ACS_OK) or a negative ACS_E* status; no exceptions cross the ABI.
 *    acs_last_error() returns a thread-local message for the last non-zero status.
 *  - The handle owns every device buffer.  Callers own the host buffers they pass in; the library
 *    copies into / out of them and retains no pointer after return.
 *  - A handle is not thread-safe; distinct handles may be used from distinct threads.
 */
#ifndef ACSIM_H
#define ACSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACS_ABI_VERSION 3   /* 2: acs_config.delay_max (bounded-delay rounds);
                               3: acs_config.missing_policy (was reserved0), acs_get_all_values */

/* status codes */
#define ACS_OK            0
#define ACS_EINVAL       (-1)
#define ACS_ENOMEM       (-2)
#define ACS_EDEVICE      (-3)
#define ACS_ECOMM        (-4)
#define ACS_EUNSUPPORTED (-5)

/* backends.  The product library implements ACS_HIP only; the CPU spec reference lives in
 * oracle/ as test infrastructure and is not reachable through this library (ACS_CPU returns
 * ACS_EUNSUPPORTED here). */
#define ACS_CPU 0
#define ACS_HIP 1

/* topology (§A.3) */
#define ACS_TOPO_COMPLETE        0
#define ACS_TOPO_RANDOM_REGULAR  1
#define ACS_TOPO_CSR             2   /* user-supplied adjacency, see acs_create_csr (§8(f) row 1) */

/* update rule (§A.7) */
#define ACS_RULE_AVERAGE       0
#define ACS_RULE_TRIMMED_MEAN  1
#define ACS_RULE_MIDPOINT      2
#define ACS_RULE_DLPSW_SELECT  3
/* W-MSR (LeBlanc et al. 2013): drop up to t entries strictly below the receiver's
 * own value (the smallest ones) and up to t strictly above it (the largest), average the rest */
#define ACS_RULE_WMSR          4

/* fault model (§A.4) */
#define ACS_FAULT_NONE       0
#define ACS_FAULT_CRASH      1
#define ACS_FAULT_BYZANTINE  2

/* Byzantine strategy (§A.4) */
#define ACS_BYZ_SPLIT     0
#define ACS_BYZ_RANDOM    1
#define ACS_BYZ_CONSTANT  2

/* termination (§A.8) */
#define ACS_TERM_EPS    0
#define ACS_TERM_FIXED  1

/* missing-message policy (§A.6): a crashed-silent or dropped message is replaced
 * by the receiver's own value (SELF, the §A.6 default), or removed from S_i (OMIT: m_i shrinks;
 * the trimming rules keep x_i when m_i <= 2t) */
#define ACS_MISSING_SELF 0
#define ACS_MISSING_OMIT 1

/* value type (§A.0): fp64, or binary32 throughout */
#define ACS_F64 0
#define ACS_F32 1

/* Philox streams (§A.1) */
#define ACS_STREAM_INIT          0u
#define ACS_STREAM_DROP          1u
#define ACS_STREAM_FAULTSET      2u
#define ACS_STREAM_CRASH_ROUND   3u
#define ACS_STREAM_CRASH_PARTIAL 4u
#define ACS_STREAM_BYZ           5u
#define ACS_STREAM_GRAPH         6u
#define ACS_STREAM_DELAY         7u   /* bounded-delay rounds */

/* Opaque simulation handle. */
typedef struct acs_sim acs_sim;

/* One simulation configuration.  POD; struct_size must equal sizeof(acs_config). */
typedef struct acs_config {
    uint32_t struct_size;
    uint64_t n_nodes;          /* N */
    uint64_t n_instances;      /* B: independent instances held by this handle */
    uint32_t topology;         /* ACS_TOPO_* */
    uint32_t degree;           /* d (even, >= 2) for RANDOM_REGULAR */
    uint32_t rule;             /* ACS_RULE_* */
    uint32_t trim;             /* t */
    uint32_t fault_model;      /* ACS_FAULT_* */
    uint32_t n_faulty;         /* f */
    uint32_t byz_strategy;     /* ACS_BYZ_* */
    double   byz_delta;        /* Δ */
    double   byz_const;        /* c */
    uint32_t crash_window;     /* W >= 1 */
    double   loss_p;           /* message-loss probability in [0,1) */
    uint32_t mask_group;       /* G >= 1: instances b with equal b - b%G share drop masks */
    double   eps;              /* ε */
    uint32_t max_rounds;       /* round cap (EPS) or exact round count (FIXED) */
    uint32_t termination;      /* ACS_TERM_* */
    uint32_t dtype;            /* ACS_F64 | ACS_F32 */
    uint64_t seed;             /* Philox key for every stream except GRAPH */
    uint64_t graph_seed;       /* Philox key for GRAPH; 0 means "use seed" */
    uint32_t trace_spread;     /* 1: keep spread^r for every round (per instance) */
    uint32_t omp_threads;      /* CPU oracle only; ignored by the HIP library */
    uint64_t instance_offset;  /* global id of local instance 0 (multi-GPU instance sharding, §8e) */
    uint32_t delay_max;        /* D: bounded-delay rounds; 0 = synchronous (§A.6) */
    uint32_t missing_policy;   /* ACS_MISSING_*: what a missing message becomes */
} acs_config;

/* Result of acs_round. For B > 1: round = max rounds over instances,
 * spread = max current spread over instances, lo/hi = instance 0's honest min/max. */
typedef struct acs_round_info {
    uint32_t round;            /* rounds executed so far (max over instances) */
    uint32_t done;             /* 1 when every instance has terminated */
    double   spread;
    double   lo;
    double   hi;
    uint64_t instances_done;
} acs_round_info;

/* Result of acs_run. */
typedef struct acs_result {
    uint32_t rounds_max;       /* max over instances of rounds executed */
    uint32_t n_converged;      /* instances with final spread <= eps */
    uint64_t node_rounds;      /* Σ_b N · rounds_executed(b) */
    double   wall_seconds;     /* host wall time of this call */
    double   final_spread_max; /* max over instances of final spread */
    uint64_t n_instances;
} acs_result;

/* §8b: create a simulation (validates the §A.8 constraints, allocates HBM, builds the graph,
 * the fault schedule and x^0 on the device).  devices/n_devices: exactly one device id. */
int acs_create(const acs_config* cfg, int backend, const int* devices, int n_devices,
               struct acs_sim** out);

/* §8(f) row 1: a simulation on a user-supplied graph in CSR form (cfg->topology = ACS_TOPO_CSR;
 * cfg->degree is ignored).  Receiver i's entries are itself (entry 0, no slot) followed by the
 * senders colidx[rowptr[i] + t], t < deg(i) = rowptr[i+1] - rowptr[i], on slot s = rowptr[i] + t;
 * m_i = deg(i) + 1 varies per receiver (trim rules need m_i > 2t for every i).  rowptr has N+1
 * entries (rowptr[0] = 0, non-decreasing, rowptr[N] < 2^34), colidx rowptr[N] entries < N.
 * Both arrays are copied to the device. */
int acs_create_csr(const acs_config* cfg, const uint64_t* rowptr, const uint32_t* colidx, int device,
                   struct acs_sim** out);

/* §8(e) node partitioning of ONE RANDOM_REGULAR instance over n_ranks GPUs (cfg5), one process
 * (or thread) per GPU.  Rank r owns the 64-aligned row block [r*R, (r+1)*R) ∩ [0, N),
 * R = ceil(ceil(N/n_ranks)/64)*64, keeps the full x on its GPU, and after every round exchanges
 * x^{r+1} with an in-place RCCL all-gather over xGMI plus an all-reduce of the honest
 * (-min, max) for the ε test, so every rank holds identical state.
 *   acs_get_comm_id: rank 0 creates the RCCL unique id (acs_comm_id_size() bytes) that every
 *   rank passes to acs_create_partitioned (any out-of-band channel, e.g. torch.distributed).
 *   comm_id == NULL with n_ranks > 1 simulates all n_ranks partitions on `device` with private
 *   x copies and a device-memcpy all-gather (validation of the partitioned data flow on one GPU;
 *   rank must be 0).  n_ranks == 1 behaves like acs_create. */
int acs_comm_id_size(void);
int acs_get_comm_id(void* out, uint64_t n);
int acs_create_partitioned(const acs_config* cfg, int device, int n_ranks, int rank,
                           const void* comm_id, uint64_t id_len, struct acs_sim** out);
/* Virtual partitions only: the private x copy of one partition (all copies are identical after
 * every round's all-gather; partition 0's copy is what acs_get_values returns). */
int acs_get_partition_values(struct acs_sim* sim, int partition, void* out, uint64_t n);

/* §8(a) a10/a9: advance every unfinished instance by at most k rounds; stops at convergence. */
int acs_round(struct acs_sim* sim, uint32_t k, acs_round_info* out);

/* §8(a) a11: run to convergence (EPS) or exactly max_rounds (FIXED). */
int acs_run(struct acs_sim* sim, acs_result* out);

/* Copy instance's current node values (N values of the config dtype) into a caller buffer. */
int acs_get_values(struct acs_sim* sim, uint64_t instance, void* out, uint64_t n);

/* Every instance's current values (B*N values, instance-major) in one call; instances that
 * terminated at different rounds are each read from their own round's buffer. */
int acs_get_all_values(struct acs_sim* sim, void* out, uint64_t n);

/* Per-instance rounds executed / converged flag / current spread. */
int acs_get_instance_rounds(struct acs_sim* sim, uint32_t* out, uint64_t n_instances);
int acs_get_instance_converged(struct acs_sim* sim, uint8_t* out, uint64_t n_instances);
int acs_get_instance_spread(struct acs_sim* sim, double* out, uint64_t n_instances);

/* Spread trace spread^0..spread^rounds of one instance (needs trace_spread = 1).
 * *n_out receives the number of values written (rounds + 1, capped at n). */
int acs_get_spread_trace(struct acs_sim* sim, uint64_t instance, double* out, uint64_t n,
                         uint64_t* n_out);

/* Resume (§A.9): set every instance to round `round` with values x (B*N values, instance-major).
 * Instances become unfinished unless the EPS test already holds at `round`. */
int acs_set_state(struct acs_sim* sim, uint32_t round, const void* x, uint64_t n);

/* Device-side fault schedule (§A.4): per node u32 status, 0xFFFFFFFF honest, 0xFFFFFFFE
 * Byzantine, otherwise the crash round r_v.  out holds B*N words. */
int acs_get_fault_status(struct acs_sim* sim, uint32_t* out, uint64_t n);

/* Adjacency (§A.3) of a RANDOM_REGULAR graph: out[i*d + t] = nbr(i, t). */
int acs_get_neighbors(struct acs_sim* sim, uint32_t* out, uint64_t n);

/* Kernel timing (bench measurement, §8d): while enabled, HIP events bracket the launches of the
 * round kernel on the handle's stream — every round for enable == 1, every enable-th round for
 * enable > 1 (each event pair idles the stream for a few µs, so the bench samples); enable < 0
 * brackets runs of -enable consecutive rounds with one pair each (a run ends at the end of an
 * acs_round / acs_run call at the latest) and counts every round of a run as one launch; 0 disables.
 * A run's pair brackets EVERYTHING the handle enqueues between its first and last round, not only
 * the round kernels: on node-partitioned handles the RCCL exchange, the (-min, max) all-reduce and
 * the finalize; on EPS runs of long rounds, which wait for each 16-round chunk's verdict before
 * enqueuing the next, the host round trip at a chunk boundary inside the run.  Use enable >= 1
 * for a kernel-only figure there (bench.py uses run mode on the one-instance cfg4 legs only).
 * acs_get_kernel_timing returns the summed device time and bracketed launch count since the
 * last reset, plus the name of the round kernel in use. */
int acs_set_kernel_timing(struct acs_sim* sim, int enable);
int acs_get_kernel_timing(struct acs_sim* sim, double* total_ms, uint64_t* launches,
                          char* kernel_name, uint64_t name_cap);

/* Wait for all device work of this handle. */
int acs_sync(struct acs_sim* sim);

/* Process-level facts for multi-GPU launchers (bench.py, acsim.rendezvous): the number of HIP
 * devices visible (hipGetDeviceCount), and the HIP runtime and RCCL versions this library is
 * running on, as "hip <hipRuntimeGetVersion> rccl <ncclGetVersion>" (NUL-terminated, cut to cap). */
int acs_device_count(void);
int acs_runtime_info(char* out, uint64_t cap);

void acs_destroy(struct acs_sim* sim);
const char* acs_last_error(void);
int acs_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ACSIM_H */
