/*
 * acs_oracle.h — CPU restatement of the approximate-consensus spec.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline.  The product (libacsim.so) never links or
 * calls it.
 *
 * Parity status: the upstream reference has no code (/root/reference/README.md:1 is its only
 * line), so there is nothing upstream to pin against: upstream parity is UNPINNED.  This file
 * restates SURVEY.md Appendix A (the frozen spec that replaces the missing reference); every
 * function cites the §A rule it follows.  The restatement is pinned by (1) the Random123
 * Philox4x32-10 known-answer vectors (tests/golden/philox_kat.json), (2) an independent numpy
 * restatement (tests/spec_np.py) that must agree bit for bit, and (3) committed golden vectors
 * (tests/golden/) generated from the two in agreement.
 */
#ifndef ACS_ORACLE_H
#define ACS_ORACLE_H

#include <stdint.h>
#include "../include/acsim.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct acso_sim acso_sim;

/* primitives (§A.1, §A.3, §A.5, §A.7) */
void     acso_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint32_t acso_draw(uint64_t seed, uint32_t stream, uint32_t b, uint32_t r, uint64_t s);
double   acso_u53(uint32_t w0, uint32_t w1);
uint64_t acso_feistel_perm(uint64_t n, uint64_t graph_seed, uint32_t k, uint64_t v, int inverse);
uint32_t acso_drop_threshold(double p);
double   acso_tree_sum(const double* a, uint64_t n);
int      acso_validate(const acs_config* cfg);

/* simulation (§A.2–§A.9) */
int  acso_create(const acs_config* cfg, acso_sim** out);
int  acso_create_csr(const acs_config* cfg, const uint64_t* rowptr, const uint32_t* colidx, acso_sim** out);
int  acso_round(acso_sim* sim, uint32_t k, acs_round_info* out);
int  acso_run(acso_sim* sim, acs_result* out);
int  acso_get_values(acso_sim* sim, uint64_t instance, double* out, uint64_t n);
int  acso_get_instance_rounds(acso_sim* sim, uint32_t* out, uint64_t n);
int  acso_get_instance_converged(acso_sim* sim, uint8_t* out, uint64_t n);
int  acso_get_instance_spread(acso_sim* sim, double* out, uint64_t n);
int  acso_get_spread_trace(acso_sim* sim, uint64_t instance, double* out, uint64_t n,
                           uint64_t* n_out);
int  acso_set_state(acso_sim* sim, uint32_t round, const double* x, uint64_t n);
int  acso_get_fault_status(acso_sim* sim, uint32_t* out, uint64_t n);
int  acso_get_neighbors(acso_sim* sim, uint32_t* out, uint64_t n);
void acso_destroy(acso_sim* sim);
const char* acso_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
