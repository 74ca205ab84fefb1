/*
 * selftest.c — drives the CPU oracle through every config family under AddressSanitizer and
 * UndefinedBehaviorSanitizer ("race detection / sanitizers": the CPU reference built
 * with -fsanitize=address,undefined).  TEST INFRASTRUCTURE ONLY, built by `make -C oracle asan`
 * and run by tests/test_oracle.py.  Prints one line per case and "selftest ok" at the end; any
 * sanitizer report aborts with a non-zero status.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "acs_oracle.h"

static acs_config base(void) {
    acs_config c;
    memset(&c, 0, sizeof c);
    c.struct_size = sizeof c;
    c.n_instances = 1;
    c.crash_window = 1;
    c.mask_group = 1;
    c.eps = 1e-6;
    c.max_rounds = 200;
    c.trace_spread = 1;
    c.omp_threads = 2;
    return c;
}

static int run_case(const char* name, const acs_config* c, const uint64_t* rowptr, const uint32_t* colidx) {
    acso_sim* s = NULL;
    int rc = rowptr ? acso_create_csr(c, rowptr, colidx, &s) : acso_create(c, &s);
    if (rc) {
        printf("%s: create failed %d (%s)\n", name, rc, acso_last_error());
        return 1;
    }
    acs_round_info info;
    rc = acso_round(s, 3, &info);
    const uint64_t n = c->n_nodes * c->n_instances;
    double* x = (double*)malloc(n * sizeof(double));
    for (uint64_t b = 0; !rc && b < c->n_instances; ++b) rc = acso_get_values(s, b, x + b * c->n_nodes, c->n_nodes);
    if (!rc) rc = acso_set_state(s, info.round, x, n);   /* resume from the state just read */
    acs_result res;
    if (!rc) rc = acso_run(s, &res);
    double tr[256];
    uint64_t got = 0;
    if (!rc) rc = acso_get_spread_trace(s, 0, tr, 256, &got);
    uint32_t* st = (uint32_t*)malloc(n * sizeof(uint32_t));
    if (!rc) rc = acso_get_fault_status(s, st, n);
    if (!rc && c->topology == ACS_TOPO_RANDOM_REGULAR) {
        uint32_t* nb = (uint32_t*)malloc(c->n_nodes * c->degree * sizeof(uint32_t));
        rc = acso_get_neighbors(s, nb, c->n_nodes * c->degree);
        free(nb);
    }
    printf("%s: rc %d rounds %u trace %llu\n", name, rc, rc ? 0u : res.rounds_max, (unsigned long long)got);
    free(x);
    free(st);
    acso_destroy(s);
    return rc != 0;
}

int main(void) {
    int bad = 0;
    acs_config c = base();
    c.n_nodes = 16; c.topology = ACS_TOPO_COMPLETE; c.rule = ACS_RULE_MIDPOINT;
    c.fault_model = ACS_FAULT_CRASH; c.n_faulty = 1; c.eps = 1e-3;
    bad |= run_case("cfg1", &c, NULL, NULL);

    c = base();
    c.n_nodes = 256; c.topology = ACS_TOPO_COMPLETE; c.rule = ACS_RULE_TRIMMED_MEAN; c.trim = 85;
    c.fault_model = ACS_FAULT_BYZANTINE; c.n_faulty = 85; c.byz_strategy = ACS_BYZ_SPLIT;
    bad |= run_case("cfg2_small", &c, NULL, NULL);

    c = base();
    c.n_nodes = 64; c.n_instances = 40; c.topology = ACS_TOPO_COMPLETE; c.rule = ACS_RULE_AVERAGE;
    c.loss_p = 0.2; c.mask_group = 4; c.instance_offset = 7;
    bad |= run_case("cfg3_small", &c, NULL, NULL);

    c = base();
    c.n_nodes = 3001; c.topology = ACS_TOPO_RANDOM_REGULAR; c.degree = 32; c.rule = ACS_RULE_TRIMMED_MEAN;
    c.trim = 5; c.fault_model = ACS_FAULT_BYZANTINE; c.n_faulty = 30; c.byz_strategy = ACS_BYZ_RANDOM;
    c.byz_delta = 0.1; c.loss_p = 0.1;
    bad |= run_case("cfg4_byz_lossy", &c, NULL, NULL);

    c = base();
    c.n_nodes = 2000; c.topology = ACS_TOPO_RANDOM_REGULAR; c.degree = 8; c.rule = ACS_RULE_WMSR; c.trim = 2;
    c.fault_model = ACS_FAULT_CRASH; c.n_faulty = 40; c.crash_window = 5; c.delay_max = 3;
    bad |= run_case("wmsr_crash_delay", &c, NULL, NULL);

    c = base();
    c.n_nodes = 500; c.topology = ACS_TOPO_RANDOM_REGULAR; c.degree = 12; c.rule = ACS_RULE_DLPSW_SELECT;
    c.trim = 3; c.dtype = ACS_F32; c.fault_model = ACS_FAULT_BYZANTINE; c.n_faulty = 10;
    c.byz_strategy = ACS_BYZ_CONSTANT; c.byz_const = 0.25;
    bad |= run_case("f32_dlpsw", &c, NULL, NULL);

    /* CSR: a ring with chords, variable degree */
    {
        const uint32_t N = 300;
        uint64_t* rp = (uint64_t*)malloc((N + 1) * sizeof(uint64_t));
        uint32_t* ci = (uint32_t*)malloc(N * 8 * sizeof(uint32_t));
        uint64_t k = 0;
        for (uint32_t i = 0; i < N; ++i) {
            rp[i] = k;
            const uint32_t deg = 3 + i % 5;
            for (uint32_t t = 0; t < deg; ++t) ci[k++] = (i + 1 + t * 37) % N;
        }
        rp[N] = k;
        c = base();
        c.n_nodes = N; c.topology = ACS_TOPO_CSR; c.rule = ACS_RULE_TRIMMED_MEAN; c.trim = 1; c.loss_p = 0.05;
        bad |= run_case("csr_variable_degree", &c, rp, ci);
        free(rp);
        free(ci);
    }
    /* set_state admission: NaN must be rejected */
    {
        c = base();
        c.n_nodes = 64; c.topology = ACS_TOPO_RANDOM_REGULAR; c.degree = 4; c.rule = ACS_RULE_TRIMMED_MEAN; c.trim = 1;
        acso_sim* s = NULL;
        if (acso_create(&c, &s) == 0) {
            double x[64];
            for (int i = 0; i < 64; ++i) x[i] = i / 64.0;
            x[9] = NAN;
            if (acso_set_state(s, 0, x, 64) == 0) { printf("set_state accepted NaN\n"); bad = 1; }
            acso_destroy(s);
        } else {
            bad = 1;
        }
    }
    printf(bad ? "selftest FAILED\n" : "selftest ok\n");
    return bad;
}
