/*
 * acs_oracle.c — single-threaded (optionally OpenMP over receivers) CPU restatement of the
 * approximate-consensus spec.  TEST INFRASTRUCTURE ONLY: see acs_oracle.h for who may load it.
 *
 * Upstream parity: UNPINNED (the reference mount holds only README.md:1).  Every function below
 * cites the SURVEY.md Appendix A rule ("§A.k") it restates.  Written for clarity, not speed:
 * plain loops, insertion sort, no SIMD, -ffp-contract=off (no FMA anywhere).
 */
#include "acs_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define HONEST 0xFFFFFFFFu
#define BYZ    0xFFFFFFFEu

static __thread char g_err[512];

static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

const char* acso_last_error(void) { return g_err; }

/* ---------------------------------------------------------------- §A.1 RNG */

/* Philox4x32-10, Random123 constants (PHILOX_H:62-65), round (PHILOX_H:286-296),
 * key bump between rounds (PHILOX_H:298-302), 10 rounds (PHILOX_H:270-281). */
void acso_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int rnd = 0; rnd < 10; ++rnd) {
        if (rnd > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* §A.1: draw(stream, b, r, s) = philox(ctr = (s>>2, r, b, stream), key(seed))[s & 3]. */
uint32_t acso_draw(uint64_t seed, uint32_t stream, uint32_t b, uint32_t r, uint64_t s) {
    uint32_t ctr[4] = {(uint32_t)(s >> 2), r, b, stream};
    uint32_t key[2] = {(uint32_t)(seed & 0xFFFFFFFFu), (uint32_t)(seed >> 32)};
    uint32_t out[4];
    acso_philox4x32_10(ctr, key, out);
    return out[s & 3u];
}

/* §A.1: u53(w0, w1) = ((w0>>5)·2^26 + (w1>>6)) · 2^-53, exact in fp64. */
double acso_u53(uint32_t w0, uint32_t w1) {
    uint64_t m = ((uint64_t)(w0 >> 5) << 26) | (uint64_t)(w1 >> 6);
    return (double)m * 0x1p-53;
}

/* ---------------------------------------------------------------- §A.3 topology */

static int bit_length(uint64_t v) {
    int n = 0;
    while (v) { ++n; v >>= 1; }
    return n;
}

/* §A.3: Feistel permutation π_k of [0,N) (4 rounds, cycle walking), or its inverse. */
uint64_t acso_feistel_perm(uint64_t n, uint64_t graph_seed, uint32_t k, uint64_t v, int inverse) {
    int mb = bit_length(n - 1);
    if (mb < 2) mb = 2;
    if (mb & 1) mb += 1;
    const int h = mb / 2;
    const uint64_t mask = (1ull << h) - 1ull;
    const uint32_t key[2] = {(uint32_t)(graph_seed & 0xFFFFFFFFu), (uint32_t)(graph_seed >> 32)};
    do {
        uint64_t L = v >> h, R = v & mask;
        if (!inverse) {
            for (uint32_t j = 0; j < 4; ++j) {
                uint32_t ctr[4] = {(uint32_t)R, j, k, ACS_STREAM_GRAPH}, o[4];
                acso_philox4x32_10(ctr, key, o);
                uint64_t nl = R, nr = L ^ ((uint64_t)o[0] & mask);
                L = nl; R = nr;
            }
        } else {
            for (int j = 3; j >= 0; --j) {
                uint32_t ctr[4] = {(uint32_t)L, (uint32_t)j, k, ACS_STREAM_GRAPH}, o[4];
                acso_philox4x32_10(ctr, key, o);
                uint64_t nl = R ^ ((uint64_t)o[0] & mask), nr = L;
                L = nl; R = nr;
            }
        }
        v = (L << h) | R;
    } while (v >= n);
    return v;
}

/* ---------------------------------------------------------------- §A.5 loss */

/* §A.5: thr = (u32) floor(p · 2^32), computed in fp64. */
uint32_t acso_drop_threshold(double p) {
    double t = floor(p * 4294967296.0);
    if (t <= 0.0) return 0u;
    if (t >= 4294967295.0) return 0xFFFFFFFFu;
    return (uint32_t)t;
}

/* ---------------------------------------------------------------- §A.0 value type */

/* DESIGN.md §9 fp32 mode (ACS_F32): values are binary32 and every arithmetic step rounds to
 * binary32.  The oracle keeps them in doubles and rounds each +, -, *, / result with rnd():
 * for these operations on binary32 operands, the double result rounded to binary32 equals the
 * binary32 result (53 >= 2*24 + 2), so this is exact binary32 arithmetic.  Comparisons, min
 * and max need no rounding. */
static double rnd(int f32, double v) { return f32 ? (double)(float)v : v; }

/* ---------------------------------------------------------------- §A.7 rules */

/* §A.7 tree_sum: pad to the next power of two with +0.0, then stride-halving pairwise adds. */
static double tree_sum_t(const double* a, uint64_t n, int f32) {
    if (n == 0) return 0.0;
    uint64_t P = 1;
    while (P < n) P <<= 1;
    double stackbuf[128];
    double* w = P <= 128 ? stackbuf : (double*)malloc(P * sizeof(double));
    for (uint64_t k = 0; k < P; ++k) w[k] = k < n ? a[k] : 0.0;
    for (uint64_t s = P / 2; s >= 1; s /= 2)
        for (uint64_t k = 0; k < s; ++k) w[k] = rnd(f32, w[k] + w[k + s]);
    double r = w[0];
    if (w != stackbuf) free(w);
    return r;
}

double acso_tree_sum(const double* a, uint64_t n) { return tree_sum_t(a, n, 0); }

static int cmp_double(const void* a, const void* b) {
    double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

static void sort_asc(double* a, uint64_t m) {
    if (m <= 64) {
        for (uint64_t i = 1; i < m; ++i) {
            double v = a[i];
            uint64_t j = i;
            while (j > 0 && v < a[j - 1]) { a[j] = a[j - 1]; --j; }
            a[j] = v;
        }
    } else {
        qsort(a, (size_t)m, sizeof(double), cmp_double);
    }
}

/* §A.7: apply the rule to the m entries of S (S is reordered in place); xi is the receiver's own
 * value (W-MSR only). */
static double apply_rule(uint32_t rule, uint32_t t, double* S, uint64_t m, double* scratch, double xi, int f32) {
    if (rule == ACS_RULE_AVERAGE) return rnd(f32, tree_sum_t(S, m, f32) / (double)m);
    sort_asc(S, m);
    if (rule == ACS_RULE_WMSR) {
        /* drop min(t, #below) smallest and min(t, #above) largest entries, where
         * below / above are strictly less / greater than xi; tree_sum the rest in sorted order */
        uint64_t nl = 0, ng = 0;
        for (uint64_t k = 0; k < m; ++k) {
            if (S[k] < xi) ++nl;
            else if (S[k] > xi) ++ng;
        }
        const uint64_t lo = nl < t ? nl : t, hi = ng < t ? ng : t, nw = m - lo - hi;
        return rnd(f32, tree_sum_t(S + lo, nw, f32) / (double)nw);
    }
    const double* R = S + t;
    const uint64_t nr = m - 2ull * t;
    if (rule == ACS_RULE_TRIMMED_MEAN) return rnd(f32, tree_sum_t(R, nr, f32) / (double)nr);
    if (rule == ACS_RULE_MIDPOINT) return rnd(f32, rnd(f32, R[0] + R[nr - 1]) * 0.5);
    /* DLPSW_SELECT: Q = R[0], R[t], R[2t], ... */
    uint64_t nq = 0;
    for (uint64_t k = 0; k < nr; k += t) scratch[nq++] = R[k];
    return rnd(f32, tree_sum_t(scratch, nq, f32) / (double)nq);
}

/* DESIGN.md §9, missing_policy = OMIT: the m entries of S in entry order, miss[k] set for the
 * missing ones (never the self entry), m' = #present >= 1.  AVERAGE: tree_sum over the m entries
 * in entry order with every missing entry +0.0 (it keeps its place in the tree), divided by m'.
 * The other rules see only the m' present entries; TRIMMED / MIDPOINT / DLPSW need m' > 2t and
 * otherwise keep x_i; W-MSR applies as is (its window is never empty). */
static double apply_rule_omit(uint32_t rule, uint32_t t, double* S, const uint8_t* miss, uint64_t m, double* scratch,
                              double xi, int f32) {
    uint64_t mp = 0;
    if (rule == ACS_RULE_AVERAGE) {
        for (uint64_t k = 0; k < m; ++k) {
            if (miss[k]) S[k] = 0.0;
            else ++mp;
        }
        return rnd(f32, tree_sum_t(S, m, f32) / (double)mp);
    }
    for (uint64_t k = 0; k < m; ++k)
        if (!miss[k]) S[mp++] = S[k];
    if (rule != ACS_RULE_WMSR && mp <= 2ull * t) return xi;
    return apply_rule(rule, t, S, mp, scratch, xi, f32);
}

/* ---------------------------------------------------------------- validation (§A.8 constraints) */

int acso_validate(const acs_config* c) {
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
        m = 0;       /* per receiver: checked against the arrays by acso_create_csr */
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

/* ---------------------------------------------------------------- simulation state */

struct acso_sim {
    acs_config c;
    uint64_t N, B, m;
    uint32_t thr;            /* §A.5 drop threshold */
    uint32_t* nbr;           /* RANDOM_REGULAR: N*d neighbour ids (§A.3) */
    uint64_t* rowptr;        /* CSR: N+1 row offsets (slot of entry 1+t of i = rowptr[i]+t) */
    uint32_t* colidx;        /* CSR: rowptr[N] sender ids */
    uint32_t* status;        /* B*N: HONEST / BYZ / crash round (§A.4) */
    double* x;               /* B*N current values */
    double* xn;              /* B*N next values */
    double* hist;            /* (D+1)*B*N: x^q in slot q % (D+1) for the last D+1 rounds (delay_max D > 0) */
    uint32_t* rounds;        /* B */
    uint8_t* done;           /* B */
    uint8_t* converged;      /* B */
    double* lo;              /* B: honest min of current x */
    double* hi;              /* B */
    double* trace;           /* B*(max_rounds+1) or NULL */
    int threads;
    int f32;                 /* ACS_F32: binary32 values, held exactly in the double arrays */
};

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

/* §A.8: spread over the honest set H. */
static void honest_minmax(const acso_sim* s, uint64_t b) {
    const double* x = s->x + b * s->N;
    const uint32_t* st = s->status + b * s->N;
    double lo = INFINITY, hi = -INFINITY;
    for (uint64_t i = 0; i < s->N; ++i) {
        if (st[i] != HONEST) continue;
        if (x[i] < lo) lo = x[i];
        if (x[i] > hi) hi = x[i];
    }
    s->lo[b] = lo;
    s->hi[b] = hi;
}

static void after_update(acso_sim* s, uint64_t b) {
    honest_minmax(s, b);
    const double spread = rnd(s->f32, s->hi[b] - s->lo[b]);
    const uint32_t r = s->rounds[b];
    if (s->trace) s->trace[b * ((uint64_t)s->c.max_rounds + 1) + r] = spread;
    s->converged[b] = spread <= s->c.eps;
    s->done[b] = (s->c.termination == ACS_TERM_EPS && spread <= s->c.eps) || r >= s->c.max_rounds;
}

int acso_create(const acs_config* cfg, acso_sim** out) {
    if (!out) return fail(ACS_EINVAL, "null out");
    *out = NULL;
    int rc = acso_validate(cfg);
    if (rc) return rc;
    acso_sim* s = (acso_sim*)calloc(1, sizeof *s);
    if (!s) return fail(ACS_ENOMEM, "oom");
    s->c = *cfg;
    s->N = cfg->n_nodes;
    s->B = cfg->n_instances;
    s->m = cfg->topology == ACS_TOPO_COMPLETE ? s->N : (uint64_t)cfg->degree + 1;
    s->thr = acso_drop_threshold(cfg->loss_p);
    s->threads = cfg->omp_threads ? (int)cfg->omp_threads : 1;
    s->f32 = cfg->dtype == ACS_F32;
    const uint64_t gseed = cfg->graph_seed ? cfg->graph_seed : cfg->seed;
    const uint64_t BN = s->B * s->N;
    s->status = (uint32_t*)malloc(BN * sizeof(uint32_t));
    s->x = (double*)malloc(BN * sizeof(double));
    s->xn = (double*)malloc(BN * sizeof(double));
    s->rounds = (uint32_t*)calloc(s->B, sizeof(uint32_t));
    s->done = (uint8_t*)calloc(s->B, 1);
    s->converged = (uint8_t*)calloc(s->B, 1);
    s->lo = (double*)malloc(s->B * sizeof(double));
    s->hi = (double*)malloc(s->B * sizeof(double));
    if (cfg->trace_spread) {
        const uint64_t nt = s->B * ((uint64_t)cfg->max_rounds + 1);
        s->trace = (double*)malloc(nt * sizeof(double));
        if (s->trace) for (uint64_t k = 0; k < nt; ++k) s->trace[k] = NAN;
    }
    if (cfg->delay_max) s->hist = (double*)malloc(((uint64_t)cfg->delay_max + 1) * BN * sizeof(double));
    if (!s->status || !s->x || !s->xn || !s->rounds || !s->done || !s->converged || !s->lo ||
        !s->hi || (cfg->trace_spread && !s->trace) || (cfg->delay_max && !s->hist)) {
        acso_destroy(s);
        return fail(ACS_ENOMEM, "oom");
    }
    /* §A.3 neighbour table: t even -> π_{t/2}(i), t odd -> π_{t/2}^{-1}(i). */
    if (cfg->topology == ACS_TOPO_RANDOM_REGULAR) {
        const uint64_t d = cfg->degree;
        s->nbr = (uint32_t*)malloc(s->N * d * sizeof(uint32_t));
        if (!s->nbr) { acso_destroy(s); return fail(ACS_ENOMEM, "oom"); }
        const int64_t N = (int64_t)s->N;
#pragma omp parallel for num_threads(s->threads) schedule(static)
        for (int64_t i = 0; i < N; ++i)
            for (uint64_t t = 0; t < d; ++t)
                s->nbr[(uint64_t)i * d + t] =
                    (uint32_t)acso_feistel_perm(s->N, gseed, (uint32_t)(t >> 1), (uint64_t)i, (int)(t & 1));
    }
    for (uint64_t lb = 0; lb < s->B; ++lb) {
        const uint32_t b = (uint32_t)(cfg->instance_offset + lb);
        uint32_t* st = s->status + lb * s->N;
        double* x = s->x + lb * s->N;
        /* §A.2 initial values (fp32: (draw(INIT,b,0,2i) >> 8) * 2^-24, exact in binary32) */
        for (uint64_t i = 0; i < s->N; ++i)
            x[i] = s->f32 ? (double)(acso_draw(cfg->seed, ACS_STREAM_INIT, b, 0, 2 * i) >> 8) * 0x1p-24
                          : acso_u53(acso_draw(cfg->seed, ACS_STREAM_INIT, b, 0, 2 * i),
                                     acso_draw(cfg->seed, ACS_STREAM_INIT, b, 0, 2 * i + 1));
        /* §A.4 fault set: the f smallest (draw(FAULTSET,b,0,i), i) pairs */
        for (uint64_t i = 0; i < s->N; ++i) st[i] = HONEST;
        if (cfg->fault_model != ACS_FAULT_NONE && cfg->n_faulty > 0) {
            uint64_t* keys = (uint64_t*)malloc(s->N * sizeof(uint64_t));
            if (!keys) { acso_destroy(s); return fail(ACS_ENOMEM, "oom"); }
            for (uint64_t i = 0; i < s->N; ++i)
                keys[i] = ((uint64_t)acso_draw(cfg->seed, ACS_STREAM_FAULTSET, b, 0, i) << 32) | i;
            qsort(keys, (size_t)s->N, sizeof(uint64_t), cmp_u64);
            for (uint32_t k = 0; k < cfg->n_faulty; ++k) {
                const uint32_t v = (uint32_t)(keys[k] & 0xFFFFFFFFu);
                st[v] = cfg->fault_model == ACS_FAULT_BYZANTINE
                            ? BYZ
                            : acso_draw(cfg->seed, ACS_STREAM_CRASH_ROUND, b, 0, v) % cfg->crash_window;
            }
            free(keys);
        }
        s->rounds[lb] = 0;
        after_update(s, lb);
        if (s->hist) memcpy(s->hist + lb * s->N, x, s->N * sizeof(double));   /* x^0 in slot 0 */
    }
    *out = s;
    return ACS_OK;
}

/* §8(f) row 1 / §A.3 (CSR extension): receiver i's entries are itself then the senders
 * colidx[rowptr[i] + t] on slot rowptr[i] + t; m_i = deg(i) + 1. */
int acso_create_csr(const acs_config* cfg, const uint64_t* rowptr, const uint32_t* colidx, acso_sim** out) {
    if (!out) return fail(ACS_EINVAL, "null out");
    *out = NULL;
    if (!cfg || cfg->topology != ACS_TOPO_CSR) return fail(ACS_EINVAL, "config topology must be ACS_TOPO_CSR");
    int rc = acso_validate(cfg);
    if (rc) return rc;
    if (!rowptr || !colidx) return fail(ACS_EINVAL, "null CSR arrays");
    const uint64_t N = cfg->n_nodes;
    if (rowptr[0] != 0) return fail(ACS_EINVAL, "rowptr[0] must be 0");
    uint64_t mmax = 1;
    for (uint64_t i = 0; i < N; ++i) {
        if (rowptr[i + 1] < rowptr[i]) return fail(ACS_EINVAL, "rowptr must be non-decreasing");
        const uint64_t m = rowptr[i + 1] - rowptr[i] + 1;
        if (cfg->rule != ACS_RULE_AVERAGE && m <= 2ull * cfg->trim)
            return fail(ACS_EINVAL, "receiver %llu has m = %llu <= 2t", (unsigned long long)i, (unsigned long long)m);
        if (m > mmax) mmax = m;
    }
    const uint64_t nnz = rowptr[N];
    if (nnz >= (1ull << 34)) return fail(ACS_EINVAL, "slot count must be < 2^34");
    if (cfg->fault_model == ACS_FAULT_BYZANTINE && cfg->byz_strategy == ACS_BYZ_RANDOM && nnz > (1ull << 33))
        return fail(ACS_EINVAL, "BYZ RANDOM needs slot count <= 2^33");
    for (uint64_t k = 0; k < nnz; ++k)
        if (colidx[k] >= N) return fail(ACS_EINVAL, "colidx[%llu] out of range", (unsigned long long)k);
    acs_config c2 = *cfg;
    c2.topology = ACS_TOPO_COMPLETE;   /* build everything but the graph through acso_create */
    c2.n_nodes = N;
    const uint32_t rule = c2.rule, trim = c2.trim;
    c2.rule = ACS_RULE_AVERAGE;       /* topology-free validation of the rest */
    c2.trim = 0;
    if (N * N >= (1ull << 34)) c2.topology = ACS_TOPO_RANDOM_REGULAR, c2.degree = 2;
    acso_sim* s = NULL;
    rc = acso_create(&c2, &s);
    if (rc) return rc;
    free(s->nbr);
    s->nbr = NULL;
    s->c = *cfg;
    s->c.rule = rule;
    s->c.trim = trim;
    s->m = mmax;
    s->rowptr = (uint64_t*)malloc((N + 1) * sizeof(uint64_t));
    s->colidx = (uint32_t*)malloc((nnz ? nnz : 1) * sizeof(uint32_t));
    if (!s->rowptr || !s->colidx) { acso_destroy(s); return fail(ACS_ENOMEM, "oom"); }
    memcpy(s->rowptr, rowptr, (N + 1) * sizeof(uint64_t));
    memcpy(s->colidx, colidx, nnz * sizeof(uint32_t));
    *out = s;
    return ACS_OK;
}

void acso_destroy(acso_sim* s) {
    if (!s) return;
    free(s->rowptr); free(s->colidx);
    free(s->nbr); free(s->status); free(s->x); free(s->xn); free(s->hist); free(s->rounds); free(s->done);
    free(s->converged); free(s->lo); free(s->hi); free(s->trace);
    free(s);
}

/* §A.4 Byzantine value on slot s to receiver i in round r.  fp32: Δ and c are
 * rounded to binary32 once, RANDOM uses u24 = (draw(BYZ,b,r,2s) >> 8) * 2^-24, and every step
 * rounds to binary32 in the order written below. */
static double byz_value(const acso_sim* s, uint32_t b, uint32_t r, uint64_t i, uint64_t slot,
                        double lo, double hi) {
    const acs_config* c = &s->c;
    if (s->f32) {
        const double dl = (double)(float)c->byz_delta;
        if (c->byz_strategy == ACS_BYZ_SPLIT) return (i & 1u) == 0 ? rnd(1, hi + dl) : rnd(1, lo - dl);
        if (c->byz_strategy == ACS_BYZ_CONSTANT) return (double)(float)c->byz_const + 0.0;
        const double u = (double)(acso_draw(c->seed, ACS_STREAM_BYZ, b, r, 2 * slot) >> 8) * 0x1p-24;
        const double width = rnd(1, rnd(1, hi - lo) + 2.0 * dl);
        return rnd(1, rnd(1, lo - dl) + rnd(1, u * width));
    }
    if (c->byz_strategy == ACS_BYZ_SPLIT) return (i & 1u) == 0 ? hi + c->byz_delta : lo - c->byz_delta;
    if (c->byz_strategy == ACS_BYZ_CONSTANT) return c->byz_const + 0.0;   /* canonical +0.0 */
    const double u = acso_u53(acso_draw(c->seed, ACS_STREAM_BYZ, b, r, 2 * slot),
                              acso_draw(c->seed, ACS_STREAM_BYZ, b, r, 2 * slot + 1));
    const double width = (hi - lo) + 2.0 * c->byz_delta;
    return (lo - c->byz_delta) + u * width;
}

/* the delivered value of sender j on slot `slot` in round r is x_j^{r - delta} with
 * delta = min(r, draw(DELAY, b, r, slot) mod (D + 1)); D = 0 is the synchronous §A.6 model. */
static double delayed_value(const acso_sim* s, uint64_t lb, uint32_t b, uint32_t r, uint64_t j, uint64_t slot) {
    const uint32_t D = s->c.delay_max;
    uint32_t delta = acso_draw(s->c.seed, ACS_STREAM_DELAY, b, r, slot) % (D + 1);
    if (delta > r) delta = r;
    return s->hist[((uint64_t)((r - delta) % (D + 1)) * s->B + lb) * s->N + j];
}

/* §A.6: resolve entry (i <- j, slot, round r) for an active receiver i != j-as-self.  A missing
 * entry is x_i under the default policy; under missing_policy = OMIT *miss is set
 * and the returned value is unused. */
static double resolve(const acso_sim* s, uint32_t b, uint32_t bG, uint32_t r, const double* x,
                      const uint32_t* st, uint64_t i, uint64_t j, uint64_t slot, double lo, double hi,
                      int* miss) {
    const uint32_t sj = st[j];
    int missing = 0;
    if (sj != HONEST && sj != BYZ) {           /* crash-faulty sender, crash round sj */
        if (r > sj) missing = 1;
        else if (r == sj) missing = acso_draw(s->c.seed, ACS_STREAM_CRASH_PARTIAL, b, sj, slot) >= 0x80000000u;
    }
    if (!missing && s->thr > 0)
        missing = acso_draw(s->c.seed, ACS_STREAM_DROP, bG, r, slot) < s->thr;
    *miss = missing;
    if (missing) return x[i];
    if (sj == BYZ) return byz_value(s, b, r, i, slot, lo, hi);
    if (s->c.delay_max) return delayed_value(s, (uint64_t)(b - (uint32_t)s->c.instance_offset), b, r, j, slot);
    return x[j];
}

/* §A.9: one Jacobi step x^r -> x^{r+1} of local instance lb. */
static void step_instance(acso_sim* s, uint64_t lb) {
    const acs_config* c = &s->c;
    const uint32_t b = (uint32_t)(c->instance_offset + lb);
    const uint32_t bG = b - b % c->mask_group;
    const uint32_t r = s->rounds[lb];
    const double* x = s->x + lb * s->N;
    double* xn = s->xn + lb * s->N;
    const uint32_t* st = s->status + lb * s->N;
    const double lo = s->lo[lb], hi = s->hi[lb];
    const uint64_t N = s->N, m = s->m;
    const int64_t Ni = (int64_t)N;
#pragma omp parallel num_threads(s->threads)
    {
        double* S = (double*)malloc(2 * m * sizeof(double));
        double* scratch = S + m;
        uint8_t* miss = (uint8_t*)malloc(m);
#pragma omp for schedule(static)
        for (int64_t ii = 0; ii < Ni; ++ii) {
            const uint64_t i = (uint64_t)ii;
            const uint32_t si = st[i];
            const int active = si == HONEST || (si != BYZ && r < si);
            if (!active) { xn[i] = x[i]; continue; }
            uint64_t mi = m;
            if (c->topology == ACS_TOPO_COMPLETE) {
                for (uint64_t j = 0; j < N; ++j) {
                    miss[j] = 0;
                    int mj = 0;
                    S[j] = j == i ? x[i] : resolve(s, b, bG, r, x, st, i, j, i * N + j, lo, hi, &mj);
                    miss[j] = (uint8_t)mj;
                }
            } else if (c->topology == ACS_TOPO_CSR) {
                const uint64_t rp = s->rowptr[i], deg = s->rowptr[i + 1] - rp;
                S[0] = x[i];
                miss[0] = 0;
                for (uint64_t t = 0; t < deg; ++t) {
                    int mj = 0;
                    S[1 + t] = resolve(s, b, bG, r, x, st, i, s->colidx[rp + t], rp + t, lo, hi, &mj);
                    miss[1 + t] = (uint8_t)mj;
                }
                mi = deg + 1;
            } else {
                const uint64_t d = c->degree;
                S[0] = x[i];
                miss[0] = 0;
                for (uint64_t t = 0; t < d; ++t) {
                    int mj = 0;
                    S[1 + t] = resolve(s, b, bG, r, x, st, i, s->nbr[i * d + t], i * d + t, lo, hi, &mj);
                    miss[1 + t] = (uint8_t)mj;
                }
            }
            xn[i] = c->missing_policy == ACS_MISSING_OMIT ? apply_rule_omit(c->rule, c->trim, S, miss, mi, scratch, x[i], s->f32)
                                                         : apply_rule(c->rule, c->trim, S, mi, scratch, x[i], s->f32);
        }
        free(S);
        free(miss);
    }
    /* swap x / xn for this instance; keep x^{r+1} in the delay history */
    memcpy(s->x + lb * N, xn, N * sizeof(double));
    if (s->hist)
        memcpy(s->hist + ((uint64_t)((r + 1) % (c->delay_max + 1)) * s->B + lb) * N, xn, N * sizeof(double));
    s->rounds[lb] = r + 1;
    after_update(s, lb);
}

static void fill_info(const acso_sim* s, acs_round_info* out) {
    if (!out) return;
    memset(out, 0, sizeof *out);
    uint64_t nd = 0;
    double sp = -INFINITY;
    uint32_t rmax = 0;
    for (uint64_t b = 0; b < s->B; ++b) {
        nd += s->done[b];
        const double v = rnd(s->f32, s->hi[b] - s->lo[b]);
        if (v > sp) sp = v;
        if (s->rounds[b] > rmax) rmax = s->rounds[b];
    }
    out->round = rmax;
    out->done = nd == s->B;
    out->spread = sp;
    out->lo = s->lo[0];
    out->hi = s->hi[0];
    out->instances_done = nd;
}

int acso_round(acso_sim* s, uint32_t k, acs_round_info* out) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    for (uint64_t b = 0; b < s->B; ++b)
        for (uint32_t q = 0; q < k && !s->done[b]; ++q) step_instance(s, b);
    fill_info(s, out);
    return ACS_OK;
}

int acso_run(acso_sim* s, acs_result* out) {
    if (!s) return fail(ACS_EINVAL, "null sim");
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t b = 0; b < s->B; ++b)
        while (!s->done[b]) step_instance(s, b);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (out) {
        memset(out, 0, sizeof *out);
        out->n_instances = s->B;
        out->final_spread_max = -INFINITY;
        for (uint64_t b = 0; b < s->B; ++b) {
            if (s->rounds[b] > out->rounds_max) out->rounds_max = s->rounds[b];
            out->n_converged += s->converged[b];
            out->node_rounds += s->N * (uint64_t)s->rounds[b];
            const double v = rnd(s->f32, s->hi[b] - s->lo[b]);
            if (v > out->final_spread_max) out->final_spread_max = v;
        }
        out->wall_seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    }
    return ACS_OK;
}

int acso_get_values(acso_sim* s, uint64_t b, double* out, uint64_t n) {
    if (!s || !out || b >= s->B || n < s->N) return fail(ACS_EINVAL, "bad get_values args");
    memcpy(out, s->x + b * s->N, s->N * sizeof(double));
    return ACS_OK;
}

int acso_get_instance_rounds(acso_sim* s, uint32_t* out, uint64_t n) {
    if (!s || !out || n < s->B) return fail(ACS_EINVAL, "bad args");
    memcpy(out, s->rounds, s->B * sizeof(uint32_t));
    return ACS_OK;
}

int acso_get_instance_converged(acso_sim* s, uint8_t* out, uint64_t n) {
    if (!s || !out || n < s->B) return fail(ACS_EINVAL, "bad args");
    memcpy(out, s->converged, s->B);
    return ACS_OK;
}

int acso_get_instance_spread(acso_sim* s, double* out, uint64_t n) {
    if (!s || !out || n < s->B) return fail(ACS_EINVAL, "bad args");
    for (uint64_t b = 0; b < s->B; ++b) out[b] = rnd(s->f32, s->hi[b] - s->lo[b]);
    return ACS_OK;
}

int acso_get_spread_trace(acso_sim* s, uint64_t b, double* out, uint64_t n, uint64_t* n_out) {
    if (!s || !out || b >= s->B) return fail(ACS_EINVAL, "bad args");
    if (!s->trace) return fail(ACS_EINVAL, "trace_spread was not enabled");
    uint64_t cnt = (uint64_t)s->rounds[b] + 1;
    if (cnt > n) cnt = n;
    memcpy(out, s->trace + b * ((uint64_t)s->c.max_rounds + 1), cnt * sizeof(double));
    if (n_out) *n_out = cnt;
    return ACS_OK;
}

int acso_set_state(acso_sim* s, uint32_t round, const double* x, uint64_t n) {
    if (!s || !x || n != s->B * s->N) return fail(ACS_EINVAL, "set_state needs B*N values");
    if (round > s->c.max_rounds) return fail(ACS_EINVAL, "round > max_rounds");
    /* finite and bounded (fp64 |x| <= 1e300, fp32 |x| <= 1e30), -0.0 canonicalised to +0.0:
     * the same admission rule as the engine's acs_set_state */
    for (uint64_t k = 0; k < n; ++k) {
        if (!(fabs(x[k]) <= (s->f32 ? 1e30 : 1e300))) return fail(ACS_EINVAL, "set_state: value not finite or too large");
        if (s->f32 && (double)(float)x[k] != x[k]) return fail(ACS_EINVAL, "fp32 set_state: values must be binary32");
    }
    for (uint64_t k = 0; k < n; ++k) s->x[k] = x[k] + 0.0;
    /* bounded-delay history restarts from x: every past slot holds x^round */
    if (s->hist)
        for (uint64_t q = 0; q <= s->c.delay_max; ++q) memcpy(s->hist + q * n, s->x, n * sizeof(double));
    for (uint64_t b = 0; b < s->B; ++b) {
        s->rounds[b] = round;
        after_update(s, b);
    }
    return ACS_OK;
}

int acso_get_fault_status(acso_sim* s, uint32_t* out, uint64_t n) {
    if (!s || !out || n < s->B * s->N) return fail(ACS_EINVAL, "bad args");
    memcpy(out, s->status, s->B * s->N * sizeof(uint32_t));
    return ACS_OK;
}

int acso_get_neighbors(acso_sim* s, uint32_t* out, uint64_t n) {
    if (!s || !out) return fail(ACS_EINVAL, "bad args");
    if (!s->nbr) return fail(ACS_EINVAL, "not a RANDOM_REGULAR topology");
    if (n < s->N * s->c.degree) return fail(ACS_EINVAL, "buffer too small");
    memcpy(out, s->nbr, s->N * s->c.degree * sizeof(uint32_t));
    return ACS_OK;
}
