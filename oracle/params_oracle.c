/*
 * params_oracle.c -- CPU ORACLE for parameter-draw ingestion.
 * TEST INFRASTRUCTURE ONLY (same rule as hhmm_oracle.c).
 *
 * Restates, one draw at a time, how stanc's write_array reads each program's
 * parameters block from the unconstrained vector (declaration order; arrays
 * element-major; a simplex[n] consumes n - 1 values) with Stan Math 2.14's
 * constraining transforms:
 *   simplex_constrain: stick = 1; z_k = inv_logit(y_k - log(n - 1 - k));
 *                      x_k = stick * z_k; stick -= x_k; x_{n-1} = stick
 *   inv_logit(a):      a < 0: exp(a) if a < log(epsilon), else exp(a) / (1 + exp(a));
 *                      a >= 0: 1 / (1 + exp(-a))
 *   ordered_constrain: x_0 = y_0; x_k = x_{k-1} + exp(y_k)
 *   lb_constrain:      exp(y) + lb
 *   lub_constrain(0,1): inv_logit with the 1 - 1e-15 / 1e-15 clamps
 * (restated from the published Stan Math sources; not vendored here, so
 * parity with Stan is unpinned -- pinned instead by a Python transcription
 * and by round trips, tests/test_params.py).
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>

#include "hhmm_params.h"

#define HHMM_MATH_FN static inline
#define HHMM_MATH_TABLE static
#include "hhmm_crmath.h"

#ifdef HHMM_ORACLE_LIBM_LOG
#define P_EXP(x) exp(x)
#define P_LOG(x) log(x)
#else
#define P_EXP(x) hhmm_cr_exp(x)
#define P_LOG(x) hhmm_cr_log(x)
#endif

static double inv_logit(double a)
{
    if (a < 0) {
        double e = P_EXP(a);
        if (a < log(2.220446049250313e-16))
            return e;
        return e / (1 + e);
    }
    return 1.0 / (1 + P_EXP(-a));
}

static double lub01(double x)
{
    double il;
    if (x > 0) {
        il = 1.0 / (1.0 + P_EXP(-x));
        if (x < INFINITY && il == 1)
            il = 1 - 1e-15;
    } else {
        il = 1.0 - 1.0 / (1.0 + P_EXP(x));
        if (x > -INFINITY && il == 0)
            il = 1e-15;
    }
    return 0.0 + (1.0 - 0.0) * il;
}

typedef struct reader {
    const double *theta;
    int64_t S, s, pos;
} reader;

static double next(reader *r) { return r->theta[r->s + r->S * r->pos++]; }

/* out[s + S*(a + count*v)] */
#define PUT(out, a, count, v, val) \
    do { if (out) (out)[r->s + r->S * ((int64_t)(a) + (int64_t)(count) * (v))] = (val); } while (0)

static void rd_simplex(reader *r, int count, int n, double *out)
{
    for (int a = 0; a < count; ++a) {
        double stick = 1.0;
        for (int k = 0; k < n - 1; ++k) {
            const double z = inv_logit(next(r) - P_LOG((double)(n - 1 - k)));
            const double x = stick * z;
            stick -= x;
            PUT(out, a, count, k, x);
        }
        PUT(out, a, count, n - 1, stick);
    }
}

static void rd_ordered(reader *r, int count, int n, double *out)
{
    for (int a = 0; a < count; ++a) {
        double y = next(r);
        PUT(out, a, count, 0, y);
        for (int k = 1; k < n; ++k) {
            y = y + P_EXP(next(r));
            PUT(out, a, count, k, y);
        }
    }
}

static void rd_plain(reader *r, int count, int n, double *out, int kind, double lb)
{
    for (int a = 0; a < count; ++a)
        for (int k = 0; k < n; ++k) {
            const double u = next(r);
            const double v = kind == 1 ? P_EXP(u) + lb : (kind == 2 ? lub01(u) : u);
            PUT(out, a, count, k, v);
        }
}

/* Returns the unconstrained length consumed per draw, or -1. */
int64_t hhmm_oracle_constrain(int model, int K, int L, int M, int64_t S, const double *theta, hhmm_param_out *o)
{
    int64_t len = -1;
    for (int64_t s = 0; s < S; ++s) {
        reader rr = {theta, S, s, 0}, *r = &rr;
        switch (model) {
        case HHMM_MODEL_HMM_GAUSS: /* hmm.stan:13-22 */
            rd_simplex(r, 1, K, o->p_1k);
            rd_simplex(r, K, K, o->A_ij);
            rd_ordered(r, 1, K, o->mu_k);
            rd_plain(r, K, 1, o->sigma_k, 1, 0.0001);
            break;
        case HHMM_MODEL_HMM_MULTINOM:
        case HHMM_MODEL_HMM_MULTINOM_SEMISUP:
            rd_simplex(r, 1, K, o->p_1k);
            rd_simplex(r, K, K, o->A_ij);
            rd_simplex(r, K, L, o->phi_k);
            break;
        case HHMM_MODEL_IOHMM_REG: /* iohmm-reg.stan:16-24 */
            rd_simplex(r, 1, K, o->p_1k);
            rd_plain(r, K, M, o->w_km, 0, 0);
            rd_plain(r, K, M, o->b_km, 0, 0);
            rd_plain(r, K, 1, o->s_k, 1, 0.0001);
            break;
        case HHMM_MODEL_IOHMM_MIX:
        case HHMM_MODEL_IOHMM_HMIX:
        case HHMM_MODEL_IOHMM_HMIX_LITE: /* iohmm-mix.stan:17-26, iohmm-hmix(-lite).stan:13-23 */
            rd_simplex(r, 1, K, o->p_1k);
            rd_plain(r, K, M, o->w_km, 0, 0);
            rd_simplex(r, K, L, o->lambda_kl);
            rd_ordered(r, K, L, o->mu_kl);
            rd_plain(r, K, L, o->s_kl, 1, 0.0);
            if (model == HHMM_MODEL_IOHMM_HMIX)
                rd_ordered(r, 1, K, o->hypermu_k);
            if (model == HHMM_MODEL_IOHMM_HMIX_LITE)
                rd_plain(r, K, 1, o->hypermu_k, 0, 0);
            break;
        case HHMM_MODEL_TAYAL:
        case HHMM_MODEL_TAYAL_LITE: /* hhmm-tayal2009.stan:15-22 */
            rd_plain(r, 1, 1, o->p_11, 2, 0);
            rd_simplex(r, 2, 2, o->A_row);
            rd_simplex(r, K, L, o->phi_k);
            break;
        default:
            return -1;
        }
        len = rr.pos;
    }
    return len;
}
