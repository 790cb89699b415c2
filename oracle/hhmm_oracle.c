/*
 * hhmm_oracle.c -- CPU ORACLE for the batched HMM-family path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU baseline.  The product (libhhmm.so) never links,
 * loads or falls back to it.
 *
 * What it is: a scalar, one-pair-at-a-time restatement of the Stan programs'
 * transformed-parameters / model / generated-quantities blocks, in stanc's
 * evaluation order, with the reference's quirks and
 * the Stan Math 2.14 semantics it relies on (Appendix B).  Every function
 * cites the reference lines it follows.  It consumes the same hhmm_request /
 * hhmm_result structs as the engine (include/hhmm.h), with host pointers.
 *
 * Parity status: UNPINNED against the reference's own outputs -- the
 * reference has no tests, golden vectors or saved fits, and R/Stan are not
 * available here or on the GPU box.  The restatement is
 * cross-checked instead by an independent NumPy transcription
 * (tests/oracle_numpy.py), analytic known-answer tests, and committed
 * fixtures (tests/golden/).
 *
 * Transcendentals: `log` and `exp` are hhmm_cr_log / hhmm_cr_exp (correctly
 * rounded; the identical code runs on the GPU wherever a bit-exact result
 * depends on them) unless built with -DHHMM_ORACLE_LIBM_LOG, which uses the
 * host libm `log` and `exp` exactly as Stan would.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hhmm.h"

#define HHMM_MATH_FN static inline
#define HHMM_MATH_TABLE static
#include "hhmm_crmath.h"
#include "hhmm_detmath.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#ifdef HHMM_ORACLE_LIBM_LOG
#define OR_LOG(x) log(x)
#define OR_EXP(x) exp(x)
#else
#define OR_LOG(x) hhmm_cr_log(x)
#define OR_EXP(x) hhmm_cr_exp(x)
#endif

#define NEG_INF (-INFINITY)
#define STAN_INT_UNSET INT_MIN /* stanc 2.x fills local ints with INT_MIN */

/* ------------------------------------------------------------------ */
/* Stan Math 2.14 primitives                    */
/* ------------------------------------------------------------------ */

/* log_sum_exp(std::vector<double>) and the Eigen-vector overload:
 * max by strict `>` (NaN ignored), sum of exp(x - max) over x != -inf,
 * sequential; max + log(sum).  Used by every `real accumulator[K]`
 * (e.g. hmm/stan/hmm.stan:39,81) and by `target +=` (hmm.stan:46). */
static double stan_log_sum_exp(const double *x, int n)
{
    double mx = NEG_INF;
    for (int i = 0; i < n; ++i)
        if (x[i] > mx)
            mx = x[i];
    double sum = 0.0;
    for (int i = 0; i < n; ++i)
        if (x[i] != NEG_INF)
            sum += OR_EXP(x[i] - mx);
    return mx + OR_LOG(sum);
}

/* softmax(v): theta = exp(v - max(v)); theta / sum(theta) (sequential). */
static void stan_softmax(const double *v, int n, double *out)
{
    double mx = v[0];
    for (int i = 1; i < n; ++i)
        if (v[i] > mx)
            mx = v[i];
    double sum = 0.0;
    for (int i = 0; i < n; ++i) {
        out[i] = OR_EXP(v[i] - mx);
        sum += out[i];
    }
    for (int i = 0; i < n; ++i)
        out[i] = out[i] / sum;
}

/* sum(vector) = Eigen redux on x86-64 SSE2: two 2-wide partial sums over
 * blocks of 4, one more packet, horizontal add, scalar tail. */
static double stan_sum_vec(const double *a, int n)
{
    if (n < 2)
        return n == 1 ? a[0] : 0.0;
    const int aligned = n & ~1, aligned2 = n & ~3;
    double r0a = a[0], r0b = a[1];
    if (aligned > 2) {
        double r1a = a[2], r1b = a[3];
        for (int i = 4; i < aligned2; i += 4) {
            r0a = r0a + a[i];
            r0b = r0b + a[i + 1];
            r1a = r1a + a[i + 2];
            r1b = r1b + a[i + 3];
        }
        r0a = r0a + r1a;
        r0b = r0b + r1b;
        if (aligned > aligned2) {
            r0a = r0a + a[aligned2];
            r0b = r0b + a[aligned2 + 1];
        }
    }
    double res = r0a + r0b;
    for (int i = aligned; i < n; ++i)
        res = res + a[i];
    return res;
}

/* normalize(x) = x / sum(x)  (every functions{} block, e.g. hmm.stan:2-4). */
static void stan_normalize(const double *x, int n, double *out)
{
    const double sum = stan_sum_vec(x, n);
    for (int i = 0; i < n; ++i)
        out[i] = x[i] / sum;
}

/* max(std::vector<double>) = Eigen::Map<VectorXd>(...).maxCoeff() on x86-64
 * (SSE2 packet reduction, 16-byte aligned heap rows): maxpd / maxsd return
 * their SECOND operand when either is NaN, the scalar tail is std::max.
 * Values only differ from a plain max when NaN is present, i.e. the Viterbi
 * delta_tk[1] row left NaN by the Q3 initialisation (T == 1). */
static inline double sse_max(double a, double b) { return a > b ? a : b; }
static inline double std_max(double a, double b) { return a < b ? b : a; }
static double stan_max_vec(const double *d, int n)
{
    if (n == 0)
        return NEG_INF;
    if (n < 2) {
        return d[0];
    }
    const int aligned = n & ~1, aligned2 = n & ~3;
    double r0a = d[0], r0b = d[1];
    if (aligned > 2) {
        double r1a = d[2], r1b = d[3];
        for (int i = 4; i < aligned2; i += 4) {
            r0a = sse_max(r0a, d[i]);
            r0b = sse_max(r0b, d[i + 1]);
            r1a = sse_max(r1a, d[i + 2]);
            r1b = sse_max(r1b, d[i + 3]);
        }
        r0a = sse_max(r0a, r1a);
        r0b = sse_max(r0b, r1b);
        if (aligned > aligned2) {
            r0a = sse_max(r0a, d[aligned2]);
            r0b = sse_max(r0b, d[aligned2 + 1]);
        }
    }
    double res = sse_max(r0a, r0b);
    for (int i = aligned; i < n; ++i)
        res = std_max(res, d[i]);
    return res;
}

/* row_vector * vector = Eigen dot on x86-64 SSE2: two 2-wide partial sums
 * over blocks of 4, one more packet, horizontal add, scalar tail.
 * (iohmm-reg/stan/iohmm-reg.stan:45,54). */
static double stan_dot(const double *a, const double *b, int n)
{
    if (n < 2) {
        return n == 1 ? a[0] * b[0] : 0.0;
    }
    const int aligned = n & ~1, aligned2 = n & ~3;
    double r0a = a[0] * b[0], r0b = a[1] * b[1];
    if (aligned > 2) {
        double r1a = a[2] * b[2], r1b = a[3] * b[3];
        for (int i = 4; i < aligned2; i += 4) {
            r0a = r0a + a[i] * b[i];
            r0b = r0b + a[i + 1] * b[i + 1];
            r1a = r1a + a[i + 2] * b[i + 2];
            r1b = r1b + a[i + 3] * b[i + 3];
        }
        r0a = r0a + r1a;
        r0b = r0b + r1b;
        if (aligned > aligned2) {
            r0a = r0a + a[aligned2] * b[aligned2];
            r0b = r0b + a[aligned2 + 1] * b[aligned2 + 1];
        }
    }
    double res = r0a + r0b;
    for (int i = aligned; i < n; ++i)
        res = res + a[i] * b[i];
    return res;
}

/* normal_lpdf(y | mu, sigma), not propto: logp = 0; logp += NEG_LOG_SQRT_TWO_PI;
 * logp -= log(sigma); logp += -0.5 * ((y - mu) * (1/sigma))^2. */
static double stan_normal_lpdf(double y, double mu, double sigma)
{
    const double inv_sigma = 1.0 / sigma;
    const double log_sigma = OR_LOG(sigma);
    const double z = (y - mu) * inv_sigma;
    const double z2 = z * z;
    double logp = 0.0;
    logp += HHMM_NEG_LOG_SQRT_TWO_PI;
    logp -= log_sigma;
    logp += -0.5 * z2;
    return logp;
}

/* Vectorised normal_lpdf(y | mu_k, sigma_k): the SUM over k of the terms,
 * accumulated in the same order (hmm/stan/hmm.stan:30). */
static double stan_normal_lpdf_vec(double y, const double *mu, const double *sigma, int K)
{
    double logp = 0.0;
    for (int k = 0; k < K; ++k) {
        const double inv_sigma = 1.0 / sigma[k];
        const double log_sigma = OR_LOG(sigma[k]);
        const double z = (y - mu[k]) * inv_sigma;
        const double z2 = z * z;
        logp += HHMM_NEG_LOG_SQRT_TWO_PI;
        logp -= log_sigma;
        logp += -0.5 * z2;
    }
    return logp;
}

/* ------------------------------------------------------------------ */
/* Per-pair working set                                                 */
/* ------------------------------------------------------------------ */

typedef struct pair_ctx {
    int K, L, M, T, T_oos;
    /* series data, gathered contiguous (0-based t) */
    int32_t *x, *g, *sgn, *x_oos, *sgn_oos;
    double *xr, *u; /* u[t*M + m] */
    /* draw parameters, natural Stan index order */
    double *p;      /* [K] */
    double *A;      /* [K*K] A[i*K + j] */
    double *phi;    /* [K*L] phi[k*L + l] */
    double *mu, *sigma;          /* [K] */
    double *w, *b;               /* [K*M] */
    double *sk;                  /* [K] */
    double *lambda, *mukl, *skl; /* [K*L] */
    /* work arrays [T*K] */
    double *unalpha, *alpha, *unbeta, *beta, *ungamma, *gamma;
    double *oblik, *Arow, *logA, *delta, *acc, *tmp;
    int32_t *bp, *zstar;
    double *oblik_t;
    double *unalpha_oos, *alpha_oos;
    double loglik, logp_zstar;
    int status;
    /* FFBS (contract of §8 A14, see ffbs_contract below) */
    double *ffbs_u;     /* [T] caller uniforms of this pair */
    int32_t *zf;        /* [T] draws, 1-based (0 = undefined) */
    double *ff;         /* [T*K] filter f_t */
    /* fitted-output draws (see fitted_draws below) */
    double *hat_rand;   /* [T*3] caller uniform (hatz), uniform (hatl), normal deviate (hatx) */
    double *hatpi;      /* [T*K] */
    int32_t *hatz, *hatl; /* [T], 1-based */
    double *hatx;       /* [T] */
} pair_ctx;

static void *xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) {
        fprintf(stderr, "hhmm_oracle: out of memory\n");
        abort();
    }
    return p;
}

static void ctx_alloc(pair_ctx *c, int K, int L, int M, int Tm, int Toos)
{
    memset(c, 0, sizeof(*c));
    int TT = Tm > Toos ? Tm : Toos;
    if (TT < 1)
        TT = 1;
    size_t tk = (size_t)TT * K;
    int KL = K * (L > 0 ? L : 1);
    int KM = K * (M > 0 ? M : 1);
    c->x = xmalloc(sizeof(int32_t) * TT);
    c->g = xmalloc(sizeof(int32_t) * TT);
    c->sgn = xmalloc(sizeof(int32_t) * TT);
    c->x_oos = xmalloc(sizeof(int32_t) * TT);
    c->sgn_oos = xmalloc(sizeof(int32_t) * TT);
    c->xr = xmalloc(sizeof(double) * TT);
    c->u = xmalloc(sizeof(double) * (size_t)TT * (M > 0 ? M : 1));
    c->p = xmalloc(sizeof(double) * K);
    c->A = xmalloc(sizeof(double) * K * K);
    c->phi = xmalloc(sizeof(double) * KL);
    c->mu = xmalloc(sizeof(double) * K);
    c->sigma = xmalloc(sizeof(double) * K);
    c->w = xmalloc(sizeof(double) * KM);
    c->b = xmalloc(sizeof(double) * KM);
    c->sk = xmalloc(sizeof(double) * K);
    c->lambda = xmalloc(sizeof(double) * KL);
    c->mukl = xmalloc(sizeof(double) * KL);
    c->skl = xmalloc(sizeof(double) * KL);
    c->unalpha = xmalloc(sizeof(double) * tk);
    c->alpha = xmalloc(sizeof(double) * tk);
    c->unbeta = xmalloc(sizeof(double) * tk);
    c->beta = xmalloc(sizeof(double) * tk);
    c->ungamma = xmalloc(sizeof(double) * tk);
    c->gamma = xmalloc(sizeof(double) * tk);
    c->oblik = xmalloc(sizeof(double) * tk);
    c->Arow = xmalloc(sizeof(double) * tk);
    c->logA = xmalloc(sizeof(double) * tk);
    c->delta = xmalloc(sizeof(double) * tk);
    c->acc = xmalloc(sizeof(double) * (K > KL ? K : KL));
    c->tmp = xmalloc(sizeof(double) * 2 * (K > KL ? K : KL)); /* FFBS: w and A_{t+1} */
    c->bp = xmalloc(sizeof(int32_t) * tk);
    c->zstar = xmalloc(sizeof(int32_t) * TT);
    c->oblik_t = xmalloc(sizeof(double) * TT);
    c->unalpha_oos = xmalloc(sizeof(double) * tk);
    c->alpha_oos = xmalloc(sizeof(double) * tk);
    c->ffbs_u = xmalloc(sizeof(double) * TT);
    c->zf = xmalloc(sizeof(int32_t) * TT);
    c->ff = xmalloc(sizeof(double) * tk);
    c->hat_rand = xmalloc(sizeof(double) * (size_t)TT * 3);
    c->hatpi = xmalloc(sizeof(double) * tk);
    c->hatz = xmalloc(sizeof(int32_t) * TT);
    c->hatl = xmalloc(sizeof(int32_t) * TT);
    c->hatx = xmalloc(sizeof(double) * TT);
}

static void ctx_free(pair_ctx *c)
{
    void *ptrs[] = {c->x, c->g, c->sgn, c->x_oos, c->sgn_oos, c->xr, c->u, c->p, c->A, c->phi,
                    c->mu, c->sigma, c->w, c->b, c->sk, c->lambda, c->mukl, c->skl,
                    c->unalpha, c->alpha, c->unbeta, c->beta, c->ungamma, c->gamma, c->oblik,
                    c->Arow, c->logA, c->delta, c->acc, c->tmp, c->bp, c->zstar, c->oblik_t,
                    c->unalpha_oos, c->alpha_oos, c->ffbs_u, c->zf, c->ff,
                    c->hat_rand, c->hatpi, c->hatz, c->hatl, c->hatx};
    for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i)
        free(ptrs[i]);
}

#define TK(a, t, k) ((a)[(size_t)(t) * K + (k)])

/* ------------------------------------------------------------------ */
/* Shared GQ blocks                                                     */
/* ------------------------------------------------------------------ */

/* alpha_tk[t] = softmax(unalpha_tk[t])  (hmm.stan:60-63 and every model). */
static void gq_softmax_rows(const double *un, double *out, int T, int K)
{
    for (int t = 0; t < T; ++t)
        stan_softmax(&un[(size_t)t * K], K, &out[(size_t)t * K]);
}

/* ungamma = alpha .* beta; gamma = normalize(ungamma)  (hmm.stan:89-96). */
static void gq_gamma(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    for (int t = 0; t < T; ++t) {
        for (int k = 0; k < K; ++k)
            TK(c->ungamma, t, k) = TK(c->alpha, t, k) * TK(c->beta, t, k);
        stan_normalize(&TK(c->ungamma, t, 0), K, &TK(c->gamma, t, 0));
    }
}

/* Viterbi epilogue (hmm.stan:120-128): logp = max(delta[T]); zstar[T] = LAST j
 * with delta[T, j] == logp; backtrack through a_tk.  An unset back-pointer
 * (INT_MIN) is where Stan throws: the pair is flagged and zstar zeroed. */
static void viterbi_finish(pair_ctx *c, int T)
{
    const int K = c->K;
    c->logp_zstar = stan_max_vec(&TK(c->delta, T - 1, 0), K);
    int z = STAN_INT_UNSET;
    for (int j = 0; j < K; ++j)
        if (TK(c->delta, T - 1, j) == c->logp_zstar)
            z = j + 1;
    c->zstar[T - 1] = z;
    int bad = (z == STAN_INT_UNSET);
    for (int t = 1; t < T && !bad; ++t) {
        const int zn = c->zstar[T - t];
        const int zp = TK(c->bp, T - t, zn - 1);
        if (zp == STAN_INT_UNSET) {
            bad = 1;
            break;
        }
        c->zstar[T - 1 - t] = zp;
    }
    if (bad) {
        c->status = HHMM_PAIR_INVALID_BACKPOINTER;
        for (int t = 0; t < T; ++t)
            c->zstar[t] = 0;
    }
}

static void viterbi_reset(pair_ctx *c, int T)
{
    const int K = c->K;
    for (int t = 0; t < T; ++t)
        for (int k = 0; k < K; ++k) {
            TK(c->delta, t, k) = NAN;        /* stanc fills local reals with NaN */
            TK(c->bp, t, k) = STAN_INT_UNSET;
        }
}

/* ------------------------------------------------------------------ */
/* hmm/stan/hmm.stan -- Gaussian emissions                              */
/* ------------------------------------------------------------------ */
static void model_hmm_gauss(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    double *acc = c->acc;
    /* TP forward, hmm.stan:27-42.  t = 1 adds the SUM over k of the
     * per-state densities (vectorised normal_lpdf, Q2). */
    {
        const double s = stan_normal_lpdf_vec(c->xr[0], c->mu, c->sigma, K);
        for (int j = 0; j < K; ++j)
            TK(c->unalpha, 0, j) = OR_LOG(c->p[j]) + s;
    }
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i)
                acc[i] = TK(c->unalpha, t - 1, i) + OR_LOG(c->A[i * K + j]) +
                         stan_normal_lpdf(c->xr[t], c->mu[j], c->sigma[j]);
            TK(c->unalpha, t, j) = stan_log_sum_exp(acc, K);
        }
    /* model block, hmm.stan:46 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K);
    /* GQ forward, hmm.stan:60-63 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);
    /* GQ backward, hmm.stan:65-87 (unbeta[T] = 1, Q1) */
    for (int j = 0; j < K; ++j)
        TK(c->unbeta, T - 1, j) = 1;
    for (int tf = 0; tf <= T - 2; ++tf) {
        const int t = T - 1 - tf; /* 0-based; Stan's t = T - tforward */
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i)
                acc[i] = TK(c->unbeta, t, i) + OR_LOG(c->A[j * K + i]) +
                         stan_normal_lpdf(c->xr[t], c->mu[i], c->sigma[i]);
            TK(c->unbeta, t - 1, j) = stan_log_sum_exp(acc, K);
        }
    }
    gq_softmax_rows(c->unbeta, c->beta, T, K);
    gq_gamma(c); /* hmm.stan:89-96 */
    /* Viterbi, hmm.stan:98-130 (Q3: only delta[1, K] is written) */
    viterbi_reset(c, T);
    for (int j = 0; j < K; ++j)
        TK(c->delta, 0, K - 1) = stan_normal_lpdf(c->xr[0], c->mu[j], c->sigma[j]);
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            TK(c->delta, t, j) = NEG_INF;
            for (int i = 0; i < K; ++i) {
                const double logp = TK(c->delta, t - 1, i) + OR_LOG(c->A[i * K + j]) +
                                    stan_normal_lpdf(c->xr[t], c->mu[j], c->sigma[j]);
                if (logp > TK(c->delta, t, j)) {
                    TK(c->bp, t, j) = i + 1;
                    TK(c->delta, t, j) = logp;
                }
            }
        }
    viterbi_finish(c, T);
}

/* ------------------------------------------------------------------ */
/* hmm/stan/hmm-multinom.stan -- multinomial emissions                  */
/* ------------------------------------------------------------------ */
#define PHI(k, l) (c->phi[(size_t)(k) * c->L + (l)])

static void model_hmm_multinom(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    double *acc = c->acc;
    /* TP forward, hmm-multinom.stan:27-44 */
    for (int j = 0; j < K; ++j)
        TK(c->unalpha, 0, j) = OR_LOG(c->p[j]) + OR_LOG(PHI(j, c->x[0] - 1));
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i)
                acc[i] = TK(c->unalpha, t - 1, i) + OR_LOG(c->A[i * K + j]) +
                         OR_LOG(PHI(j, c->x[t] - 1));
            TK(c->unalpha, t, j) = stan_log_sum_exp(acc, K);
        }
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :48 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :62-65 */
    /* backward, hmm-multinom.stan:67-89 */
    for (int j = 0; j < K; ++j)
        TK(c->unbeta, T - 1, j) = 1;
    for (int tf = 0; tf <= T - 2; ++tf) {
        const int t = T - 1 - tf;
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i)
                acc[i] = TK(c->unbeta, t, i) + OR_LOG(c->A[j * K + i]) + OR_LOG(PHI(i, c->x[t] - 1));
            TK(c->unbeta, t - 1, j) = stan_log_sum_exp(acc, K);
        }
    }
    gq_softmax_rows(c->unbeta, c->beta, T, K);
    gq_gamma(c); /* :91-98 */
    /* Viterbi, hmm-multinom.stan:100-132 */
    viterbi_reset(c, T);
    for (int j = 0; j < K; ++j)
        TK(c->delta, 0, K - 1) = OR_LOG(PHI(j, c->x[0] - 1));
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            TK(c->delta, t, j) = NEG_INF;
            for (int i = 0; i < K; ++i) {
                const double logp = TK(c->delta, t - 1, i) + OR_LOG(c->A[i * K + j]) +
                                    OR_LOG(PHI(j, c->x[t] - 1));
                if (logp > TK(c->delta, t, j)) {
                    TK(c->bp, t, j) = i + 1;
                    TK(c->delta, t, j) = logp;
                }
            }
        }
    viterbi_finish(c, T);
}

/* ------------------------------------------------------------------ */
/* hmm/stan/hmm-multinom-semisup.stan -- group-masked forward            */
/* ------------------------------------------------------------------ */
static int semisup_mask(int g, int j1)
{
    /* hmm-multinom-semisup.stan:42 (j1 is 1-based) */
    return (g == 1 && (j1 == 1 || j1 == 4)) || (g == 2 && (j1 == 2 || j1 == 3));
}

static void model_hmm_multinom_semisup(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    double *acc = c->acc;
    /* TP forward, semisup.stan:29-49 (transition only under the mask, Q7) */
    for (int j = 0; j < K; ++j)
        TK(c->unalpha, 0, j) = OR_LOG(c->p[j]) + OR_LOG(PHI(j, c->x[0] - 1));
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i) {
                acc[i] = TK(c->unalpha, t - 1, i) + OR_LOG(PHI(j, c->x[t] - 1));
                if (semisup_mask(c->g[t], j + 1))
                    acc[i] = acc[i] + OR_LOG(c->A[i * K + j]);
            }
            TK(c->unalpha, t, j) = stan_log_sum_exp(acc, K);
        }
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :53 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :67-70 */
    /* backward, semisup.stan:72-94 (unmasked) */
    for (int j = 0; j < K; ++j)
        TK(c->unbeta, T - 1, j) = 1;
    for (int tf = 0; tf <= T - 2; ++tf) {
        const int t = T - 1 - tf;
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i)
                acc[i] = TK(c->unbeta, t, i) + OR_LOG(c->A[j * K + i]) + OR_LOG(PHI(i, c->x[t] - 1));
            TK(c->unbeta, t - 1, j) = stan_log_sum_exp(acc, K);
        }
    }
    gq_softmax_rows(c->unbeta, c->beta, T, K);
    gq_gamma(c); /* :96-103 */
    /* Viterbi, semisup.stan:105-137 (unmasked) */
    viterbi_reset(c, T);
    for (int j = 0; j < K; ++j)
        TK(c->delta, 0, K - 1) = OR_LOG(PHI(j, c->x[0] - 1));
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            TK(c->delta, t, j) = NEG_INF;
            for (int i = 0; i < K; ++i) {
                const double logp = TK(c->delta, t - 1, i) + OR_LOG(c->A[i * K + j]) +
                                    OR_LOG(PHI(j, c->x[t] - 1));
                if (logp > TK(c->delta, t, j)) {
                    TK(c->bp, t, j) = i + 1;
                    TK(c->delta, t, j) = logp;
                }
            }
        }
    viterbi_finish(c, T);
}

/* ------------------------------------------------------------------ */
/* IOHMM shared blocks                                                  */
/* ------------------------------------------------------------------ */

/* Transition TP: unA[1] = A[1] = p_1k (filler); A[t] = softmax(u_t' w_j)
 * (iohmm-reg.stan:40-49; iohmm-mix.stan:42-51).  Arow[t*K + i]. */
static void iohmm_transitions(pair_ctx *c)
{
    const int K = c->K, T = c->T, M = c->M;
    for (int k = 0; k < K; ++k)
        TK(c->Arow, 0, k) = c->p[k];
    for (int t = 1; t < T; ++t) {
        for (int j = 0; j < K; ++j)
            c->tmp[j] = stan_dot(&c->u[(size_t)t * M], &c->w[(size_t)j * M], M);
        stan_softmax(c->tmp, K, &TK(c->Arow, t, 0));
    }
}

/* hmix: logA[1] = log(p_1k); logA[t] = log(softmax(u_t' w_j))
 * (iohmm-hmix.stan:36-48; iohmm-hmix-lite.stan:32-44). */
static void iohmm_log_transitions(pair_ctx *c)
{
    const int K = c->K, T = c->T, M = c->M;
    for (int k = 0; k < K; ++k)
        TK(c->logA, 0, k) = OR_LOG(c->p[k]);
    for (int t = 1; t < T; ++t) {
        for (int j = 0; j < K; ++j)
            c->tmp[j] = stan_dot(&c->u[(size_t)t * M], &c->w[(size_t)j * M], M);
        stan_softmax(c->tmp, K, c->acc);
        for (int j = 0; j < K; ++j)
            TK(c->logA, t, j) = OR_LOG(c->acc[j]);
    }
}

/* Gaussian-mixture emission: loglambda = log(lambda_kl);
 * oblik[t][j] = LSE_l(loglambda[j][l] + normal_lpdf(x_t | mu_kl, s_kl))
 * (iohmm-mix.stan:53-65; iohmm-hmix.stan:50-62; iohmm-hmix-lite.stan:46-58). */
static void iohmm_mixture_oblik(pair_ctx *c)
{
    const int K = c->K, T = c->T, L = c->L;
    double *ll = c->tmp; /* [K*L] */
    for (int k = 0; k < K * L; ++k)
        ll[k] = OR_LOG(c->lambda[k]);
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            for (int l = 0; l < L; ++l)
                c->acc[l] = ll[j * L + l] +
                            stan_normal_lpdf(c->xr[t], c->mukl[j * L + l], c->skl[j * L + l]);
            TK(c->oblik, t, j) = stan_log_sum_exp(c->acc, L);
        }
}

/* Forward with the prev-state-indexed K-vector transition (Q5):
 * acc[i] = unalpha[t-1, i] + logA_t(i) + oblik[t][j]. */
static void iohmm_forward(pair_ctx *c, int use_logA_table)
{
    const int K = c->K, T = c->T;
    double *acc = c->acc;
    for (int j = 0; j < K; ++j)
        TK(c->unalpha, 0, j) = OR_LOG(c->p[j]) + TK(c->oblik, 0, j);
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i) {
                const double la = use_logA_table ? TK(c->logA, t, i) : OR_LOG(TK(c->Arow, t, i));
                acc[i] = TK(c->unalpha, t - 1, i) + la + TK(c->oblik, t, j);
            }
            TK(c->unalpha, t, j) = stan_log_sum_exp(acc, K);
        }
}

/* Backward: acc[i] = unbeta[t, i] + logA_t(i) + oblik[t][i], the same for
 * every j (iohmm-reg.stan:80-102; iohmm-hmix.stan:85-108). */
static void iohmm_backward(pair_ctx *c, int use_logA_table)
{
    const int K = c->K, T = c->T;
    double *acc = c->acc;
    for (int j = 0; j < K; ++j)
        TK(c->unbeta, T - 1, j) = 1;
    for (int tf = 0; tf <= T - 2; ++tf) {
        const int t = T - 1 - tf;
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i) {
                const double la = use_logA_table ? TK(c->logA, t, i) : OR_LOG(TK(c->Arow, t, i));
                acc[i] = TK(c->unbeta, t, i) + la + TK(c->oblik, t, i);
            }
            TK(c->unbeta, t - 1, j) = stan_log_sum_exp(acc, K);
        }
    }
}

/* Viterbi: (delta + logA_t(i)) + oblik[t][j]; buggy init unless fixed_init
 * (iohmm-reg.stan:150-181; iohmm-hmix.stan:160-193 has the fixed init, :166-167). */
static void iohmm_viterbi(pair_ctx *c, int use_logA_table, int fixed_init)
{
    const int K = c->K, T = c->T;
    viterbi_reset(c, T);
    if (fixed_init) {
        for (int j = 0; j < K; ++j)
            TK(c->delta, 0, j) = TK(c->oblik, 0, j);
    } else {
        for (int j = 0; j < K; ++j)
            TK(c->delta, 0, K - 1) = TK(c->oblik, 0, j);
    }
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            TK(c->delta, t, j) = NEG_INF;
            for (int i = 0; i < K; ++i) {
                const double la = use_logA_table ? TK(c->logA, t, i) : OR_LOG(TK(c->Arow, t, i));
                const double logp = TK(c->delta, t - 1, i) + la + TK(c->oblik, t, j);
                if (logp > TK(c->delta, t, j)) {
                    TK(c->bp, t, j) = i + 1;
                    TK(c->delta, t, j) = logp;
                }
            }
        }
    viterbi_finish(c, T);
}

/* iohmm-reg/stan/iohmm-reg.stan */
static void model_iohmm_reg(pair_ctx *c)
{
    const int K = c->K, T = c->T, M = c->M;
    iohmm_transitions(c); /* :40-49 */
    for (int t = 0; t < T; ++t) /* emission, :51-57 */
        for (int j = 0; j < K; ++j)
            TK(c->oblik, t, j) = stan_normal_lpdf(
                c->xr[t], stan_dot(&c->u[(size_t)t * M], &c->b[(size_t)j * M], M), c->sk[j]);
    iohmm_forward(c, 0);                                        /* :59-75 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :76-77 */
    iohmm_backward(c, 0);                                       /* :80-98 */
    gq_softmax_rows(c->unbeta, c->beta, T, K);                  /* :100-101 */
    gq_gamma(c);                                                /* :104-110 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :120 (priors excluded) */
    iohmm_viterbi(c, 0, 0);                                     /* :150-181 */
}

/* iohmm-mix/stan/iohmm-mix.stan */
static void model_iohmm_mix(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    iohmm_transitions(c);  /* :42-51 */
    iohmm_mixture_oblik(c); /* :53-65 */
    /* forward uses `logA_ij = log(A_ij)` (:69, :79) */
    for (int t = 0; t < T; ++t)
        for (int k = 0; k < K; ++k)
            TK(c->logA, t, k) = OR_LOG(TK(c->Arow, t, k));
    iohmm_forward(c, 1);                                        /* :67-83 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :85-86 */
    iohmm_backward(c, 0);                                       /* :89-107, log(A_ij) */
    gq_softmax_rows(c->unbeta, c->beta, T, K);                  /* :109-110 */
    gq_gamma(c);                                                /* :113-119 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :129 */
    iohmm_viterbi(c, 0, 0);                                     /* :164-195, log(A_ij) */
}

/* oblik_t[t] = log_sum_exp(log(alpha_tk[t]) + oblik_tk[t]) (iohmm-hmix.stan:118-121);
 * lite recomputes log(softmax(unalpha)) (iohmm-hmix-lite.stan:78-81, Q10). */
static void iohmm_oblik_t(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    for (int t = 0; t < T; ++t) {
        for (int k = 0; k < K; ++k)
            c->acc[k] = OR_LOG(TK(c->alpha, t, k)) + TK(c->oblik, t, k);
        c->oblik_t[t] = stan_log_sum_exp(c->acc, K);
    }
}

/* iohmm-mix/stan/iohmm-hmix.stan */
static void model_iohmm_hmix(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    iohmm_log_transitions(c);                                   /* :36-48 */
    iohmm_mixture_oblik(c);                                     /* :50-62 */
    iohmm_forward(c, 1);                                        /* :64-79 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :81-82 */
    iohmm_backward(c, 1);                                       /* :85-104 */
    gq_softmax_rows(c->unbeta, c->beta, T, K);                  /* :106-107 */
    for (int t = 0; t < T; ++t) {                               /* :110-116 */
        for (int k = 0; k < K; ++k)
            TK(c->ungamma, t, k) = TK(c->alpha, t, k) * TK(c->beta, t, k);
        const double s = stan_sum_vec(&TK(c->ungamma, t, 0), K);
        for (int k = 0; k < K; ++k)
            TK(c->gamma, t, k) = TK(c->ungamma, t, k) / s;
    }
    iohmm_oblik_t(c);                                           /* :118-121 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :134 */
    iohmm_viterbi(c, 1, 1);                                     /* :160-193 */
}

/* iohmm-mix/stan/iohmm-hmix-lite.stan */
static void model_iohmm_hmix_lite(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    iohmm_log_transitions(c);                                   /* :32-44 */
    iohmm_mixture_oblik(c);                                     /* :46-58 */
    iohmm_forward(c, 1);                                        /* :60-76 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* softmax in :80 */
    iohmm_oblik_t(c);                                           /* :78-81 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :94 */
}

/* ------------------------------------------------------------------ */
/* tayal2009/stan -- flattened HHMM with sign-masked transitions         */
/* ------------------------------------------------------------------ */

/* Expansion p_1k / A_ij from p_11, A_row (hhmm-tayal2009.stan:30-44). */
static void tayal_expand(pair_ctx *c, double p11, const double Arow[2][2])
{
    const int K = 4;
    for (int k = 0; k < K; ++k)
        c->p[k] = 0;
    c->p[0] = p11;
    c->p[2] = 1 - p11;
    for (int k = 0; k < K * K; ++k)
        c->A[k] = 0;
    c->A[0 * K + 1] = Arow[0][0];
    c->A[0 * K + 2] = Arow[0][1];
    c->A[1 * K + 0] = 1;
    c->A[2 * K + 0] = Arow[1][0];
    c->A[2 * K + 3] = Arow[1][1];
    c->A[3 * K + 2] = 1;
}

static int tayal_pred(int sign, int j1)
{
    /* hhmm-tayal2009.stan:62 / :109 / :144 (j1 is 1-based) */
    return (sign == 1 && (j1 == 2 || j1 == 3)) || (sign == 2 && (j1 == 1 || j1 == 4));
}

static int tayal_init_pred(int sign, int j1)
{
    return (sign == 1 && j1 == 3) || (sign == 2 && j1 == 1); /* :51 */
}

/* Tayal forward over (x, sign) of length T into un (hhmm-tayal2009.stan:46-70). */
static void tayal_forward(pair_ctx *c, const int32_t *x, const int32_t *sg, int T, double *un)
{
    const int K = c->K;
    double *acc = c->acc;
    for (int j = 0; j < K; ++j) {
        TK(un, 0, j) = OR_LOG(PHI(j, x[0] - 1));
        if (tayal_init_pred(sg[0], j + 1))
            TK(un, 0, j) = TK(un, 0, j) + OR_LOG(c->p[j]);
    }
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i) {
                acc[i] = TK(un, t - 1, i) + OR_LOG(PHI(j, x[t] - 1));
                if (tayal_pred(sg[t], j + 1))
                    acc[i] = acc[i] + OR_LOG(c->A[i * K + j]);
            }
            TK(un, t, j) = stan_log_sum_exp(acc, K);
        }
}

/* Tayal Viterbi over (x, sign) (hhmm-tayal2009.stan:130-165; lite :123-158). */
static void tayal_viterbi(pair_ctx *c, const int32_t *x, const int32_t *sg, int T)
{
    const int K = c->K;
    viterbi_reset(c, T);
    for (int j = 0; j < K; ++j)
        TK(c->delta, 0, K - 1) = OR_LOG(PHI(j, x[0] - 1));
    for (int t = 1; t < T; ++t)
        for (int j = 0; j < K; ++j) {
            TK(c->delta, t, j) = NEG_INF;
            for (int i = 0; i < K; ++i) {
                double logp = TK(c->delta, t - 1, i) + OR_LOG(PHI(j, x[t] - 1));
                if (tayal_pred(sg[t], j + 1))
                    logp = logp + OR_LOG(c->A[i * K + j]);
                if (logp > TK(c->delta, t, j)) {
                    TK(c->bp, t, j) = i + 1;
                    TK(c->delta, t, j) = logp;
                }
            }
        }
    viterbi_finish(c, T);
}

static void model_tayal(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    double *acc = c->acc;
    tayal_forward(c, c->x, c->sgn, T, c->unalpha);              /* :46-70 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :74 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :88-91 */
    /* backward, :93-119 (predicate on j = previous state, Q6) */
    for (int j = 0; j < K; ++j)
        TK(c->unbeta, T - 1, j) = 1;
    for (int tf = 0; tf <= T - 2; ++tf) {
        const int t = T - 1 - tf;
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i) {
                acc[i] = TK(c->unbeta, t, i) + OR_LOG(PHI(i, c->x[t] - 1));
                if (tayal_pred(c->sgn[t], j + 1))
                    acc[i] = acc[i] + OR_LOG(c->A[j * K + i]);
            }
            TK(c->unbeta, t - 1, j) = stan_log_sum_exp(acc, K);
        }
    }
    gq_softmax_rows(c->unbeta, c->beta, T, K);
    gq_gamma(c);                          /* :121-128 */
    tayal_viterbi(c, c->x, c->sgn, T);    /* :130-165 */
}

static void model_tayal_lite(pair_ctx *c)
{
    const int K = c->K, T = c->T;
    tayal_forward(c, c->x, c->sgn, T, c->unalpha);              /* lite :50-74 */
    c->loglik = stan_log_sum_exp(&TK(c->unalpha, T - 1, 0), K); /* :78 */
    gq_softmax_rows(c->unalpha, c->alpha, T, K);                /* :89-92 */
    tayal_forward(c, c->x_oos, c->sgn_oos, c->T_oos, c->unalpha_oos); /* :94-117 */
    gq_softmax_rows(c->unalpha_oos, c->alpha_oos, c->T_oos, K);       /* :119-120 */
    tayal_viterbi(c, c->x_oos, c->sgn_oos, c->T_oos);                 /* :123-158 */
}

/* ------------------------------------------------------------------ */
/* FFBS -- forward filtering, backward sampling        */
/* ------------------------------------------------------------------ */
/*
 * The reference has no FFBS: techreview/Rmd/hmm.Rmd:193-221 describes it in
 * prose (z_T ~ alpha_T, then z_t | z_{t+1} ~ p(z_t | z_{t+1}, x_{1:t})) and
 * stops at "= \dots" (:213).  This is the engine's CONTRACT, stated in the
 * exact arithmetic the gfx950 kernels perform, so that draws are bit-exact
 * given the caller's uniforms u[t] in (0, 1):
 *
 *   filter f_t (K-vector, linear space, renormalised each step):
 *     e_t(j) = emission: phi_k[j, x_t] (multinomial / semisup / Tayal);
 *              det_exp(lpdf_j - m) with m = fmax over j (hmm.stan Gaussian);
 *              IOHMM regression: det_exp(ob_t(j) - m), m = fmax over j (0 if -inf);
 *              IOHMM mixture: sum_l det_exp(acc_t(j,l) - m) in l order over the
 *              finite acc (acc = log lambda_jl + normal_lpdf, the summands of the
 *              model's log_sum_exp), m = fmax over j of (max_l by '>') (0 if -inf):
 *              exp(ob_t(j) - m) without forming ob_t, so a step takes K*L det_exp
 *              and no det_log
 *     det_exp / det_log: the deterministic exp / log of hhmm_detmath.h (the
 *     contract's own transcendentals: bit-identical on both sides, cheaper
 *     than the correctly rounded ones the Viterbi needs)
 *     f_0(j) = p_j * e_0(j); hmm.stan: p_j (Q2, the summed emission cancels);
 *              Tayal: e_0(j) * p_j only where the init predicate holds, else e_0(j)
 *     f_t(j) = s_t(j) * e_t(j), s_t(j) = f(0) A(0,j), then fma(f(i), A(i,j), s) for i = 1..K-1;
 *              a masked transition (semisup g_t / Tayal sign_t, as in the model's
 *              FORWARD pass) replaces s_t(j) by ((f(0) + f(1)) + ...) + f(K-1)
 *     renorm: f <- ldexp(f, -E), E = frexp exponent of fmax_j f(j) (0 if 0/inf/NaN)
 *   sampling, cat(w, u) = Stan's categorical_rng(w / sum w) with the caller's
 *     uniform, without the divisions: sum = ((w0 + w1) + ...); us = u * sum;
 *     b = 0, c = w_0; while (b < K-1 && us > c) c = c + w_{++b};  draw b + 1
 *     (0 and every earlier draw 0 if sum is not a positive finite number)
 *     z_{T-1} = cat(f_{T-1}, u_{T-1});
 *     z_t     = cat(w, u_t), w_i = f_t(i) * A(i, z_{t+1}), or w_i = f_t(i) where the
 *               model's forward mask switches the transition off at (t+1, z_{t+1})
 *   IOHMM (Q5: the transition K-vector A_t does not depend on the next state,
 *     so f_t is proportional to e_t for t >= 1 and the draws decouple):
 *     v_0 = p .* e_0, v_t = e_t (t >= 1); z_t = cat(v_t .* th_{t+1}, u_t); z_{T-1} = cat(v_{T-1}, u_{T-1}),
 *     th_t = the softmax numerators det_exp(u_t' w_j - max_j) (A_t = th_t / sum: cat
 *     normalises, so the division is left out).  ob_t and th_t follow the model's
 *     emission and softmax transition in the model's operation order
 *     (iohmm-reg.stan:40-57, iohmm-mix.stan:42-65, iohmm-hmix.stan:36-62) with
 *     det_exp / det_log in place of exp / log.
 */
static void ffbs_renorm(double *v, int K)
{
    double mx = v[0];
    for (int k = 1; k < K; ++k)
        mx = fmax(mx, v[k]);
    int e = 0;
    if (isfinite(mx) && mx != 0.0)
        (void)frexp(mx, &e);
    for (int k = 0; k < K; ++k)
        v[k] = ldexp(v[k], -e);
}

static int ffbs_cat(const double *w, int K, double u)
{
    double sum = w[0];
    for (int i = 1; i < K; ++i)
        sum = sum + w[i];
    if (!(sum > 0.0) || !isfinite(sum))
        return 0;
    /* u against the cumulative weights scaled by the sum: no division */
    const double us = u * sum;
    int b = 0;
    double cum = w[0];
    while (b < K - 1 && us > cum) {
        ++b;
        cum = cum + w[b];
    }
    return b + 1;
}

/* e_t for the HMM family (discrete tables exact; Gaussian normalised by the max). */
static void ffbs_emission_hmm(const pair_ctx *c, int gauss, const int32_t *x, int t, double *e)
{
    const int K = c->K;
    if (gauss) {
        double m = NEG_INF;
        for (int j = 0; j < K; ++j) {
            e[j] = stan_normal_lpdf(c->xr[t], c->mu[j], c->sigma[j]);
            m = fmax(m, e[j]);
        }
        for (int j = 0; j < K; ++j)
            e[j] = hhmm_det_exp(e[j] - m);
    } else {
        for (int j = 0; j < K; ++j)
            e[j] = PHI(j, x[t] - 1);
    }
}

static int ffbs_mask(int model, const pair_ctx *c, int t, int j1)
{
    if (model == HHMM_MODEL_HMM_MULTINOM_SEMISUP)
        return semisup_mask(c->g[t], j1);
    if (model == HHMM_MODEL_TAYAL)
        return tayal_pred(c->sgn[t], j1);
    return 1;
}

/* The IOHMM emission factor e_t (K-vector, scaled by exp(-m)) of the FFBS
 * contract, from the model's emission (model_iohmm_reg's normal_lpdf,
 * iohmm_mixture_oblik's summands) with det_exp / det_log. */
static void ffbs_iohmm_emission(const pair_ctx *c, int model, int t, double *e)
{
    const int K = c->K, M = c->M, L = c->L;
    double m = NEG_INF;
    if (model == HHMM_MODEL_IOHMM_REG) {
        for (int j = 0; j < K; ++j) { /* normal_lpdf(x_t | u_t' b_j, s_j) (iohmm-reg.stan:51-57) */
            const double mu = stan_dot(&c->u[(size_t)t * M], &c->b[(size_t)j * M], M);
            const double z = (c->xr[t] - mu) * (1.0 / c->sk[j]);
            e[j] = (HHMM_NEG_LOG_SQRT_TWO_PI - hhmm_det_log(c->sk[j])) + (-0.5 * (z * z));
            m = (j == 0) ? e[j] : fmax(m, e[j]);
        }
        if (m == NEG_INF)
            m = 0.0;
        for (int j = 0; j < K; ++j)
            e[j] = hhmm_det_exp(e[j] - m);
        return;
    }
    /* the summands of LSE_l(log lambda_jl + normal_lpdf(x_t | mu_jl, s_jl)) (iohmm-mix.stan:53-65) */
    double acc[K * (L > 0 ? L : 1)];
    for (int j = 0; j < K; ++j) {
        double mx = NEG_INF;
        for (int l = 0; l < L; ++l) {
            const double s = c->skl[j * L + l];
            const double z = (c->xr[t] - c->mukl[j * L + l]) * (1.0 / s);
            const double a = hhmm_det_log(c->lambda[j * L + l]) + ((HHMM_NEG_LOG_SQRT_TWO_PI - hhmm_det_log(s)) + (-0.5 * (z * z)));
            acc[j * L + l] = a;
            if (a > mx)
                mx = a;
        }
        m = (j == 0) ? mx : fmax(m, mx);
    }
    if (m == NEG_INF)
        m = 0.0;
    for (int j = 0; j < K; ++j) {
        double sum = 0.0;
        for (int l = 0; l < L; ++l)
            if (acc[j * L + l] != NEG_INF)
                sum += hhmm_det_exp(acc[j * L + l] - m);
        e[j] = sum;
    }
}

/* The softmax numerators th_t(j) = det_exp(u_t' w_j - max) (t >= 1). */
static void ffbs_iohmm_transition(const pair_ctx *c, int t, double *th)
{
    const int K = c->K, M = c->M;
    double mx = NEG_INF;
    for (int j = 0; j < K; ++j) {
        th[j] = stan_dot(&c->u[(size_t)t * M], &c->w[(size_t)j * M], M);
        if (j == 0 || th[j] > mx)
            mx = th[j];
    }
    for (int j = 0; j < K; ++j)
        th[j] = hhmm_det_exp(th[j] - mx);
}

static void ffbs_contract(pair_ctx *c, int model)
{
    const int K = c->K, T = c->T;
    double *e = c->acc, *w = c->tmp;
    const int iohmm = (model == HHMM_MODEL_IOHMM_REG || model == HHMM_MODEL_IOHMM_MIX ||
                       model == HHMM_MODEL_IOHMM_HMIX);
    if (iohmm) {
        double *A1 = w + K; /* A_{t+1} */
        for (int t = 0; t < T; ++t) {
            ffbs_iohmm_emission(c, model, t, e);
            for (int k = 0; k < K; ++k)
                TK(c->ff, t, k) = (t == 0) ? c->p[k] * e[k] : e[k];
            if (t + 1 < T)
                ffbs_iohmm_transition(c, t + 1, A1);
            for (int i = 0; i < K; ++i)
                w[i] = (t + 1 < T) ? TK(c->ff, t, i) * A1[i] : TK(c->ff, t, i);
            c->zf[t] = ffbs_cat(w, K, c->ffbs_u[t]);
        }
        return;
    }
    const int gauss = (model == HHMM_MODEL_HMM_GAUSS);
    /* forward filter */
    ffbs_emission_hmm(c, gauss, c->x, 0, e);
    for (int j = 0; j < K; ++j) {
        if (gauss)
            TK(c->ff, 0, j) = c->p[j];
        else if (model == HHMM_MODEL_TAYAL)
            TK(c->ff, 0, j) = tayal_init_pred(c->sgn[0], j + 1) ? e[j] * c->p[j] : e[j];
        else
            TK(c->ff, 0, j) = c->p[j] * e[j];
    }
    ffbs_renorm(&TK(c->ff, 0, 0), K);
    for (int t = 1; t < T; ++t) {
        ffbs_emission_hmm(c, gauss, c->x, t, e);
        const double *fp = &TK(c->ff, t - 1, 0);
        double tot = fp[0];
        for (int i = 1; i < K; ++i)
            tot = tot + fp[i];
        for (int j = 0; j < K; ++j) {
            double s = fp[0] * c->A[0 * K + j];
            for (int i = 1; i < K; ++i)
                s = fma(fp[i], c->A[i * K + j], s);
            if (!ffbs_mask(model, c, t, j + 1))
                s = tot;
            TK(c->ff, t, j) = s * e[j];
        }
        ffbs_renorm(&TK(c->ff, t, 0), K);
    }
    /* backward sampling */
    c->zf[T - 1] = ffbs_cat(&TK(c->ff, T - 1, 0), K, c->ffbs_u[T - 1]);
    for (int t = T - 2; t >= 0; --t) {
        const int zn = c->zf[t + 1];
        if (zn == 0) {
            c->zf[t] = 0;
            continue;
        }
        const int on = ffbs_mask(model, c, t + 1, zn);
        for (int i = 0; i < K; ++i)
            w[i] = on ? TK(c->ff, t, i) * c->A[i * K + (zn - 1)] : TK(c->ff, t, i);
        c->zf[t] = ffbs_cat(w, K, c->ffbs_u[t]);
    }
}

/* ------------------------------------------------------------------ */
/* Fitted-output draws                                   */
/* ------------------------------------------------------------------ */

/* Stan Math categorical_rng(theta, rng) with the caller's uniform u in
 * place of uniform_01(rng): index = cumulative_sum(theta); b = 0;
 * while (u > index[b]) b++ -- bounded to n - 1 (a u above a total that
 * rounded below 1 takes the last category).  Returns 1-based. */
static int stan_categorical(const double *theta, int n, double u)
{
    int b = 0;
    double cum = theta[0];
    while (b < n - 1 && u > cum) {
        ++b;
        cum = cum + theta[b];
    }
    return b + 1;
}

/* iohmm-reg.stan:131-148, iohmm-mix.stan:140-160, iohmm-hmix.stan:146-157:
 *   reg_tk[t, j] = u_tm[t]' * to_vector(w_km[j]); hatpi_tk[t] = softmax(reg_tk[t]);
 *   hatz_t[t] = categorical_rng(hatpi_tk[t]);
 *   reg:  hatx_t[t] = normal_rng(u_tm[t]' * b_km[hatz_t[t]], s_k[hatz_t[t]]);
 *   mix:  hatl_t[t] = categorical_rng(lambda_kl[hatz_t[t]]);
 *         hatx_t[t] = normal_rng(mu_kl[hatz][hatl], s_kl[hatz][hatl]).
 * normal_rng(mu, sigma) is boost's normal_distribution: unit deviate * sigma
 * + mu, the unit deviate supplied by the caller (hat_rand[.,.,2]). */
static void fitted_draws(pair_ctx *c, int model, int have_rand)
{
    const int K = c->K, T = c->T, M = c->M, L = c->L;
    double *v = c->acc;
    for (int t = 0; t < T; ++t) {
        for (int j = 0; j < K; ++j)
            v[j] = stan_dot(&c->u[(size_t)t * M], &c->w[(size_t)j * M], M);
        stan_softmax(v, K, &TK(c->hatpi, t, 0));
        if (!have_rand)
            continue;
        const double *rnd = &c->hat_rand[(size_t)t * 3];
        const int z = stan_categorical(&TK(c->hatpi, t, 0), K, rnd[0]);
        c->hatz[t] = z;
        if (model == HHMM_MODEL_IOHMM_REG) {
            const double mu = stan_dot(&c->u[(size_t)t * M], &c->b[(size_t)(z - 1) * M], M);
            c->hatl[t] = 0;
            c->hatx[t] = rnd[2] * c->sk[z - 1] + mu;
        } else {
            const int l = stan_categorical(&c->lambda[(size_t)(z - 1) * L], L, rnd[1]);
            c->hatl[t] = l;
            c->hatx[t] = rnd[2] * c->skl[(z - 1) * L + (l - 1)] + c->mukl[(z - 1) * L + (l - 1)];
        }
    }
}

/* ------------------------------------------------------------------ */
/* Batch driver                                                         */
/* ------------------------------------------------------------------ */

static int64_t num_pairs(const hhmm_request *r)
{
    if (r->pairing == HHMM_PAIR_ZIP)
        return r->data.n_series == r->draws.n_draws ? r->data.n_series : -1;
    if (r->pairing == HHMM_PAIR_BLOCK)
        return r->draws.n_draws % r->data.n_series == 0 ? r->draws.n_draws : -1;
    return r->data.n_series * r->draws.n_draws;
}

/* pair p -> (series n, draw s), include/hhmm.h pairing modes */
static void pair_of(const hhmm_request *r, int64_t p, int64_t *n, int64_t *s)
{
    const int64_t N = r->data.n_series, S = r->draws.n_draws;
    if (r->pairing == HHMM_PAIR_ZIP) {
        *n = p;
        *s = p;
    } else if (r->pairing == HHMM_PAIR_BLOCK) {
        *n = p / (S / N);
        *s = p;
    } else {
        *n = p / S;
        *s = p % S;
    }
}

static void gather(pair_ctx *c, const hhmm_request *r, int64_t p, int64_t n, int64_t s)
{
    const hhmm_data *d = &r->data;
    const hhmm_draws *w = &r->draws;
    const int64_t N = d->n_series, S = w->n_draws;
    const int K = c->K, L = c->L, M = c->M;
    const int Tm = d->T_max;
    for (int t = 0; t < c->T; ++t) {
        const size_t ix = (size_t)n + (size_t)N * t;
        if (d->x_int) c->x[t] = d->x_int[ix];
        if (d->x_real) c->xr[t] = d->x_real[ix];
        if (d->g) c->g[t] = d->g[ix];
        if (d->sign) c->sgn[t] = d->sign[ix];
        if (d->u)
            for (int m = 0; m < M; ++m)
                c->u[(size_t)t * M + m] = d->u[(size_t)n + (size_t)N * ((size_t)t + (size_t)Tm * m)];
    }
    if (r->ffbs_u) {
        const size_t P = (size_t)num_pairs(r), pp = (size_t)p;
        for (int t = 0; t < c->T; ++t)
            c->ffbs_u[t] = r->ffbs_u[pp + P * (size_t)t];
    }
    if (r->hat_rand) {
        const size_t P = (size_t)num_pairs(r), pp = (size_t)p;
        for (int t = 0; t < c->T; ++t)
            for (int q = 0; q < 3; ++q)
                c->hat_rand[(size_t)t * 3 + q] = r->hat_rand[pp + P * ((size_t)t + (size_t)Tm * q)];
    }
    for (int t = 0; t < c->T_oos; ++t) {
        const size_t ix = (size_t)n + (size_t)N * t;
        c->x_oos[t] = d->x_oos[ix];
        c->sgn_oos[t] = d->sign_oos[ix];
    }
#define DRAW1(arr, k) ((arr)[(size_t)s + (size_t)S * (size_t)(k)])
#define DRAW2(arr, a, b, A_) ((arr)[(size_t)s + (size_t)S * ((size_t)(a) + (size_t)(A_) * (size_t)(b))])
    if (w->p_1k) for (int k = 0; k < K; ++k) c->p[k] = DRAW1(w->p_1k, k);
    if (w->A_ij) for (int i = 0; i < K; ++i) for (int j = 0; j < K; ++j) c->A[i * K + j] = DRAW2(w->A_ij, i, j, K);
    if (w->phi_k) for (int k = 0; k < K; ++k) for (int l = 0; l < L; ++l) c->phi[k * L + l] = DRAW2(w->phi_k, k, l, K);
    if (w->mu_k) for (int k = 0; k < K; ++k) c->mu[k] = DRAW1(w->mu_k, k);
    if (w->sigma_k) for (int k = 0; k < K; ++k) c->sigma[k] = DRAW1(w->sigma_k, k);
    if (w->w_km) for (int k = 0; k < K; ++k) for (int m = 0; m < M; ++m) c->w[k * M + m] = DRAW2(w->w_km, k, m, K);
    if (w->b_km) for (int k = 0; k < K; ++k) for (int m = 0; m < M; ++m) c->b[k * M + m] = DRAW2(w->b_km, k, m, K);
    if (w->s_k) for (int k = 0; k < K; ++k) c->sk[k] = DRAW1(w->s_k, k);
    if (w->lambda_kl) for (int k = 0; k < K; ++k) for (int l = 0; l < L; ++l) c->lambda[k * L + l] = DRAW2(w->lambda_kl, k, l, K);
    if (w->mu_kl) for (int k = 0; k < K; ++k) for (int l = 0; l < L; ++l) c->mukl[k * L + l] = DRAW2(w->mu_kl, k, l, K);
    if (w->s_kl) for (int k = 0; k < K; ++k) for (int l = 0; l < L; ++l) c->skl[k * L + l] = DRAW2(w->s_kl, k, l, K);
    if (r->model == HHMM_MODEL_TAYAL || r->model == HHMM_MODEL_TAYAL_LITE) {
        double ar[2][2];
        for (int a = 0; a < 2; ++a)
            for (int b2 = 0; b2 < 2; ++b2)
                ar[a][b2] = DRAW2(w->A_row, a, b2, 2);
        tayal_expand(c, DRAW1(w->p_11, 0), ar);
    }
#undef DRAW1
#undef DRAW2
}

static void scatter(const pair_ctx *c, const hhmm_request *r, hhmm_result *o, int64_t p, int64_t P)
{
    const uint32_t out = r->outputs;
    const int K = c->K, T = c->T, Tm = r->data.T_max, To = r->data.T_oos_max;
#define PTK(arr, t, k, TT) (arr)[(size_t)p + (size_t)P * ((size_t)(t) + (size_t)(TT) * (size_t)(k))]
#define PUT_TK(bit, dst, src)                                     \
    if ((out & (bit)) && (dst))                                   \
        for (int t = 0; t < T; ++t)                               \
            for (int k = 0; k < K; ++k)                           \
                PTK(dst, t, k, Tm) = src[(size_t)t * K + k];
    if ((out & HHMM_OUT_LOGLIK) && o->loglik)
        o->loglik[p] = c->loglik;
    PUT_TK(HHMM_OUT_UNALPHA, o->unalpha_tk, c->unalpha)
    PUT_TK(HHMM_OUT_ALPHA, o->alpha_tk, c->alpha)
    PUT_TK(HHMM_OUT_UNBETA, o->unbeta_tk, c->unbeta)
    PUT_TK(HHMM_OUT_BETA, o->beta_tk, c->beta)
    PUT_TK(HHMM_OUT_UNGAMMA, o->ungamma_tk, c->ungamma)
    PUT_TK(HHMM_OUT_GAMMA, o->gamma_tk, c->gamma)
    PUT_TK(HHMM_OUT_OBLIK_TK, o->oblik_tk, c->oblik)
    if ((out & HHMM_OUT_LOGA) && o->logA_ij) {
        const double *src = (r->model == HHMM_MODEL_IOHMM_HMIX || r->model == HHMM_MODEL_IOHMM_HMIX_LITE)
                                ? c->logA : c->Arow;
        PUT_TK(HHMM_OUT_LOGA, o->logA_ij, src)
    }
    if ((out & HHMM_OUT_OBLIK_T) && o->oblik_t)
        for (int t = 0; t < T; ++t)
            o->oblik_t[(size_t)p + (size_t)P * t] = c->oblik_t[t];
    const int Tz = (r->model == HHMM_MODEL_TAYAL_LITE) ? c->T_oos : T;
    if ((out & HHMM_OUT_ZSTAR) && o->zstar_t)
        for (int t = 0; t < Tz; ++t)
            o->zstar_t[(size_t)p + (size_t)P * t] = c->zstar[t];
    if ((out & HHMM_OUT_LOGP_ZSTAR) && o->logp_zstar)
        o->logp_zstar[p] = c->logp_zstar;
    if (r->model == HHMM_MODEL_TAYAL_LITE) {
        if ((out & HHMM_OUT_ALPHA_OOS) && o->alpha_tk_oos)
            for (int t = 0; t < c->T_oos; ++t)
                for (int k = 0; k < K; ++k)
                    PTK(o->alpha_tk_oos, t, k, To) = c->alpha_oos[(size_t)t * K + k];
        if ((out & HHMM_OUT_UNALPHA_OOS) && o->unalpha_tk_oos)
            for (int t = 0; t < c->T_oos; ++t)
                for (int k = 0; k < K; ++k)
                    PTK(o->unalpha_tk_oos, t, k, To) = c->unalpha_oos[(size_t)t * K + k];
    }
    if ((out & HHMM_OUT_FFBS) && o->z_ffbs)
        for (int t = 0; t < T; ++t)
            o->z_ffbs[(size_t)p + (size_t)P * t] = c->zf[t];
    PUT_TK(HHMM_OUT_HATPI, o->hatpi_tk, c->hatpi)
    if ((out & HHMM_OUT_HATZ) && o->hatz_t)
        for (int t = 0; t < T; ++t)
            o->hatz_t[(size_t)p + (size_t)P * t] = c->hatz[t];
    if ((out & HHMM_OUT_HATL) && o->hatl_t)
        for (int t = 0; t < T; ++t)
            o->hatl_t[(size_t)p + (size_t)P * t] = c->hatl[t];
    if ((out & HHMM_OUT_HATX) && o->hatx_t)
        for (int t = 0; t < T; ++t)
            o->hatx_t[(size_t)p + (size_t)P * t] = c->hatx[t];
    if (o->pair_status)
        o->pair_status[p] = c->status;
#undef PUT_TK
#undef PTK
}

static void run_pair(pair_ctx *c, const hhmm_request *r)
{
    switch (r->model) {
    case HHMM_MODEL_HMM_GAUSS: model_hmm_gauss(c); break;
    case HHMM_MODEL_HMM_MULTINOM: model_hmm_multinom(c); break;
    case HHMM_MODEL_HMM_MULTINOM_SEMISUP: model_hmm_multinom_semisup(c); break;
    case HHMM_MODEL_IOHMM_REG: model_iohmm_reg(c); break;
    case HHMM_MODEL_IOHMM_MIX: model_iohmm_mix(c); break;
    case HHMM_MODEL_IOHMM_HMIX: model_iohmm_hmix(c); break;
    case HHMM_MODEL_IOHMM_HMIX_LITE: model_iohmm_hmix_lite(c); break;
    case HHMM_MODEL_TAYAL: model_tayal(c); break;
    case HHMM_MODEL_TAYAL_LITE: model_tayal_lite(c); break;
    default: break;
    }
    if ((r->outputs & HHMM_OUT_FFBS) && r->ffbs_u)
        ffbs_contract(c, r->model);
    if (r->outputs & (HHMM_OUT_HATPI | HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX))
        fitted_draws(c, r->model, r->hat_rand != NULL);
}

/* Runs pairs [p0, p1) of the request; nthreads <= 0 uses the OpenMP default.
 * Returns 0, or 1 if some pair failed its Viterbi backtrack, or -1 on a bad request. */
int hhmm_oracle_run_range(const hhmm_request *r, hhmm_result *o, int64_t p0, int64_t p1, int nthreads)
{
    const int64_t P = num_pairs(r);
    if (P < 0 || r->model < 1 || r->model > 9)
        return -1;
    if (p1 > P)
        p1 = P;
    const int K = r->data.K;
    const int L = r->data.L, M = r->data.M;
    int failures = 0;
#ifdef _OPENMP
    if (nthreads > 0)
        omp_set_num_threads(nthreads);
#pragma omp parallel reduction(+ : failures)
#endif
    {
        pair_ctx c;
        ctx_alloc(&c, K, L, M, r->data.T_max, r->data.T_oos_max);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t p = p0; p < p1; ++p) {
            int64_t n, s;
            pair_of(r, p, &n, &s);
            c.K = K;
            c.L = L;
            c.M = M;
            c.T = r->data.T ? r->data.T[n] : r->data.T_max;
            c.T_oos = (r->model == HHMM_MODEL_TAYAL_LITE)
                          ? (r->data.T_oos ? r->data.T_oos[n] : r->data.T_oos_max) : 0;
            c.status = 0;
            c.loglik = NAN;
            c.logp_zstar = NAN;
            gather(&c, r, p, n, s);
            run_pair(&c, r);
            if (c.status)
                failures += 1;
            scatter(&c, r, o, p, P);
        }
        ctx_free(&c);
    }
    return failures ? 1 : 0;
}

int hhmm_oracle_run(const hhmm_request *r, hhmm_result *o, int nthreads)
{
    return hhmm_oracle_run_range(r, o, 0, INT64_MAX, nthreads);
}

/* The oracle's log (correctly rounded unless built with HHMM_ORACLE_LIBM_LOG). */
void hhmm_oracle_log_array(const double *in, double *out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        out[i] = OR_LOG(in[i]);
}

void hhmm_oracle_exp_array(const double *in, double *out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        out[i] = OR_EXP(in[i]);
}

/* The FFBS contract's deterministic log / exp (hhmm_detmath.h; every build). */
void hhmm_oracle_det_log_array(const double *in, double *out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        out[i] = hhmm_det_log(in[i]);
}

void hhmm_oracle_det_exp_array(const double *in, double *out, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        out[i] = hhmm_det_exp(in[i]);
}

/* Self-check of hhmm_crmath.h's quick phases against its accurate phases
 * (which = 0: log, 1: exp) over in[0..n): stats[0] = max relative distance
 * between the two double-double values where the quick phase applies,
 * stats[1] = arguments whose rounding test failed (accurate fallback),
 * stats[2] = arguments where hhmm_cr_* differs from the accurate value rounded
 * once (must be 0), stats[3] = arguments the quick phase covered. */
void hhmm_oracle_crmath_quick_check(int which, const double *in, int64_t n, double *stats)
{
    double maxrel = 0.0, fails = 0.0, bad = 0.0, covered = 0.0, zfails = 0.0, zbad = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        const double x = in[i];
        hhmm_dd q, a;
        double acc, bound;
        int eq = 0, ea = 0;
        if (which == 0) {
            if (!(x >= 0x1p-1022) || x == __builtin_inf() || x == 1.0)
                continue;
            q = hhmm_cr_log_quick_dd(x);
            a = hhmm_cr_log_acc_dd(x);
            acc = a.hi + a.lo;
            bound = fabs(q.hi) * 0x1p-68;
            bad += (hhmm_cr_log(x) != acc);
            /* the device's test (hhmm_round_ziv): where it accepts, q.hi must be the CR value */
            const int zok = hhmm_round_ziv(q.hi, q.lo, HHMM_CR_LOG_ZIV);
            zfails += !zok;
            zbad += zok && q.hi != acc;
        } else {
            if (!(x > -707.0 && x < 693.0))
                continue;
            q = hhmm_cr_exp_quick_dd(x, &eq);
            a = hhmm_cr_exp_acc_dd(x, &ea);
            if (eq != ea) {
                bad += 1.0;
                continue;
            }
            acc = a.hi + a.lo;
            bound = q.hi * 0x1p-72;
            bad += (hhmm_cr_exp(x) != acc * ldexp(1.0, ea));
            const int zok = hhmm_round_ziv(q.hi, q.lo, HHMM_CR_EXP_ZIV);
            zfails += !zok;
            zbad += zok && q.hi != acc;
        }
        covered += 1.0;
        const double rel = fabs((q.hi - a.hi) + (q.lo - a.lo)) / fabs(a.hi);
        if (rel > maxrel)
            maxrel = rel;
        fails += !hhmm_round_safe(q.hi, q.lo, bound);
    }
    stats[0] = maxrel;
    stats[1] = fails;
    stats[2] = bad;
    stats[3] = covered;
    stats[4] = zfails;
    stats[5] = zbad;
}

const char *hhmm_oracle_variant(void)
{
#ifdef HHMM_ORACLE_LIBM_LOG
    return "libm-log";
#else
    return "cr-log";
#endif
}
