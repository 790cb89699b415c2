/*
 * hhmm_params.h -- C ABI of parameter-draw ingestion, part
 * of libhhmm.so: Stan's constraining transforms applied to a batch of
 * unconstrained draws, producing the hhmm_draws arrays the engine consumes.
 *
 * Replaces, for all draws at once, what rstan does per draw when it maps a
 * point of the sampler's unconstrained space to the parameters block
 * (`constrain_pars(fit, upars)`, the inverse of `unconstrain_pars`; stanc's
 * generated `write_array` reads the block with `in__.<type>_constrain()`).
 * The parameter blocks are those of the nine programs:
 *   hmm.stan:13-22                 simplex[K] p_1k; simplex[K] A_ij[K]; ordered[K] mu_k;
 *                                  real<lower=0.0001> sigma_k[K]
 *   hmm-multinom.stan:14-22,       simplex[K] p_1k; simplex[K] A_ij[K]; simplex[L] phi_k[K]
 *   hmm-multinom-semisup.stan:16-24
 *   iohmm-reg.stan:16-24           simplex[K] p_1k; vector[M] w_km[K]; vector[M] b_km[K];
 *                                  real<lower=0.0001> s_k[K]
 *   iohmm-mix.stan:17-26           simplex[K] p_1k; vector[M] w_km[K]; simplex[L] lambda_kl[K];
 *                                  ordered[L] mu_kl[K]; vector<lower=0>[L] s_kl[K]
 *   iohmm-hmix.stan:13-23          ... + ordered[K] hypermu_k
 *   iohmm-hmix-lite.stan:13-23     ... + real hypermu_k[K]
 *   hhmm-tayal2009(-lite).stan     real<lower=0,upper=1> p_11; simplex[2] A_row[2];
 *                                  simplex[L] phi_k[K]    (K = 4)
 *
 * Unconstrained layout (Stan's): the parameters in declaration order; an
 * array of vectors is array-index major, vector index minor; a simplex[n]
 * takes n - 1 values.  theta is [S, n_unc], draw fastest: theta[s + S*i].
 * Transforms (Stan Math): simplex = stick-breaking with
 * z_k = inv_logit(y_k - log(n - 1 - k)); ordered: x_0 = y_0,
 * x_k = x_{k-1} + exp(y_k); lower bound: exp(y) + lb; (0, 1) bound: Stan's
 * lub_constrain with its 1 - 1e-15 / 1e-15 clamps.  exp / log are the
 * correctly rounded functions shared with the oracle.
 */
#ifndef HHMM_PARAMS_H
#define HHMM_PARAMS_H

#include "hhmm.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Constrained outputs in the hhmm_draws layouts ([S, ...], S fastest);
 * NULL = not materialised.  hypermu_k ([S, K]) is a parameter of
 * iohmm-hmix(-lite) that no path output reads. */
typedef struct hhmm_param_out {
    double *p_1k, *A_ij, *phi_k, *mu_k, *sigma_k, *w_km, *b_km, *s_k;
    double *lambda_kl, *mu_kl, *s_kl, *p_11, *A_row, *hypermu_k;
} hhmm_param_out;

/* Length of one draw's unconstrained vector, or -1 for a bad model / dims. */
int64_t hhmm_num_unconstrained(int model, int K, int L, int M);

/* Host pointers: uploads theta [S, n_unc], constrains on `device` (-1 =
 * current), downloads every non-NULL output. */
hhmm_status hhmm_constrain_draws(int model, int K, int L, int M, int64_t S, const double *theta,
                                 hhmm_param_out *out, int device);

/* Device pointers on the current device, enqueued on `stream`. */
hhmm_status hhmm_constrain_draws_device(int model, int K, int L, int M, int64_t S, const double *theta,
                                        hhmm_param_out *out, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HHMM_PARAMS_H */
