/*
 * hhmm_fitted.hip -- fitted-output draws of the IOHMM generated quantities
 * (SURVEY.md §8 F4):
 *   iohmm-reg.stan:131-148   hatpi_tk, hatz_t, hatx_t
 *   iohmm-mix.stan:140-160   hatpi_tk, hatz_t, hatl_t, hatx_t
 *   iohmm-hmix.stan:146-157  hatz_t, hatl_t, hatx_t (hatpi_tk is a local)
 *
 * Per step t (independent of the recursions: only u_t and the draw):
 *   reg_tk[t, j] = u_t' w_km[j]                     (Eigen SSE2 dot order)
 *   hatpi_tk[t]  = softmax(reg_tk[t])               (Stan Math softmax, CR exp)
 *   hatz_t[t]    = categorical_rng(hatpi_tk[t])     uniform hat_rand[p, t, 0]
 *   hatl_t[t]    = categorical_rng(lambda_kl[hatz]) uniform hat_rand[p, t, 1]
 *   hatx_t[t]    = normal_rng(mu, sigma) = z * sigma + mu,  z = hat_rand[p, t, 2]
 * with mu, sigma = u_t' b_km[hatz], s_k[hatz] (reg) or mu_kl[hatz][hatl],
 * s_kl[hatz][hatl] (mix / hmix).  Stan draws with its own RNG; the caller's
 * uniforms / normal deviates make the draws reproducible, and every value the
 * categorical draw compares against is bit-identical to the oracle's
 * (correctly rounded exp in the softmax), so hatz / hatl / hatx match it
 * exactly.
 *
 * Layout (K <= 8): one lane per pair; every per-step load and store is a
 * coalesced pair-fastest wave transaction (u_t is a broadcast in GRID
 * pairing); 8 < K <= 32: a group of lanes per pair (hhmm_lkio.h).  The
 * kernel is HBM-bound at (K*8 hatpi + 4 + 4 + 8 outputs + 24 random inputs)
 * B per series-timestep.
 */
#include "hhmm_lkio.h"

namespace hhmm {

template <int FAM, int K, int MMAX>
__global__ void __launch_bounds__(kBlock) fitted_kernel(const DevArgs a)
{
    const int64_t p = min((int64_t)blockIdx.x * blockDim.x + threadIdx.x, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int M = a.M, L = a.L;
    const uint32_t po = (uint32_t)p;

    double w[K][MMAX];
    double b[FAM == IO_REG ? K : 1][MMAX];
    double s[FAM == IO_REG ? K : 1];
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int m = 0; m < MMAX; ++m) {
            w[k][m] = (m < M) ? a.w_km[d + a.S * ((int64_t)k + (int64_t)K * m)] : 0.0;
            if constexpr (FAM == IO_REG)
                b[k][m] = (m < M) ? a.b_km[d + a.S * ((int64_t)k + (int64_t)K * m)] : 0.0;
        }
        if constexpr (FAM == IO_REG)
            s[k] = a.s_k[d + a.S * k];
    }
    const bool draw = a.hat_rand && (a.outputs & (HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX));
    const int Tw = wave_max(Tp);
    for (int t = 0; t < Tw; ++t) {
        if (t >= Tp)
            continue;
        const int64_t row = a.N * (int64_t)t;
        double u[MMAX];
#pragma unroll
        for (int m = 0; m < MMAX; ++m)
            u[m] = (m < M) ? at(a.u + row + a.N * (int64_t)a.Tmax * m, (uint32_t)n * 8u) : 0.0;
        double v[K], th[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            v[j] = sse_dot<MMAX>(u, w[j], M);
        stan_softmax<K, true>(v, th);
        if ((a.outputs & HHMM_OUT_HATPI) && a.hatpi)
            store_tk<K>(a.hatpi, a, p, t, th);
        if (!draw)
            continue;
        const double *rnd = a.hat_rand + a.P * (int64_t)t;
        const int64_t rs = a.P * (int64_t)a.Tmax;
        const int z = stan_categorical<K>(th, K, at(rnd, po * 8u));
        const double zn = at(rnd + 2 * rs, po * 8u);
        double mu, sg;
        int l = 0;
        if constexpr (FAM == IO_REG) {
            double bz[MMAX];
            sg = s[0];
#pragma unroll
            for (int m = 0; m < MMAX; ++m)
                bz[m] = b[0][m];
#pragma unroll
            for (int j = 1; j < K; ++j)
                if (z == j) {
                    sg = s[j];
#pragma unroll
                    for (int m = 0; m < MMAX; ++m)
                        bz[m] = b[j][m];
                }
            mu = sse_dot<MMAX>(u, bz, M); /* reg_tk[t] = u_tm[t]' * b_km[hatz_t[t]] */
        } else {
            double lam[kIoLmax];
#pragma unroll
            for (int q = 0; q < kIoLmax; ++q)
                lam[q] = (q < L) ? a.lambda_kl[d + a.S * ((int64_t)z + (int64_t)K * q)] : 0.0;
            l = stan_categorical<kIoLmax>(lam, L, at(rnd + rs, po * 8u));
            const int64_t ix = d + a.S * ((int64_t)z + (int64_t)K * l);
            mu = a.mu_kl[ix];
            sg = a.s_kl[ix];
        }
        if ((a.outputs & HHMM_OUT_HATZ) && a.hatz)
            at(a.hatz + a.P * (int64_t)t, po * 4u) = z + 1;
        if constexpr (FAM == IO_MIX)
            if ((a.outputs & HHMM_OUT_HATL) && a.hatl)
                at(a.hatl + a.P * (int64_t)t, po * 4u) = l + 1;
        if ((a.outputs & HHMM_OUT_HATX) && a.hatx)
            at(a.hatx + a.P * (int64_t)t, po * 8u) = zn * sg + mu;
    }
}

template <int FAM, int K>
static hhmm_status launch_fitted_k(const DevArgs &a, hipStream_t st)
{
    const dim3 grid((unsigned)((a.P + kBlock - 1) / kBlock));
    if (a.M <= 4)
        hipLaunchKernelGGL((fitted_kernel<FAM, K, 4>), grid, dim3(kBlock), 0, st, a);
    else
        hipLaunchKernelGGL((fitted_kernel<FAM, K, 8>), grid, dim3(kBlock), 0, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("fitted_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

template <int FAM, int KK>
static hhmm_status launch_fitted_range(const DevArgs &a, hipStream_t st)
{
    if constexpr (KK > kMaxK) {
        set_error("K = %d not supported by the fitted-output path", a.K);
        return HHMM_ERR_UNSUPPORTED;
    } else {
        if (a.K == KK)
            return launch_fitted_k<FAM, KK>(a, st);
        return launch_fitted_range<FAM, KK + 1>(a, st);
    }
}

hhmm_status launch_fitted(const DevArgs &a, hipStream_t st)
{
    char why[160];
    const bool reg = a.model == HHMM_MODEL_IOHMM_REG;
    if (a.K > kMaxK && a.K <= kMaxKLarge) /* group per pair (hhmm_lkio.h lkfit_kernel) */
        return reg ? launch_lkfit<IO_REG>(a, st) : launch_lkfit<IO_MIX>(a, st);
    if (!iohmm_supported(a.K, a.M, reg ? 1 : a.L, why, sizeof(why))) {
        set_error("%s", why);
        return HHMM_ERR_UNSUPPORTED;
    }
    return reg ? launch_fitted_range<IO_REG, 1>(a, st) : launch_fitted_range<IO_MIX, 1>(a, st);
}

} // namespace hhmm
