/*
 * hhmm_iolog.hip -- log-space re-run of the IOHMM filter for the pairs whose
 * linear-space sweep underflowed (SURVEY.md §8 A6-A10 for iohmm-reg,
 * iohmm-mix, iohmm-hmix, iohmm-hmix-lite at any K <= 32).
 *
 * The IOHMM sweeps (hhmm_iohmm.h iohmm_sweep / iohmm_sp_sweep, hhmm_lkio.h
 * lkio_kernel) run the reference's forward recursion in linear space,
 * f_t = e_t * s_t with s_t = sum_i f_{t-1}(i) A_t(i) and e_t = exp(oblik_t - max).
 * Where the softmax transitions saturate, A_t is 0 in double on every state the
 * renormalised filter holds while the states whose emission factor underflowed
 * carry the mass: s_t becomes 0 and the loglik -inf, whereas the reference's
 * log-space recursion (iohmm-reg/stan/iohmm-reg.stan:59-78, iohmm-mix.stan:67-87,
 * iohmm-hmix.stan:64-83, iohmm-hmix-lite.stan:60-76) keeps every state finite.
 * The sweeps therefore check, per step, that s_t (and max f_0, and the backward
 * accumulator c_t = sum_i A_t(i) e_t(i) where beta / gamma / unbeta are
 * requested) stays above kIoWeak = 2^-960: above it every term the linear form
 * dropped or rounded in the subnormal range is below 2^-110 of the sum, so the
 * linear outputs are within the 1e-9 tolerance.  A pair that fails appends
 * itself to a.io_redo (count, then pair ids), and this kernel recomputes its
 * filter outputs with the reference's own log-space arithmetic:
 *
 *   A_t = softmax(u_t' w_j), log A_t(i) = log(A_t(i))            (:40-49, :70)
 *   unalpha[1, j] = log(p_1k[j]) + oblik[1][j]                    (:62-63)
 *   unalpha[t, j] = log_sum_exp_i((unalpha[t-1, i] + log A_t(i)) + oblik[t][j])  (:65-74)
 *   alpha = softmax(unalpha), loglik = log_sum_exp(unalpha[T])    (:76-77, :120)
 *   unbeta[T] = 1; unbeta[t-1] = unbeta[t] + log_sum_exp_i(log A_t(i) + oblik[t][i])
 *                                                                  (:80-98, Q1, Q5)
 *   beta = softmax(unbeta) (1/K, NaN where unbeta is -inf), gamma = normalize(alpha .* beta)
 *   oblik_t = log_sum_exp(log(alpha_t) + oblik_t)                 (iohmm-hmix.stan:118-121)
 *
 * in Stan Math's operation order (log_sum_exp: max by '>', the sum of
 * exp(x - max) over x != -inf, max + log(sum); the oracle's stan_log_sum_exp),
 * K^2 exps per step.  The Viterbi, oblik_tk, A_ij / logA_ij and the FFBS draws
 * are not filter outputs and are left as the sweep wrote them.  One lane per
 * listed pair (grid-stride over the list); in a batch without underflow the
 * list is empty and the launch reads one word.
 */
#include "hhmm_iohmm.h"

namespace hhmm {

namespace {

constexpr int kLogMmax = 8;

/* Stan Math log_sum_exp over the first K entries (oracle stan_log_sum_exp). */
template <int KM>
__device__ __forceinline__ double lse_rt(const double (&v)[KM], int K)
{
    double mx = dev_ninf();
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K && v[i] > mx)
            mx = v[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K && v[i] != dev_ninf())
            sum += exp(v[i] - mx);
    return mx + log(sum);
}

/* softmax(v) over the first K entries, the numerators in place (oracle stan_softmax). */
template <int KM>
__device__ __forceinline__ void softmax_rt(double (&v)[KM], int K)
{
    double mx = v[0];
#pragma unroll
    for (int i = 1; i < KM; ++i)
        if (i < K && v[i] > mx)
            mx = v[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K) {
            v[i] = exp(v[i] - mx);
            sum += v[i];
        }
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K)
            v[i] = v[i] / sum;
}

/* Row k of a draw-major [S, K, M] regressor array (w_km, b_km), zero-padded. */
__device__ __forceinline__ void io_row(const double *arr, const DevArgs &a, int64_t d, int k,
                                       double (&r)[kLogMmax])
{
#pragma unroll
    for (int m = 0; m < kLogMmax; ++m)
        r[m] = (m < a.M) ? arr[d + a.S * ((int64_t)k + (int64_t)a.K * m)] : 0.0;
}

/* oblik_t(k): regression normal_lpdf(x | u' b_k, s_k) (iohmm-reg.stan:51-57) or the
 * mixture log_sum_exp_l(log lambda_kl + normal_lpdf(x | mu_kl, s_kl)) (iohmm-mix.stan:53-65),
 * io_emission's arithmetic for one state with libm. */
template <int FAM>
__device__ __forceinline__ double io_oblik(const DevArgs &a, int64_t d, int k, double x, const double (&u)[kLogMmax])
{
    if constexpr (FAM == IO_REG) {
        double br[kLogMmax];
        io_row(a.b_km, a, d, k, br);
        const double mu = sse_dot<kLogMmax>(u, br, a.M);
        const double s = a.s_k[d + a.S * k];
        const double z = (x - mu) * (1.0 / s);
        const double z2 = z * z;
        return (HHMM_NEG_LOG_SQRT_TWO_PI - log(s)) + (-0.5 * z2);
    } else {
        double acc[kIoLmax];
        double mx = dev_ninf();
#pragma unroll
        for (int l = 0; l < kIoLmax; ++l) {
            acc[l] = dev_ninf();
            if (l < a.L) {
                const int64_t ix = d + a.S * ((int64_t)k + (int64_t)a.K * l);
                const double s = a.s_kl[ix];
                const double z = (x - a.mu_kl[ix]) * (1.0 / s);
                const double z2 = z * z;
                acc[l] = log(a.lambda_kl[ix]) + ((HHMM_NEG_LOG_SQRT_TWO_PI - log(s)) + (-0.5 * z2));
                if (acc[l] > mx)
                    mx = acc[l];
            }
        }
        double sum = 0.0;
#pragma unroll
        for (int l = 0; l < kIoLmax; ++l)
            if (l < a.L && acc[l] != dev_ninf())
                sum += exp(acc[l] - mx);
        return mx + log(sum);
    }
}

/* One listed pair: the filter outputs in log space, written over the sweep's. */
template <int FAM, int KM>
__device__ void iohmm_log_pair(const DevArgs &a, int64_t p)
{
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int K = a.K;
    const uint32_t out = a.outputs;
    const uint32_t po = (uint32_t)p;
    double ua[KM], la[KM], ob[KM], nu[KM];
    double u[kLogMmax];
    int tneg = 0; /* unbeta is -inf / NaN (beta and gamma NaN) at t < tneg */
    auto put_k = [&](double *arr, int t, int k, double v) {
        if (arr)
            put_out(arr + a.P * ((int64_t)t + (int64_t)a.Tout * k), po * 8u, v);
    };
    for (int t = 0; t < Tp; ++t) {
        const double x = a.xr[n + a.N * (int64_t)t];
#pragma unroll
        for (int m = 0; m < kLogMmax; ++m)
            u[m] = (m < a.M) ? a.u[n + a.N * ((int64_t)t + (int64_t)a.Tmax * m)] : 0.0;
#pragma unroll
        for (int k = 0; k < KM; ++k)
            if (k < K)
                ob[k] = io_oblik<FAM>(a, d, k, x, u);
        if (t == 0) {
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    ua[k] = log(a.p_1k[d + a.S * k]) + ob[k];
        } else {
            /* log A_t = log(softmax(u_t' w_j)) */
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K) {
                    double wr[kLogMmax];
                    io_row(a.w_km, a, d, k, wr);
                    la[k] = sse_dot<kLogMmax>(u, wr, a.M);
                }
            softmax_rt<KM>(la, K);
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    la[k] = log(la[k]);
            /* unalpha[t, j] = LSE_i((unalpha[t-1, i] + log A_t(i)) + oblik[t][j]) */
#pragma unroll
            for (int j = 0; j < KM; ++j) {
                if (j < K) { /* lse_rt over acc[i] = (ua[i] + la[i]) + ob[j], formed twice */
                    double mx = dev_ninf();
#pragma unroll
                    for (int i = 0; i < KM; ++i)
                        if (i < K && (ua[i] + la[i]) + ob[j] > mx)
                            mx = (ua[i] + la[i]) + ob[j];
                    double sum = 0.0;
#pragma unroll
                    for (int i = 0; i < KM; ++i)
                        if (i < K && (ua[i] + la[i]) + ob[j] != dev_ninf())
                            sum += exp(((ua[i] + la[i]) + ob[j]) - mx);
                    nu[j] = mx + log(sum);
                }
            }
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    ua[k] = nu[k];
            /* the backward accumulator of step t: LSE_i(log A_t(i) + oblik[t][i]) */
#pragma unroll
            for (int k = 0; k < KM; ++k)
                nu[k] = (k < K) ? la[k] + ob[k] : dev_ninf();
            const double dt = lse_rt<KM>(nu, K);
            if (!(dt > dev_ninf()))
                tneg = t;
            if ((out & HHMM_OUT_UNBETA) && a.lam)
                at(a.lam + a.P * (int64_t)t, po * 8u) = dt;
        }
        if ((out & HHMM_OUT_UNALPHA) && a.unalpha)
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    put_k(a.unalpha, t, k, ua[k]);
        /* alpha = softmax(unalpha) */
#pragma unroll
        for (int k = 0; k < KM; ++k)
            nu[k] = ua[k];
        softmax_rt<KM>(nu, K);
        if ((out & HHMM_OUT_ALPHA) && a.alpha)
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    put_k(a.alpha, t, k, nu[k]);
        if ((out & (HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA | HHMM_OUT_BETA))) {
            /* beta = 1/K where unbeta is finite (the NaN rows are patched below);
             * ungamma = alpha .* beta; gamma = ungamma / sum(ungamma) */
            const double bk = 1.0 / K;
            double sg = 0.0;
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    sg += nu[k] * bk;
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K) {
                    if ((out & HHMM_OUT_BETA))
                        put_k(a.beta, t, k, bk);
                    if ((out & HHMM_OUT_UNGAMMA))
                        put_k(a.ungamma, t, k, nu[k] * bk);
                    if ((out & HHMM_OUT_GAMMA))
                        put_k(a.gamma, t, k, (nu[k] * bk) / sg);
                }
        }
        if ((out & HHMM_OUT_OBLIK_T) && a.oblik_t) {
            /* oblik_t = log_sum_exp(log(alpha_t) + oblik_t) */
#pragma unroll
            for (int k = 0; k < KM; ++k)
                nu[k] = (k < K) ? log(nu[k]) + ob[k] : dev_ninf();
            at(a.oblik_t + a.P * (int64_t)t, po * 8u) = lse_rt<KM>(nu, K);
        }
    }
    if ((out & HHMM_OUT_LOGLIK) && a.loglik)
        a.loglik[p] = lse_rt<KM>(ua, K);
    if ((out & HHMM_OUT_UNBETA) && a.unbeta && a.lam) {
        /* unbeta[T] = 1 (Q1); unbeta[t-1] = unbeta[t] + d_t, the same for every j (Q5) */
        double B = 1.0;
        for (int t = Tp - 1; t >= 0; --t) {
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < K)
                    put_k(a.unbeta, t, k, B);
            if (t > 0)
                B = B + at(a.lam + a.P * (int64_t)t, po * 8u);
        }
    }
    /* softmax of an all -inf (or NaN) unbeta row is NaN: beta, ungamma, gamma */
    for (int t = 0; t < tneg; ++t)
#pragma unroll
        for (int k = 0; k < KM; ++k)
            if (k < K) {
                if (out & HHMM_OUT_BETA)
                    put_k(a.beta, t, k, dev_nan());
                if (out & HHMM_OUT_UNGAMMA)
                    put_k(a.ungamma, t, k, dev_nan());
                if (out & HHMM_OUT_GAMMA)
                    put_k(a.gamma, t, k, dev_nan());
            }
}

template <int FAM, int KM>
__global__ void __launch_bounds__(64) iohmm_log_kernel(const DevArgs a)
{
    const int64_t cnt = a.io_redo[0];
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < cnt; q += (int64_t)gridDim.x * blockDim.x)
        iohmm_log_pair<FAM, KM>(a, a.io_redo[1 + q]);
}

template <int FAM>
void launch_log_fam(const DevArgs &a, hipStream_t st, dim3 grid)
{
    if (a.K <= 8)
        hipLaunchKernelGGL((iohmm_log_kernel<FAM, 8>), grid, dim3(64), 0, st, a);
    else if (a.K <= 16)
        hipLaunchKernelGGL((iohmm_log_kernel<FAM, 16>), grid, dim3(64), 0, st, a);
    else
        hipLaunchKernelGGL((iohmm_log_kernel<FAM, kMaxKLarge>), grid, dim3(64), 0, st, a);
}

} // namespace

hhmm_status launch_iohmm_log(const DevArgs &a, hipStream_t st)
{
    if (!a.io_redo || !(a.outputs & kIoFilt))
        return HHMM_OK;
    if (a.K > kMaxKLarge || a.M > kLogMmax || (a.model != HHMM_MODEL_IOHMM_REG && a.L > kIoLmax)) {
        set_error("IOHMM log-space fallback: K = %d, M = %d, L = %d out of range", a.K, a.M, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    /* up to 1024 one-wave workgroups; each lane walks the list with a grid stride */
    const int64_t waves = (a.P + 63) / 64;
    const dim3 grid((unsigned)(waves < 1024 ? waves : 1024));
    if (a.model == HHMM_MODEL_IOHMM_REG)
        launch_log_fam<IO_REG>(a, st, grid);
    else
        launch_log_fam<IO_MIX>(a, st, grid);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("iohmm_log_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

} // namespace hhmm
