/*
 * hhmm_lkio.h -- the IOHMM programs at large K (8 < K <= 32): iohmm-reg,
 * iohmm-mix, iohmm-hmix, iohmm-hmix-lite with free `int<lower=1> K`
 * (iohmm-reg/stan/iohmm-reg.stan:9, iohmm-mix/stan/iohmm-hmix.stan:7).
 *
 * Layout as hhmm_large.h: a GROUP of G lanes owns one (series, draw) pair,
 * lane j state j (lanes j >= K idle; G = 16 up to K = 16, 32 above).  Lane j
 * keeps state j's parameters in registers (w_j, b_j, s_j; the mixture rows of
 * state j sit in the group's LDS block) and computes everything that belongs
 * to state j in the reference's own operation order:
 *   v_j = u_t' w_j        (Eigen's SSE2 dot order, sse_dot)
 *   oblik_t(j)            (normal_lpdf / the mixture log_sum_exp, io_emission's
 *                          arithmetic for one state)
 * The softmax over states (iohmm-reg.stan:40-49) needs the group's vector: the
 * lanes exchange v and then the numerators through a per-group LDS slot, and
 * every lane forms the max by the strict '>' scan and the SEQUENTIAL sum in
 * state order exactly as stan_softmax does, so A_t(j) and log A_t(j) are the
 * lane kernel's doubles.  The Viterbi candidate (delta_{t-1}(i) + log A_t(i))
 * + oblik_t(j) is the lane kernel's: lane i contributes delta(i) + log A(i),
 * lane j scans the K of them with strict '>' (first i wins), so paths and
 * logp_zstar are bit-exact with the oracle.
 *
 * The IOHMM "transition" is a K-vector, so the forward
 * step is f_t(j) = e_t(j) * s_t with ONE group sum s_t = sum_i f_{t-1}(i) A_t(i),
 * and beta is 1/K exactly (hhmm_iohmm.h header): one forward sweep produces
 * loglik, alpha, beta, ungamma, gamma, unalpha, oblik_tk, oblik_t, A_ij /
 * logA_ij and the Viterbi; unbeta adds a second pass over the stored log c_t.
 * Back-pointers and the backtrack are lk_viterbi_kernel's ([P][T_b/16][K][16]
 * bytes, one 16-byte store per lane and block).  FFBS (IO_DET, its own sweep):
 * the transition does not depend on the next state, so each draw z_{t-1} =
 * cat(v_{t-1} .* th_t, u_{t-1}) is formed in the forward sweep from the
 * exchanged weights.  The fitted-output draws (hatpi / hatz /
 * hatl / hatx) run in lkfit_kernel below, the same group layout.
 */
#pragma once
#include <hip/hip_runtime.h>

#include "hhmm_large.h"
#include "hhmm_iohmm.h"

namespace hhmm {

constexpr int kLkioMmax = 8; /* inputs per step on the device path (as the lane kernels' MMAX) */

/* ffbs_cat over the first K entries of a KM-capacity vector (the same
 * sequential sum and running-sum comparison; -1 when the sum is not a
 * positive finite number) */
template <int KM>
__device__ __forceinline__ int lkio_cat(const double (&w)[KM], int K, double u)
{
    double sum = w[0];
#pragma unroll
    for (int i = 1; i < KM; ++i)
        if (i < K)
            sum = sum + w[i];
    const double us = u * sum;
    int b = 0;
    double cum = w[0];
#pragma unroll
    for (int i = 1; i < KM; ++i) {
        if (i < K) {
            const bool step = (b == i - 1) & (us > cum);
            b = step ? i : b;
            cum = step ? cum + w[i] : cum;
        }
    }
    return ((sum > 0.0) & __builtin_isfinite(sum)) ? b : -1;
}

template <int FAM, int G, int KM, int MATH>
__global__ void __launch_bounds__(kBlock) lkio_kernel(const DevArgs a)
{
    constexpr int MMAX = kLkioMmax;
    HIP_DYNAMIC_SHARED(double, lds)
    const int tid = threadIdx.x;
    const int g = tid / G, gpb = blockDim.x / G;
    const int j = tid % G;
    const int K = a.K, M = a.M, L = a.L;
    const bool on = j < K;
    const int jj = on ? j : 0;
    const int64_t p = lk_group<G>(a.P);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int64_t S = a.S;
    const uint32_t out = a.outputs;
    const bool want_vit = MATH == IO_CR && (out & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR));
    const bool fixed_init = (a.model == HHMM_MODEL_IOHMM_HMIX); /* iohmm-hmix.stan:166-167 */
    const bool log_A_out = (a.model == HHMM_MODEL_IOHMM_HMIX || a.model == HHMM_MODEL_IOHMM_HMIX_LITE);
    const bool need_lA = want_vit || (log_A_out && (out & HHMM_OUT_LOGA) && a.logA);
    const bool gate = (out & kIoFilt) && a.io_redo; /* iohmm_sweep's underflow check (group-uniform) */
    bool weak = false;

    /* ---- state jj's parameters ---- */
    const double pj = a.p_1k[d + S * jj];
    double w[MMAX], b[MMAX];
#pragma unroll
    for (int m = 0; m < MMAX; ++m) {
        w[m] = (m < M) ? a.w_km[d + S * ((int64_t)jj + (int64_t)K * m)] : 0.0;
        b[m] = (FAM == IO_REG && m < M) ? a.b_km[d + S * ((int64_t)jj + (int64_t)K * m)] : 0.0;
    }
    double isig = 0.0, c0 = 0.0;
    if constexpr (FAM == IO_REG) {
        const double s = a.s_k[d + S * jj];
        isig = 1.0 / s;
        c0 = HHMM_NEG_LOG_SQRT_TWO_PI - io_log<MATH>(s);
    }
    /* LDS: [groups][3][G] exchange slots, then [groups][L][4][G] mixture rows
     * (mu, 1/s, log lambda, C - log s) */
    double *xch = lds + (size_t)g * 3 * G;
    double *mix = lds + (size_t)gpb * 3 * G + (size_t)g * L * 4 * G;
    if constexpr (FAM == IO_MIX) {
        for (int l = 0; l < L; ++l) { /* loglambda_kl = log(lambda_kl) (iohmm-mix.stan:55) */
            const int64_t ix = d + S * ((int64_t)jj + (int64_t)K * l);
            const double s = a.s_kl[ix];
            mix[(l * 4 + 0) * G + j] = a.mu_kl[ix];
            mix[(l * 4 + 1) * G + j] = 1.0 / s;
            mix[(l * 4 + 2) * G + j] = io_log<MATH>(a.lambda_kl[ix]);
            mix[(l * 4 + 3) * G + j] = HHMM_NEG_LOG_SQRT_TWO_PI - io_log<MATH>(s);
        }
    }
    /* IO_DET: the contract exp's table in LDS after the mixture rows (io_stage_exp2) */
    const hhmm_exp2_entry *etab =
        io_stage_exp2<MATH>(lds + (size_t)gpb * 3 * G + (FAM == IO_MIX ? (size_t)gpb * L * 4 * G : 0));
    __syncthreads();

    /* oblik_t(j): reg normal_lpdf(x | u' b_j, s_j) (iohmm-reg.stan:51-57); mix
     * LSE_l(log lambda_jl + normal_lpdf(x | mu_jl, s_jl)) (iohmm-mix.stan:53-65) */
    auto emission = [&](double x, const double (&u)[MMAX]) -> double {
        if constexpr (FAM == IO_REG) {
            const double mu = sse_dot<MMAX>(u, b, M);
            const double z = (x - mu) * isig;
            const double z2 = z * z;
            return c0 + (-0.5 * z2);
        } else {
            double acc[kIoLmax];
            double mx = dev_ninf();
#pragma unroll
            for (int l = 0; l < kIoLmax; ++l) {
                acc[l] = dev_ninf();
                if (l < L) {
                    const double z = (x - mix[(l * 4 + 0) * G + j]) * mix[(l * 4 + 1) * G + j];
                    const double z2 = z * z;
                    acc[l] = mix[(l * 4 + 2) * G + j] + (mix[(l * 4 + 3) * G + j] + (-0.5 * z2));
                    if (acc[l] > mx)
                        mx = acc[l];
                }
            }
            double sum = 0.0;
#pragma unroll
            for (int l = 0; l < kIoLmax; ++l)
                if (l < L && acc[l] != dev_ninf())
                    sum += io_exp<MATH>(acc[l] - mx, etab);
            return mx + io_log<MATH>(sum);
        }
    };
    auto load = [&](int t, double &x, double (&u)[MMAX]) {
        const int tc = min(max(t, 0), a.Tmax - 1);
        x = a.xr[n + a.N * (int64_t)tc];
#pragma unroll
        for (int m = 0; m < MMAX; ++m)
            u[m] = (m < M) ? a.u[n + a.N * ((int64_t)tc + (int64_t)a.Tmax * m)] : 0.0;
    };
    auto put = [&](double *arr, int t, double v) {
        if (on && arr)
            arr[p + a.P * ((int64_t)t + (int64_t)a.Tout * j)] = v;
    };

    /* back-pointers [P][NB][K][16] bytes (lk_viterbi_kernel's layout) */
    const int Tb = lk_row_bytes(a.Tmax), NB = Tb / kLBack;
    uint8_t *bpb = reinterpret_cast<uint8_t *>(a.bp) + (int64_t)p * NB * K * kLBack;
    auto bp_at = [&](int blk) { return bpb + ((int64_t)blk * K + jj) * kLBack; };

    double f = 0.0, lsc = 0.0, lam = 0.0;
    int ex = 0;
    double dl = dev_ninf();
    uint32_t wd0 = 0u, wd1 = 0u, wd2 = 0u, wd3 = 0u;
    double vx[KM];
    double x, xn, u[MMAX], un[MMAX];
    double vprev = 0.0, uprev = 0.5; /* FFBS (IO_DET): v_{t-1}, the uniform of step t - 1 */
    load(0, x, u);
    const int Tw = wave_max(Tp);
#pragma unroll 1
    for (int t = 0; t < Tw; ++t) {
        load(t + 1, xn, un);
        if constexpr (MATH == IO_DET) {
            /* FFBS (oracle ffbs_contract): the K-vector transition
             * does not depend on the next state, so z_{t-1} = cat(v_{t-1} .* th_t,
             * u_{t-1}) with v the contract's emission factor (p .* e_0 at t = 0)
             * and th_t the softmax numerators -- iohmm_sweep's IO_DET arithmetic */
            if (t < Tp) {
                double e;
                if constexpr (FAM == IO_REG) {
                    const double o = on ? emission(x, u) : dev_ninf();
                    double m = grp_max<G>(o);
                    if (m == dev_ninf())
                        m = 0.0;
                    e = on ? hhmm_det_exp_tab(o - m, etab) : 0.0;
                } else { /* io_mix_factor: the largest summand over every state and component */
                    double acc[kIoLmax];
                    double mx = dev_ninf();
#pragma unroll
                    for (int l = 0; l < kIoLmax; ++l) {
                        acc[l] = dev_ninf();
                        if (l < L) {
                            const double z = (x - mix[(l * 4 + 0) * G + j]) * mix[(l * 4 + 1) * G + j];
                            const double z2 = z * z;
                            acc[l] = mix[(l * 4 + 2) * G + j] + (mix[(l * 4 + 3) * G + j] + (-0.5 * z2));
                            if (acc[l] > mx)
                                mx = acc[l];
                        }
                    }
                    double mm = grp_max<G>(on ? mx : dev_ninf());
                    if (mm == dev_ninf())
                        mm = 0.0;
                    double sum = 0.0;
#pragma unroll
                    for (int l = 0; l < kIoLmax; ++l)
                        if (l < L && acc[l] != dev_ninf())
                            sum += hhmm_det_exp_tab(acc[l] - mm, etab);
                    e = on ? sum : 0.0;
                }
                if (t == 0) {
                    vprev = on ? pj * e : 0.0;
                } else {
                    const double v = on ? sse_dot<MMAX>(u, w, M) : 0.0;
                    grp_exchange<G, KM>(xch, 0, j, v, vx);
                    double mx = vx[0];
#pragma unroll
                    for (int i = 1; i < KM; ++i)
                        if (i < K && vx[i] > mx)
                            mx = vx[i];
                    const double th = on ? hhmm_det_exp_tab(v - mx, etab) : 0.0;
                    grp_exchange<G, KM>(xch, 1, j, vprev * th, vx);
                    const int z = lkio_cat<KM>(vx, K, uprev);
                    if (j == 0)
                        a.z_ffbs[p + a.P * (int64_t)(t - 1)] = z + 1;
                    vprev = on ? e : 0.0;
                }
                uprev = a.ffbs_u[p + a.P * (int64_t)t];
            }
            x = xn;
#pragma unroll
            for (int m2 = 0; m2 < MMAX; ++m2)
                u[m2] = un[m2];
            continue;
        }
        if (t < Tp) { /* group-uniform */
            const double o = on ? emission(x, u) : dev_ninf();
            double A, lA = 0.0;
            if (t == 0) {
                /* A_ij[1] = p_1k (iohmm-reg.stan:41-42); logA_ij[1] = log(p_1k) (iohmm-hmix.stan:40) */
                A = pj;
                if (log_A_out)
                    lA = io_log<MATH>(pj);
            } else {
                /* A_t = softmax(u_t' w_j) (iohmm-reg.stan:43-48): max by the strict '>'
                 * scan, numerators, sequential sum, quotient -- stan_softmax per state */
                const double v = on ? sse_dot<MMAX>(u, w, M) : 0.0;
                grp_exchange<G, KM>(xch, 0, j, v, vx);
                double mx = vx[0];
#pragma unroll
                for (int i = 1; i < KM; ++i)
                    if (i < K && vx[i] > mx)
                        mx = vx[i];
                const double num = on ? io_exp<MATH>(v - mx, etab) : 0.0;
                grp_exchange<G, KM>(xch, 1, j, num, vx);
                double sum = 0.0;
#pragma unroll
                for (int i = 0; i < KM; ++i)
                    if (i < K)
                        sum += vx[i];
                A = num / sum;
                if (need_lA)
                    lA = io_log<MATH>(A);
            }
            if (out & HHMM_OUT_OBLIK_TK)
                put(a.oblik, t, o);
            if (out & HHMM_OUT_LOGA)
                put(a.logA, t, log_A_out ? lA : A);

            /* forward (iohmm-reg.stan:59-78): f_t(j) = e_t(j) * sum_i f_{t-1}(i) A_t(i) */
            double m = grp_max<G>(o);
            if (m == dev_ninf())
                m = 0.0; /* every emission impossible: f_t = 0, alpha = NaN as in Stan */
            const double e = on ? exp(o - m) : 0.0;
            double ua_base = 0.0, fj;
            if (t == 0) {
                fj = on ? pj * e : 0.0;
                weak = gate && !(grp_max<G>(fj) >= kIoWeak0);
            } else {
                const double s = grp_sum<G>(on ? f * A : 0.0);
                ua_base = log(s) + (lsc + kLn2 * ex);
                weak |= gate && !(s >= kIoWeak);
                const int es = __builtin_amdgcn_frexp_exp(s); /* iohmm_sweep: s into [0.5, 1) first */
                ex += es;
                fj = e * ldexp(s, -es);
                if (out & kIoBack) { /* log c_t = m + log sum_i A_t(i) e_t(i) (:94) */
                    const double c = grp_sum<G>(on ? A * e : 0.0);
                    weak |= gate && !(c >= kIoWeak);
                    if (out & HHMM_OUT_UNBETA) {
                        lam += m + log(c);
                        if (j == 0)
                            a.lam[p + a.P * (int64_t)t] = lam;
                    }
                }
            }
            lsc += m;
            f = grp_renorm<G>(fj, ex);
            const double rfs = fast_rcp(grp_sum<G>(f));
            const double al = f * rfs;
            if (out & HHMM_OUT_ALPHA)
                put(a.alpha, t, al);
            if (out & HHMM_OUT_GAMMA) /* gamma = normalize(alpha .* 1/K) = alpha */
                put(a.gamma, t, al);
            if (out & HHMM_OUT_UNGAMMA)
                put(a.ungamma, t, al * (1.0 / K));
            if (out & HHMM_OUT_BETA) /* softmax of a repeated scalar */
                put(a.beta, t, 1.0 / K);
            if (out & HHMM_OUT_UNALPHA) /* t = 0: log(p_1k[j]) + oblik (:62-63); else oblik + log s_t + scale */
                put(a.unalpha, t, (t == 0) ? log(pj) + o : o + ua_base);
            if ((out & HHMM_OUT_OBLIK_T) && a.oblik_t) {
                /* oblik_t = LSE(log(alpha_t) + oblik_t) (iohmm-hmix.stan:118-121) */
                const double num = grp_sum<G>(on ? f * e : 0.0);
                if (j == 0)
                    a.oblik_t[p + a.P * (int64_t)t] = m + log(num * rfs);
            }

            /* Viterbi (iohmm-reg.stan:150-181; iohmm-mix.stan:164-195; iohmm-hmix.stan:160-193) */
            if (want_vit) {
                if (t == 0) {
                    /* delta_tk[1, K] = oblik_tk[1][j] for j = 1..K (Q3); hmix: every j */
                    dl = !on ? dev_ninf() : ((fixed_init || j == K - 1) ? o : dev_nan());
                } else {
                    grp_exchange<G, KM>(xch, 2, j, on ? dl + lA : dev_ninf(), vx);
                    double best = dev_ninf();
                    int arg = 0;
#pragma unroll
                    for (int i = 0; i < KM; ++i) { /* idle i: -inf, never greater */
                        const double cand = vx[i] + o;
                        const bool gt = cand > best;
                        best = fmax(best, cand);
                        arg = gt ? i : arg;
                    }
                    dl = on ? best : dev_ninf();
                    const int v = t % kLBack;
                    const uint32_t bits = (uint32_t)arg << (8 * (v & 3));
                    wd0 |= (v >> 2) == 0 ? bits : 0u;
                    wd1 |= (v >> 2) == 1 ? bits : 0u;
                    wd2 |= (v >> 2) == 2 ? bits : 0u;
                    wd3 |= (v >> 2) == 3 ? bits : 0u;
                }
                if (t % kLBack == kLBack - 1 || t == Tp - 1) {
                    if (on)
                        *reinterpret_cast<uint4 *>(bp_at(t / kLBack)) = make_uint4(wd0, wd1, wd2, wd3);
                    wd0 = wd1 = wd2 = wd3 = 0u;
                }
            }
        }
        x = xn;
#pragma unroll
        for (int m2 = 0; m2 < MMAX; ++m2)
            u[m2] = un[m2];
    }
    if constexpr (MATH == IO_DET) { /* z_{T-1} = cat(v_{T-1}, u_{T-1}) */
        grp_exchange<G, KM>(xch, 2, j, vprev, vx);
        const int z = lkio_cat<KM>(vx, K, uprev);
        if (j == 0)
            a.z_ffbs[p + a.P * (int64_t)(Tp - 1)] = z + 1;
        return;
    }
    if (weak && j == 0 && lk_group_raw<G>() < a.P)
        a.io_redo[1 + atomicAdd(&a.io_redo[0], 1)] = (int32_t)p; /* re-run in log space (launch_iohmm_log) */
    if ((out & HHMM_OUT_LOGLIK) && a.loglik) { /* target += log_sum_exp(unalpha_tk[T]) (iohmm-reg.stan:120) */
        const double fs = grp_sum<G>(f);
        if (j == 0)
            a.loglik[p] = log(fs) + (lsc + kLn2 * ex);
    }
    if ((out & HHMM_OUT_UNBETA) && a.unbeta) { /* B_T = 1 (Q1); B_t = 1 + (Lambda_T - Lambda_t) (:80-98) */
        for (int t = 0; t < Tp; ++t) {
            const double lt = (t == 0) ? 0.0 : a.lam[p + a.P * (int64_t)t];
            put(a.unbeta, t, 1.0 + (lam - lt));
        }
    }
    if (!want_vit)
        return;

    /* logp_zstar = max(delta_T) (SSE2 order); zstar_T = LAST j attaining it */
    grp_exchange<G, KM>(xch, 0, j, dl, vx);
    const double lp = stan_max_rt<KM>(vx, K);
    int z = -1;
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K && vx[i] == lp)
            z = i;
    const bool invalid = (z < 0) || (Tp >= 2 && lp == dev_ninf());
    if (j == 0) {
        if ((out & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
            a.logp_zstar[p] = lp;
        if (a.pair_status)
            a.pair_status[p] = invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
    }
    if (!((out & HHMM_OUT_ZSTAR) && a.zstar))
        return;
    if (invalid) {
        for (int t = j; t < Tp; t += G)
            a.zstar[p + a.P * (int64_t)t] = 0;
        return;
    }
    /* backtrack (lk_viterbi_kernel's) */
    const int nb = (Tp + kLBack - 1) / kLBack;
    auto ld = [&](int c) -> uint4 {
        const int cc = min(max(c, 0), NB - 1);
        return *reinterpret_cast<const uint4 *>(bp_at(cc));
    };
    uint4 q0 = ld(nb - 1), q1 = ld(nb - 2);
    for (int c = nb - 1; c >= 0; --c) {
        const uint4 q2 = ld(c - 2);
        const uint32_t wq[4] = {q0.x, q0.y, q0.z, q0.w};
        int mine = 0;
#pragma unroll
        for (int u2 = kLBack - 1; u2 >= 0; --u2) {
            const int t = c * kLBack + u2;
            if (t < Tp) {
                if ((j & (kLBack - 1)) == u2)
                    mine = z + 1;
                if (t > 0)
                    z = __shfl((int)((wq[u2 >> 2] >> (8 * (u2 & 3))) & 0xffu), z, G);
            }
        }
        const int t = c * kLBack + (j & (kLBack - 1));
        if (j < kLBack && t < Tp)
            a.zstar[p + a.P * (int64_t)t] = mine;
        q0 = q1;
        q1 = q2;
    }
}

template <int FAM, int G, int KM>
static hhmm_status launch_lkio_g(const DevArgs &a, hipStream_t st)
{
    const int gpb = kBlock / G;
    const size_t lds = ((size_t)gpb * 3 * G + (FAM == IO_MIX ? (size_t)gpb * a.L * 4 * G : 0)) * sizeof(double);
    const size_t tab = 128 * sizeof(hhmm_exp2_entry); /* the IO_DET launch's io_stage_exp2 copy */
    if (lds + tab > kLdsLimit) {
        set_error("large-K IOHMM: mixture table L = %d does not fit in LDS", a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const dim3 grid((unsigned)((a.P + gpb - 1) / gpb));
    if (a.outputs & HHMM_OUT_FFBS) { /* the draws in their own sweep (the contract's arithmetic) */
        DevArgs f = a;
        f.outputs = HHMM_OUT_FFBS;
        hipLaunchKernelGGL((lkio_kernel<FAM, G, KM, IO_DET>), grid, dim3(kBlock), lds + tab, st, f);
    }
    DevArgs b = a;
    b.outputs &= ~HHMM_OUT_FFBS;
    const bool vit = (b.outputs & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR)) != 0;
    if (vit)
        hipLaunchKernelGGL((lkio_kernel<FAM, G, KM, IO_CR>), grid, dim3(kBlock), lds, st, b);
    else if (b.outputs)
        hipLaunchKernelGGL((lkio_kernel<FAM, G, KM, IO_LIBM>), grid, dim3(kBlock), lds, st, b);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("lkio_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

template <int FAM>
static hhmm_status launch_lkio(const DevArgs &a, hipStream_t st)
{
    constexpr uint32_t kHat = HHMM_OUT_HATPI | HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX;
    if (a.outputs & kHat) { /* launch_all hands the fitted draws to launch_fitted */
        set_error("internal: lkio_kernel got fitted-output bits");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (a.M > kLkioMmax || (FAM == IO_MIX && a.L > kIoLmax)) {
        set_error("large-K IOHMM: M = %d (at most %d), L = %d (at most %d)", a.M, kLkioMmax, a.L, kIoLmax);
        return HHMM_ERR_UNSUPPORTED;
    }
    return a.K <= 16 ? launch_lkio_g<FAM, 16, 16>(a, st)
           : a.K <= 24 ? launch_lkio_g<FAM, 32, 24>(a, st)
                       : launch_lkio_g<FAM, 32, 32>(a, st);
}

/* ---- fitted-output draws at large K (fitted_kernel's arithmetic) ----
 * iohmm-reg.stan:131-148, iohmm-mix.stan:140-160, iohmm-hmix.stan:146-157 with
 * K free data (iohmm-reg.stan:9).  A group of G lanes per pair, lane j state j:
 *   v_j = u_t' w_j (sse_dot), exchanged through LDS; every lane forms the max
 *   by the strict '>' scan, its numerator dev_cr_exp(v_j - max), and after a
 *   second exchange the SEQUENTIAL sum in state order and th_i = num_i / sum for
 *   every i -- stan_softmax<K, IO_CR>'s doubles, so hatpi_tk and the draws
 *   match fitted_kernel and the oracle bit for bit;
 *   hatz = categorical_rng(th) with the caller's uniform (stan_categorical over
 *   the first K entries, evaluated by every lane alike);
 *   reg: hatx = z sigma + mu with mu = u_t' b_hatz (lane hatz's sse_dot) and
 *   sigma = s_hatz, both read from lane hatz; mix / hmix: hatl =
 *   categorical_rng(lambda_kl[hatz]), mu / sigma = mu_kl / s_kl[hatz][hatl]. */
template <int FAM, int G, int KM>
__global__ void __launch_bounds__(kBlock) lkfit_kernel(const DevArgs a)
{
    constexpr int MMAX = kLkioMmax;
    HIP_DYNAMIC_SHARED(double, lds)
    const int tid = threadIdx.x;
    const int g = tid / G;
    const int j = tid % G;
    const int K = a.K, M = a.M, L = a.L;
    const bool on = j < K;
    const int jj = on ? j : 0;
    const int64_t p = lk_group<G>(a.P);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int64_t S = a.S;
    const uint32_t out = a.outputs;
    double w[MMAX], b[MMAX];
#pragma unroll
    for (int m = 0; m < MMAX; ++m) {
        w[m] = (m < M) ? a.w_km[d + S * ((int64_t)jj + (int64_t)K * m)] : 0.0;
        b[m] = (FAM == IO_REG && m < M) ? a.b_km[d + S * ((int64_t)jj + (int64_t)K * m)] : 0.0;
    }
    const double sj = (FAM == IO_REG) ? a.s_k[d + S * jj] : 0.0;
    double *xch = lds + (size_t)g * 2 * G;
    const bool draw = a.hat_rand && (out & (HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX));
    const int64_t rs = a.P * (int64_t)a.Tmax;
    const int base = tid - j; /* lane of state 0 in this group (shuffle source) */
    double vx[KM];
    const int Tw = wave_max(Tp);
#pragma unroll 1
    for (int t = 0; t < Tw; ++t) {
        if (t >= Tp) /* group-uniform */
            continue;
        double u[MMAX];
#pragma unroll
        for (int m = 0; m < MMAX; ++m)
            u[m] = (m < M) ? a.u[n + a.N * ((int64_t)t + (int64_t)a.Tmax * m)] : 0.0;
        const double v = on ? sse_dot<MMAX>(u, w, M) : 0.0;
        grp_exchange<G, KM>(xch, 0, j, v, vx);
        double mx = vx[0];
#pragma unroll
        for (int i = 1; i < KM; ++i)
            if (i < K && vx[i] > mx)
                mx = vx[i];
        const double num = on ? dev_cr_exp(v - mx) : 0.0;
        grp_exchange<G, KM>(xch, 1, j, num, vx);
        double sum = 0.0;
#pragma unroll
        for (int i = 0; i < KM; ++i)
            if (i < K)
                sum += vx[i];
        if ((out & HHMM_OUT_HATPI) && a.hatpi && on)
            a.hatpi[p + a.P * ((int64_t)t + (int64_t)a.Tout * j)] = num / sum;
        if (!draw)
            continue;
        double th[KM];
#pragma unroll
        for (int i = 0; i < KM; ++i)
            th[i] = vx[i] / sum;
        const double *rnd = a.hat_rand + a.P * (int64_t)t;
        const int z = stan_categorical<KM>(th, K, rnd[p]);
        const double zn = rnd[2 * rs + p];
        double mu, sg;
        int l = 0;
        if constexpr (FAM == IO_REG) {
            const double mj = sse_dot<MMAX>(u, b, M); /* reg_tk[t] = u_tm[t]' * b_km[hatz_t[t]] on lane hatz */
            mu = __shfl(mj, base + z);
            sg = __shfl(sj, base + z);
        } else {
            double lam[kIoLmax];
#pragma unroll
            for (int q = 0; q < kIoLmax; ++q)
                lam[q] = (q < L) ? a.lambda_kl[d + S * ((int64_t)z + (int64_t)K * q)] : 0.0;
            l = stan_categorical<kIoLmax>(lam, L, rnd[rs + p]);
            const int64_t ix = d + S * ((int64_t)z + (int64_t)K * l);
            mu = a.mu_kl[ix];
            sg = a.s_kl[ix];
        }
        if (j == 0) {
            if ((out & HHMM_OUT_HATZ) && a.hatz)
                a.hatz[p + a.P * (int64_t)t] = z + 1;
            if (FAM == IO_MIX && (out & HHMM_OUT_HATL) && a.hatl)
                a.hatl[p + a.P * (int64_t)t] = l + 1;
            if ((out & HHMM_OUT_HATX) && a.hatx)
                a.hatx[p + a.P * (int64_t)t] = zn * sg + mu;
        }
    }
}

template <int FAM, int G, int KM>
static hhmm_status launch_lkfit_g(const DevArgs &a, hipStream_t st)
{
    const int gpb = kBlock / G;
    const size_t lds = (size_t)gpb * 2 * G * sizeof(double);
    const dim3 grid((unsigned)((a.P + gpb - 1) / gpb));
    hipLaunchKernelGGL((lkfit_kernel<FAM, G, KM>), grid, dim3(kBlock), lds, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("lkfit_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

template <int FAM>
static hhmm_status launch_lkfit(const DevArgs &a, hipStream_t st)
{
    if (a.M > kLkioMmax || (FAM == IO_MIX && a.L > kIoLmax)) {
        set_error("large-K fitted draws: M = %d (at most %d), L = %d (at most %d)", a.M, kLkioMmax, a.L, kIoLmax);
        return HHMM_ERR_UNSUPPORTED;
    }
    return a.K <= 16 ? launch_lkfit_g<FAM, 16, 16>(a, st)
           : a.K <= 24 ? launch_lkfit_g<FAM, 32, 24>(a, st)
                       : launch_lkfit_g<FAM, 32, 32>(a, st);
}

} // namespace hhmm
