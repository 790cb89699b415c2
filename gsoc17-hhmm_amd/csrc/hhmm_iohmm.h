/*
 * hhmm_iohmm.h -- gfx950 kernel for the input-output HMM family (templates;
 * hhmm_io_*.hip instantiate one family / K range each):
 *   iohmm-reg/stan/iohmm-reg.stan        (regression emission)
 *   iohmm-mix/stan/iohmm-mix.stan        (Gaussian-mixture emission)
 *   iohmm-mix/stan/iohmm-hmix.stan       (+ oblik_t, fixed Viterbi init)
 *   iohmm-mix/stan/iohmm-hmix-lite.stan  (forward + oblik_t only)
 * SURVEY.md §8 rows A3 (regression emission), A4 (mixture emission), A5
 * (softmax input-driven transitions), A6-A9 (forward / backward / gamma),
 * A10 (oblik_t), A11 (Viterbi), A14 (FFBS).
 *
 * Structure of the reference's IOHMM recursions: the
 * "transition" is a K-vector A_t = softmax(u_t' w_j) that depends only on the
 * step, indexed by the PREVIOUS state i in the forward pass and Viterbi
 * (iohmm-reg.stan:70,163) and by the NEXT state i in the backward pass
 * (:94).  Two consequences this kernel is built on:
 *   * forward: unalpha_t(j) = LSE_i(unalpha_{t-1}(i) + log A_t(i)) + oblik_t(j),
 *     i.e. in linear space f_t = e_t * s_t with ONE scalar s_t = sum_i f_{t-1}(i) A_t(i);
 *   * backward: the accumulator (:94) does not depend on j, so every unbeta_t
 *     row is one repeated scalar B_t, beta_t = softmax(unbeta_t) = 1/K exactly,
 *     and B_{t-1} = B_t + log c_t with c_t = sum_i A_t(i) exp(oblik_t(i)).
 * So forward, loglik, alpha, beta, gamma, oblik_t and Viterbi all come out of
 * ONE sweep over t that computes each step's transcendentals once; only the
 * unbeta output needs a second (cheap) sweep, for B_t = 1 + (Lambda_T - Lambda_t).
 *
 * One LANE = one (series, draw) pair.  Layout as hhmm_kernels.hip: every
 * per-step load/store is a coalesced wave transaction (pair-fastest), and in
 * GRID pairing the 64 lanes of a wave share one series, so x_t / u_t are
 * broadcast loads.  w_km (and b_km) live in registers; the mixture tables
 * (log lambda, mu, 1/s, NEG_LOG_SQRT_TWO_PI - log s) in a per-lane LDS slab.
 *
 * Arithmetic modes (template MATH, chosen per request by launch_io3):
 *   IO_LIBM  no bit-exact output: device libm everywhere (within the 1e-9
 *            tolerance of the float outputs);
 *   IO_CR    zstar / logp_zstar requested: every transcendental the Viterbi
 *            consumes -- the softmax exps, log A, the mixture LSE, the
 *            log(sigma) of normal_lpdf -- is the shared correctly rounded
 *            exp / log (dev_cr_exp / dev_cr_log = hhmm_cr_exp / hhmm_cr_log),
 *            in the reference's operation order (Eigen SSE2 dot order,
 *            sequential softmax sum, Stan's log_sum_exp), so paths are
 *            bit-exact with the oracle; the filter's e_t stays libm;
 *   IO_DET   FFBS draws requested: the same transcendentals, plus the
 *            filter's e_t, are the deterministic hhmm_det_exp / hhmm_det_log
 *            of the FFBS contract (cheap, no rounding test,
 *            bit-identical in the oracle; the exp's table read from an LDS
 *            copy, io_stage_exp2).
 * A request with both Viterbi and FFBS outputs runs an IO_CR sweep and an
 * IO_DET sweep (FFBS only).  log A_t is evaluated only when the Viterbi or the
 * logA_ij output consumes it.
 */
#pragma once
#include <hip/hip_runtime.h>

#include <stdio.h>

#include "hhmm_device.h"

namespace hhmm {

constexpr int kIoLmax = 8; /* mixture components per state on the device path */

enum IoFam { IO_REG = 0, IO_MIX = 1 };

enum IoMath { IO_LIBM = 0, IO_CR = 1, IO_DET = 2 };

/* tab: the FFBS contract's 2^(j/128) table (IO_DET; hhmm_det_exp_tab) -- the
 * sweeps pass their LDS copy, staged by io_stage_exp2 */
template <int MATH>
__device__ __forceinline__ double io_exp(double x, const hhmm_exp2_entry *tab = hhmm_exp2_tab)
{
    if constexpr (MATH == IO_CR)
        return dev_cr_exp(x);
    else if constexpr (MATH == IO_DET)
        return hhmm_det_exp_tab(x, tab);
    else
        return exp(x);
}
template <int MATH>
__device__ __forceinline__ double io_log(double x)
{
    if constexpr (MATH == IO_CR)
        return dev_cr_log(x);
    else if constexpr (MATH == IO_DET)
        return hhmm_det_log(x);
    else
        return log(x);
}

/* IO_DET: copy the FFBS contract exp's 2^(j/128) table (2 KB) to `dst` in LDS
 * and return it; a read of the global table would sit on the dependency chain
 * of every exp (C4's lane sweep 70.9 against 62.0 ms with the table form reading
 * it from global memory, profiles/r05i_ab_c4.log).  Other modes: the global
 * table, unread.  Every thread of the block calls it (a barrier). */
template <int MATH>
__device__ __forceinline__ const hhmm_exp2_entry *io_stage_exp2(void *dst)
{
    if constexpr (MATH == IO_DET) {
        hhmm_exp2_entry *t = reinterpret_cast<hhmm_exp2_entry *>(dst);
        for (int i = threadIdx.x; i < 128; i += blockDim.x)
            t[i] = hhmm_exp2_tab[i];
        __syncthreads();
        return t;
    } else {
        return hhmm_exp2_tab;
    }
}

/* row_vector * vector as Eigen evaluates it on x86-64 SSE2 (oracle stan_dot):
 * two 2-wide partial sums over blocks of 4, one more packet, horizontal add,
 * scalar tail.  n <= MMAX is wave-uniform (scalar branches). */
template <int MMAX>
__device__ __forceinline__ double sse_dot(const double (&a)[MMAX], const double (&b)[MMAX], int n)
{
    static_assert(MMAX >= 4 && MMAX % 4 == 0, "MMAX is 4 or 8");
    if (n < 2)
        return n == 1 ? a[0] * b[0] : 0.0;
    const int aligned = n & ~1, aligned2 = n & ~3;
    double r0a = a[0] * b[0], r0b = a[1] * b[1];
    if (aligned > 2) {
        double r1a = a[2] * b[2], r1b = a[3] * b[3];
#pragma unroll
        for (int i = 4; i + 4 <= MMAX; i += 4) {
            if (i < aligned2) {
                r0a = r0a + a[i] * b[i];
                r0b = r0b + a[i + 1] * b[i + 1];
                r1a = r1a + a[i + 2] * b[i + 2];
                r1b = r1b + a[i + 3] * b[i + 3];
            }
        }
        r0a = r0a + r1a;
        r0b = r0b + r1b;
        if (aligned > aligned2) {
#pragma unroll
            for (int q = 4; q + 2 <= MMAX; q += 4) {
                if (q == aligned2) {
                    r0a = r0a + a[q] * b[q];
                    r0b = r0b + a[q + 1] * b[q + 1];
                }
            }
        }
    }
    double res = r0a + r0b;
#pragma unroll
    for (int i = 2; i < MMAX; ++i)
        if (i >= aligned && i < n)
            res = res + a[i] * b[i];
    return res;
}

/* Stan Math categorical_rng(theta) with the caller's uniform:
 * index = cumulative_sum(theta); b = 0; while (c > index[b]) ++b (bounded to
 * n - 1: a uniform above a rounded-down total lands in the last category). */
template <int NMAX>
__device__ __forceinline__ int stan_categorical(const double (&th)[NMAX], int n, double u)
{
    int b = 0;
    double cum = th[0];
#pragma unroll
    for (int i = 1; i < NMAX; ++i) {
        if (i < n && b == i - 1 && u > cum) {
            b = i;
            cum = cum + th[i];
        }
    }
    return b;
}

/* Stan Math softmax(v): theta = exp(v - max v); theta / sequential sum.
 * num: the numerators exp(v - max v) (the FFBS contract's weights). */
template <int K, int MATH>
__device__ __forceinline__ void stan_softmax(const double (&v)[K], double (&th)[K], double (&num)[K], double &den,
                                             const hhmm_exp2_entry *tab = hhmm_exp2_tab)
{
    double mx = v[0];
#pragma unroll
    for (int i = 1; i < K; ++i)
        if (v[i] > mx)
            mx = v[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        num[i] = io_exp<MATH>(v[i] - mx, tab);
        sum += num[i];
    }
#pragma unroll
    for (int i = 0; i < K; ++i)
        th[i] = num[i] / sum;
    den = sum;
}

/* stan_softmax<K, IO_CR> together with lA[i] = dev_cr_log(A[i]) -- the same
 * doubles -- from ONE log per step instead of K:
 *   log A_i = log th_i - log(sum) + log(A_i sum / th_i),
 *   log th_i = y_i - log1p(rho_i), y_i = v_i - max v, rho_i = E.lo / E.hi where
 *     the exp's quick phase gives exp(y_i) = (E.hi + E.lo) 2^e and th_i = E.hi 2^e;
 *   A_i sum / th_i = 1 + rem_i / th_i, rem_i = fma(A_i, sum, -th_i) exact (the
 *     remainder of a rounded quotient);
 *   log(sum) as the log quick phase's double-double (relative error < 2^-72).
 * Summed in double-double, the value is within
 *   err = 2^-71 |log sum| + 2^-76 (the log and exp quick phases' bounds, the
 *   dropped second-order terms < 2^-106, the reciprocal refinements)
 * of log A_i, so where the rounding test passes the rounded head IS the
 * correctly rounded log; elsewhere (the rounding test fails, the exp took its
 * accurate phase, A_i within ~2^-18 of 1) the lane calls the full function. */
/* Always on for the correctly rounded profile.  With w / b in registers it
 * measured slower at C3 (60.95 against 58.6 ms: the sweep is capped at 256
 * registers and the extra live doubles grew its spill from 144 to 224 bytes);
 * with w / b in the LDS slab (io_wb_lds, 245 registers, no spill) it measured
 * 53.8 against 58.5 ms (tools/ab_workload.py, one box, profiles/r02zh_ab_c3.log). */
__device__ __forceinline__ double rcp_refined(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return r;
}

template <int K>
__device__ __forceinline__ void softmax_cr_log(const double (&v)[K], double (&A)[K], double (&lA)[K])
{
    double mx = v[0];
#pragma unroll
    for (int i = 1; i < K; ++i)
        if (v[i] > mx)
            mx = v[i];
    double y[K], th[K], rho[K];
    bool ok[K];
    bool all_ok = true;
    /* the K quick phases first, straight-line (independent chains that
     * interleave), then one branch for the rare lanes whose rounding test
     * failed, then the sum in order: the same doubles as calling dev_cr_exp
     * per state */
#pragma unroll
    for (int i = 0; i < K; ++i) {
        y[i] = v[i] - mx;
        /* dev_cr_exp, keeping the quick phase's low part */
        const bool in = (y[i] > -707.0) & (y[i] < 693.0); /* NaN: false */
        int e;
        const hhmm_dd f = hhmm_cr_exp_quick_dd(in ? y[i] : 0.0, &e);
        ok[i] = in & cr_fast_ok(f.hi, f.lo, kCrExpC);
        th[i] = f.hi * hhmm_bits_to_double((uint64_t)(e + 1023) << 52);
        rho[i] = f.lo * rcp_refined(f.hi);
        all_ok &= ok[i];
    }
    if (!all_ok) {
#pragma unroll
        for (int i = 0; i < K; ++i)
            if (!ok[i])
                th[i] = cr_exp_cold(y[i]);
    }
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i)
        sum += th[i];
#pragma unroll
    for (int i = 0; i < K; ++i)
        A[i] = th[i] / sum;
    /* sum >= 1 (the max term is exp(0) = 1): log(1) = 0 exactly */
    const bool one = (sum == 1.0);
    const bool sok = one | ((sum > 1.0) & (sum < 0x1p+1000));
    hhmm_dd ls = hhmm_cr_log_quick_dd((sok & !one) ? sum : 2.0);
    if (one)
        ls = hhmm_dd_make(0.0, 0.0);
    const double err = __builtin_fabs(ls.hi) * 0x1p-71 + 0x1p-76;
    bool lok[K];
    bool all_lok = true;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double rem = fma(A[i], sum, -th[i]);
        const double corr = (rem * rcp_refined(th[i]) - rho[i]) - ls.lo;
        const hhmm_dd s = hhmm_two_sum(y[i], -ls.hi);
        const hhmm_dd r = hhmm_two_sum(s.hi, s.lo + corr);
        lA[i] = r.hi;
        lok[i] = ok[i] & sok & cr_round_safe(r.hi, r.lo, err);
        all_lok &= lok[i];
    }
    if (!all_lok) {
#pragma unroll
        for (int i = 0; i < K; ++i)
            if (!lok[i])
                lA[i] = cr_log_cold(A[i]);
    }
}

template <int K, int MATH>
__device__ __forceinline__ void stan_softmax(const double (&v)[K], double (&th)[K])
{
    double num[K], den;
    stan_softmax<K, MATH>(v, th, num, den);
}

/* Per-lane mixture table entry (j, l): (mu, 1/s) and (log lambda, C - log s). */
__device__ __forceinline__ const double2 *mix_row(const double2 *slab, int L, int j, int l, int f)
{
    return slab + ((j * L + l) * 2 + f) * 64;
}

/* The regression sweep keeps w and b (2 K MMAX doubles per lane) in a per-lane
 * LDS slab instead of registers: the correctly rounded functions of the
 * Viterbi profile need the registers (two waves per SIMD, 256 of them), and
 * the slab costs 16 ds_read_b128 per step against ~1,400 VALU. */
template <int FAM>
constexpr bool io_wb_lds() { return FAM == IO_REG; }

/* Row `row` of the w / b slab (rows 0..K-1: w_j, K..2K-1: b_j). */
template <int MMAX>
__device__ __forceinline__ void wb_row(const double2 *wb, int row, double (&r)[MMAX])
{
#pragma unroll
    for (int mp = 0; mp < MMAX / 2; ++mp) {
        const double2 v = wb[(row * (MMAX / 2) + mp) * 64];
        r[2 * mp] = v.x;
        r[2 * mp + 1] = v.y;
    }
}

/* Per-lane parameters. */
template <int FAM, int K, int MMAX>
struct IoParams {
    double p[K];
    double w[K][MMAX];
    double b[FAM == IO_REG ? K : 1][MMAX];
    double isig[FAM == IO_REG ? K : 1];
    double c0[FAM == IO_REG ? K : 1];
};

/* One step's per-state quantities. */
template <int K>
struct IoStep {
    double o[K];  /* oblik_tk[t] */
    double A[K];  /* A_ij[t] (t = 0: p_1k filler) */
    double th[K]; /* the softmax numerators of A_ij[t] (FFBS weights) */
    double den;   /* their sum */
    double lA[K]; /* log A_ij[t] (t = 0: log p_1k) */
};

/* Emission oblik_t(j).
 * reg: normal_lpdf(x_t | u_t' b_j, s_j)          (iohmm-reg.stan:51-57)
 * mix: LSE_l(log lambda_jl + normal_lpdf(x_t | mu_jl, s_jl))
 *                                                 (iohmm-mix.stan:53-65; hmix :50-62; lite :46-58)
 * normal_lpdf = ((NEG_LOG_SQRT_TWO_PI - log s) + (-0.5 * z^2)), z = (x - mu) * (1/s);
 * log_sum_exp(std::vector): max by '>', sum of exp(x - max) over x != -inf
 * in order, max + log(sum). */
template <int FAM, int K, int MMAX, int MATH>
__device__ __forceinline__ void io_emission(const IoParams<FAM, K, MMAX> &pp, const double2 *slab, int L, int M,
                                            double x, const double (&u)[MMAX], double (&o)[K],
                                            const double2 *wb = nullptr, const hhmm_exp2_entry *tab = hhmm_exp2_tab)
{
    if constexpr (FAM == IO_REG) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            double br[MMAX];
            if constexpr (io_wb_lds<FAM>())
                wb_row<MMAX>(wb, K + j, br);
            const double mu = sse_dot<MMAX>(u, io_wb_lds<FAM>() ? br : pp.b[j], M);
            const double z = (x - mu) * pp.isig[j];
            const double z2 = z * z;
            o[j] = pp.c0[j] + (-0.5 * z2);
        }
    } else {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            double acc[kIoLmax];
            double mx = dev_ninf();
#pragma unroll
            for (int l = 0; l < kIoLmax; ++l) {
                if (l < L) {
                    const double2 ms = *mix_row(slab, L, j, l, 0);
                    const double2 lc = *mix_row(slab, L, j, l, 1);
                    const double z = (x - ms.x) * ms.y;
                    const double z2 = z * z;
                    acc[l] = lc.x + (lc.y + (-0.5 * z2));
                    if (acc[l] > mx)
                        mx = acc[l];
                }
            }
            double sum = 0.0;
#pragma unroll
            for (int l = 0; l < kIoLmax; ++l)
                if (l < L && acc[l] != dev_ninf())
                    sum += io_exp<MATH>(acc[l] - mx, tab);
            o[j] = mx + io_log<MATH>(sum);
        }
    }
}

/* Mixture emission factor without the log (MATH != IO_CR: the FFBS
 * contract's, or libm within tolerance): e(j) = sum_l exp(acc(j,l) - m) over
 * the finite summands acc(j,l) = log lambda_jl + normal_lpdf of the model's
 * log_sum_exp, m = fmax over j of max_l acc(j,l) (0 if -inf) -- exp(oblik(j) - m)
 * with K*L exps and no log (oracle ffbs_iohmm_emission). */
template <int K, int MATH>
__device__ __forceinline__ void io_mix_factor(const double2 *slab, int L, double x, double (&e)[K], double &m,
                                              const hhmm_exp2_entry *tab = hhmm_exp2_tab)
{
    double acc[K][kIoLmax];
    double mm = dev_ninf();
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double mx = dev_ninf();
#pragma unroll
        for (int l = 0; l < kIoLmax; ++l) {
            acc[j][l] = dev_ninf();
            if (l < L) {
                const double2 ms = *mix_row(slab, L, j, l, 0);
                const double2 lc = *mix_row(slab, L, j, l, 1);
                const double z = (x - ms.x) * ms.y;
                const double z2 = z * z;
                acc[j][l] = lc.x + (lc.y + (-0.5 * z2));
                if (acc[j][l] > mx)
                    mx = acc[j][l];
            }
        }
        mm = (j == 0) ? mx : fmax(mm, mx);
    }
    if (mm == dev_ninf())
        mm = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double sum = 0.0;
#pragma unroll
        for (int l = 0; l < kIoLmax; ++l)
            if (l < L && acc[j][l] != dev_ninf())
                sum += io_exp<MATH>(acc[j][l] - mm, tab);
        e[j] = sum;
    }
    m = mm;
}

/* Transition vector of step t >= 1: A_t = softmax(u_t' w_j), log A_t
 * (iohmm-reg.stan:40-49; iohmm-mix.stan:42-51, :69; iohmm-hmix.stan:36-48). */
template <int FAM, int K, int MMAX, int MATH>
__device__ __forceinline__ void io_transition(const IoParams<FAM, K, MMAX> &pp, int M, const double (&u)[MMAX],
                                              IoStep<K> &st, bool need_lA, const double2 *wb = nullptr,
                                              const hhmm_exp2_entry *tab = hhmm_exp2_tab)
{
    double v[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double wr[MMAX];
        if constexpr (io_wb_lds<FAM>())
            wb_row<MMAX>(wb, j, wr);
        v[j] = sse_dot<MMAX>(u, io_wb_lds<FAM>() ? wr : pp.w[j], M);
    }
    if constexpr (MATH == IO_CR) {
        if (need_lA) { /* the Viterbi's log A from the softmax's own exps */
            softmax_cr_log<K>(v, st.A, st.lA);
            return;
        }
    }
    stan_softmax<K, MATH>(v, st.A, st.th, st.den, tab);
    if (need_lA) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            st.lA[j] = io_log<MATH>(st.A[j]);
    }
}

/* Loads x_t and u_t[0..M) of one series (clamped, unconditional). */
template <int MMAX>
__device__ __forceinline__ void io_load(const DevArgs &a, uint32_t n, int t, double &x, double (&u)[MMAX])
{
    const int tc = min(max(t, 0), a.Tmax - 1);
    x = at(a.xr + a.N * (int64_t)tc, n * 8u);
#pragma unroll
    for (int m = 0; m < MMAX; ++m) {
        u[m] = 0.0;
        if (m < a.M)
            u[m] = at(a.u + a.N * ((int64_t)tc + (int64_t)a.Tmax * m), n * 8u);
    }
}

/* HOT: the request asks for nothing outside kIoHot, so the other outputs'
 * code (and their pointers, which would otherwise stay live in SGPRs through
 * the loop and spill) is compiled out. */
constexpr uint32_t kIoHot = HHMM_OUT_LOGLIK | HHMM_OUT_GAMMA | HHMM_OUT_ALPHA | HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR;

template <int FAM, int K, int MMAX, int MATH, bool HOT = false>
__device__ __forceinline__ void iohmm_sweep(const DevArgs &a)
{
    HIP_DYNAMIC_SHARED(double2, lds)
    constexpr int BITS = bp_bits(K);
    constexpr int SPW = bp_steps_per_word(K);
    constexpr int STEPB = K * BITS;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t pg = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t p = min(pg, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int M = a.M, L = a.L;
    const uint32_t out = HOT ? (a.outputs & kIoHot) : a.outputs;
    /* the linear filter's underflow check (hhmm_iolog.hip): s_t, max f_0 and,
     * where a backward output is read, c_t must stay above kIoWeak */
    const bool gate = (out & kIoFilt) && a.io_redo;
    bool weak = false;
    const bool want_vit = MATH == IO_CR && (out & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR));
    const bool want_ffbs = MATH == IO_DET && (out & HHMM_OUT_FFBS) && a.z_ffbs;
    const bool fixed_init = (a.model == HHMM_MODEL_IOHMM_HMIX); /* iohmm-hmix.stan:166-167 */
    const bool log_A_out = (a.model == HHMM_MODEL_IOHMM_HMIX || a.model == HHMM_MODEL_IOHMM_HMIX_LITE);
    const bool need_lA = want_vit || (log_A_out && (out & HHMM_OUT_LOGA) && a.logA);

    /* ---- per-pair parameters ---- */
    IoParams<FAM, K, MMAX> pp;
    double2 *wb = lds + (size_t)wave * K * MMAX * 64 + lane; /* io_wb_lds: K*MMAX double2 per lane */
#pragma unroll
    for (int k = 0; k < K; ++k) {
        pp.p[k] = a.p_1k[d + a.S * k];
#pragma unroll
        for (int m = 0; m < MMAX; ++m) {
            pp.w[k][m] = (m < M) ? a.w_km[d + a.S * ((int64_t)k + (int64_t)K * m)] : 0.0;
            if constexpr (FAM == IO_REG)
                pp.b[k][m] = (m < M) ? a.b_km[d + a.S * ((int64_t)k + (int64_t)K * m)] : 0.0;
        }
        if constexpr (io_wb_lds<FAM>()) {
#pragma unroll
            for (int mp = 0; mp < MMAX / 2; ++mp) {
                wb[(k * (MMAX / 2) + mp) * 64] = make_double2(pp.w[k][2 * mp], pp.w[k][2 * mp + 1]);
                wb[((K + k) * (MMAX / 2) + mp) * 64] = make_double2(pp.b[k][2 * mp], pp.b[k][2 * mp + 1]);
            }
        }
        if constexpr (FAM == IO_REG) {
            const double s = a.s_k[d + a.S * k];
            pp.isig[k] = 1.0 / s;
            pp.c0[k] = HHMM_NEG_LOG_SQRT_TWO_PI - io_log<MATH>(s);
        }
    }
    double2 *slab = lds + (size_t)wave * K * L * 2 * 64 + lane;
    if constexpr (FAM == IO_MIX) {
        /* loglambda_kl = log(lambda_kl) (iohmm-mix.stan:55) */
        for (int j = 0; j < K; ++j)
            for (int l = 0; l < L; ++l) {
                const int64_t ix = d + a.S * ((int64_t)j + (int64_t)K * l);
                const double s = a.s_kl[ix];
                *const_cast<double2 *>(mix_row(slab, L, j, l, 0)) = make_double2(a.mu_kl[ix], 1.0 / s);
                *const_cast<double2 *>(mix_row(slab, L, j, l, 1)) =
                    make_double2(io_log<MATH>(a.lambda_kl[ix]), HHMM_NEG_LOG_SQRT_TWO_PI - io_log<MATH>(s));
            }
    }
    /* IO_DET: the contract exp's table in LDS, after the waves' slabs */
    const hhmm_exp2_entry *etab = io_stage_exp2<MATH>(
        lds + (size_t)(blockDim.x >> 6) * (FAM == IO_MIX ? K * L * 2 * 64 : (io_wb_lds<FAM>() ? K * MMAX * 64 : 0)));
    const int Tw_min = wave_min(Tp);
    const int Tw_max = wave_max(Tp);

    /* ---- the sweep ---- */
    double f[K];         /* scaled linear-space forward state */
    double lsc = 0.0;    /* log scale, excluding the binary exponent ex */
    int ex = 0;
    double lam = 0.0;    /* Lambda_t = sum_{2 <= tau <= t} log c_tau (unbeta pass) */
    double dl[K];        /* Viterbi delta */
    uint32_t word = 0;
    /* the filter on the softmax numerators (no division; the sums in psum * 2^pex)
     * wherever nothing reads the normalised s_t (unalpha) and no Viterbi shares A */
    const bool num_filter = MATH != IO_CR && !(out & HHMM_OUT_UNALPHA);
    double psum = 1.0;
    int pex = 0;
    double vprev[K];     /* FFBS: v_{t-1} (p .* e_0 at t = 0, e_t after) */
    double uprev = 0.5;  /* FFBS: the uniform of step t - 1 */
    double x, xn;
    double u[MMAX], un[MMAX];
    io_load<MMAX>(a, (uint32_t)n, 0, x, u);
    for (int t = 0; t < Tw_max; ++t) {
        io_load<MMAX>(a, (uint32_t)n, t + 1, xn, un); /* one step ahead */
        if (t < Tp) {
            IoStep<K> st;
            /* mixture without a bit-exact Viterbi: the filter's factor comes
             * without the log-sum-exp's log (io_mix_factor); oblik itself only
             * where an output reads it */
            constexpr bool MIXF = (FAM == IO_MIX && MATH != IO_CR);
            if (!MIXF || (out & (HHMM_OUT_OBLIK_TK | HHMM_OUT_UNALPHA)))
                io_emission<FAM, K, MMAX, MATH>(pp, slab, L, M, x, u, st.o, wb, etab);
            if (t == 0) {
                /* A_ij[1] = p_1k (filler, iohmm-reg.stan:41-42); logA_ij[1] = log(p_1k) (iohmm-hmix.stan:40) */
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    st.A[k] = st.th[k] = pp.p[k];
                    st.lA[k] = log_A_out ? io_log<MATH>(pp.p[k]) : 0.0;
                }
                st.den = 1.0;
            } else {
                io_transition<FAM, K, MMAX, MATH>(pp, M, u, st, need_lA, wb, etab);
            }
            if ((out & HHMM_OUT_OBLIK_TK) && a.oblik)
                store_tk<K>(a.oblik, a, p, t, st.o);
            if ((out & HHMM_OUT_LOGA) && a.logA)
                store_tk<K>(a.logA, a, p, t, log_A_out ? st.lA : st.A);

            /* forward (iohmm-reg.stan:59-78): f_t = e_t * sum_i f_{t-1}(i) A_t(i) */
            double m = 0.0;
            double e[K];
            if constexpr (MIXF) {
                io_mix_factor<K, MATH>(slab, L, x, e, m, etab);
            } else {
            m = st.o[0];
#pragma unroll
            for (int k = 1; k < K; ++k)
                m = fmax(m, st.o[k]);
            if (m == dev_ninf())
                m = 0.0; /* every emission impossible: f_t = 0, alpha = NaN as in Stan */
            if constexpr (MATH == IO_DET) { /* the FFBS contract's e_t */
#pragma unroll
                for (int k = 0; k < K; ++k)
                    e[k] = hhmm_det_exp_tab(st.o[k] - m, etab);
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    e[k] = exp(st.o[k] - m);
            }
            }
            /* FFBS: the K-vector transition does not depend on the
             * next state, so z_{t-1} = cat(v_{t-1} .* th_t, u_{t-1}) is drawn here
             * (th_t = A_t's softmax numerators: cat normalises) */
            if (want_ffbs) {
                if (t > 0) {
                    double w[K];
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        w[k] = vprev[k] * st.th[k];
                    at(a.z_ffbs + a.P * (int64_t)(t - 1), (uint32_t)p * 4u) = ffbs_cat<K>(w, uprev) + 1;
                }
#pragma unroll
                for (int k = 0; k < K; ++k)
                    vprev[k] = (t == 0) ? pp.p[k] * e[k] : e[k];
                uprev = at(a.ffbs_u + a.P * (int64_t)t, (uint32_t)p * 8u);
            }
            /* unalpha in log space, so that a state whose emission underflows
             * exp(o - m) keeps Stan's finite value:
             *   t = 0: log(p_1k[j]) + oblik_1(j)                    (iohmm-reg.stan:62-63)
             *   t > 0: oblik_t(j) + log(s_t) + log-scale of f_{t-1}   (:65-74) */
            double ua_base;
            if (t == 0) {
                ua_base = 0.0;
#pragma unroll
                for (int k = 0; k < K; ++k)
                    f[k] = pp.p[k] * e[k];
                double f0 = f[0];
#pragma unroll
                for (int k = 1; k < K; ++k)
                    f0 = fmax(f0, f[k]);
                weak = gate && !(f0 >= kIoWeak0);
            } else {
                /* num_filter: the softmax numerators, the sum in the log scale
                 * (psum, pex) -- iohmm_sp_sweep's arithmetic, bit for bit */
                double s = f[0] * (num_filter ? st.th[0] : st.A[0]);
#pragma unroll
                for (int i = 1; i < K; ++i)
                    s = fma(f[i], num_filter ? st.th[i] : st.A[i], s);
                if (num_filter) {
                    int pe;
                    psum = frexp(psum * st.den, &pe);
                    pex += pe;
                }
                ua_base = log(s) + (lsc + kLn2 * ex);
                weak |= gate && !(s >= kIoWeak);
                /* s into [0.5, 1) first (exact): f_t = e_t * s then keeps every
                 * emission factor e_t(j) the reference's alpha keeps (a tiny s
                 * would flush e_t(j) * s below the subnormals) */
                const int es = __builtin_amdgcn_frexp_exp(s);
                ex += es;
                const double sn = ldexp(s, -es);
#pragma unroll
                for (int k = 0; k < K; ++k)
                    f[k] = e[k] * sn;
                /* log c_t = m + log sum_i A_t(i) e_t(i) (backward accumulator, :94) */
                if (out & kIoBack) {
                    double c = st.A[0] * e[0];
#pragma unroll
                    for (int i = 1; i < K; ++i)
                        c = fma(st.A[i], e[i], c);
                    weak |= gate && !(c >= kIoWeak);
                    if (out & HHMM_OUT_UNBETA) {
                        lam += m + log(c);
                        at(a.lam + a.P * (int64_t)t, (uint32_t)p * 8u) = lam;
                    }
                }
            }
            lsc += m;
            renorm<K>(f, ex);

            /* posteriors of step t */
            const double fs = vsum<K>(f);
            const double rfs = fast_rcp(fs); /* renormalised: fs >= 1/2 (or 0 / NaN) */
            if ((out & HHMM_OUT_ALPHA) && a.alpha) {
                double v[K];
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[k] = f[k] * rfs;
                store_tk<K>(a.alpha, a, p, t, v);
            }
            if ((out & HHMM_OUT_UNALPHA) && a.unalpha) {
                double v[K];
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[k] = (t == 0) ? log(pp.p[k]) + st.o[k] : st.o[k] + ua_base;
                store_tk<K>(a.unalpha, a, p, t, v);
            }
            if ((out & HHMM_OUT_BETA) && a.beta) { /* softmax of a repeated scalar */
                double v[K];
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[k] = 1.0 / K;
                store_tk<K>(a.beta, a, p, t, v);
            }
            if ((out & (HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA)) && (a.gamma || a.ungamma)) {
                /* ungamma = alpha .* (1/K); gamma = normalize(ungamma) = alpha */
                double v[K];
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[k] = f[k] * rfs;
                if ((out & HHMM_OUT_GAMMA) && a.gamma)
                    store_tk<K>(a.gamma, a, p, t, v);
                if ((out & HHMM_OUT_UNGAMMA) && a.ungamma) {
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        v[k] = v[k] * (1.0 / K);
                    store_tk<K>(a.ungamma, a, p, t, v);
                }
            }
            if ((out & HHMM_OUT_OBLIK_T) && a.oblik_t) {
                /* oblik_t = LSE(log(alpha_t) + oblik_t) = m + log(sum_j f_j e_j / sum_j f_j)
                 * (iohmm-hmix.stan:118-121; lite :78-81) */
                double num = f[0] * e[0];
#pragma unroll
                for (int k = 1; k < K; ++k)
                    num = fma(f[k], e[k], num);
                at(a.oblik_t + a.P * (int64_t)t, (uint32_t)p * 8u) = m + log(num * rfs);
            }

            /* Viterbi (iohmm-reg.stan:150-181; iohmm-mix.stan:164-195; iohmm-hmix.stan:160-193) */
            if (want_vit) {
                if (t == 0) {
                    if (fixed_init) {
#pragma unroll
                        for (int k = 0; k < K; ++k)
                            dl[k] = st.o[k];
                    } else { /* delta_tk[1, K] = oblik_tk[1][j] for j = 1..K (Q3) */
#pragma unroll
                        for (int k = 0; k < K - 1; ++k)
                            dl[k] = dev_nan();
                        dl[K - 1] = st.o[K - 1];
                    }
                } else {
                    /* logp = (delta_{t-1}(i) + log A_t(i)) + oblik_t(j); strict '>' from -inf */
                    double ai[K];
#pragma unroll
                    for (int i = 0; i < K; ++i)
                        ai[i] = dl[i] + st.lA[i];
                    const int slot = t % SPW;
#pragma unroll
                    for (int j = 0; j < K; ++j) {
                        double best = dev_ninf();
                        uint32_t arg = 0;
#pragma unroll
                        for (int i = 0; i < K; ++i) {
                            const double cand = ai[i] + st.o[j];
                            if (cand > best) {
                                best = cand;
                                arg = (uint32_t)i;
                            }
                        }
                        dl[j] = best;
                        word |= arg << (slot * STEPB + j * BITS);
                    }
                    if (slot == SPW - 1) {
                        a.bp[p + a.P * (int64_t)(t / SPW)] = word;
                        word = 0;
                    }
                }
            }
        }
        x = xn;
#pragma unroll
        for (int m2 = 0; m2 < MMAX; ++m2)
            u[m2] = un[m2];
    }
    if (want_ffbs)
        at(a.z_ffbs + a.P * (int64_t)(Tp - 1), (uint32_t)p * 4u) = ffbs_cat<K>(vprev, uprev) + 1;
    if (weak && pg < a.P) /* re-run in log space (launch_iohmm_log) */
        a.io_redo[1 + atomicAdd(&a.io_redo[0], 1)] = (int32_t)p;
    if ((out & HHMM_OUT_LOGLIK) && a.loglik) /* target += log_sum_exp(unalpha_tk[T]) (iohmm-reg.stan:120) */
        a.loglik[p] = (log(vsum<K>(f)) + (lsc + kLn2 * ex)) - (log(psum) + kLn2 * pex);

    /* unbeta_tk: B_T = 1 (Q1); B_t = 1 + (Lambda_T - Lambda_t) (iohmm-reg.stan:80-98) */
    if ((out & HHMM_OUT_UNBETA) && a.unbeta) {
        const double lamT = lam;
        for (int t = 0; t < Tp; ++t) {
            const double lt = (t == 0) ? 0.0 : a.lam[p + a.P * (int64_t)t];
            double v[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                v[k] = 1.0 + (lamT - lt);
            store_tk<K>(a.unbeta, a, p, t, v);
        }
    }
    if (want_vit)
        viterbi_epilogue<K>(a, p, Tp, Tw_min, Tw_max, dl, word);
}

/* The regression family's exact sweep needs ~290 registers: uncapped it runs
 * one wave per SIMD.  Capped at two waves (256 registers, a 144-byte spill)
 * it ran C3 in 87 ms against 156 ms on one box; the mixture family runs
 * faster uncapped (C4: 147 against 160 ms), so only the regression kernel
 * carries the cap. */
#ifndef HHMM_IO_REG_WAVES
#define HHMM_IO_REG_WAVES 2
#endif
template <int K, int MMAX, int MATH, bool HOT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(HHMM_IO_REG_WAVES))) iohmm_reg_kernel(const DevArgs a)
{
    iohmm_sweep<IO_REG, K, MMAX, MATH, HOT>(a);
}

template <int K, int MMAX, int MATH, bool HOT>
__global__ void __launch_bounds__(kBlock) iohmm_mix_kernel(const DevArgs a)
{
    iohmm_sweep<IO_MIX, K, MMAX, MATH, HOT>(a);
}


/* ---- state-parallel sweep (few pairs; C4) ------------------------------ *
 * One lane per (pair, state j), a pair's K <= 4 states in one lane quad.  A
 * step's transcendentals are per state -- the mixture log_sum_exp of state j,
 * its softmax exp, its filter exp -- so each lane evaluates only its own
 * state's, and the quad exchanges the K-vectors it needs by DPP broadcasts:
 * softmax max / sum, the emission max, A_t and e_t.  Everything that mixes
 * states (the softmax sum, the forward dot, the FFBS category) is then
 * evaluated by every lane of the quad from the gathered vectors in the lane
 * sweep's order, so outputs and draws are bit-identical to iohmm_sweep.  At
 * C4 (65,536 pairs) lane-per-pair runs one wave per SIMD, each step a
 * latency-bound chain of ~24 exps; here it runs four with a quarter of the
 * chain.  The lane's mixture entries sit in its LDS column (registers held the
 * kernel at three waves per SIMD).  Profile: loglik, alpha / gamma (= alpha,
 * Q5) and FFBS. */
template <int FAM, int K, int MMAX, int MATH, int LM>
__device__ __forceinline__ void iohmm_sp_sweep(const DevArgs &a)
{
    static_assert(K >= 2 && K <= 4, "one lane quad per pair");
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = (g >> 2) < a.P;
    const int64_t p = min(g >> 2, a.P - 1);
    const int j = (int)(g & 3);
    const int js = min(j, K - 1);
    const bool owns = live && j < K;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    /* LM == 3 is launched for L == 3 exactly (launch_io_sp): the mixture loops
     * are straight-line code, so the step's three exps interleave */
    const int M = a.M, L = (FAM == IO_MIX && LM == 3) ? 3 : a.L;
    const uint32_t out = a.outputs;
    const bool want_ffbs = MATH == IO_DET && (out & HHMM_OUT_FFBS) && a.z_ffbs;
    const bool gate = (out & kIoFilt) && a.io_redo; /* iohmm_sweep's underflow check */
    bool weak = false;

    /* ---- parameters: p_1k whole, state js's rows and tables ---- */
    double pk[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        pk[k] = a.p_1k[d + a.S * k];
    double w[MMAX], b[MMAX];
#pragma unroll
    for (int m = 0; m < MMAX; ++m) {
        w[m] = (m < M) ? a.w_km[d + a.S * ((int64_t)js + (int64_t)K * m)] : 0.0;
        b[m] = 0.0;
        if constexpr (FAM == IO_REG)
            b[m] = (m < M) ? a.b_km[d + a.S * ((int64_t)js + (int64_t)K * m)] : 0.0;
    }
    double isig = 0.0, c0 = 0.0;
    /* state js's mixture entries in the lane's LDS column: (mu, 1/s), (log lambda, C - log s) */
    HIP_DYNAMIC_SHARED(double2, lds)
    double2 *col = lds + (threadIdx.x >> 6) * (size_t)(2 * LM * 64) + (threadIdx.x & 63);
    if constexpr (FAM == IO_REG) {
        const double sg = a.s_k[d + a.S * js];
        isig = 1.0 / sg;
        c0 = HHMM_NEG_LOG_SQRT_TWO_PI - io_log<MATH>(sg);
    } else {
#pragma unroll
        for (int l = 0; l < LM; ++l) {
            if (l < L) {
                const int64_t ix = d + a.S * ((int64_t)js + (int64_t)K * l);
                const double sg = a.s_kl[ix];
                col[(2 * l) * 64] = make_double2(a.mu_kl[ix], 1.0 / sg);
                col[(2 * l + 1) * 64] =
                    make_double2(io_log<MATH>(a.lambda_kl[ix]), HHMM_NEG_LOG_SQRT_TWO_PI - io_log<MATH>(sg));
            }
        }
    }
    /* the FFBS contract's exp reads its 2^(j/128) table from a copy in LDS
     * after the columns (hhmm_det_exp_tab): a global read would sit on the
     * dependency chain of each of the step's exps */
    const hhmm_exp2_entry *etab =
        io_stage_exp2<MATH>(lds + (FAM == IO_MIX ? (blockDim.x >> 6) * (size_t)(2 * LM * 64) : 0));
    auto sexp = [&](double v) -> double { return io_exp<MATH>(v, etab); };
    const int Tw_max = wave_max(Tp);

    double f[K];
    double lsc = 0.0;
    int ex = 0;
    double vprev[K];
    double uprev = 0.5;
    double psum = 1.0; /* product of the softmax sums the filter did not divide by, */
    int pex = 0;       /* as psum * 2^pex */
    double x, xn;
    double u[MMAX], un[MMAX];
    io_load<MMAX>(a, (uint32_t)n, 0, x, u);
    for (int t = 0; t < Tw_max; ++t) {
        io_load<MMAX>(a, (uint32_t)n, t + 1, xn, un);
        if (t < Tp) {
            /* emission of state js (io_emission's arithmetic); the mixture
             * yields only its summands' max mx and the filter factor comes from
             * them below (io_mix_factor's arithmetic: no log) */
            double o = 0.0, acc[LM], mxs = 0.0;
            if constexpr (FAM == IO_REG) {
                const double mv = sse_dot<MMAX>(u, b, M);
                const double z = (x - mv) * isig;
                const double z2 = z * z;
                o = c0 + (-0.5 * z2);
            } else {
                double mx = dev_ninf();
#pragma unroll
                for (int l = 0; l < LM; ++l) {
                    acc[l] = dev_ninf();
                    if (l < L) {
                        const double2 ms = col[(2 * l) * 64];
                        const double2 lg = col[(2 * l + 1) * 64];
                        const double z = (x - ms.x) * ms.y;
                        const double z2 = z * z;
                        acc[l] = lg.x + (lg.y + (-0.5 * z2));
                        if (acc[l] > mx)
                            mx = acc[l];
                    }
                }
                mxs = mx;
            }
            /* transition A_t = softmax(u_t' w) (stan_softmax's order); t = 0: p_1k */
            double AA[K];
            if (t == 0) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    AA[k] = pk[k];
            } else {
                const double v = sse_dot<MMAX>(u, w, M);
                double vv[K];
                quad_gather<K>(v, vv);
                double mx = vv[0];
#pragma unroll
                for (int i = 1; i < K; ++i)
                    if (vv[i] > mx)
                        mx = vv[i];
                /* the numerators exp(v - max) only: the FFBS weights take them as
                 * they are (cat normalises), and the filter carries the sum in a
                 * separate log scale (psum, pex) instead of dividing */
                quad_gather<K>(sexp(v - mx), AA);
                double sum = 0.0;
#pragma unroll
                for (int i = 0; i < K; ++i)
                    sum += AA[i];
                int e;
                psum = frexp(psum * sum, &e);
                pex += e;
            }
            /* e_t = exp(o - max o); mixture: sum_l exp(acc_l - m) */
            double oo[K];
            quad_gather<K>(FAM == IO_REG ? o : mxs, oo);
            double m = oo[0];
#pragma unroll
            for (int k = 1; k < K; ++k)
                m = fmax(m, oo[k]);
            if (m == dev_ninf())
                m = 0.0;
            double ej;
            if constexpr (FAM == IO_REG) {
                ej = MATH == IO_DET ? sexp(o - m) : exp(o - m);
            } else {
                /* every summand's exp first (independent: their table reads
                 * overlap), then the model's sum over the finite ones in order
                 * (a skipped -inf summand and an added +0 give the same bits) */
                double ye[LM];
#pragma unroll
                for (int l = 0; l < LM; ++l)
                    ye[l] = (l < L) ? sexp(acc[l] - m) : 0.0;
                ej = 0.0;
#pragma unroll
                for (int l = 0; l < LM; ++l)
                    if (l < L)
                        ej += (acc[l] != dev_ninf()) ? ye[l] : 0.0;
            }
            double ee[K];
            quad_gather<K>(ej, ee);
            if (want_ffbs) {
                if (t > 0) {
                    double wv[K];
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        wv[k] = vprev[k] * AA[k];
                    const int z = ffbs_cat<K>(wv, uprev) + 1;
                    if (live && j == 0)
                        at(a.z_ffbs + a.P * (int64_t)(t - 1), (uint32_t)p * 4u) = z;
                }
#pragma unroll
                for (int k = 0; k < K; ++k)
                    vprev[k] = (t == 0) ? pk[k] * ee[k] : ee[k];
                uprev = at(a.ffbs_u + a.P * (int64_t)t, (uint32_t)p * 8u);
            }
            /* forward: f_t = e_t * sum_i f_{t-1}(i) A_t(i) (times the softmax sum) */
            if (t == 0) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    f[k] = pk[k] * ee[k];
                double f0 = f[0];
#pragma unroll
                for (int k = 1; k < K; ++k)
                    f0 = fmax(f0, f[k]);
                weak = gate && !(f0 >= kIoWeak0);
            } else {
                double sv = f[0] * AA[0];
#pragma unroll
                for (int i = 1; i < K; ++i)
                    sv = fma(f[i], AA[i], sv);
                weak |= gate && !(sv >= kIoWeak);
                const int es = __builtin_amdgcn_frexp_exp(sv); /* iohmm_sweep: s into [0.5, 1) first */
                ex += es;
                const double sn = ldexp(sv, -es);
#pragma unroll
                for (int k = 0; k < K; ++k)
                    f[k] = ee[k] * sn;
                if (out & kIoBack) { /* the backward accumulator sum_i A_t(i) e_t(i) (numerators) */
                    double c = AA[0] * ee[0];
#pragma unroll
                    for (int i = 1; i < K; ++i)
                        c = fma(AA[i], ee[i], c);
                    weak |= gate && !(c >= kIoWeak);
                }
            }
            lsc += m;
            renorm<K>(f, ex);
            if ((out & (HHMM_OUT_ALPHA | HHMM_OUT_GAMMA)) && owns) {
                double fj = f[0];
#pragma unroll
                for (int k = 1; k < K; ++k)
                    fj = (js == k) ? f[k] : fj;
                const double v = fj * fast_rcp(vsum<K>(f)); /* renormalised: the sum is >= 1/2 (or 0 / NaN) */
                if ((out & HHMM_OUT_ALPHA) && a.alpha)
                    put_out(a.alpha + a.P * ((int64_t)t + (int64_t)a.Tout * js), (uint32_t)p * 8u, v);
                if ((out & HHMM_OUT_GAMMA) && a.gamma)
                    put_out(a.gamma + a.P * ((int64_t)t + (int64_t)a.Tout * js), (uint32_t)p * 8u, v);
            }
        }
        x = xn;
#pragma unroll
        for (int m2 = 0; m2 < MMAX; ++m2)
            u[m2] = un[m2];
    }
    if (live && j == 0) {
        if (want_ffbs)
            at(a.z_ffbs + a.P * (int64_t)(Tp - 1), (uint32_t)p * 4u) = ffbs_cat<K>(vprev, uprev) + 1;
        if (weak) /* re-run in log space (launch_iohmm_log) */
            a.io_redo[1 + atomicAdd(&a.io_redo[0], 1)] = (int32_t)p;
        if ((out & HHMM_OUT_LOGLIK) && a.loglik)
            a.loglik[p] = (log(vsum<K>(f)) + (lsc + kLn2 * ex)) - (log(psum) + kLn2 * pex);
    }
}

/* Capped at four waves per SIMD (128 registers, a 12-register spill): C4 45.9
 * against 47.5 ms uncapped (138 registers, three waves). */
#ifndef HHMM_IO_SP_WAVES
#define HHMM_IO_SP_WAVES 4
#endif
template <int FAM, int K, int MMAX, int MATH, int LM>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(HHMM_IO_SP_WAVES)))
iohmm_sp_kernel(const DevArgs a)
{
    if constexpr (K >= 2 && K <= 4)
        iohmm_sp_sweep<FAM, K, MMAX, MATH, LM>(a);
}

/* The state-parallel sweep's profile and range: K = 2..4, outputs within
 * loglik / alpha / gamma / FFBS, a batch that leaves lane-per-pair below two
 * waves per SIMD (HHMM_FLAG_VIT_LANES / _VIT_STATES force one layout). */
static bool io_states(const DevArgs &a)
{
    const uint32_t sp_out = HHMM_OUT_LOGLIK | HHMM_OUT_ALPHA | HHMM_OUT_GAMMA | HHMM_OUT_FFBS;
    if (a.K < 2 || a.K > 4 || (a.outputs & ~sp_out) || (a.flags & HHMM_FLAG_VIT_LANES))
        return false;
    return (a.flags & HHMM_FLAG_VIT_STATES) || a.P < 131072;
}

/* ------------------------------------------------------------------ */
/* Host-side launch                                                      */
/* ------------------------------------------------------------------ */

template <int FAM, int K, int MMAX, int MATH, bool HOT>
static hhmm_status launch_io5(const DevArgs &a, hipStream_t st)
{
    const size_t per_wave = (FAM == IO_MIX) ? (size_t)K * a.L * 2 * 64 * sizeof(double2)
                                            : (io_wb_lds<FAM>() ? (size_t)K * MMAX * 64 * sizeof(double2) : 0);
    const size_t tab = MATH == IO_DET ? 128 * sizeof(hhmm_exp2_entry) : 0; /* io_stage_exp2's copy */
    int waves = 4;
    while (per_wave > 0 && waves > 1 && per_wave * waves + tab > kLdsLimit)
        --waves;
    if (per_wave * waves + tab > kLdsLimit) {
        set_error("IOHMM mixture table K*L = %d*%d does not fit in LDS", K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const int threads = 64 * waves;
    const dim3 grid((unsigned)((a.P + threads - 1) / threads));
    if constexpr (FAM == IO_REG)
        hipLaunchKernelGGL((iohmm_reg_kernel<K, MMAX, MATH, HOT>), grid, dim3(threads), per_wave * waves + tab, st, a);
    else
        hipLaunchKernelGGL((iohmm_mix_kernel<K, MMAX, MATH, HOT>), grid, dim3(threads), per_wave * waves + tab, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("iohmm kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* The hot profile is instantiated for the Viterbi sweep at K <= 4 (C3's). */
template <int FAM, int K, int MMAX, int MATH>
static hhmm_status launch_io4(const DevArgs &a, hipStream_t st)
{
    if constexpr (MATH == IO_CR && K <= 4) {
        if (!(a.outputs & ~kIoHot))
            return launch_io5<FAM, K, MMAX, MATH, true>(a, st);
    }
    return launch_io5<FAM, K, MMAX, MATH, false>(a, st);
}

template <int FAM, int K, int MMAX, int MATH>
static hhmm_status launch_io_sp(const DevArgs &a, hipStream_t st)
{
    const int64_t lanes = 4 * a.P;
    const dim3 grid((unsigned)((lanes + kBlock - 1) / kBlock));
    /* the mixture tables of a lane's state sit in registers: L <= 4 or <= 8 */
    const size_t tab = MATH == IO_DET ? 128 * sizeof(hhmm_exp2_entry) : 0; /* hhmm_det_exp_tab's copy */
    const int lm = (FAM == IO_MIX && a.L == 3) ? 3 : (a.L <= 4 ? 4 : kIoLmax);
    const size_t lds = ((FAM == IO_MIX) ? (size_t)(kBlock / 64) * 2 * lm * 64 * sizeof(double2) : 0) + tab;
    if (FAM == IO_REG)
        hipLaunchKernelGGL((iohmm_sp_kernel<FAM, K, MMAX, MATH, 1>), grid, dim3(kBlock), tab, st, a);
    else if (lm == 3)
        hipLaunchKernelGGL((iohmm_sp_kernel<FAM, K, MMAX, MATH, 3>), grid, dim3(kBlock), lds, st, a);
    else if (a.L <= 4)
        hipLaunchKernelGGL((iohmm_sp_kernel<FAM, K, MMAX, MATH, 4>), grid, dim3(kBlock), lds, st, a);
    else
        hipLaunchKernelGGL((iohmm_sp_kernel<FAM, K, MMAX, MATH, kIoLmax>), grid, dim3(kBlock), lds, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("iohmm state-parallel kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

template <int FAM, int K, int MATH>
static hhmm_status launch_io_m(const DevArgs &a, hipStream_t st)
{
    if constexpr (K >= 2 && K <= 4 && MATH != IO_CR) {
        if (io_states(a))
            return a.M <= 4 ? launch_io_sp<FAM, K, 4, MATH>(a, st) : launch_io_sp<FAM, K, 8, MATH>(a, st);
    }
    return a.M <= 4 ? launch_io4<FAM, K, 4, MATH>(a, st) : launch_io4<FAM, K, 8, MATH>(a, st);
}

/* The arithmetic mode(s) of a request (see the header comment). */
template <int FAM, int K>
static hhmm_status launch_io3(const DevArgs &a, hipStream_t st)
{
    const bool vit = (a.outputs & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR)) != 0;
    const bool ffbs = (a.outputs & HHMM_OUT_FFBS) != 0 && a.z_ffbs;
    if (!ffbs)
        return vit ? launch_io_m<FAM, K, IO_CR>(a, st) : launch_io_m<FAM, K, IO_LIBM>(a, st);
    if (!vit)
        return launch_io_m<FAM, K, IO_DET>(a, st);
    DevArgs b = a;
    b.outputs = a.outputs & ~(uint32_t)HHMM_OUT_FFBS;
    const hhmm_status s = launch_io_m<FAM, K, IO_CR>(b, st);
    if (s != HHMM_OK)
        return s;
    b.outputs = HHMM_OUT_FFBS;
    return launch_io_m<FAM, K, IO_DET>(b, st);
}

/* Dispatch on K for the K values [KK, KHI] this translation unit instantiates. */
template <int FAM, int KK, int KHI>
static hhmm_status launch_io_range(const DevArgs &a, hipStream_t st)
{
    if constexpr (KK > KHI) {
        set_error("K = %d not supported by this IOHMM build", a.K);
        return HHMM_ERR_UNSUPPORTED;
    } else {
        if (a.K == KK)
            return launch_io3<FAM, KK>(a, st);
        return launch_io_range<FAM, KK + 1, KHI>(a, st);
    }
}

} // namespace hhmm
