/*
 * hhmm_hmm.h -- gfx950 kernels for the HMM family (hmm, hmm-multinom, semisup,
 * Tayal full / lite), as templates; each hhmm_m_*.hip instantiates one model
 * (one translation unit per model so the library builds in parallel).
 *
 * Layout in HBM (include/hhmm.h): every array is pair-/series-/draw-fastest,
 * so one wave of 64 lanes = 64 consecutive pairs reads and writes 64
 * consecutive elements per (t, k): every global access below is a fully
 * coalesced 256 B (int32) or 512 B (fp64) wave transaction.
 *
 * One LANE owns one (series, draw) PAIR for the whole sequence; the K-state
 * vectors live in registers.  Per-pair emission tables (phi_k and log phi_k,
 * K*L doubles) live in LDS, one slab per wave, laid out
 *     slab[(l * KP + kp) * 64 + lane]  (double2: states 2kp, 2kp+1)
 * so a 16-lane ds_read_b128 group touches 16 consecutive 16-B slots = all 64
 * banks once: conflict-free for any per-lane symbol.
 *
 * Kernels:
 *   fb_kernel      A2/A1 emissions, A6 forward + loglik, A7 alpha, A8 backward,
 *                  A9 gamma, A12/A13 masks.  LINEAR-space scaled recursion
 *                  (K^2 FMAs per step, an exact power-of-two renormalisation
 *                  per step; no exp/log in the discrete loop);
 *                  forward checkpoints every C steps, recomputed chunk by chunk
 *                  in the backward sweep.  Tolerance 1e-9 rel.
 * Latency rules used throughout (the kernels are latency-, not issue-bound at
 * the 2 waves/SIMD the LDS tables allow): observation loads are issued
 * unconditionally (clamped index) one chunk ahead, checkpoints and
 * back-pointer words one chunk ahead, and each step's LDS emission row is
 * fetched one step ahead.
 *   viterbi_kernel A11 max-plus recursion in LOG space with exactly the
 *                  reference's operation order and tie rules, log tables from
 *                  the correctly rounded hhmm_cr_log (bit-identical to the
 *                  oracle); back-pointers packed 2 bits/state to HBM, backtrack
 *                  in the same kernel.  Bit-exact.
 * Build with -ffp-contract=off: the Viterbi sums must round exactly as written.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <vector>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "hhmm_device.h"

namespace hhmm {


/* hmm-multinom-semisup.stan:42 -- j0 is 0-based */
__device__ __forceinline__ bool semisup_mask(int g, int j0)
{
    const int j = j0 + 1;
    return (g == 1 && (j == 1 || j == 4)) || (g == 2 && (j == 2 || j == 3));
}
/* hhmm-tayal2009.stan:62 / :109 / :144 */
__device__ __forceinline__ bool tayal_pred(int s, int j0)
{
    const int j = j0 + 1;
    return (s == 1 && (j == 2 || j == 3)) || (s == 2 && (j == 1 || j == 4));
}
/* tayal_pred for a compile-time sign class sg (1, 2, or 3 = any other sign):
 * the kernels whose wave shares one step's sign (one series under many draws,
 * C5) take the masks as constants, so the masked-off terms cost nothing. */
__host__ __device__ constexpr bool tayal_on(int sg, int j0)
{
    return (sg == 1 && (j0 == 1 || j0 == 2)) || (sg == 2 && (j0 == 0 || j0 == 3));
}
/* The flattened HHMM's transition matrix (hhmm-tayal2009.stan:36-44), as ONE
 * table both load_params (which builds A) and tayal_nz (which skips its
 * structural zeros) read: entry (i, j) is 0 (a structural zero), 1 (one), or
 * 2 + 2r + c for A_row[r][c]. */
constexpr int kTayalA[4][4] = {{0, 2, 3, 0}, {1, 0, 0, 0}, {4, 0, 0, 5}, {0, 0, 1, 0}};
/* Entry (i, j) can be nonzero.  A term with a structural zero adds exactly
 * nothing (0 x f to a linear sum of finite terms, a -inf candidate to a
 * max-plus one), so the sign-class paths skip it -- in the linear filters only
 * where the wave's parameters are probabilities (PairParams::skip_ok), so no
 * NaN or infinity can meet a skipped zero (the reference's 0 x NaN = NaN). */
__host__ __device__ constexpr bool tayal_nz(int i, int j) { return kTayalA[i][j] != 0; }
/* hhmm-tayal2009.stan:51 */
__device__ __forceinline__ bool tayal_init_pred(int s, int j0)
{
    const int j = j0 + 1;
    return (s == 1 && j == 3) || (s == 2 && j == 1);
}

template <int MODEL>
struct ModelTraits {
    static constexpr bool kGauss = (MODEL == HHMM_MODEL_HMM_GAUSS);
    static constexpr bool kSemisup = (MODEL == HHMM_MODEL_HMM_MULTINOM_SEMISUP);
    static constexpr bool kTayal = (MODEL == HHMM_MODEL_TAYAL || MODEL == HHMM_MODEL_TAYAL_LITE);
    static constexpr bool kDiscrete = !kGauss;
    static constexpr bool kAux = kSemisup || kTayal; /* needs g[] or sign[] per step */
};

/* One observation step of a series. */
struct Obs {
    int x;     /* symbol 1..L (discrete models) */
    int aux;   /* g (semisup) or sign (tayal) */
    double xr; /* real observation (gauss) */
};

/* Observation streams of one series (series-fastest arrays): uniform base
 * pointers + this lane's 32-bit series index.  A time row t is the uniform
 * pointer base + N*t, so hipcc can address it as SGPR base + VGPR offset. */
struct SeriesPtrs {
    const int32_t *x;
    const int32_t *aux;
    const double *xr;
    int64_t stride; /* N: elements between consecutive time steps */
    uint32_t n;     /* this lane's series */
    int tmax;       /* padded time extent of the arrays */
};

/* Loads the C observations of chunk [t0, t0+C).  Every load is issued
 * unconditionally from a wave-uniform time index clamped into [0, Tmax-1]: a
 * conditional load makes hipcc branch around it and drain vmcnt(0) per
 * element (cdna_hip_programming.md §5, trap (c)); rows past a lane's own
 * length are padding that is never consumed. */
template <int MODEL, int C, bool AUX>
__device__ __forceinline__ void load_chunk(Obs (&dst)[C], const SeriesPtrs &sp, int t0)
{
#pragma unroll
    for (int u = 0; u < C; ++u) {
        const int tc = min(max(t0 + u, 0), sp.tmax - 1);
        const int64_t row = (int64_t)tc * sp.stride;
        dst[u].x = 1;
        dst[u].aux = 0;
        dst[u].xr = 0.0;
        if constexpr (!ModelTraits<MODEL>::kGauss)
            dst[u].x = at(sp.x + row, sp.n * 4u);
        if constexpr (AUX)
            dst[u].aux = at(sp.aux + row, sp.n * 4u);
        if constexpr (ModelTraits<MODEL>::kGauss)
            dst[u].xr = at(sp.xr + row, sp.n * 8u);
    }
}

/* Per-pair parameters held in registers. */
template <int MODEL, int K>
struct PairParams {
    double A[K][K];  /* probability (FB) or log (Viterbi) */
    double p[K];
    double mu[K], isig[K], lsig[K], c0[K]; /* gauss: 1/sigma, log sigma, NEG_LOG_SQRT_TWO_PI - log sigma */
    bool skip_ok;    /* tayal: p_11, A_row (load_params) and phi (fill_table) all in [0, 1] */
};

template <int K>
__device__ __forceinline__ double draw1(const double *arr, const DevArgs &a, int64_t d, int k)
{
    return arr[d + a.S * (int64_t)k];
}
template <int K>
__device__ __forceinline__ double draw2(const double *arr, const DevArgs &a, int64_t d, int i, int j, int I)
{
    return arr[d + a.S * ((int64_t)i + (int64_t)I * j)];
}

/* 0 <= v <= 1 (false for NaN) */
__device__ __forceinline__ bool in01(double v) { return (v >= 0.0) & (v <= 1.0); }

/* Loads p_1k, A_ij (Tayal: expands p_11 / A_row, hhmm-tayal2009.stan:30-44)
 * and the Gaussian constants.  LOG = true puts log A in params.A.
 * Every global load is issued before the first log consumes one: with the
 * load -> correctly rounded log pairs interleaved, hipcc waits vmcnt(0) per
 * parameter, i.e. one HBM round trip per entry (K^2 + K of them) before the
 * first step. */
template <int MODEL, int K, bool LOG>
__device__ __forceinline__ void load_params(PairParams<MODEL, K> &pp, const DevArgs &a, int64_t d)
{
    if constexpr (ModelTraits<MODEL>::kTayal) {
        static_assert(K == 4, "tayal is a K = 4 model");
        const double p11 = a.p_11[d];
        const double r00 = a.A_row[d + a.S * 0], r10 = a.A_row[d + a.S * 1];
        const double r01 = a.A_row[d + a.S * 2], r11 = a.A_row[d + a.S * 3];
        const double src[6] = {0.0, 1.0, r00, r01, r10, r11}; /* kTayalA's codes */
        double A[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                A[i][j] = src[kTayalA[i][j]];
        pp.skip_ok = in01(p11) && in01(r00) && in01(r01) && in01(r10) && in01(r11);
        pp.p[0] = p11;
        pp.p[1] = 0;
        pp.p[2] = 1 - p11;
        pp.p[3] = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                pp.A[i][j] = LOG ? dev_cr_log(A[i][j]) : A[i][j];
    } else {
        pp.skip_ok = false;
        double raw[K][K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            pp.p[k] = draw1<K>(a.p_1k, a, d, k);
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                raw[i][j] = draw2<K>(a.A_ij, a, d, i, j, K);
        double mu[ModelTraits<MODEL>::kGauss ? K : 1], sg[ModelTraits<MODEL>::kGauss ? K : 1];
        if constexpr (ModelTraits<MODEL>::kGauss) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                sg[k] = draw1<K>(a.sigma_k, a, d, k);
                mu[k] = draw1<K>(a.mu_k, a, d, k);
            }
        }
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                pp.A[i][j] = LOG ? dev_cr_log(raw[i][j]) : raw[i][j];
        if constexpr (ModelTraits<MODEL>::kGauss) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                pp.mu[k] = mu[k];
                pp.isig[k] = 1.0 / sg[k];
                pp.lsig[k] = dev_cr_log(sg[k]);
                pp.c0[k] = HHMM_NEG_LOG_SQRT_TWO_PI - pp.lsig[k];
            }
        }
    }
}

/* Fills this lane's LDS slab with phi_k (LOG: log phi_k).  Rows are fetched
 * kRowBatch at a time, all loads of a batch in flight together (a load per
 * row followed by its LDS store costs one HBM round trip per row). */
constexpr int kRowBatch = 4;
template <int K, bool LOG>
__device__ __forceinline__ bool fill_table(double2 *slab, const DevArgs &a, int64_t d)
{
    constexpr int KP = (K + 1) / 2;
    bool ok = true; /* every phi entry in [0, 1] (PairParams::skip_ok) */
    for (int l0 = 0; l0 < a.L; l0 += kRowBatch) {
        double v[kRowBatch][2 * KP];
#pragma unroll
        for (int r = 0; r < kRowBatch; ++r) {
            const int l = min(l0 + r, a.L - 1); /* clamped: a short last batch re-reads row L-1 */
#pragma unroll
            for (int k = 0; k < 2 * KP; ++k)
                v[r][k] = (k < K) ? draw2<K>(a.phi_k, a, d, k, l, K) : 0.0;
        }
#pragma unroll
        for (int r = 0; r < kRowBatch; ++r) {
            if (l0 + r < a.L) {
#pragma unroll
                for (int kp = 0; kp < KP; ++kp) {
                    double v0 = v[r][2 * kp], v1 = v[r][2 * kp + 1];
                    ok = ok && in01(v0) && in01(v1);
                    if (LOG) {
                        v0 = dev_cr_log(v0);
                        v1 = dev_cr_log(v1);
                    }
                    slab[((l0 + r) * KP + kp) * 64] = make_double2(v0, v1);
                }
            }
        }
    }
    return ok;
}

template <int K>
__device__ __forceinline__ void read_table(const double2 *slab, int x, int L, double (&e)[K])
{
    constexpr int KP = (K + 1) / 2;
    /* row x (1-based, clamped) from the slab's base one row back, so the
     * state pairs sit at non-negative immediate offsets of one address */
    const int xc = min(max(x, 1), L);
    const double2 *r = (slab - KP * 64) + xc * (KP * 64);
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
        const double2 v = r[kp * 64];
        e[2 * kp] = v.x;
        if (2 * kp + 1 < K)
            e[2 * kp + 1] = v.y;
    }
}

/* Stan's scalar normal_lpdf(y | mu_j, sigma_j) with cached c0 = C - log(sigma),
 * isig = 1/sigma: ((C - log sigma) + (-0.5 * z*z)), z = (y - mu) * isig. */
template <int MODEL, int K>
__device__ __forceinline__ double gauss_lpdf(const PairParams<MODEL, K> &pp, double y, int j)
{
    const double z = (y - pp.mu[j]) * pp.isig[j];
    const double z2 = z * z;
    return pp.c0[j] + (-0.5 * z2);
}

/* Emission of one step for the linear-space filter: e[j] (probabilities,
 * Gaussian densities divided by their max m over states) and log m. */
template <int K>
struct Em {
    double e[K];
    double m;
};

/* DETEXP: the Gaussian exp is hhmm_det_exp (FFBS contract, DESIGN.md §5: the
 * filter the draws come from is bit-reproducible by the oracle). */
template <int MODEL, int K, bool DETEXP = false>
__device__ __forceinline__ void emit_prob(const PairParams<MODEL, K> &pp, const double2 *slab, int L,
                                          const Obs &o, Em<K> &em, const hhmm_exp2_entry *etab = hhmm_exp2_tab)
{
    if constexpr (ModelTraits<MODEL>::kGauss) {
        double lp[K];
        double m = dev_ninf();
#pragma unroll
        for (int j = 0; j < K; ++j) {
            lp[j] = gauss_lpdf<MODEL, K>(pp, o.xr, j);
            m = fmax(m, lp[j]);
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
            em.e[j] = DETEXP ? hhmm_det_exp_tab(lp[j] - m, etab) : exp(lp[j] - m);
        em.m = m;
    } else {
        read_table<K>(slab, o.x, L, em.e);
        em.m = 0.0;
    }
}

/* out = e_t .* (in M_t), with the model's FORWARD transition masks (semisup
 * g_t on the current state, hmm-multinom-semisup.stan:42-44; Tayal sign_t on
 * the current state, hhmm-tayal2009.stan:62-64); no renormalisation.  in may
 * alias out. */
template <int MODEL, int K, int SG = -1>
__device__ __forceinline__ void fwd_step_raw(const double (&al)[K], double (&out)[K], const PairParams<MODEL, K> &pp,
                                             const double (&e)[K], const Obs &o)
{
    double s[K];
    if constexpr (SG > 0 && ModelTraits<MODEL>::kTayal) {
        /* the sign class is known: the off columns take the row total (the
         * same additions), the on ones the same fma chain -- the same bits */
        double tot = al[0];
#pragma unroll
        for (int i = 1; i < K; ++i)
            tot += al[i];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if (tayal_on(SG, j)) {
                /* the structurally nonzero terms in the same order (a zero term
                 * 0 x f adds nothing to the chain: the same bits) */
                double acc = 0.0;
                bool first = true;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    if (tayal_nz(i, j)) {
                        acc = first ? al[i] * pp.A[i][j] : fma(al[i], pp.A[i][j], acc);
                        first = false;
                    }
                }
                s[j] = acc;
            } else {
                s[j] = tot;
            }
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
            out[j] = s[j] * e[j];
        return;
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double acc = al[0] * pp.A[0][j];
#pragma unroll
        for (int i = 1; i < K; ++i)
            acc = fma(al[i], pp.A[i][j], acc);
        s[j] = acc;
    }
    if constexpr (ModelTraits<MODEL>::kAux) {
        double tot = al[0];
#pragma unroll
        for (int i = 1; i < K; ++i)
            tot += al[i];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            bool on;
            if constexpr (ModelTraits<MODEL>::kSemisup)
                on = semisup_mask(o.aux, j);
            else
                on = tayal_pred(o.aux, j);
            s[j] = on ? s[j] : tot;
        }
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        out[j] = s[j] * e[j];
}

/* rn: renormalise after this step (every step, except the FB_BIG gamma
 * profile's every kBigRenorm-th; the flag is a compile-time constant after
 * unrolling) */
/* F(sg) with sg a std::integral_constant: the Tayal sign class of the step
 * when every lane of the wave has the same sign (readfirstlane + ballot: a
 * wave of one series under many draws, the T-scan's chunks at C5), else -1
 * (the masks per lane).  Other models: always -1. */
template <int MODEL, typename F>
__device__ __forceinline__ void tayal_dispatch(const Obs &o, bool skip_ok, F &&f)
{
    if constexpr (ModelTraits<MODEL>::kTayal) {
        const int s0 = __builtin_amdgcn_readfirstlane(o.aux);
        if (__ballot((o.aux != s0) | !skip_ok) == 0) {
            if (s0 == 1)
                f(std::integral_constant<int, 1>());
            else if (s0 == 2)
                f(std::integral_constant<int, 2>());
            else
                f(std::integral_constant<int, 3>());
            return;
        }
    }
    f(std::integral_constant<int, -1>());
}

template <int MODEL, int K>
__device__ __forceinline__ void fwd_step_to(const double (&al)[K], double (&out)[K], const PairParams<MODEL, K> &pp,
                                            const double (&e)[K], const Obs &o, int &ex, bool rn = true)
{
    tayal_dispatch<MODEL>(o, pp.skip_ok, [&](auto sgc) { fwd_step_raw<MODEL, K, decltype(sgc)::value>(al, out, pp, e, o); });
    if (rn)
        renorm<K>(out, ex);
}

template <int MODEL, int K>
__device__ __forceinline__ void fwd_step(double (&al)[K], const PairParams<MODEL, K> &pp, const double (&e)[K],
                                         const Obs &o, int &ex, bool rn = true)
{
    fwd_step_to<MODEL, K>(al, al, pp, e, o, ex, rn);
}

/* beta_{t-1} from beta_t and step t's emission / masks. */
template <int MODEL, int K, int SG>
__device__ __forceinline__ void bwd_step_sg(double (&be)[K], const PairParams<MODEL, K> &pp, const double (&e)[K],
                                            const Obs &o)
{
    double b[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        b[i] = e[i] * be[i];
    double s[K];
    double tot = 0.0;
    if constexpr (ModelTraits<MODEL>::kTayal) {
        tot = b[0];
#pragma unroll
        for (int i = 1; i < K; ++i)
            tot += b[i];
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (SG > 0 && !tayal_on(SG, j)) { /* known off: the row total alone (the same bits) */
            s[j] = tot;
            continue;
        }
        if constexpr (SG > 0 && ModelTraits<MODEL>::kTayal) {
            /* known on: row j's structurally nonzero terms in the same order */
            double acc = 0.0;
            bool first = true;
#pragma unroll
            for (int i = 0; i < K; ++i) {
                if (tayal_nz(j, i)) {
                    acc = first ? pp.A[j][i] * b[i] : fma(pp.A[j][i], b[i], acc);
                    first = false;
                }
            }
            s[j] = acc;
            continue;
        }
        double acc = pp.A[j][0] * b[0];
#pragma unroll
        for (int i = 1; i < K; ++i)
            acc = fma(pp.A[j][i], b[i], acc);
        s[j] = acc;
    }
    if constexpr (ModelTraits<MODEL>::kTayal && SG < 0) { /* predicate on the PREVIOUS state j (Q6) */
#pragma unroll
        for (int j = 0; j < K; ++j)
            s[j] = tayal_pred(o.aux, j) ? s[j] : tot;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        be[j] = s[j];
}

template <int MODEL, int K>
__device__ __forceinline__ void bwd_step(double (&be)[K], const PairParams<MODEL, K> &pp,
                                         const double (&e)[K], const Obs &o, int &ex, bool rn = true)
{
    tayal_dispatch<MODEL>(o, pp.skip_ok, [&](auto sgc) { bwd_step_sg<MODEL, K, decltype(sgc)::value>(be, pp, e, o); });
    if (rn)
        renorm<K>(be, ex);
}

/* alpha_1 (t = 0) from the step-0 observation / emission. */
template <int MODEL, int K>
__device__ __forceinline__ void fwd_init(double (&al)[K], const PairParams<MODEL, K> &pp, const Em<K> &em,
                                         const Obs &o, double &lsc, int &ex)
{
    if constexpr (ModelTraits<MODEL>::kGauss) {
        /* hmm.stan:30 -- log(p_1k) + SUM_k normal_lpdf(x[1] | mu_k, sigma_k) (Q2) */
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double z = (o.xr - pp.mu[k]) * pp.isig[k];
            const double z2 = z * z;
            s += HHMM_NEG_LOG_SQRT_TWO_PI;
            s -= pp.lsig[k];
            s += -0.5 * z2;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            al[k] = pp.p[k];
        lsc += s;
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if constexpr (ModelTraits<MODEL>::kTayal)
                al[k] = tayal_init_pred(o.aux, k) ? em.e[k] * pp.p[k] : em.e[k];
            else
                al[k] = pp.p[k] * em.e[k];
        }
    }
    renorm<K>(al, ex);
}


template <int MODEL, bool AUX>
__device__ __forceinline__ SeriesPtrs series_ptrs(const DevArgs &a, int64_t n)
{
    SeriesPtrs sp;
    sp.stride = a.N;
    sp.n = (uint32_t)n;
    sp.tmax = a.Tmax;
    sp.x = a.x;
    sp.aux = nullptr;
    if constexpr (AUX && ModelTraits<MODEL>::kSemisup)
        sp.aux = a.g;
    if constexpr (AUX && ModelTraits<MODEL>::kTayal)
        sp.aux = a.sign;
    sp.xr = a.xr;
    return sp;
}

/* ------------------------------------------------------------------ */
/* Forward / backward / posteriors                                       */
/* ------------------------------------------------------------------ */

/* Output profile of the forward-backward kernel (compile time). */
enum FbMode {
    FB_GAMMA = 0, /* loglik + gamma_tk: the hot path, no per-output branches */
    FB_FULL = 1,  /* any mix of alpha/beta/unalpha/unbeta/ungamma/gamma (+ per-step log scale) */
    FB_FWD = 2,   /* forward only: loglik / alpha / unalpha (tayal-lite, no backward output) */
    FB_FFBS = 4,  /* flag: FFBS draws in the backward sweep */
    FB_PACK = 8,  /* flag: the forward sweep packs each chunk's symbols (4 bits, L <= 16)
                   * into the checkpoint record; the backward sweep reads those
                   * instead of re-reading x (hmm-multinom: 4 B -> 1 B per step) */
    FB_BIG = 16,  /* flag (gamma profile): checkpoints every kBigChunk steps, and a
                   * two-level recompute in the backward sweep (every kGroup-th
                   * state kept, each group recomputed before it is consumed):
                   * checkpoint traffic 8 -> 4 B per step for ~1.44 forward
                   * recomputes per step instead of 1 */
    FB_RN1 = 32   /* flag (with FB_BIG): renormalise every step -- the waves whose
                   * pairs' parameters do not bound the kBigRenorm-step shrink
                   * (renorm_sparse_safe) */
};
constexpr int fb_base(int mode) { return mode & 3; }
constexpr bool fb_ffbs(int mode) { return (mode & FB_FFBS) != 0; }
constexpr bool fb_pack(int mode) { return (mode & FB_PACK) != 0; }
constexpr bool fb_big(int mode) { return (mode & FB_BIG) != 0; }
/* steps between renormalisations */
constexpr int fb_rp(int mode);
constexpr int kFwdGroup = 4;  /* forward chunks per observation prefetch group */
constexpr int kVitGroup = 2;  /* Viterbi chunks per observation prefetch group */
#ifndef HHMM_BIG_CHUNK
#define HHMM_BIG_CHUNK 16
#endif
constexpr int kBigChunk = HHMM_BIG_CHUNK; /* checkpoint interval of FB_BIG (a multiple of fb_chunk(K) = 8) */
/* Phases of one forward-backward launch: both sweeps (the default), or the
 * split schedule's two launches (HHMM_FLAG_FB_SPLIT): the forward sweep
 * (loglik, checkpoints, packed symbols) and then the backward sweep, with the
 * Viterbi decoding the packed symbols beside the latter. */
enum FbPhase { FB_PH_BOTH = 0, FB_PH_FWD = 1, FB_PH_BWD = 2 };
/* FB_BIG renormalises every kBigRenorm-th step (every checkpoint step
 * included): the max-exponent renormalisation is ~9 VALU on each step's
 * chain, and over four steps the state only shrinks by the emission x
 * transition mass, far above the subnormal range. */
#ifndef HHMM_BIG_RENORM
#define HHMM_BIG_RENORM 4
#endif
constexpr int kBigRenorm = HHMM_BIG_RENORM;
/* the gate's bound 2^-(156 / kBigRenorm) below is a shift of at most 52 bits */
static_assert(kBigRenorm >= 3 && kBigRenorm <= 8, "HHMM_BIG_RENORM must be 3..8");
constexpr int fb_rp(int mode) { return (fb_big(mode) && !(mode & FB_RN1)) ? kBigRenorm : 1; }
/* Is the kBigRenorm-step cadence safe for this pair?  Renormalisation leaves
 * the filter's max in [0.5, 1).  One forward step keeps the max at least
 * max * min_i max_j A(i,j) phi(j,x) >= max * (min_i rowmax_i) * phi_min, one
 * backward step at least max * (min_i colmax_i) * phi_min (rowmax / colmax:
 * the largest entry of row / column i of A; phi_min: the smallest emission
 * probability).  With b = phi_min * min(rowmax, colmax) >= 2^-39, kBigRenorm = 4
 * unrenormalised steps keep the max above 2^-157, so every component down to
 * 2^-865 of it stays a normal double -- far below the 1e-250 tolerance floor,
 * as with per-step renormalisation.  Pairs with a smaller b (rare symbols,
 * near-zero transitions; the reference's log space stays finite there) make
 * their wave renormalise every step (FB_RN1), the exact per-step form. */
constexpr double kRenormSafeBound = 1.0 / (double)(1ull << (156 / kBigRenorm)); /* 2^-39 at 4 steps */
template <int MODEL, int K>
__device__ __forceinline__ bool renorm_sparse_safe(const PairParams<MODEL, K> &pp, const double2 *slab, int L)
{
    static_assert(!ModelTraits<MODEL>::kGauss, "discrete emissions only");
    double tmin = 1.0 / 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double rmax = pp.A[i][0], cmax = pp.A[0][i];
#pragma unroll
        for (int j = 1; j < K; ++j) {
            rmax = fmax(rmax, pp.A[i][j]);
            cmax = fmax(cmax, pp.A[j][i]);
        }
        tmin = fmin(tmin, fmin(rmax, cmax));
    }
    double emin = 1.0 / 0.0;
    for (int l = 1; l <= L; ++l) {
        double e[K];
        read_table<K>(slab, l, L, e);
#pragma unroll
        for (int k = 0; k < K; ++k)
            emin = fmin(emin, e[k]);
    }
    return emin * tmin >= kRenormSafeBound; /* NaN: unsafe */
}
/* true when any lane of the wave is unsafe (wave-uniform) */
__device__ __forceinline__ bool wave_any(bool v)
{
    return __builtin_amdgcn_readfirstlane((int)(__ballot(v) != 0)) != 0;
}
#ifndef HHMM_BIG_GROUP
#define HHMM_BIG_GROUP 2
#endif
constexpr int kGroup = HHMM_BIG_GROUP; /* pass 1 keeps every kGroup-th state (32 steps / groups of 4 need
                               * ~300 VGPRs: occupancy 1) */


/* Writes the forward-side outputs of step t (alpha, unalpha). */
template <int K>
__device__ __forceinline__ void emit_alpha(const DevArgs &a, int64_t p, int t, const double (&al)[K], double lsc)
{
    if ((a.outputs & HHMM_OUT_ALPHA) && a.alpha) {
        const double r = 1.0 / vsum<K>(al);
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            v[k] = al[k] * r;
        store_tk<K>(a.alpha, a, p, t, v);
    }
    if ((a.outputs & HHMM_OUT_UNALPHA) && a.unalpha) {
        double v[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            v[k] = log(al[k]) + lsc;
        store_tk<K>(a.unalpha, a, p, t, v);
    }
}

/* Outputs of step t once alpha_t and beta_t are known. */
template <int K, int MODE>
__device__ __forceinline__ void emit_posteriors(const DevArgs &a, int64_t p, int t, const double (&al)[K],
                                                const double (&be)[K], double lsa, double lsb)
{
    if constexpr (fb_base(MODE) == FB_GAMMA) {
        /* gamma = (alpha .* beta) / sum: the normalisations of alpha and beta
         * cancel, one division per step (hmm.stan:89-96 up to rounding) */
        if (fb_ffbs(MODE) && !a.gamma) /* FFBS alone */
            return;
        double ug[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            ug[k] = al[k] * be[k];
        double sg = vsum<K>(ug);
        double r;
        if (__builtin_expect(sg > kGammaDirect, 1)) {
            r = fast_rcp(sg);
        } else {
            /* alpha and beta nearly disjoint (e.g. the Tayal masks of Q6 on a
             * long series): form the product from the normalised vectors as
             * the reference does, so that its underflow to 0 (and gamma = NaN)
             * happens where Stan's does */
            const double ra = 1.0 / vsum<K>(al), rb = 1.0 / vsum<K>(be);
#pragma unroll
            for (int k = 0; k < K; ++k)
                ug[k] = (al[k] * ra) * (be[k] * rb);
            sg = vsum<K>(ug);
            r = 1.0 / sg;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            ug[k] = ug[k] * r;
        store_tk<K>(a.gamma, a, p, t, ug);
    } else {
        const uint32_t o = a.outputs;
        emit_alpha<K>(a, p, t, al, lsa);
        const double sb = vsum<K>(be);
        if ((o & HHMM_OUT_BETA) && a.beta) {
            const double r = 1.0 / sb;
            double v[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                v[k] = be[k] * r;
            store_tk<K>(a.beta, a, p, t, v);
        }
        if ((o & HHMM_OUT_UNBETA) && a.unbeta) {
            /* unbeta_tk[T] = 1 (Q1): every unbeta carries +1 */
            double v[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                v[k] = (log(be[k]) + lsb) + 1.0;
            store_tk<K>(a.unbeta, a, p, t, v);
        }
        if (o & (HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA)) {
            const double ra = 1.0 / vsum<K>(al), rb = 1.0 / sb;
            double ug[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                ug[k] = (al[k] * ra) * (be[k] * rb);
            if ((o & HHMM_OUT_UNGAMMA) && a.ungamma)
                store_tk<K>(a.ungamma, a, p, t, ug);
            if ((o & HHMM_OUT_GAMMA) && a.gamma) {
                const double rg = 1.0 / vsum<K>(ug);
                double v[K];
#pragma unroll
                for (int k = 0; k < K; ++k)
                    v[k] = ug[k] * rg;
                store_tk<K>(a.gamma, a, p, t, v);
            }
        }
    }
}


/* The device entry's data check done inline by a whole-series sweep that reads
 * x anyway (HHMM_PAIR_INVALID_DATA): the running max of x - 1 as unsigned (an
 * x < 1 wraps above L), one sub and one max per symbol; steps at or past the
 * lane's own length count only on the wave's partial chunks (FULL: none). */
template <int C, bool FULL>
__device__ __forceinline__ void xcheck_acc(uint32_t &xm, const Obs (&o)[C], int c, int Tp)
{
#pragma unroll
    for (int v = 0; v < C; ++v)
        xm = max(xm, (FULL || c * C + v < Tp) ? (uint32_t)(o[v].x - 1) : 0u);
}

/* Per-lane state of the forward-backward kernel. */
template <int MODEL, int K>
struct FbLane {
    PairParams<MODEL, K> pp;
    const double2 *slab;
    int L;
    int64_t p;   /* output pair */
    int t0;      /* first step of this lane's sweep (0, or a scan chunk's start) */
    int Tp;      /* one past its last step */
    int cb;      /* t0 / C: first checkpoint row */
    int64_t q;   /* checkpoint column (the pair, or the scan lane) */
    int64_t Qs;  /* checkpoint row stride */
    bool noinit = false; /* step 0 is not the series' first (a segment window's chunk 0) */
    int64_t n = 0;       /* the series (fb_block: the inline data check's flag) */
    const hhmm_exp2_entry *etab = hhmm_exp2_tab; /* DETEXP: the LDS copy (fb_kernel) */
};

/* One forward chunk [t0, t0+C).  FULLC: every lane of the wave has all C
 * steps (no per-step predicate).  The emission of step u+1 is fetched before
 * step u is computed (LDS latency hidden behind the K^2 FMAs). */
template <int MODEL, int K, int C, int MODE, bool FULLC>
__device__ __forceinline__ void fwd_chunk(const DevArgs &a, const FbLane<MODEL, K> &ln, int c, const Obs (&cur)[C],
                                          const Obs &nxt0, Em<K> &ecur, double (&al)[K], double &lsc, int &ex)
{
    const int t0 = c * C;
#pragma unroll
    for (int u = 0; u < C; ++u) {
        const int t = t0 + u;
        Em<K> enx;
        emit_prob<MODEL, K, fb_ffbs(MODE)>(ln.pp, ln.slab, ln.L, (u + 1 < C) ? cur[u + 1 < C ? u + 1 : 0] : nxt0,
                                           enx, ln.etab);
        if (FULLC || t < ln.Tp) {
            if (u == 0 && c == 0 && !ln.noinit) {
                fwd_init<MODEL, K>(al, ln.pp, ecur, cur[0], lsc, ex);
            } else {
                lsc += ecur.m;
                fwd_step<MODEL, K>(al, ln.pp, ecur.e, cur[u], ex, u % fb_rp(MODE) == 0);
            }
            if constexpr (fb_base(MODE) == FB_FWD) {
                emit_alpha<K>(a, ln.p, t, al, lsc + kLn2 * ex);
            } else if (u == 0 && (!fb_big(MODE) || (c - ln.cb) % (kBigChunk / C) == 0)) {
                /* checkpoint row: one per C-chunk, or one per kBigChunk steps (FB_BIG) */
                const int64_t row = fb_big(MODE) ? (c - ln.cb) / (kBigChunk / C) : (c - ln.cb);
#pragma unroll
                for (int k = 0; k < K; ++k)
                    put_tmp(a.ckpt + ln.Qs * (row * K + k), (uint32_t)ln.q * 8u, al[k]);
                if constexpr (fb_base(MODE) == FB_FULL)
                    put_tmp(a.ckpt_ls + ln.Qs * (int64_t)(c - ln.cb), (uint32_t)ln.q * 8u, lsc + kLn2 * ex);
            }
            if (fb_pack(MODE) && u == 0) {
                /* the chunk's C <= 8 symbols, 4 bits each, for the backward sweep */
                uint32_t w = 0;
#pragma unroll
                for (int v = 0; v < C; ++v)
                    w |= ((uint32_t)(cur[v].x - 1) & 15u) << (4 * v);
                at(a.xpk + ln.Qs * (int64_t)(c - ln.cb), (uint32_t)ln.q * 4u) = w;
            }
        }
        ecur = enx;
    }
}

/* FFBS draw of step t (oracle ffbs_contract): z_{T-1} ~ cat(f_{T-1}),
 * z_t ~ cat(f_t(i) * A(i, z_{t+1})) -- or f_t(i) where the model's forward mask
 * switches the transition off at (t+1, z_{t+1}).  z is 0-based, -1 = undefined. */
template <int MODEL, int K>
__device__ __forceinline__ int ffbs_draw(const PairParams<MODEL, K> &pp, const double (&f)[K], bool last,
                                         const Obs &onext, int z, double u)
{
    double w[K];
    if (last) {
#pragma unroll
        for (int i = 0; i < K; ++i)
            w[i] = f[i];
    } else {
        if (z < 0)
            return -1;
        bool on = true;
        if constexpr (ModelTraits<MODEL>::kSemisup)
            on = semisup_mask(onext.aux, z);
        if constexpr (ModelTraits<MODEL>::kTayal)
            on = tayal_pred(onext.aux, z);
#pragma unroll
        for (int i = 0; i < K; ++i) {
            double az = pp.A[i][0];
#pragma unroll
            for (int j = 1; j < K; ++j)
                az = (z == j) ? pp.A[i][j] : az;
            w[i] = on ? f[i] * az : f[i];
        }
    }
    return ffbs_cat<K>(w, u);
}

/* One backward chunk: recompute alpha over the chunk from its checkpoint,
 * then walk t = t0+C-1 .. t0 emitting the posteriors and stepping beta
 * (and drawing the FFBS state from the recomputed, bit-identical filter). */
template <int MODEL, int K, int C, int MODE, bool FULLC>
__device__ __forceinline__ void bwd_chunk(const DevArgs &a, const FbLane<MODEL, K> &ln, int c, const Obs (&cur)[C],
                                          const double (&ck)[K], double ck_ls, double (&be)[K], double &blsc,
                                          int &bex, const double (&uu)[fb_ffbs(MODE) ? C : 1], const Obs &onext,
                                          int &z)
{
    constexpr bool DETEXP = fb_ffbs(MODE);
    const int t0 = c * C;
    double abuf[C][K];
    double lsbuf[fb_base(MODE) == FB_FULL ? C : 1];
#pragma unroll
    for (int k = 0; k < K; ++k)
        abuf[0][k] = ck[k];
    lsbuf[0] = ck_ls;
    {
        double lsacc = 0.0;
        int exb = 0;
        Em<K> ecur;
        emit_prob<MODEL, K, DETEXP>(ln.pp, ln.slab, ln.L, cur[1 < C ? 1 : 0], ecur, ln.etab);
#pragma unroll
        for (int u = 1; u < C; ++u) {
            Em<K> enx;
            emit_prob<MODEL, K, DETEXP>(ln.pp, ln.slab, ln.L, cur[u + 1 < C ? u + 1 : u], enx, ln.etab);
            if (FULLC || t0 + u < ln.Tp) {
                lsacc += ecur.m;
                fwd_step_to<MODEL, K>(abuf[u - 1], abuf[u], ln.pp, ecur.e, cur[u], exb);
            }
            if constexpr (fb_base(MODE) == FB_FULL)
                lsbuf[u] = ck_ls + (lsacc + kLn2 * exb);
            ecur = enx;
        }
    }
    Em<K> ecur;
    emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, cur[C - 1], ecur);
#pragma unroll
    for (int u = C - 1; u >= 0; --u) {
        const int t = t0 + u;
        Em<K> enx;
        emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, cur[u > 0 ? u - 1 : 0], enx);
        if (FULLC || t < ln.Tp) {
            emit_posteriors<K, MODE>(a, ln.p, t, abuf[u], be, lsbuf[fb_base(MODE) == FB_FULL ? u : 0],
                                     blsc + kLn2 * bex);
            if constexpr (fb_ffbs(MODE)) {
                z = ffbs_draw<MODEL, K>(ln.pp, abuf[u], t == ln.Tp - 1, (u + 1 < C) ? cur[u + 1 < C ? u + 1 : u] : onext,
                                        z, uu[u]);
                at(a.z_ffbs + a.P * (int64_t)t, (uint32_t)ln.p * 4u) = z + 1;
            }
            if (t > ln.t0) {
                if constexpr (fb_base(MODE) == FB_FULL)
                    blsc += ecur.m;
                bwd_step<MODEL, K>(be, ln.pp, ecur.e, cur[u], bex);
            }
        }
        ecur = enx;
    }
}

/* FB_BIG applies to hmm-multinom's packed gamma profile with 8-step chunks. */
template <int MODEL, int K>
constexpr bool fb_big_ok()
{
    return MODEL == HHMM_MODEL_HMM_MULTINOM && fb_chunk(K) == 8;
}

/* Observation u of a kBigChunk-step block from its packed words (FB_PACK). */
__device__ __forceinline__ Obs unpack_obs(const uint32_t (&w)[kBigChunk / 8], int u)
{
    Obs o;
    o.x = (int)((w[u >> 3] >> (4 * (u & 7))) & 15u) + 1;
    o.aux = 0;
    o.xr = 0.0;
    return o;
}

/* One kBigChunk-step block of the FB_BIG backward sweep: pass 1 recomputes
 * the block's forward states from its checkpoint keeping every kGroup-th;
 * pass 2 takes the groups from the end, recomputes each group's states and
 * walks it backwards (posteriors, beta step). */
template <int MODEL, int K, int MODE, bool FULLB>
__device__ __forceinline__ void bwd_block_big(const DevArgs &a, const FbLane<MODEL, K> &ln, int t0,
                                              const uint32_t (&w)[kBigChunk / 8], const double (&ck)[K],
                                              double (&be)[K], int &bex)
{
    constexpr int B = kBigChunk, G = kGroup, NG = B / G;
    double ga[NG][K];
    double al[K];
    int exb = 0;
#pragma unroll
    for (int k = 0; k < K; ++k)
        al[k] = ga[0][k] = ck[k];
    /* pass 1; each step's emission row is fetched one step ahead, and a
     * scheduling barrier per step keeps the compiler from hoisting every
     * LDS read of the unrolled block into registers at once */
    Em<K> ecur, enx;
    emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, unpack_obs(w, 1), ecur);
#pragma unroll
    for (int u = 1; u < B; ++u) {
        if (u + 1 < B)
            emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, unpack_obs(w, u + 1 < B ? u + 1 : u), enx);
        if (FULLB || t0 + u < ln.Tp)
            fwd_step<MODEL, K>(al, ln.pp, ecur.e, unpack_obs(w, u), exb, u % fb_rp(MODE) == 0);
        if (u % G == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                ga[u / G][k] = al[k];
        }
        ecur = enx;
        __builtin_amdgcn_sched_barrier(0);
    }
    /* pass 2: emission rows re-read from LDS one step ahead (keeping a
     * group's rows in registers would cost 40 VGPRs) */
#pragma unroll
    for (int g = NG - 1; g >= 0; --g) {
        double gb[G][K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            gb[0][k] = ga[g][k];
        Em<K> e1, e2;
        emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, unpack_obs(w, g * G + 1), e1);
#pragma unroll
        for (int r = 1; r < G; ++r) {
            const int u = g * G + r;
            /* next: the following recompute step, or (after the last) the group's last step again */
            emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, unpack_obs(w, r + 1 < G ? u + 1 : g * G + G - 1), e2);
            if (FULLB || t0 + u < ln.Tp)
                fwd_step_to<MODEL, K>(gb[r - 1], gb[r], ln.pp, e1.e, unpack_obs(w, u), exb, u % fb_rp(MODE) == 0);
            e1 = e2;
        }
        /* e1 = emission of step g*G + G-1 */
#pragma unroll
        for (int r = G - 1; r >= 0; --r) {
            const int u = g * G + r;
            const int t = t0 + u;
            if (r > 0)
                emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, unpack_obs(w, r > 0 ? u - 1 : u), e2);
            if (FULLB || t < ln.Tp) {
                emit_posteriors<K, MODE>(a, ln.p, t, gb[r], be, 0.0, 0.0);
                if (t > ln.t0)
                    bwd_step<MODEL, K>(be, ln.pp, e1.e, unpack_obs(w, u), bex, u % fb_rp(MODE) == 0);
            }
            e1 = e2;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

/* FB_BIG backward sweep (gamma profile, packed symbols): kBigChunk-step
 * blocks from the end, each block's checkpoint and packed words prefetched
 * one block ahead. */
template <int MODEL, int K, int MODE>
__device__ __forceinline__ void fb_backward_big(const DevArgs &a, const FbLane<MODEL, K> &ln, int Tw_min, int Tw_max,
                                                double (&be)[K], int &bex)
{
    static_assert(fb_pack(MODE) && fb_base(MODE) == FB_GAMMA && !fb_ffbs(MODE), "FB_BIG: packed gamma profile");
    constexpr int B = kBigChunk, C = fb_chunk(K), NW = B / 8;
    static_assert(C == 8, "FB_BIG packs 8-step chunks");
    const int nblk = (Tw_max + B - 1) / B;
    const int nfullb = Tw_min / B;
    auto load_blk = [&](int blk, double (&ck)[K], uint32_t (&w)[NW]) {
        const int bb = max(blk, 0);
#pragma unroll
        for (int k = 0; k < K; ++k)
            ck[k] = get_tmp(a.ckpt + ln.Qs * ((int64_t)bb * K + k), (uint32_t)ln.q * 8u);
#pragma unroll
        for (int i = 0; i < NW; ++i)
            w[i] = at(a.xpk + ln.Qs * (int64_t)(bb * NW + i), (uint32_t)ln.q * 4u);
    };
    double ck[K], ckn[K];
    uint32_t w[NW], wn[NW];
    load_blk(nblk - 1, ck, w);
    for (int blk = nblk - 1; blk >= 0; --blk) {
        load_blk(blk - 1, ckn, wn);
        if (blk < nfullb)
            bwd_block_big<MODEL, K, MODE, true>(a, ln, blk * B, w, ck, be, bex);
        else
            bwd_block_big<MODEL, K, MODE, false>(a, ln, blk * B, w, ck, be, bex);
#pragma unroll
        for (int k = 0; k < K; ++k)
            ck[k] = ckn[k];
#pragma unroll
        for (int i = 0; i < NW; ++i)
            w[i] = wn[i];
    }
}

/* The forward-backward sweep of one lane over [ln.t0, ln.Tp): a whole series
 * (fb_kernel) or one T-chunk of the parallel scan (fb_scan_kernel, SURVEY §8
 * A16), which enters with the boundary vectors the scan computed: al = the
 * forward state f_{t0-1} (ignored at t0 = 0, where the model's init runs),
 * be = beta at the chunk's last step, with their log scales. */
template <int MODEL, int K, int MODE, bool SCAN, int PH = FB_PH_BOTH>
__device__ __forceinline__ void fb_sweep(const DevArgs &a, const FbLane<MODEL, K> &ln, const SeriesPtrs &sp,
                                         double (&al)[K], double lsc, double (&be)[K], double blsc)
{
    static_assert(PH == FB_PH_BOTH || (fb_big(MODE) && !SCAN), "split sweeps: FB_BIG gamma profile only");
    constexpr int C = fb_chunk(K);
    constexpr bool AUX = ModelTraits<MODEL>::kAux;
    const int64_t p = ln.p;
    const int Tw_min = wave_min(ln.Tp);
    const int Tw_max = wave_max(ln.Tp);
    const int nfull = Tw_min / C;              /* chunks complete for every lane */
    const int nchunk = (Tw_max + C - 1) / C;   /* chunks any lane needs */
    const int cb = ln.cb;

    Obs cur[C];
    if constexpr (PH != FB_PH_BWD) {
    /* ---- forward sweep ---- */
    int ex = 0;       /* sum of binary exponents removed */
    /* Full chunks go kFwdGroup at a time with the next group's observations
     * in flight: one chunk of forward steps (~40 VALU each) is far shorter
     * than an HBM round trip under load, so a one-chunk prefetch stalled
     * every chunk (the forward sweep alone measured 2.6 ms at C2 against
     * ~0.9 ms of issue).  The last, partial chunks keep the one-ahead loop. */
    constexpr int D = kFwdGroup;
    Obs grp[D][C];
#pragma unroll
    for (int i = 0; i < D; ++i)
        load_chunk<MODEL, C, AUX>(grp[i], sp, (cb + i) * C);
    Em<K> ecur;
    emit_prob<MODEL, K, fb_ffbs(MODE)>(ln.pp, ln.slab, ln.L, grp[0][0], ecur, ln.etab);
    /* whole-series sweeps over x alone check it inline (xcheck_acc) */
    constexpr bool XCHK = !SCAN && !AUX && ModelTraits<MODEL>::kDiscrete;
    uint32_t xm = 0;
    int c = cb;
    for (; c + D <= nfull; c += D) {
        Obs nxt[D][C];
#pragma unroll
        for (int i = 0; i < D; ++i)
            load_chunk<MODEL, C, AUX>(nxt[i], sp, (c + D + i) * C);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            fwd_chunk<MODEL, K, C, MODE, true>(a, ln, c + i, grp[i], (i + 1 < D) ? grp[i + 1 < D ? i + 1 : 0][0]
                                                                              : nxt[0][0], ecur, al, lsc, ex);
            if constexpr (XCHK)
                xcheck_acc<C, true>(xm, grp[i], c + i, ln.Tp);
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int u = 0; u < C; ++u)
                grp[i][u] = nxt[i][u];
    }
#pragma unroll
    for (int u = 0; u < C; ++u)
        cur[u] = grp[0][u];
    for (; c < nchunk; ++c) { /* < D full chunks, then the partial ones (one code copy) */
        Obs nxt[C];
        load_chunk<MODEL, C, AUX>(nxt, sp, (c + 1) * C);
        fwd_chunk<MODEL, K, C, MODE, false>(a, ln, c, cur, nxt[0], ecur, al, lsc, ex);
        if constexpr (XCHK)
            xcheck_acc<C, false>(xm, cur, c, ln.Tp);
#pragma unroll
        for (int u = 0; u < C; ++u)
            cur[u] = nxt[u];
    }
    if constexpr (XCHK)
        if (a.dc_flag && xm >= (uint32_t)ln.L)
            a.dc_flag[ln.n] = 1;
    if (!SCAN && (a.outputs & HHMM_OUT_LOGLIK) && a.loglik)
        a.loglik[p] = log(vsum<K>(al)) + (lsc + kLn2 * ex);
    } /* forward sweep */
    if constexpr (fb_base(MODE) == FB_FWD || PH == FB_PH_FWD)
        return;

    /* ---- backward sweep, chunk by chunk from the end ---- */
    int bex = 0;
    if constexpr (fb_big(MODE)) {
        fb_backward_big<MODEL, K, MODE>(a, ln, Tw_min, Tw_max, be, bex);
        return;
    }
    const int clast = nchunk - 1;
    /* observations of chunk cc: x itself, or the packed record of the forward sweep */
    auto obs_chunk = [&](Obs (&dst)[C], int cc) {
        if constexpr (fb_pack(MODE)) {
            const uint32_t w = at(a.xpk + ln.Qs * (int64_t)(max(cc, cb) - cb), (uint32_t)ln.q * 4u);
#pragma unroll
            for (int v = 0; v < C; ++v) {
                dst[v].x = (int)((w >> (4 * v)) & 15u) + 1;
                dst[v].aux = 0;
                dst[v].xr = 0.0;
            }
        } else {
            load_chunk<MODEL, C, AUX>(dst, sp, cc * C);
        }
    };
    obs_chunk(cur, clast);
    /* checkpoint rows are wave-uniform: a lane shorter than the wave reads
     * (unused) slots past its own last chunk, never past the allocation */
    double ck[K], ck_ls = 0.0;
    {
        const int cc = clast - cb;
#pragma unroll
        for (int k = 0; k < K; ++k)
            ck[k] = get_tmp(a.ckpt + ln.Qs * ((int64_t)cc * K + k), (uint32_t)ln.q * 8u);
        if constexpr (fb_base(MODE) == FB_FULL)
            ck_ls = get_tmp(a.ckpt_ls + ln.Qs * (int64_t)cc, (uint32_t)ln.q * 8u);
    }
    /* FFBS: the caller's uniforms, prefetched one chunk ahead like the observations */
    double uu[fb_ffbs(MODE) ? C : 1], un[fb_ffbs(MODE) ? C : 1];
    if constexpr (fb_ffbs(MODE)) {
#pragma unroll
        for (int u = 0; u < C; ++u)
            uu[u] = at(a.ffbs_u + a.P * (int64_t)min(clast * C + u, a.Tmax - 1), (uint32_t)p * 8u);
    }
    Obs onext = cur[0];
    int z = -1;
    for (int c = clast; c >= cb; --c) {
        Obs nxt[C];
        obs_chunk(nxt, c - 1);
        if constexpr (fb_ffbs(MODE)) {
#pragma unroll
            for (int u = 0; u < C; ++u)
                un[u] = at(a.ffbs_u + a.P * (int64_t)max((c - 1) * C + u, 0), (uint32_t)p * 8u);
        }
        double cn[K], cn_ls = 0.0;
        {
            const int cc = max(c - 1, cb) - cb;
#pragma unroll
            for (int k = 0; k < K; ++k)
                cn[k] = get_tmp(a.ckpt + ln.Qs * ((int64_t)cc * K + k), (uint32_t)ln.q * 8u);
            if constexpr (fb_base(MODE) == FB_FULL)
                cn_ls = get_tmp(a.ckpt_ls + ln.Qs * (int64_t)cc, (uint32_t)ln.q * 8u);
        }
        if (c < nfull)
            bwd_chunk<MODEL, K, C, MODE, true>(a, ln, c, cur, ck, ck_ls, be, blsc, bex, uu, onext, z);
        else
            bwd_chunk<MODEL, K, C, MODE, false>(a, ln, c, cur, ck, ck_ls, be, blsc, bex, uu, onext, z);
        onext = cur[0];
#pragma unroll
        for (int u = 0; u < C; ++u)
            cur[u] = nxt[u];
        if constexpr (fb_ffbs(MODE)) {
#pragma unroll
            for (int u = 0; u < C; ++u)
                uu[u] = un[u];
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            ck[k] = cn[k];
        ck_ls = cn_ls;
    }
}

/* One wave of the forward-backward: pairs [64 gwave, 64 gwave + 64) (gwave =
 * block * waves per block + wave in fb_kernel). */
template <int MODEL, int K, int MODE, int PH>
__device__ __forceinline__ void fb_block(const DevArgs &a, int64_t gwave, const hhmm_exp2_entry *etab = hhmm_exp2_tab)
{
    constexpr bool AUX = ModelTraits<MODEL>::kAux;
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    /* lanes past the last pair redo pair P-1 (identical values, benign
     * duplicate stores): every lane stays in the wave-wide reductions */
    const int64_t p = min(gwave * 64 + lane, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    constexpr int KP = (K + 1) / 2;

    FbLane<MODEL, K> ln;
    ln.p = p;
    ln.n = n;
    ln.L = a.L;
    ln.t0 = 0;
    ln.Tp = pair_len(a, n);
    ln.cb = 0;
    ln.q = p;
    ln.Qs = a.P;
    ln.slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    ln.etab = etab;
    load_params<MODEL, K, false>(ln.pp, a, d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        ln.pp.skip_ok &= fill_table<K, false>(lds + (size_t)wave * a.L * KP * 64 + lane, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, AUX>(a, n);
    double al[K], be[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        al[k] = 0.0;
        be[k] = 1.0; /* unbeta_tk[T] = 1 (Q1): beta_T uniform */
    }
    if constexpr (fb_big(MODE) && !(MODE & FB_RN1)) {
        const bool dense = wave_any(!renorm_sparse_safe<MODEL, K>(ln.pp, ln.slab, a.L));
        if constexpr (PH == FB_PH_BOTH) {
            /* a wave holding a pair without the bound appends itself to the
             * list a.rnw (count, then wave ids) and leaves its sweep to
             * fb_dense_kernel (per-step renormalisation), launched right after
             * this kernel: the hot kernel carries one copy of the sweep */
            if (dense) {
                if (lane == 0) {
                    const int slot = atomicAdd(&a.rnw[0], 1);
                    a.rnw[1 + slot] = (int32_t)gwave;
                }
                return;
            }
        } else if (dense) { /* the split schedule's two launches decide alike */
            fb_sweep<MODEL, K, MODE | FB_RN1, false, PH>(a, ln, sp, al, 0.0, be, 0.0);
            return;
        }
    }
    fb_sweep<MODEL, K, MODE, false, PH>(a, ln, sp, al, 0.0, be, 0.0);
}

/* The FB_BIG waves fb_kernel listed in a.rnw, with per-step renormalisation:
 * one-wave workgroups (one emission slab each) take list entries in turn;
 * with none listed the launch reads the count and ends. */
constexpr int kDenseBlocks = 256;
template <int MODEL, int K, int MODE>
__global__ void __launch_bounds__(64) fb_dense_kernel(const DevArgs a)
{
    const int n = __builtin_amdgcn_readfirstlane(a.rnw[0]);
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const int64_t gw = __builtin_amdgcn_readfirstlane(a.rnw[1 + i]);
        fb_block<MODEL, K, MODE | FB_RN1, FB_PH_BOTH>(a, gw);
    }
}

/* fb_exp2_lds: the FFBS contract's Gaussian exps (DETEXP) read their 2^(j/128)
 * table from an LDS copy -- the Gaussian models have no emission slab, so the
 * copy sits at the start of the launch's LDS (launch_fb sizes it) */
template <int MODEL, int MODE>
constexpr bool fb_exp2_lds() { return ModelTraits<MODEL>::kGauss && fb_ffbs(MODE); }
constexpr size_t kExp2TabBytes = 128 * sizeof(hhmm_exp2_entry);

template <int MODEL, int K, int MODE, int PH = FB_PH_BOTH>
__global__ void __launch_bounds__(kBlock) fb_kernel(const DevArgs a)
{
    const hhmm_exp2_entry *etab = hhmm_exp2_tab;
    if constexpr (fb_exp2_lds<MODEL, MODE>()) {
        HIP_DYNAMIC_SHARED(hhmm_exp2_entry, t)
        for (int i = threadIdx.x; i < 128; i += blockDim.x)
            t[i] = hhmm_exp2_tab[i];
        __syncthreads();
        etab = t;
    }
    fb_block<MODEL, K, MODE, PH>(a, (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), etab);
}

/* ------------------------------------------------------------------ */
/* Viterbi                                                                */
/* ------------------------------------------------------------------ */

/* Log emission of state j at one step, bit-identical to the reference. */
template <int MODEL, int K>
__device__ __forceinline__ void emit_log(const PairParams<MODEL, K> &pp, const double2 *slab, int L,
                                         const Obs &o, double (&le)[K])
{
    if constexpr (ModelTraits<MODEL>::kGauss) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            le[j] = gauss_lpdf<MODEL, K>(pp, o.xr, j);
    } else {
        read_table<K>(slab, o.x, L, le);
    }
}


/* One max-plus step t >= 1: delta_t(j) = max_i cand(i, j) with the
 * reference's strict '>' from -inf (first maximising i wins, NaN never
 * wins); back-pointer i packed into `word` at `slot`.
 * VALU form: the running max is one v_max_f64 (maxNum: a NaN candidate
 * leaves it unchanged, and an equal one leaves its value unchanged) and the
 * back-pointer one select on the strict compare, so each candidate costs
 * 2 adds + cmp + max + select.  Value-identical to the reference loop; the
 * back-pointer differs only where every candidate is -inf / NaN (the
 * reference leaves it unset, here 0), which the epilogue flags through
 * delta_T = -inf exactly as before. */
template <int MODEL, int K, bool NANIN = false>
__device__ __forceinline__ void vit_step(double (&dl)[K], const PairParams<MODEL, K> &pp, const double (&le)[K],
                                         const Obs &o, uint32_t &word, int slot)
{
    /* NANIN: delta_{t-1} may hold NaN -- only the step after the t = 1 row of
     * Q3.  Every later delta is a max over candidates that include a non-NaN
     * one (state K's row at t = 2, then every state), so the running max can
     * start from the first candidate instead of from fmax(-inf, candidate). */
    constexpr int BITS = bp_bits(K);
    constexpr int STEPB = K * BITS;
    double nd[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        bool on = true;
        if constexpr (ModelTraits<MODEL>::kTayal)
            on = tayal_pred(o.aux, j);
        const int sh = slot * STEPB + j * BITS;
        double best = dev_ninf();
        uint32_t argsh = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            double cand;
            if constexpr (ModelTraits<MODEL>::kTayal) {
                /* (delta + log phi) [+ log A] (hhmm-tayal2009.stan:143-146) */
                cand = dl[i] + le[j];
                cand = on ? cand + pp.A[i][j] : cand;
            } else {
                /* (delta + log A) + emission (hmm.stan:111) */
                cand = (dl[i] + pp.A[i][j]) + le[j];
            }
            if (i == 0) {
                best = NANIN ? fmax(best, cand) : cand;
            } else {
                const bool gt = cand > best;
                best = fmax(best, cand);
                argsh = gt ? ((uint32_t)i << sh) : argsh;
            }
        }
        nd[j] = best;
        word |= argsh;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        dl[j] = nd[j];
}

template <int MODEL, int K, int CV, bool FULLC, bool FIRST = false>
__device__ __forceinline__ void vit_fwd_chunk(const DevArgs &a, int64_t p, const PairParams<MODEL, K> &pp,
                                              const double2 *slab, int Tp, int c, const Obs (&cur)[CV],
                                              const Obs &nxt0, double (&le)[K], double (&dl)[K], uint32_t &word)
{
    constexpr int SPW = bp_steps_per_word(K);
    const int t0 = c * CV;
#pragma unroll
    for (int u = 0; u < CV; ++u) {
        const int t = t0 + u;
        double ln[K];
        emit_log<MODEL, K>(pp, slab, a.L, (u + 1 < CV) ? cur[u + 1 < CV ? u + 1 : 0] : nxt0, ln);
        if (FULLC || t < Tp) {
            /* FIRST: chunk 0, whose step 0 is the init row and step 1 the NaN step */
            if (FIRST && u == 1)
                vit_step<MODEL, K, true>(dl, pp, le, cur[u], word, u % SPW);
            else if (!(FIRST && u == 0))
                vit_step<MODEL, K, false>(dl, pp, le, cur[u], word, u % SPW);
            if (u % SPW == SPW - 1) {
                put_tmp(a.bp + a.P * (int64_t)(t / SPW), (uint32_t)p * 4u, word);
                word = 0;
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            le[k] = ln[k];
    }
}

/* One workgroup of the Viterbi decoder: pairs [block * blockDim, +blockDim).
 * PK: the observations come from the packed symbol words the split
 * schedule's forward launch wrote (a.xpk: one 4-bit symbol per step, one word
 * per 8-step chunk; hmm-multinom, L <= 16), 0.5 instead of 4 bytes per step. */
template <int MODEL, int K, bool PK = false>
__device__ __forceinline__ void viterbi_block(const DevArgs &a, uint32_t block)
{
    constexpr int CV = vit_chunk(K);
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal; /* semisup Viterbi is unmasked (Q7) */
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t p = min((int64_t)block * blockDim.x + threadIdx.x, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    constexpr int KP = (K + 1) / 2;
    double2 *slab = lds + (size_t)wave * a.L * KP * 64 + lane;

    PairParams<MODEL, K> pp;
    load_params<MODEL, K, true>(pp, a, d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        fill_table<K, true>(slab, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, n);
    static_assert(!PK || (!VAUX && !ModelTraits<MODEL>::kGauss && CV == 8), "packed symbols: 8-step chunks, x only");
    const int pkrows = (a.Tmax + CV - 1) / CV;
    auto vload = [&](Obs (&dst)[CV], const SeriesPtrs &s, int t0) {
        if constexpr (PK) {
            /* rows past a lane's own length hold padding that is never consumed */
            const int cc = min(max(t0 / CV, 0), pkrows - 1);
            const uint32_t w = at(a.xpk + a.P * (int64_t)cc, (uint32_t)p * 4u);
#pragma unroll
            for (int v = 0; v < CV; ++v) {
                dst[v].x = (int)((w >> (4 * v)) & 15u) + 1;
                dst[v].aux = 0;
                dst[v].xr = 0.0;
            }
        } else {
            load_chunk<MODEL, CV, VAUX>(dst, s, t0);
        }
    };
    const int Tw_min = wave_min(Tp);
    const int Tw_max = wave_max(Tp);
    const int nfull = Tw_min / CV;
    const int nchunk = (Tw_max + CV - 1) / CV;

    /* delta_tk[1, K] = emission of j for j = 1..K: only column K is written,
     * the others keep stanc's NaN (Q3, e.g. hmm-multinom.stan:105-106). */
    double dl[K];
    Obs cur[CV];
    vload(cur, sp, 0);
    /* chunks 1.. go kVitGroup at a time with the next group's observations in
     * flight (a one-chunk prefetch is shorter than an HBM round trip) */
    constexpr int D = kVitGroup;
    Obs grp[D][CV];
#pragma unroll
    for (int i = 0; i < D; ++i)
        vload(grp[i], sp, (1 + i) * CV);
    double le[K];
    emit_log<MODEL, K>(pp, slab, a.L, cur[0], le);
#pragma unroll
    for (int k = 0; k < K - 1; ++k)
        dl[k] = dev_nan();
    dl[K - 1] = le[K - 1];
    uint32_t word = 0;
    /* chunk 0: the t = 1 row and the NaN step (Q3) */
    vit_fwd_chunk<MODEL, K, CV, false, true>(a, p, pp, slab, Tp, 0, cur, grp[0][0], le, dl, word);
    /* decoding x itself: the data check inline (xcheck_acc) */
    constexpr bool XCHK = !PK && !ModelTraits<MODEL>::kAux && ModelTraits<MODEL>::kDiscrete;
    uint32_t xm = 0;
    if constexpr (XCHK)
        xcheck_acc<CV, false>(xm, cur, 0, Tp);
    int c = 1;
    for (; c + D <= nfull; c += D) {
        Obs nxt[D][CV];
#pragma unroll
        for (int i = 0; i < D; ++i)
            vload(nxt[i], sp, (c + D + i) * CV);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            vit_fwd_chunk<MODEL, K, CV, true>(a, p, pp, slab, Tp, c + i, grp[i],
                                              (i + 1 < D) ? grp[i + 1 < D ? i + 1 : 0][0] : nxt[0][0], le, dl, word);
            if constexpr (XCHK)
                xcheck_acc<CV, true>(xm, grp[i], c + i, Tp);
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int u = 0; u < CV; ++u)
                grp[i][u] = nxt[i][u];
    }
#pragma unroll
    for (int u = 0; u < CV; ++u)
        cur[u] = grp[0][u];
    for (; c < nchunk; ++c) { /* < D full chunks, then the partial ones (one code copy) */
        Obs nxt[CV];
        vload(nxt, sp, (c + 1) * CV);
        vit_fwd_chunk<MODEL, K, CV, false>(a, p, pp, slab, Tp, c, cur, nxt[0], le, dl, word);
        if constexpr (XCHK)
            xcheck_acc<CV, false>(xm, cur, c, Tp);
#pragma unroll
        for (int u = 0; u < CV; ++u)
            cur[u] = nxt[u];
    }
    if constexpr (XCHK)
        if (a.dc_flag && xm >= (uint32_t)a.L)
            a.dc_flag[n] = 1;
    viterbi_epilogue<K>(a, p, Tp, Tw_min, Tw_max, dl, word);
}

template <int MODEL, int K, bool PK = false>
__global__ void __launch_bounds__(kBlock) viterbi_kernel(const DevArgs a)
{
    if constexpr (!PK || (fb_big_ok<MODEL, K>() && vit_chunk(K) == 8))
        viterbi_block<MODEL, K, PK>(a, blockIdx.x);
}

/* ---- fused forward-backward + Viterbi (C2's profile) -------------------- *
 * One lane, one pair, ONE pass over the observations for both halves of the
 * hot path (hmm-multinom.stan:27-132): the forward sweep runs the scaled
 * linear-space filter (fwd_chunk) and the max-plus recursion (vit_fwd_chunk)
 * on the same observation registers, so x crosses HBM once instead of twice;
 * the backward sweep (FB_BIG blocks of kBigChunk steps) emits gamma and
 * backtracks the path over the same blocks, so the back-pointer words ride
 * the checkpoint prefetch.  Both emission tables (phi and log phi, K*L
 * doubles each) sit in the wave's LDS slab, which holds the kernel at one
 * wave per SIMD; both halves produce exactly what fb_kernel and
 * viterbi_kernel produce (same functions, same operation order).
 * K = 4 (fb_chunk = vit_chunk = 8, two back-pointer words per chunk).
 * Measured: 11.3 ms at C2 against 10.4 ms for the two concurrent kernels --
 * every wave runs the VALU-bound forward half and then the HBM-bound backward
 * half in lockstep with the others, so the pipes take turns instead of
 * overlapping -- hence opt-in (HHMM_FLAG_FUSED). */
template <int MODEL, int K>
constexpr bool fbv_ok()
{
    return fb_big_ok<MODEL, K>() && vit_chunk(K) == fb_chunk(K);
}

/* FB_BIG backward sweep and the Viterbi backtrack over the same kBigChunk-step
 * blocks from the end (fbv_kernel, vfb_kernel): gamma from the recomputed
 * filter and beta, the path from the back-pointer words, which ride the
 * checkpoint prefetch.  z = zstar_T (0-based); invalid: the path is all zeros
 * (pair flagged, the walk is discarded). */
template <int MODEL, int K, int MODE>
__device__ __forceinline__ void fbv_backward(const DevArgs &a, const FbLane<MODEL, K> &ln, int Tw_min, int Tw_max,
                                             int z, bool invalid, bool want_z)
{
    constexpr int C = fb_chunk(K);
    constexpr int SPW = bp_steps_per_word(K);
    constexpr int WPC = C / SPW;
    constexpr int B = kBigChunk, NW = B / 8, CPB = B / C; /* chunks per block */
    const int64_t p = ln.p;
    const int Tp = ln.Tp;
    const int nfull = Tw_min / C;
    double be[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        be[k] = 1.0; /* unbeta_tk[T] = 1 (Q1) */
    int bex = 0;
    const int nblk = (Tw_max + B - 1) / B;
    const int nfullb = Tw_min / B;
    const int wmax = a.Tmax / SPW;
    auto load_blk = [&](int blk, double (&ck)[K], uint32_t (&w)[NW], uint32_t (&bw)[CPB * WPC]) {
        const int bb = max(blk, 0);
#pragma unroll
        for (int k = 0; k < K; ++k)
            ck[k] = get_tmp(a.ckpt + ln.Qs * ((int64_t)bb * K + k), (uint32_t)p * 8u);
#pragma unroll
        for (int i = 0; i < NW; ++i)
            w[i] = at(a.xpk + ln.Qs * (int64_t)(bb * NW + i), (uint32_t)p * 4u);
#pragma unroll
        for (int i = 0; i < CPB * WPC; ++i)
            bw[i] = get_tmp(a.bp + a.P * (int64_t)min(bb * CPB * WPC + i, wmax), (uint32_t)p * 4u);
    };
    double ck[K], ckn[K];
    uint32_t w[NW], wn[NW], bw[CPB * WPC], bwn[CPB * WPC];
    load_blk(nblk - 1, ck, w, bw);
    for (int blk = nblk - 1; blk >= 0; --blk) {
        load_blk(blk - 1, ckn, wn, bwn);
        if (blk < nfullb)
            bwd_block_big<MODEL, K, MODE, true>(a, ln, blk * B, w, ck, be, bex);
        else
            bwd_block_big<MODEL, K, MODE, false>(a, ln, blk * B, w, ck, be, bex);
#pragma unroll
        for (int cc = CPB - 1; cc >= 0; --cc) {
            const int cidx = blk * CPB + cc;
            int zb[C];
            uint32_t wc[WPC];
#pragma unroll
            for (int i = 0; i < WPC; ++i)
                wc[i] = bw[cc * WPC + i];
            if (cidx < nfull)
                vit_back_chunk<K, C, true>(Tp, cidx, wc, z, zb);
            else
                vit_back_chunk<K, C, false>(Tp, cidx, wc, z, zb);
            if (want_z) {
                if (invalid) {
#pragma unroll
                    for (int u = 0; u < C; ++u)
                        zb[u] = 0;
                }
                vit_back_flush<C, false>(a, p, Tp, cidx, zb);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            ck[k] = ckn[k];
#pragma unroll
        for (int i = 0; i < NW; ++i)
            w[i] = wn[i];
#pragma unroll
        for (int i = 0; i < CPB * WPC; ++i)
            bw[i] = bwn[i];
    }
}

template <int MODEL, int K, int MODE = FB_GAMMA | FB_PACK | FB_BIG>
__device__ __forceinline__ void fbv_block(const DevArgs &a, uint32_t block)
{
    constexpr int C = fb_chunk(K);
    constexpr int SPW = bp_steps_per_word(K);
    constexpr int B = kBigChunk;
    constexpr int KP = (K + 1) / 2;
    static_assert(vit_chunk(K) == C && B % C == 0, "fused sweep: one chunk size for both halves");
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t p = min((int64_t)block * blockDim.x + threadIdx.x, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const size_t tab = (size_t)a.L * KP * 64; /* double2 per table per wave */
    double2 *slab = lds + (size_t)wave * 2 * tab + lane;
    const double2 *lslab = slab + tab;

    FbLane<MODEL, K> ln;
    ln.p = p;
    ln.n = n;
    ln.L = a.L;
    ln.t0 = 0;
    ln.Tp = pair_len(a, n);
    ln.cb = 0;
    ln.q = p;
    ln.Qs = a.P;
    ln.slab = slab;
    PairParams<MODEL, K> lpp; /* log A for the max-plus half */
    load_params<MODEL, K, false>(ln.pp, a, d);
    load_params<MODEL, K, true>(lpp, a, d);
    fill_table<K, false>(slab, a, d);
    fill_table<K, true>(slab + tab, a, d);
    if constexpr (!(MODE & FB_RN1)) {
        if (wave_any(!renorm_sparse_safe<MODEL, K>(ln.pp, slab, a.L))) {
            fbv_block<MODEL, K, MODE | FB_RN1>(a, block); /* per-step renormalisation (renorm_sparse_safe) */
            return;
        }
    }
    const SeriesPtrs sp = series_ptrs<MODEL, false>(a, n);
    const int Tp = ln.Tp;
    const int Tw_min = wave_min(Tp);
    const int Tw_max = wave_max(Tp);
    const int nfull = Tw_min / C;
    const int nchunk = (Tw_max + C - 1) / C;

    /* ---- forward sweep: filter + max-plus on one pass of x ---- */
    double al[K], lsc = 0.0;
    int ex = 0;
#pragma unroll
    for (int k = 0; k < K; ++k)
        al[k] = 0.0;
    constexpr int D = kFwdGroup;
    Obs cur[C];
    load_chunk<MODEL, C, false>(cur, sp, 0);
    Obs grp[D][C];
#pragma unroll
    for (int i = 0; i < D; ++i)
        load_chunk<MODEL, C, false>(grp[i], sp, (1 + i) * C);
    Em<K> ecur;
    emit_prob<MODEL, K>(ln.pp, slab, a.L, cur[0], ecur);
    double le[K], dl[K];
    emit_log<MODEL, K>(lpp, lslab, a.L, cur[0], le);
#pragma unroll
    for (int k = 0; k < K - 1; ++k)
        dl[k] = dev_nan(); /* delta_tk[1, K] only (Q3, hmm-multinom.stan:105-106) */
    dl[K - 1] = le[K - 1];
    uint32_t word = 0;
    fwd_chunk<MODEL, K, C, MODE, false>(a, ln, 0, cur, grp[0][0], ecur, al, lsc, ex);
    vit_fwd_chunk<MODEL, K, C, false, true>(a, p, lpp, lslab, Tp, 0, cur, grp[0][0], le, dl, word);
    int c = 1;
    for (; c + D <= nfull; c += D) {
        Obs nxt[D][C];
#pragma unroll
        for (int i = 0; i < D; ++i)
            load_chunk<MODEL, C, false>(nxt[i], sp, (c + D + i) * C);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const Obs &n0 = (i + 1 < D) ? grp[i + 1 < D ? i + 1 : 0][0] : nxt[0][0];
            fwd_chunk<MODEL, K, C, MODE, true>(a, ln, c + i, grp[i], n0, ecur, al, lsc, ex);
            vit_fwd_chunk<MODEL, K, C, true>(a, p, lpp, lslab, Tp, c + i, grp[i], n0, le, dl, word);
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int u = 0; u < C; ++u)
                grp[i][u] = nxt[i][u];
    }
#pragma unroll
    for (int u = 0; u < C; ++u)
        cur[u] = grp[0][u];
    for (; c < nchunk; ++c) {
        Obs nxt[C];
        load_chunk<MODEL, C, false>(nxt, sp, (c + 1) * C);
        fwd_chunk<MODEL, K, C, MODE, false>(a, ln, c, cur, nxt[0], ecur, al, lsc, ex);
        vit_fwd_chunk<MODEL, K, C, false>(a, p, lpp, lslab, Tp, c, cur, nxt[0], le, dl, word);
#pragma unroll
        for (int u = 0; u < C; ++u)
            cur[u] = nxt[u];
    }
    if ((a.outputs & HHMM_OUT_LOGLIK) && a.loglik)
        a.loglik[p] = log(vsum<K>(al)) + (lsc + kLn2 * ex);

    /* ---- Viterbi end (as viterbi_epilogue): partial word, logp_zstar, zstar_T ---- */
    if ((Tp - 1) % SPW != SPW - 1)
        put_tmp(a.bp + a.P * (int64_t)((Tp - 1) / SPW), (uint32_t)p * 4u, word);
    const double lpz = stan_max_vec<K>(dl);
    int z = -1;
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (dl[j] == lpz)
            z = j;
    const bool invalid = (z < 0) || (Tp >= 2 && lpz == dev_ninf());
    if ((a.outputs & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
        a.logp_zstar[p] = lpz;
    if (a.pair_status)
        a.pair_status[p] = invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
    const bool want_z = (a.outputs & HHMM_OUT_ZSTAR) && a.zstar;
    if (invalid)
        z = 0; /* the path is all zeros (pair flagged), the walk below is discarded */

    fbv_backward<MODEL, K, MODE>(a, ln, Tw_min, Tw_max, z, invalid, want_z);
}

template <int MODEL, int K>
__global__ void __launch_bounds__(kBlock) fbv_kernel(const DevArgs a)
{
    if constexpr (fbv_ok<MODEL, K>())
        fbv_block<MODEL, K>(a, blockIdx.x);
}


/* ---- phased sweep: the Viterbi first, then the forward-backward (C2's profile) ---- *
 * One lane, one pair, three phases over ONE emission slab (so the wave keeps
 * the single-table LDS footprint of fb_kernel / viterbi_kernel: two waves per
 * SIMD), x read from HBM once (hmm-multinom.stan:27-132):
 *   1. log phi in the slab: the max-plus recursion over x (viterbi_kernel's
 *      arithmetic), writing the back-pointer words and each 8-step chunk's
 *      symbols packed 4 bits each (the record fb_kernel's FB_PACK writes);
 *      logp_zstar, pair_status and zstar_T as viterbi_epilogue.
 *   2. phi in the slab: the scaled filter over the PACKED symbols (0.5 instead
 *      of 4 B per step), loglik, 16-step checkpoints (FB_BIG).
 *   3. the FB_BIG backward sweep with the backtrack on the same blocks
 *      (fbv_backward).
 * Against fb_kernel beside viterbi_kernel it moves x's second read and the
 * forward-backward's own symbol packing (-3.5 B per series-timestep); waves
 * in different phases share a CU the way the two kernels' waves did.  Outputs
 * are bit-identical to the two kernels (same functions, same operation order).
 * A wave holding a pair without the renormalisation bound lists itself after
 * phase 1 (zstar_T parked in zstar[T-1]) for vfb_dense_kernel. */
#ifndef HHMM_VFB_DEFAULT
#define HHMM_VFB_DEFAULT 1 /* the phased sweep for the C2 request without flags */
#endif
template <int MODEL, int K>
__device__ __forceinline__ uint32_t pack_chunk(const Obs (&cur)[8])
{
    uint32_t w = 0;
#pragma unroll
    for (int v = 0; v < 8; ++v)
        w |= ((uint32_t)(cur[v].x - 1) & 15u) << (4 * v);
    return w;
}

/* Phase 1: the max-plus forward over x, packing each chunk's symbols.  The
 * packing also checks the data block's bound on x (int<lower=1,upper=L> x[T],
 * hmm-multinom.stan:11) for the steps t < Tp: bad = some symbol is outside
 * 1..L (the device entry's HHMM_PAIR_INVALID_DATA, at no extra read of x). */
template <int MODEL, int K>
__device__ __forceinline__ void vfb_viterbi(const DevArgs &a, int64_t p, const PairParams<MODEL, K> &pp,
                                            const double2 *slab, const SeriesPtrs &sp, int Tp, int Tw_min,
                                            int Tw_max, double (&dl)[K], uint32_t &word, bool &bad)
{
    constexpr int CV = vit_chunk(K);
    static_assert(CV == 8, "phased sweep: 8-step chunks");
    const int nfull = Tw_min / CV;
    const int nchunk = (Tw_max + CV - 1) / CV;
    /* the data check inline (xcheck_acc) */
    uint32_t xm = 0;
    auto pack_put = [&](int c, const Obs (&cur)[CV], auto full) {
        if (c * CV < Tp) {
            put_tmp(a.xpk + a.P * (int64_t)c, (uint32_t)p * 4u, pack_chunk<MODEL, K>(cur));
            xcheck_acc<CV, decltype(full)::value>(xm, cur, c, Tp);
        }
    };
    const std::true_type full;
    const std::false_type tail;
    Obs cur[CV];
    load_chunk<MODEL, CV, false>(cur, sp, 0);
    constexpr int D = kVitGroup;
    Obs grp[D][CV];
#pragma unroll
    for (int i = 0; i < D; ++i)
        load_chunk<MODEL, CV, false>(grp[i], sp, (1 + i) * CV);
    double le[K];
    emit_log<MODEL, K>(pp, slab, a.L, cur[0], le);
#pragma unroll
    for (int k = 0; k < K - 1; ++k)
        dl[k] = dev_nan(); /* delta_tk[1, K] only (Q3, hmm-multinom.stan:105-106) */
    dl[K - 1] = le[K - 1];
    word = 0;
    vit_fwd_chunk<MODEL, K, CV, false, true>(a, p, pp, slab, Tp, 0, cur, grp[0][0], le, dl, word);
    pack_put(0, cur, tail);
    int c = 1;
    for (; c + D <= nfull; c += D) {
        Obs nxt[D][CV];
#pragma unroll
        for (int i = 0; i < D; ++i)
            load_chunk<MODEL, CV, false>(nxt[i], sp, (c + D + i) * CV);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            vit_fwd_chunk<MODEL, K, CV, true>(a, p, pp, slab, Tp, c + i, grp[i],
                                              (i + 1 < D) ? grp[i + 1 < D ? i + 1 : 0][0] : nxt[0][0], le, dl, word);
            pack_put(c + i, grp[i], full); /* c + i < nfull: every lane's steps are < Tp */
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int u = 0; u < CV; ++u)
                grp[i][u] = nxt[i][u];
    }
#pragma unroll
    for (int u = 0; u < CV; ++u)
        cur[u] = grp[0][u];
    for (; c < nchunk; ++c) {
        Obs nxt[CV];
        load_chunk<MODEL, CV, false>(nxt, sp, (c + 1) * CV);
        vit_fwd_chunk<MODEL, K, CV, false>(a, p, pp, slab, Tp, c, cur, nxt[0], le, dl, word);
        pack_put(c, cur, tail);
#pragma unroll
        for (int u = 0; u < CV; ++u)
            cur[u] = nxt[u];
    }
    bad = xm >= (uint32_t)a.L;
}

/* Phase 2: the scaled filter over the packed symbols (FB_BIG checkpoints),
 * the words a group of chunks ahead; loglik. */
template <int MODEL, int K, int MODE>
__device__ __forceinline__ void vfb_forward(const DevArgs &a, const FbLane<MODEL, K> &ln, int Tw_min, int Tw_max)
{
    constexpr int C = fb_chunk(K);
    constexpr int MF = MODE & ~FB_PACK; /* the symbols are packed already */
    constexpr int D = 8;                /* chunks (words) per prefetch group */
    const int nfull = Tw_min / C;
    const int nchunk = (Tw_max + C - 1) / C;
    const int pkrows = (a.Tmax + C - 1) / C;
    auto word_at = [&](int c) -> uint32_t {
        return get_tmp(a.xpk + a.P * (int64_t)min(c, pkrows - 1), (uint32_t)ln.q * 4u);
    };
    auto unpack = [&](uint32_t w, Obs (&dst)[C]) {
#pragma unroll
        for (int v = 0; v < C; ++v) {
            dst[v].x = (int)((w >> (4 * v)) & 15u) + 1;
            dst[v].aux = 0;
            dst[v].xr = 0.0;
        }
    };
    auto first_obs = [&](uint32_t w) {
        Obs o;
        o.x = (int)(w & 15u) + 1;
        o.aux = 0;
        o.xr = 0.0;
        return o;
    };
    double al[K], lsc = 0.0;
    int ex = 0;
#pragma unroll
    for (int k = 0; k < K; ++k)
        al[k] = 0.0;
    uint32_t wg[D];
#pragma unroll
    for (int i = 0; i < D; ++i)
        wg[i] = word_at(i);
    Em<K> ecur;
    emit_prob<MODEL, K>(ln.pp, ln.slab, ln.L, first_obs(wg[0]), ecur);
    int c = 0;
    for (; c + D <= nfull; c += D) {
        uint32_t wn[D];
#pragma unroll
        for (int i = 0; i < D; ++i)
            wn[i] = word_at(c + D + i);
#pragma unroll
        for (int i = 0; i < D; ++i) {
            Obs cur[C];
            unpack(wg[i], cur);
            fwd_chunk<MODEL, K, C, MF, true>(a, ln, c + i, cur, first_obs(i + 1 < D ? wg[i + 1 < D ? i + 1 : 0] : wn[0]),
                                             ecur, al, lsc, ex);
        }
#pragma unroll
        for (int i = 0; i < D; ++i)
            wg[i] = wn[i];
    }
    /* the rest one chunk at a time, the window rolling D words ahead */
    for (; c < nchunk; ++c) {
        Obs cur[C];
        unpack(wg[0], cur);
        const uint32_t w1 = wg[1];
#pragma unroll
        for (int i = 0; i + 1 < D; ++i)
            wg[i] = wg[i + 1];
        wg[D - 1] = word_at(c + D);
        fwd_chunk<MODEL, K, C, MF, false>(a, ln, c, cur, first_obs(w1), ecur, al, lsc, ex);
    }
    if ((a.outputs & HHMM_OUT_LOGLIK) && a.loglik)
        a.loglik[ln.p] = log(vsum<K>(al)) + (lsc + kLn2 * ex);
}

template <int MODEL, int K>
__device__ __forceinline__ void vfb_lane(const DevArgs &a, int64_t gwave, FbLane<MODEL, K> &ln, int64_t &d)
{
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    constexpr int KP = (K + 1) / 2;
    const int64_t p = min(gwave * 64 + lane, a.P - 1);
    int64_t n;
    pair_coords(a, p, n, d);
    ln.p = p;
    ln.L = a.L;
    ln.t0 = 0;
    ln.Tp = pair_len(a, n);
    ln.cb = 0;
    ln.q = p;
    ln.Qs = a.P;
    ln.slab = lds + (size_t)wave * a.L * KP * 64 + lane;
}

template <int MODEL, int K, int MODE = FB_GAMMA | FB_PACK | FB_BIG>
__device__ __forceinline__ void vfb_block(const DevArgs &a, int64_t gwave)
{
    FbLane<MODEL, K> ln;
    int64_t d;
    vfb_lane<MODEL, K>(a, gwave, ln, d);
    const int64_t p = ln.p;
    const int Tp = ln.Tp;
    const int Tw_min = wave_min(Tp);
    const int Tw_max = wave_max(Tp);
    double2 *slab = const_cast<double2 *>(ln.slab);
    int z;
    bool invalid;
    {
        /* ---- phase 1: Viterbi over x ---- */
        PairParams<MODEL, K> lpp;
        load_params<MODEL, K, true>(lpp, a, d);
        fill_table<K, true>(slab, a, d);
        int64_t n, dd;
        pair_coords(a, p, n, dd);
        const SeriesPtrs sp = series_ptrs<MODEL, false>(a, n);
        double dl[K];
        uint32_t word;
        bool bad;
        vfb_viterbi<MODEL, K>(a, p, lpp, slab, sp, Tp, Tw_min, Tw_max, dl, word, bad);
        if (a.T)
            bad |= a.T[n] < 1 || a.T[n] > a.Tmax;
        constexpr int SPW = bp_steps_per_word(K);
        if ((Tp - 1) % SPW != SPW - 1) /* partial last word */
            put_tmp(a.bp + a.P * (int64_t)((Tp - 1) / SPW), (uint32_t)p * 4u, word);
        const double lpz = stan_max_vec<K>(dl);
        z = -1;
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (dl[j] == lpz)
                z = j;
        invalid = (z < 0) || (Tp >= 2 && lpz == dev_ninf());
        if ((a.outputs & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
            a.logp_zstar[p] = lpz;
        if (a.pair_status)
            a.pair_status[p] = bad ? HHMM_PAIR_INVALID_DATA : invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
        if (invalid)
            z = 0;
    }
    /* ---- the slab switches to phi ---- */
    load_params<MODEL, K, false>(ln.pp, a, d);
    fill_table<K, false>(slab, a, d);
    if constexpr (!(MODE & FB_RN1)) {
        if (wave_any(!renorm_sparse_safe<MODEL, K>(ln.pp, ln.slab, a.L))) {
            /* zstar_T parked where the backtrack writes it anyway (0: invalid) */
            if (Tp >= 1)
                put_out(a.zstar + a.P * (int64_t)(Tp - 1), (uint32_t)p * 4u, invalid ? 0 : z + 1);
            if ((threadIdx.x & 63) == 0) {
                const int slot = atomicAdd(&a.rnw[0], 1);
                a.rnw[1 + slot] = (int32_t)gwave;
            }
            return;
        }
    }
    /* ---- phase 2: the filter over the packed symbols ---- */
    vfb_forward<MODEL, K, MODE>(a, ln, Tw_min, Tw_max);
    /* ---- phase 3: gamma and the backtrack ---- */
    fbv_backward<MODEL, K, MODE>(a, ln, Tw_min, Tw_max, z, invalid, true);
}

template <int MODEL, int K>
__global__ void __launch_bounds__(kBlock) vfb_kernel(const DevArgs a)
{
    if constexpr (fbv_ok<MODEL, K>())
        vfb_block<MODEL, K>(a, (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
}

/* Phases 2-3 with per-step renormalisation for the waves vfb_kernel listed
 * (a.rnw), zstar_T read back from zstar[T-1]. */
template <int MODEL, int K>
__global__ void __launch_bounds__(64) vfb_dense_kernel(const DevArgs a)
{
    if constexpr (fbv_ok<MODEL, K>()) {
        constexpr int MODE = FB_GAMMA | FB_PACK | FB_BIG | FB_RN1;
        const int nl = __builtin_amdgcn_readfirstlane(a.rnw[0]);
        for (int i = blockIdx.x; i < nl; i += gridDim.x) {
            const int64_t gw = __builtin_amdgcn_readfirstlane(a.rnw[1 + i]);
            FbLane<MODEL, K> ln;
            int64_t d;
            vfb_lane<MODEL, K>(a, gw, ln, d);
            const int zt = ln.Tp >= 1 ? a.zstar[ln.p + a.P * (int64_t)(ln.Tp - 1)] : 0;
            load_params<MODEL, K, false>(ln.pp, a, d);
            fill_table<K, false>(const_cast<double2 *>(ln.slab), a, d);
            const int Tw_min = wave_min(ln.Tp);
            const int Tw_max = wave_max(ln.Tp);
            vfb_forward<MODEL, K, MODE>(a, ln, Tw_min, Tw_max);
            fbv_backward<MODEL, K, MODE>(a, ln, Tw_min, Tw_max, zt > 0 ? zt - 1 : 0, zt <= 0, true);
        }
    }
}

/* ---- state-parallel Viterbi (few pairs, long T; C5) ------------------- *
 * One lane per (pair, state j): a pair's K <= 4 states sit in one lane quad.
 * Each step a lane fetches delta_{t-1} of the quad by DPP quad broadcasts,
 * forms its own K candidates in the reference's order and reduces them with
 * the same fmax / strict-compare rules as vit_step, so delta, the
 * back-pointers and the paths are bit-identical to the lane-per-pair decoder.
 * The per-step dependency chain is K candidates instead of K^2, which is what
 * bounds a batch too small to hide latency with other waves (250 pairs x
 * T = 1e6: 4 waves on the whole chip).  The back-pointer bits of the quad are
 * OR-reduced into the same packed word layout, so the epilogue (run by all
 * four lanes on the gathered delta_T; identical duplicate stores) and the
 * backtrack are shared. */

/* Steps per prefetched observation chunk: a multiple of the word length, two
 * Viterbi chunks deep so the (latency-bound) loads run far ahead. */
constexpr int vit_sp_chunk(int K) { return 2 * vit_chunk(K); }

template <int MODEL, int K>
struct SpLane {
    double colA[K]; /* log A[i][js] */
    double mu, isig, c0; /* gauss: state js */
    const double *slab;  /* discrete: log phi[js][.] column, stride 64 */
    const double *arow;  /* tayal: rows [sign 1 | sign 2 | other][i] of the masked column, stride 64 */
    int js;              /* state of this lane */
    int j;               /* quad position (bits only from j < K) */
};

template <int MODEL, int K>
__device__ __forceinline__ double sp_emit(const SpLane<MODEL, K> &ln, const Obs &o, int L)
{
    if constexpr (ModelTraits<MODEL>::kGauss) {
        const double z = (o.xr - ln.mu) * ln.isig;
        const double z2 = z * z;
        return ln.c0 + (-0.5 * z2);
    } else {
        return ln.slab[(min(max(o.x, 1), L) - 1) * 64];
    }
}

/* Tayal: the masked transition column of this lane for a step's sign:
 * log A[i][js] where the mask is on, -0.0 where it is off (x + -0.0 == x for
 * every double x, so the off candidate keeps its value bit for bit). */
template <int MODEL, int K>
__device__ __forceinline__ void sp_arow(const SpLane<MODEL, K> &ln, int sign, double (&ar)[K])
{
    const int r = (sign == 1) ? 0 : (sign == 2 ? 1 : 2);
#pragma unroll
    for (int i = 0; i < K; ++i)
        ar[i] = ln.arow[(r * K + i) * 64];
}

/* Stores chunk c's back-pointer words (issued after the next chunk's loads). */
template <int K, int CS>
__device__ __forceinline__ void sp_flush_words(const DevArgs &a, int64_t p, int Tp, int c,
                                               const uint32_t (&wb)[CS / bp_steps_per_word(K)])
{
    constexpr int SPW = bp_steps_per_word(K);
#pragma unroll
    for (int i = 0; i < CS / SPW; ++i) {
        const int t = c * CS + i * SPW + SPW - 1;
        if (t < Tp)
            put_tmp(a.bp + a.P * (int64_t)(t / SPW), (uint32_t)p * 4u, wb[i]);
    }
}

template <int MODEL, int K, int CS, bool FULLC>
__device__ __forceinline__ void vit_sp_chunk_run(const DevArgs &a, const SpLane<MODEL, K> &ln, int Tp, int c,
                                                 const Obs (&cur)[CS], const Obs &nxt0, double &le, double (&ar)[K],
                                                 double &dl, uint32_t &bits,
                                                 uint32_t (&wb)[CS / bp_steps_per_word(K)])
{
    constexpr int BITS = bp_bits(K);
    constexpr int STEPB = K * BITS;
    constexpr int SPW = bp_steps_per_word(K);
    const int t0 = c * CS;
    const uint32_t jbit = (uint32_t)(ln.j * BITS);
    const bool owns = ln.j < K;
#pragma unroll
    for (int u = 0; u < CS; ++u) {
        const int t = t0 + u;
        const Obs &on1 = (u + 1 < CS) ? cur[u + 1 < CS ? u + 1 : 0] : nxt0;
        const double lnx = sp_emit<MODEL, K>(ln, on1, a.L);
        double arx[K];
        if constexpr (ModelTraits<MODEL>::kTayal)
            sp_arow<MODEL, K>(ln, on1.aux, arx);
        if (FULLC || t < Tp) {
            if (!(u == 0 && c == 0)) {
                double d[K];
                quad_gather<K>(dl, d);
                double best = dev_ninf();
                uint32_t arg = 0;
#pragma unroll
                for (int i = 0; i < K; ++i) {
                    double cand;
                    if constexpr (ModelTraits<MODEL>::kTayal) {
                        /* (delta + log phi) [+ log A] (hhmm-tayal2009.stan:143-146) */
                        cand = (d[i] + le) + ar[i];
                    } else {
                        cand = (d[i] + ln.colA[i]) + le; /* (delta + log A) + emission (hmm.stan:111) */
                    }
                    if (i == 0) {
                        best = fmax(best, cand);
                    } else {
                        const bool gt = cand > best;
                        best = fmax(best, cand);
                        arg = gt ? (uint32_t)i : arg;
                    }
                }
                dl = best;
                if (owns)
                    bits |= arg << ((uint32_t)((u % SPW) * STEPB) + jbit);
            }
            if (u % SPW == SPW - 1) {
                wb[u / SPW] = quad_or(bits);
                bits = 0;
            }
        }
        le = lnx;
        if constexpr (ModelTraits<MODEL>::kTayal) {
#pragma unroll
            for (int i = 0; i < K; ++i)
                ar[i] = arx[i];
        }
    }
}

template <int MODEL, int K>
__global__ void __launch_bounds__(64) viterbi_sp_kernel(const DevArgs a)
{
    static_assert(K >= 2 && K <= 4, "state-parallel Viterbi: one lane quad per pair");
    constexpr int CS = vit_sp_chunk(K);
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal; /* semisup Viterbi is unmasked (Q7) */
    HIP_DYNAMIC_SHARED(double, ldsd)
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * 64 + lane;
    const int64_t p = min(g >> 2, a.P - 1);
    if (a.vs_redo && !a.vs_redo[p]) /* hhmm_vscan.h's fallback: only the pairs it flagged */
        return;
    SpLane<MODEL, K> ln;
    ln.j = (int)(g & 3);
    ln.js = min(ln.j, K - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);

    {
        PairParams<MODEL, K> pp;
        load_params<MODEL, K, true>(pp, a, d);
#pragma unroll
        for (int i = 0; i < K; ++i) {
            double v = pp.A[i][0];
#pragma unroll
            for (int jj = 1; jj < K; ++jj)
                v = (ln.js == jj) ? pp.A[i][jj] : v;
            ln.colA[i] = v;
        }
        ln.mu = ln.isig = ln.c0 = 0.0;
        if constexpr (ModelTraits<MODEL>::kGauss) {
            ln.mu = pp.mu[0];
            ln.isig = pp.isig[0];
            ln.c0 = pp.c0[0];
#pragma unroll
            for (int jj = 1; jj < K; ++jj) {
                ln.mu = (ln.js == jj) ? pp.mu[jj] : ln.mu;
                ln.isig = (ln.js == jj) ? pp.isig[jj] : ln.isig;
                ln.c0 = (ln.js == jj) ? pp.c0[jj] : ln.c0;
            }
        }
    }
    ln.slab = ldsd + lane;
    ln.arow = ldsd + (size_t)a.L * 64 + lane;
    if constexpr (ModelTraits<MODEL>::kDiscrete) {
        double *col = ldsd + lane;
        for (int l = 0; l < a.L; ++l)
            col[l * 64] = dev_cr_log(draw2<K>(a.phi_k, a, d, ln.js, l, K));
    }
    if constexpr (ModelTraits<MODEL>::kTayal) {
        double *rows = ldsd + (size_t)a.L * 64 + lane;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int i = 0; i < K; ++i)
                rows[(r * K + i) * 64] = tayal_pred(r + 1, ln.js) ? ln.colA[i] : -0.0;
    }
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, n);
    const int Tw_min = wave_min(Tp);
    const int Tw_max = wave_max(Tp);
    const int nfull = Tw_min / CS;
    const int nchunk = (Tw_max + CS - 1) / CS;

    __syncthreads(); /* LDS tables written (one wave per block; orders LDS) */

    Obs cur[CS];
    load_chunk<MODEL, CS, VAUX>(cur, sp, 0);
    double le = sp_emit<MODEL, K>(ln, cur[0], a.L);
    double ar[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        ar[i] = 0.0;
    /* Q3: only column K of delta_tk[1] is written, the others stay NaN */
    double dl = (ln.js == K - 1) ? le : dev_nan();
    uint32_t bits = 0;
    constexpr int WPC = CS / bp_steps_per_word(K);
    uint32_t wb[WPC];
    for (int c = 0; c < nchunk; ++c) {
        Obs nxt[CS];
        load_chunk<MODEL, CS, VAUX>(nxt, sp, (c + 1) * CS);
        if (c > 0)
            sp_flush_words<K, CS>(a, p, Tp, c - 1, wb);
        if (c < nfull)
            vit_sp_chunk_run<MODEL, K, CS, true>(a, ln, Tp, c, cur, nxt[0], le, ar, dl, bits, wb);
        else
            vit_sp_chunk_run<MODEL, K, CS, false>(a, ln, Tp, c, cur, nxt[0], le, ar, dl, bits, wb);
#pragma unroll
        for (int u = 0; u < CS; ++u)
            cur[u] = nxt[u];
    }
    if (nchunk > 0)
        sp_flush_words<K, CS>(a, p, Tp, nchunk - 1, wb);
    double dv[K];
    quad_gather<K>(dl, dv);
    viterbi_epilogue<K, true>(a, p, Tp, Tw_min, Tw_max, dv, quad_or(bits));
}

} // namespace hhmm
#include "hhmm_vscan.h"
namespace hhmm {



/* ------------------------------------------------------------------ */
/* Log-space forward-backward (the unalpha_tk / unbeta_tk profile)       */
/* ------------------------------------------------------------------ */
/*
 * The log-scale outputs unalpha_tk / unbeta_tk keep finite values for states
 * whose probability is below the double range relative to the others (Stan
 * works in log space: e.g. hhmm-tayal2009.stan:93-119 keeps unbeta ~ -2400
 * where the linear recursion's component underflows).  When either is
 * requested the recursion runs in log space like the reference -- log A and
 * log phi tabulated once per pair, Stan's log_sum_exp per (t, j) -- with the
 * same checkpoint / recompute structure as fb_kernel.  Posteriors follow the
 * reference's formulas: alpha = softmax(unalpha), beta = softmax(unbeta),
 * ungamma = alpha .* beta, gamma = ungamma / sum (hmm.stan:60-63, 85-96).
 */
template <int K>
__device__ __forceinline__ double stan_lse(const double (&x)[K])
{
    double mx = dev_ninf();
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (x[i] > mx)
            mx = x[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i)
        if (x[i] != dev_ninf())
            sum += exp(x[i] - mx);
    return mx + log(sum);
}

template <int K>
__device__ __forceinline__ void stan_softmax_v(const double (&v)[K], double (&th)[K])
{
    double mx = v[0];
#pragma unroll
    for (int i = 1; i < K; ++i)
        if (v[i] > mx)
            mx = v[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
        th[i] = exp(v[i] - mx);
        sum += th[i];
    }
#pragma unroll
    for (int i = 0; i < K; ++i)
        th[i] = th[i] / sum;
}

/* unalpha_1 (hmm.stan:29-30 with the Q2 summed emission; multinom :30-31;
 * Tayal :49-54).  pp.A holds log A. */
template <int MODEL, int K>
__device__ __forceinline__ void fwd_log_init(double (&u)[K], const PairParams<MODEL, K> &pp, const double (&le)[K],
                                             const Obs &o)
{
    if constexpr (ModelTraits<MODEL>::kGauss) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double z = (o.xr - pp.mu[k]) * pp.isig[k];
            const double z2 = z * z;
            s += HHMM_NEG_LOG_SQRT_TWO_PI;
            s -= pp.lsig[k];
            s += -0.5 * z2;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            u[k] = log(pp.p[k]) + s;
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if constexpr (ModelTraits<MODEL>::kTayal)
                u[k] = tayal_init_pred(o.aux, k) ? le[k] + log(pp.p[k]) : le[k];
            else
                u[k] = log(pp.p[k]) + le[k];
        }
    }
}

/* unalpha_t(j) = LSE_i(acc_i) with the reference's accumulator
 * (hmm.stan:37; semisup :39-44 and Tayal :60-64: transition under the mask). */
template <int MODEL, int K>
__device__ __forceinline__ void fwd_log_step(const double (&u)[K], double (&out)[K], const PairParams<MODEL, K> &pp,
                                             const double (&le)[K], const Obs &o)
{
    double nu[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double acc[K];
        if constexpr (ModelTraits<MODEL>::kAux) {
            bool on;
            if constexpr (ModelTraits<MODEL>::kSemisup)
                on = semisup_mask(o.aux, j);
            else
                on = tayal_pred(o.aux, j);
#pragma unroll
            for (int i = 0; i < K; ++i) {
                acc[i] = u[i] + le[j];
                acc[i] = on ? acc[i] + pp.A[i][j] : acc[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i)
                acc[i] = (u[i] + pp.A[i][j]) + le[j];
        }
        nu[j] = stan_lse<K>(acc);
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        out[j] = nu[j];
}

/* unbeta_{t-1}(j) = LSE_i(acc_i): (unbeta_t(i) + log A(j,i)) + le_t(i)
 * (hmm.stan:79; semisup unmasked :84); Tayal: unbeta + log phi, + log A(j,i)
 * under the predicate on the PREVIOUS state j (hhmm-tayal2009.stan:107-111). */
template <int MODEL, int K>
__device__ __forceinline__ void bwd_log_step(double (&ub)[K], const PairParams<MODEL, K> &pp, const double (&le)[K],
                                             const Obs &o)
{
    double nb[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double acc[K];
        if constexpr (ModelTraits<MODEL>::kTayal) {
            const bool on = tayal_pred(o.aux, j);
#pragma unroll
            for (int i = 0; i < K; ++i) {
                acc[i] = ub[i] + le[i];
                acc[i] = on ? acc[i] + pp.A[j][i] : acc[i];
            }
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i)
                acc[i] = (ub[i] + pp.A[j][i]) + le[i];
        }
        nb[j] = stan_lse<K>(acc);
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        ub[j] = nb[j];
}

template <int K>
__device__ __forceinline__ void emit_log_posteriors(const DevArgs &a, int64_t p, int t, const double (&u)[K],
                                                    const double (&ub)[K], bool fwd_only)
{
    const uint32_t o = a.outputs;
    double al[K], be[K];
    stan_softmax_v<K>(u, al);
    if ((o & HHMM_OUT_UNALPHA) && a.unalpha)
        store_tk<K>(a.unalpha, a, p, t, u);
    if ((o & HHMM_OUT_ALPHA) && a.alpha)
        store_tk<K>(a.alpha, a, p, t, al);
    if (fwd_only)
        return;
    stan_softmax_v<K>(ub, be);
    if ((o & HHMM_OUT_UNBETA) && a.unbeta)
        store_tk<K>(a.unbeta, a, p, t, ub);
    if ((o & HHMM_OUT_BETA) && a.beta)
        store_tk<K>(a.beta, a, p, t, be);
    if (o & (HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA)) {
        double ug[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            ug[k] = al[k] * be[k];
        if ((o & HHMM_OUT_UNGAMMA) && a.ungamma)
            store_tk<K>(a.ungamma, a, p, t, ug);
        if ((o & HHMM_OUT_GAMMA) && a.gamma) {
            const double r = 1.0 / vsum<K>(ug);
            double v[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
                v[k] = ug[k] * r;
            store_tk<K>(a.gamma, a, p, t, v);
        }
    }
}

template <int MODEL, int K, bool FWDONLY>
__global__ void __launch_bounds__(kBlock) fb_log_kernel(const DevArgs a)
{
    constexpr int C = fb_chunk(K);
    constexpr bool AUX = ModelTraits<MODEL>::kAux;
    constexpr int KP = (K + 1) / 2;
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t p = min((int64_t)blockIdx.x * blockDim.x + threadIdx.x, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    double2 *slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    PairParams<MODEL, K> pp;
    load_params<MODEL, K, true>(pp, a, d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        fill_table<K, true>(slab, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, AUX>(a, n);
    const int nchunk = (wave_max(Tp) + C - 1) / C;

    double u[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        u[k] = 0.0;
    Obs cur[C];
    load_chunk<MODEL, C, AUX>(cur, sp, 0);
    for (int c = 0; c < nchunk; ++c) {
        Obs nxt[C];
        load_chunk<MODEL, C, AUX>(nxt, sp, (c + 1) * C);
#pragma unroll
        for (int v = 0; v < C; ++v) {
            const int t = c * C + v;
            if (t < Tp) {
                double le[K];
                emit_log<MODEL, K>(pp, slab, a.L, cur[v], le);
                if (t == 0)
                    fwd_log_init<MODEL, K>(u, pp, le, cur[v]);
                else
                    fwd_log_step<MODEL, K>(u, u, pp, le, cur[v]);
                if constexpr (FWDONLY) {
                    emit_log_posteriors<K>(a, p, t, u, u, true);
                } else if (v == 0) {
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        put_tmp(a.ckpt + a.P * ((int64_t)c * K + k), (uint32_t)p * 8u, u[k]);
                }
            }
        }
#pragma unroll
        for (int v = 0; v < C; ++v)
            cur[v] = nxt[v];
    }
    if ((a.outputs & HHMM_OUT_LOGLIK) && a.loglik) /* target += log_sum_exp(unalpha_tk[T]) */
        a.loglik[p] = stan_lse<K>(u);
    if constexpr (FWDONLY)
        return;

    double ub[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        ub[k] = 1.0; /* unbeta_tk[T, j] = 1 (Q1) */
    for (int c = nchunk - 1; c >= 0; --c) {
        load_chunk<MODEL, C, AUX>(cur, sp, c * C);
        double abuf[C][K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            abuf[0][k] = get_tmp(a.ckpt + a.P * ((int64_t)c * K + k), (uint32_t)p * 8u);
#pragma unroll
        for (int v = 1; v < C; ++v) {
            if (c * C + v < Tp) {
                double le[K];
                emit_log<MODEL, K>(pp, slab, a.L, cur[v], le);
                fwd_log_step<MODEL, K>(abuf[v - 1], abuf[v], pp, le, cur[v]);
            }
        }
#pragma unroll
        for (int v = C - 1; v >= 0; --v) {
            const int t = c * C + v;
            if (t < Tp) {
                emit_log_posteriors<K>(a, p, t, abuf[v], ub, false);
                if (t > 0) {
                    double le[K];
                    emit_log<MODEL, K>(pp, slab, a.L, cur[v], le);
                    bwd_log_step<MODEL, K>(ub, pp, le, cur[v]);
                }
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* Parallel scan over T                                  */
/* ------------------------------------------------------------------ */
/*
 * For long series with few pairs (C5: Tayal, T = 1e6).  The forward filter is
 * linear: f_t = f_{t-1} F_t with F_t(i,j) = Abar_t(i,j) e_t(j), Abar = A with
 * the columns the forward mask switches off set to 1; the backward pass is
 * beta_{t-1} = B_t beta_t with B_t(j,i) = Abar'_t(j,i) e_t(i), Abar' = A with
 * the ROWS the backward mask switches off set to 1 (Tayal, Q6; the other
 * programs' backward passes are unmasked, Q7).  All entries are
 * non-negative, so chunk products keep every entry's relative precision (no
 * cancellation), like the sequential recursion.
 *   phase 1  lane = (pair, T-chunk c): Pf_c = prod_{t in c} F_t and
 *            Qb_c = prod_{t in c} B_t (chunk 0 starts from the model's init f_0,
 *            so its row 0 is f at the chunk's end)
 *   phase 2  lane = pair: f entering every chunk (a left scan over Pf), beta
 *            at every chunk's last step (a right scan over Qb), loglik
 *   phase 3  lane = (pair, T-chunk): fb_sweep over the chunk from those vectors
 * Each product is renormalised by an exact power of two after every step;
 * the exponents and the Gaussian log-scale sum of the chunk travel with it.
 */

/* Whole-matrix power-of-two renormalisation (max entry into [0.5, 1)). */
template <int K>
__device__ __forceinline__ void renorm_mat(double (&M)[K][K], int &ex)
{
    double mx = M[0][0];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            mx = fmax(mx, M[i][j]);
    const int e = __builtin_amdgcn_frexp_exp(mx);
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[i][j] = ldexp(M[i][j], -e);
    ex += e;
}

/* q <- q B_t for a row vector q: q'(i) = e(i) sum_j q(j) Abar'(j,i), with the
 * model's BACKWARD mask (hhmm-tayal2009.stan:109-111: the predicate on the
 * previous state j; unmasked otherwise). */
template <int MODEL, int K, int SG = -1>
__device__ __forceinline__ void bwd_row_raw(double (&q)[K], const PairParams<MODEL, K> &pp, const double (&e)[K],
                                            const Obs &o)
{
    if constexpr (SG > 0 && ModelTraits<MODEL>::kTayal) {
        /* the sign class is known: the off rows' terms (0 x A, + 0) dropped,
         * the rest in the same order -- the same bits */
        double qoff = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (!tayal_on(SG, j))
                qoff += q[j];
        double s[K];
#pragma unroll
        for (int i = 0; i < K; ++i) {
            double acc = 0.0;
            bool first = true;
#pragma unroll
            for (int j = 0; j < K; ++j) {
                if (tayal_on(SG, j) && tayal_nz(j, i)) {
                    acc = first ? q[j] * pp.A[j][i] : fma(q[j], pp.A[j][i], acc);
                    first = false;
                }
            }
            s[i] = acc + qoff;
        }
#pragma unroll
        for (int i = 0; i < K; ++i)
            q[i] = s[i] * e[i];
        return;
    }
    double qon[K];
    double qoff = 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        bool on = true;
        if constexpr (ModelTraits<MODEL>::kTayal)
            on = tayal_pred(o.aux, j);
        qon[j] = on ? q[j] : 0.0;
        qoff += on ? 0.0 : q[j];
    }
    double s[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double acc = qon[0] * pp.A[0][i];
#pragma unroll
        for (int j = 1; j < K; ++j)
            acc = fma(qon[j], pp.A[j][i], acc);
        s[i] = acc + qoff;
    }
#pragma unroll
    for (int i = 0; i < K; ++i)
        q[i] = s[i] * e[i];
}

/* Observation of step t (clamped, unconditional). */
template <int MODEL, bool AUX>
__device__ __forceinline__ Obs load_obs(const SeriesPtrs &sp, int t)
{
    Obs o[1];
    load_chunk<MODEL, 1, AUX>(o, sp, t);
    return o[0];
}

/* The chunk products in HBM, pair-major: chunk c of pair p is the K*K
 * record at sc_mat, its exponents / log scale the 3 doubles at sc_mxi. */
template <int K>
__device__ __forceinline__ int64_t sc_mat(const DevArgs &a, int64_t p, int c)
{
    return (p * a.scan_nc + c) * (int64_t)(K * K);
}
__device__ __forceinline__ int64_t sc_mxi(const DevArgs &a, int64_t p, int c, int f)
{
    return (p * a.scan_nc + c) * 3 + f;
}

template <int MODEL, int K, bool BWD>
__global__ void __launch_bounds__(kBlock) scan_prod_kernel(const DevArgs a)
{
    constexpr bool AUX = ModelTraits<MODEL>::kAux;
    constexpr int KP = (K + 1) / 2;
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int64_t G = a.P * (int64_t)a.scan_nc;
    const int64_t g = min((int64_t)blockIdx.x * blockDim.x + threadIdx.x, G - 1);
    const int64_t p = g % a.P;
    const int c = (int)(g / a.P);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int t0 = c * a.scan_cl;
    const int t1 = min(t0 + a.scan_cl, Tp);
    PairParams<MODEL, K> pp;
    load_params<MODEL, K, false>(pp, a, d);
    const double2 *slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        pp.skip_ok &= fill_table<K, false>(lds + (size_t)wave * a.L * KP * 64 + lane, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, AUX>(a, n);

    double F[K][K], Q[K][K];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            F[i][j] = (i == j) ? 1.0 : 0.0;
            Q[i][j] = F[i][j];
        }
    int fex = 0, qex = 0;
    double lsc = 0.0;
    int tb = t0;
    if (c == 0 && !a.seg_nofirst) { /* chunk 0 enters from the model's init vector f_0 (every row) */
        const Obs o0 = load_obs<MODEL, AUX>(sp, 0);
        Em<K> em;
        emit_prob<MODEL, K>(pp, slab, a.L, o0, em);
        double f0[K];
        fwd_init<MODEL, K>(f0, pp, em, o0, lsc, fex);
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                F[i][j] = f0[j];
        tb = 1;
    }
    auto prods = [&](auto sgc, const Obs &o, const Em<K> &em) {
        constexpr int SG = decltype(sgc)::value;
#pragma unroll
        for (int r = 0; r < K; ++r)
            fwd_step_raw<MODEL, K, SG>(F[r], F[r], pp, em.e, o);
        if constexpr (BWD) {
#pragma unroll
            for (int r = 0; r < K; ++r)
                bwd_row_raw<MODEL, K, SG>(Q[r], pp, em.e, o);
        }
    };
    auto step = [&](const Obs &o, bool rn) {
        Em<K> em;
        emit_prob<MODEL, K>(pp, slab, a.L, o, em);
        lsc += em.m;
        /* a wave whose lanes share the step's sign (one series under many
         * draws: C5) takes the masks as constants (round 4) */
        tayal_dispatch<MODEL>(o, pp.skip_ok, [&](auto sgc) { prods(sgc, o, em); });
        if (rn) {
            renorm_mat<K>(F, fex);
            if constexpr (BWD)
                renorm_mat<K>(Q, qex);
        }
    };
    /* Discrete emissions renormalise the products every kBigRenorm-th step
     * (and every step of the chunk's ragged tail) where the pair's parameters
     * bound the shrink (renorm_sparse_safe, FB_BIG's argument: the max stays
     * above 2^-156 between renormalisations; a step grows it by at most K);
     * a wave holding an unsafe pair renormalises every step.  The exponents
     * are exact powers of two either way (round 4: a quarter of the
     * renormalisations, which were a sixth of the phase's VALU at C5). */
    bool sparse = false;
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        sparse = !wave_any(!renorm_sparse_safe<MODEL, K>(pp, slab, a.L));
    Obs onx = load_obs<MODEL, AUX>(sp, tb);
    int t = tb;
    if (sparse) {
        constexpr int G = kBigRenorm;
        Obs og[G];
#pragma unroll
        for (int u = 0; u < G; ++u)
            og[u] = load_obs<MODEL, AUX>(sp, tb + u);
        for (; t + G <= t1; t += G) {
            Obs on[G];
#pragma unroll
            for (int u = 0; u < G; ++u)
                on[u] = load_obs<MODEL, AUX>(sp, t + G + u);
#pragma unroll
            for (int u = 0; u < G; ++u)
                step(og[u], u == G - 1);
#pragma unroll
            for (int u = 0; u < G; ++u)
                og[u] = on[u];
        }
        onx = og[0];
    }
    for (; t < t1; ++t) {
        const Obs o = onx;
        onx = load_obs<MODEL, AUX>(sp, t + 1);
        step(o, true);
    }
    /* pair-major records (sc_mat / sc_mxi): a lane writes whole lines, and
     * the boundary scan's lanes (consecutive chunks of one pair) read
     * consecutive lines */
    double *mf = a.sc_mf + sc_mat<K>(a, p, c);
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            mf[i * K + j] = F[i][j];
            if constexpr (BWD)
                a.sc_qb[sc_mat<K>(a, p, c) + i * K + j] = Q[i][j];
        }
    a.sc_mx[sc_mxi(a, p, c, 0)] = (double)fex;
    a.sc_mx[sc_mxi(a, p, c, 1)] = lsc;
    a.sc_mx[sc_mxi(a, p, c, 2)] = (double)qex;
}

template <int K>
__device__ __forceinline__ void load_mat(const double *base, const DevArgs &a, int c, int64_t p, double (&M)[K][K])
{
    const double *m = base + sc_mat<K>(a, p, c);
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[i][j] = m[i * K + j];
}

/* Phase 2: one wave per pair scans its chunk products, 64 chunks per step of
 * the walk, lane-parallel.  Lane l holds chunk cb + l's product; a
 * Hillis-Steele prefix over the lanes (six levels of K x K products, the
 * partner's matrix by __shfl_up) gives every lane the product of the block's
 * chunks up to its own, and every lane applies it to the vector entering the
 * block, so the vectors entering all 64 chunks come out at once and are
 * stored by their own lanes.  The serial walk (one chunk per ~700 cycles of
 * dependent latency, lane 0 storing) took 2.4 ms at C5.
 * Products of the non-negative chunk matrices keep every entry's relative
 * precision; the partial products carry one exact power-of-two exponent PER
 * ROW (a row is the map from one entering state, and rows can drift apart by
 * more than the double range over a block), as lks_bound_kernel's exponents
 * do at large K.  The reassociated sums change the boundary vectors by a few
 * ulps against the serial walk, far inside the 1e-9 parity tolerance. */
constexpr int kNoExp = -(1 << 30);

template <int K>
struct RowMat {
    double m[K][K]; /* rows with max in [0.5, 1), or zero */
    int rs[K];      /* row i of the value is 2^rs[i] m[i] */
    double ls;      /* additive log scale (nats): the Gaussian emission shifts */
};

/* out 2^ex = f diag(2^rs) m (f any non-negative vector): the terms scaled to
 * the largest entering exponent, out renormalised into [0.5, 1). f == 0:
 * out = 0, ex unchanged. */
template <int K>
__device__ __forceinline__ void vec_rowmat(const double (&f)[K], const double (&m)[K][K], const int (&rs)[K],
                                           double (&out)[K], int &ex)
{
    int E = kNoExp;
#pragma unroll
    for (int i = 0; i < K; ++i)
        E = (f[i] != 0.0) ? max(E, __builtin_amdgcn_frexp_exp(f[i]) + rs[i]) : E;
    double g[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        g[i] = (f[i] != 0.0) ? ldexp(f[i], rs[i] - E) : 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double acc = g[0] * m[0][j];
#pragma unroll
        for (int i = 1; i < K; ++i)
            acc = fma(g[i], m[i][j], acc);
        out[j] = acc;
    }
    int e2 = 0;
    renorm<K>(out, e2);
    ex += (E == kNoExp) ? 0 : E + e2;
}

/* A chunk product as stored by scan_prod_kernel (one exponent for the whole
 * matrix; TR: transposed, the backward map applied to a row vector), fetched
 * a block ahead; `ident` (past the walk's end): the identity. */
template <int K>
struct RawMat {
    double m[K][K];
    double ex, ls;
};

template <int K, bool TR>
__device__ __forceinline__ void rawmat_fetch(const double *base, const DevArgs &a, int c, int64_t p, int xf,
                                             RawMat<K> &R)
{
    const double *m = base + sc_mat<K>(a, p, c);
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            R.m[i][j] = m[(TR ? j : i) * K + (TR ? i : j)];
    R.ex = a.sc_mx[sc_mxi(a, p, c, xf)];
    R.ls = a.sc_mx[sc_mxi(a, p, c, 1)];
}

/* ... in the row-scaled form */
template <int K>
__device__ __forceinline__ void rowmat_from(const RawMat<K> &M, bool ident, RowMat<K> &R)
{
#pragma unroll
    for (int i = 0; i < K; ++i) {
        double mx = 0.0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const double v = ident ? (i == j ? 1.0 : 0.0) : M.m[i][j];
            R.m[i][j] = v;
            mx = fmax(mx, v);
        }
        const int e = __builtin_amdgcn_frexp_exp(mx); /* 0 for a zero row */
#pragma unroll
        for (int j = 0; j < K; ++j)
            R.m[i][j] = ldexp(R.m[i][j], -e);
        R.rs[i] = ident ? e : e + (int)M.ex;
    }
    R.ls = ident ? 0.0 : M.ls;
}

/* R = X Y (X the earlier chunks). */
template <int K>
__device__ __forceinline__ void rowmat_mul(const RowMat<K> &X, const RowMat<K> &Y, RowMat<K> &R)
{
#pragma unroll
    for (int i = 0; i < K; ++i) {
        int e = 0;
        vec_rowmat<K>(X.m[i], Y.m, Y.rs, R.m[i], e);
        R.rs[i] = X.rs[i] + e;
    }
    R.ls = X.ls + Y.ls;
}

template <int K>
__device__ __forceinline__ void rowmat_shfl_up(const RowMat<K> &S, RowMat<K> &D, int d)
{
#pragma unroll
    for (int i = 0; i < K; ++i) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            D.m[i][j] = __shfl_up(S.m[i][j], d);
        D.rs[i] = __shfl_up(S.rs[i], d);
    }
    D.ls = __shfl_up(S.ls, d);
}

/* Inclusive prefix product over the wave's lanes: P_l = M_0 M_1 ... M_l, for
 * the first nb lanes (wave-uniform; ceil(log2 nb) levels). */
template <int K>
__device__ __forceinline__ void rowmat_prefix(RowMat<K> &P, int lane, int nb = 64)
{
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        if (d < nb) { /* wave-uniform; a guard, not a break, so the six levels unroll */
            RowMat<K> X, R;
            rowmat_shfl_up<K>(P, X, d);
            rowmat_mul<K>(X, P, R);
            if (lane >= d)
                P = R;
        }
    }
}

/* One block of the boundary walk: lane l holds the (row-scaled) map of the
 * block's chunk l (identity past the walk's end); v / vsc enter the block
 * (wave-uniform) and leave it after its last live chunk nb - 1.  Lane l
 * returns the vector leaving its chunk, normalised, and its log scale. */
template <int K>
__device__ __forceinline__ void bound_block(RowMat<K> &P, int lane, int nb, double (&v)[K], double &vsc,
                                            double (&out)[K], double &osc)
{
    rowmat_prefix<K>(P, lane, nb);
    int ex = 0;
    vec_rowmat<K>(v, P.m, P.rs, out, ex);
    osc = vsc + (P.ls + kLn2 * ex);
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = __shfl(out[k], nb - 1);
    vsc = __shfl(osc, nb - 1);
}

/* The boundary walk of one direction over items i = 0 .. n-1 (item i is chunk
 * c0 + i forward, chunk ncp-1-i backward), split over the workgroup's
 * kBoundWaves waves (round 4): each wave first multiplies its own range's
 * chunk products into one total (block prefixes, the block totals chained),
 * the totals meet in LDS, each wave forms the vector entering its range from
 * the ones before it, then walks its range storing every boundary vector --
 * twice the products of one wave walking everything, on four waves. */
#ifndef HHMM_BOUND_WAVES
#define HHMM_BOUND_WAVES 4 /* build knob: waves per (pair, direction) of the boundary scan */
#endif
constexpr int kBoundWaves = HHMM_BOUND_WAVES;
/* A walk of at most one block (n <= 64 items: C1's 16 chunks per pair) runs on
 * wave 0 alone, without the range totals: one prefix of ceil(log2 n) levels
 * instead of two six-level prefixes and a workgroup barrier on every wave
 * (C1 0.107 -> 0.121 ms with the four-wave scan).  Build knob. */
#ifndef HHMM_BOUND_SHORT
#define HHMM_BOUND_SHORT 1
#endif

template <int K, bool BW>
__device__ __forceinline__ void bound_walk(const DevArgs &a, int64_t p, int ncp, int c0, int n, double (&v)[K],
                                           double &vsc, RowMat<K> *tot)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool one = HHMM_BOUND_SHORT && n <= 64; /* workgroup-uniform */
    if (one && wave > 0)
        return;
    const int nw = one ? 1 : kBoundWaves;
    const int lo = (int)((int64_t)n * wave / nw), hi = (int)((int64_t)n * (wave + 1) / nw);
    const double *base = BW ? a.sc_qb : a.sc_mf;
    auto chunk = [&](int i) { return BW ? ncp - 1 - i : c0 + i; };
    auto fetch = [&](int ib, RawMat<K> &r) { /* item ib + lane, clamped into the range */
        rawmat_fetch<K, BW>(base, a, chunk(max(min(ib + lane, hi - 1), 0)), p, BW ? 2 : 0, r);
    };
    RawMat<K> nx;
    if (!one) {
    /* ---- 1. the range's total ---- */
    RowMat<K> T;
    {
        RawMat<K> id;
        rowmat_from<K>(id, true, T);
    }
    if (lo < hi)
        fetch(lo, nx);
    for (int ib = lo; ib < hi; ib += 64) {
        RowMat<K> P;
        rowmat_from<K>(nx, ib + lane >= hi, P);
        fetch(ib + 64, nx);
        rowmat_prefix<K>(P, lane, min(hi - ib, 64));
        RowMat<K> B, R;
        const int last = min(hi - ib, 64) - 1;
#pragma unroll
        for (int i = 0; i < K; ++i) {
#pragma unroll
            for (int j = 0; j < K; ++j)
                B.m[i][j] = __shfl(P.m[i][j], last);
            B.rs[i] = __shfl(P.rs[i], last);
        }
        B.ls = __shfl(P.ls, last);
        rowmat_mul<K>(T, B, R);
        T = R;
    }
    if (lane == 0)
        tot[wave] = T;
    __syncthreads();
    /* ---- 2. the vector entering this wave's range ---- */
    for (int w = 0; w < wave; ++w) {
        const RowMat<K> &U = tot[w];
        double o[K];
        int ex = 0;
        vec_rowmat<K>(v, U.m, U.rs, o, ex);
        vsc += U.ls + kLn2 * ex;
#pragma unroll
        for (int k = 0; k < K; ++k)
            v[k] = o[k];
    }
    }
    /* ---- 3. the walk, every boundary vector stored by its own lane ---- */
    if (lo < hi)
        fetch(lo, nx);
    for (int ib = lo; ib < hi; ib += 64) {
        const int i = ib + lane;
        RowMat<K> P;
        rowmat_from<K>(nx, i >= hi, P);
        fetch(ib + 64, nx);
        double out[K], osc;
        bound_block<K>(P, lane, min(hi - ib, 64), v, vsc, out, osc);
        const int c = chunk(i);
        if (!BW && i < hi && c + 1 < ncp) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                a.sc_st[p + a.P * (int64_t)((c + 1) * K + k)] = out[k];
            a.sc_sl[p + a.P * (int64_t)(c + 1)] = osc;
        }
        if (BW && i < hi) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                a.sc_be[p + a.P * (int64_t)((c - 1) * K + k)] = out[k];
            a.sc_bl[p + a.P * (int64_t)(c - 1)] = osc;
        }
    }
}

/* One workgroup of kBoundWaves waves per (pair, direction): blockIdx.y == 0
 * the forward walk (f entering chunks c0 .. ncp-1, the loglik), 1 the
 * backward walk (beta leaving chunks ncp-1 .. 0; chunk c's map applied to a
 * row vector is Q_c^T).  The two are independent. */
template <int MODEL, int K, bool BWD>
__global__ void __launch_bounds__(64 * kBoundWaves) scan_bound_kernel(const DevArgs a)
{
    __shared__ RowMat<K> tot[kBoundWaves];
    const int64_t p = blockIdx.x;
    const bool t0 = threadIdx.x == 0;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + a.scan_cl - 1) / a.scan_cl;
    auto mx = [&](int c, int f) { return a.sc_mx[sc_mxi(a, p, c, f)]; };

    if (blockIdx.y == 0) {
        double f[K];
        double sc;
        int c0;
        if (!a.seg_nofirst) {
            /* chunk 0's product has every row equal to the filter leaving it */
#pragma unroll
            for (int j = 0; j < K; ++j)
                f[j] = a.sc_mf[sc_mat<K>(a, p, 0) + j];
            sc = mx(0, 1) + kLn2 * mx(0, 0);
            c0 = 1;
        } else {
            /* a segment window: chunk 0 enters from the caller's state, which then
             * goes through chunk 0's product like every later chunk */
#pragma unroll
            for (int j = 0; j < K; ++j)
                f[j] = a.seg_enter[p + a.P * (int64_t)j];
            sc = a.seg_enter[p + a.P * (int64_t)K];
            c0 = 0;
        }
        if (t0 && c0 < ncp) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                a.sc_st[p + a.P * (int64_t)(c0 * K + k)] = f[k];
            a.sc_sl[p + a.P * (int64_t)c0] = sc;
        }
        bound_walk<K, false>(a, p, ncp, c0, max(ncp - c0, 0), f, sc, tot);
        /* the last wave leaves with the filter after chunk ncp-1 (wave 0 alone
         * on a short walk; the others returned from it) */
        const int nlast = (HHMM_BOUND_SHORT && ncp - c0 <= 64) ? 0 : kBoundWaves - 1;
        if ((threadIdx.x == 64 * nlast) && (a.outputs & HHMM_OUT_LOGLIK) && a.loglik && !a.seg_nolast)
            a.loglik[p] = log(vsum<K>(f)) + sc;
        return;
    }

    if constexpr (BWD) {
        double b[K];
        /* beta at the last step: unbeta_tk[T] = 1 (Q1), or a segment window's
         * beta leaving it (the caller's) */
        double bsc = a.seg_nolast ? a.seg_leave[p + a.P * (int64_t)K] : 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            b[k] = a.seg_nolast ? a.seg_leave[p + a.P * (int64_t)k] : 1.0;
            if (t0)
                a.sc_be[p + a.P * (int64_t)((ncp - 1) * K + k)] = b[k];
        }
        if (t0)
            a.sc_bl[p + a.P * (int64_t)(ncp - 1)] = bsc;
        bound_walk<K, true>(a, p, ncp, 0, max(ncp - 1, 0), b, bsc, tot);
    }
}

/* Segment summary (hhmm_segment): one lane per pair multiplies its window's
 * chunk products in order, SF = F_0 F_1 ... and SQ = Q_0 Q_1 ..., each
 * renormalised by an exact power of two after every product, the exponents
 * and the Gaussian log scales summed alongside (the K x K
 * summary a rank contributes to the all-gather). */
template <int K>
__device__ __forceinline__ void mat_mul_acc(double (&S)[K][K], const double (&M)[K][K])
{
    double R[K][K];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            double acc = S[i][0] * M[0][j];
#pragma unroll
            for (int l = 1; l < K; ++l)
                acc = fma(S[i][l], M[l][j], acc);
            R[i][j] = acc;
        }
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            S[i][j] = R[i][j];
}

template <int MODEL, int K, bool BWD>
__global__ void __launch_bounds__(kBlock) seg_summary_kernel(const DevArgs a)
{
    const int64_t p = min((int64_t)blockIdx.x * blockDim.x + threadIdx.x, a.P - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int ncp = (pair_len(a, n) + a.scan_cl - 1) / a.scan_cl;
    double SF[K][K], SQ[K][K], M[K][K];
    load_mat<K>(a.sc_mf, a, 0, p, SF);
    if constexpr (BWD)
        load_mat<K>(a.sc_qb, a, 0, p, SQ);
    double fex = a.sc_mx[sc_mxi(a, p, 0, 0)], lsc = a.sc_mx[sc_mxi(a, p, 0, 1)], qex = a.sc_mx[sc_mxi(a, p, 0, 2)];
    for (int c = 1; c < ncp; ++c) {
        int e = 0;
        load_mat<K>(a.sc_mf, a, c, p, M);
        mat_mul_acc<K>(SF, M);
        renorm_mat<K>(SF, e);
        fex += a.sc_mx[sc_mxi(a, p, c, 0)] + e;
        lsc += a.sc_mx[sc_mxi(a, p, c, 1)];
        if constexpr (BWD) {
            e = 0;
            load_mat<K>(a.sc_qb, a, c, p, M);
            mat_mul_acc<K>(SQ, M);
            renorm_mat<K>(SQ, e);
            qex += a.sc_mx[sc_mxi(a, p, c, 2)] + e;
        }
    }
    if constexpr (!BWD) {
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                SQ[i][j] = (i == j) ? 1.0 : 0.0;
    }
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            a.seg_sum[p + a.P * (int64_t)(i * K + j)] = SF[i][j];
            a.seg_sum[p + a.P * (int64_t)(K * K + i * K + j)] = SQ[i][j];
        }
    a.seg_sum[p + a.P * (int64_t)(2 * K * K + 0)] = fex;
    a.seg_sum[p + a.P * (int64_t)(2 * K * K + 1)] = lsc;
    a.seg_sum[p + a.P * (int64_t)(2 * K * K + 2)] = qex;
}

/* Phase 3: the forward-backward sweep of one (pair, T-chunk). */
template <int MODEL, int K, int MODE>
__global__ void __launch_bounds__(kBlock) fb_scan_kernel(const DevArgs a)
{
    constexpr bool AUX = ModelTraits<MODEL>::kAux;
    constexpr int KP = (K + 1) / 2;
    constexpr int C = fb_chunk(K);
    HIP_DYNAMIC_SHARED(double2, lds)
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    /* lane g = pp + Pp * c with Pp = P rounded up to whole waves: every wave
     * lies in ONE T-chunk, so the sweep's wave-uniform chunk bounds (and its
     * unconditional checkpoint prefetches) stay inside that chunk's rows.
     * Lanes pp >= P redo pair P-1 (identical values, benign duplicate stores). */
    const int64_t Pp = scan_lanes_per_chunk(a.P);
    const int64_t G = Pp * (int64_t)a.scan_nc;
    const int64_t g = min((int64_t)blockIdx.x * blockDim.x + threadIdx.x, G - 1);
    const int64_t p = min(g % Pp, a.P - 1);
    const int c = (int)(g / Pp);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tpair = pair_len(a, n);
    FbLane<MODEL, K> ln;
    ln.p = p;
    ln.L = a.L;
    ln.t0 = c * a.scan_cl;
    ln.Tp = max(min(ln.t0 + a.scan_cl, Tpair), ln.t0); /* chunks past the pair's end do nothing */
    ln.cb = ln.t0 / C;
    ln.q = g;
    ln.Qs = G;
    ln.slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    load_params<MODEL, K, false>(ln.pp, a, d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        ln.pp.skip_ok &= fill_table<K, false>(lds + (size_t)wave * a.L * KP * 64 + lane, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, AUX>(a, n);
    const bool live = ln.t0 < Tpair;
    /* a segment window's chunk 0 enters from the state scan_bound_kernel stored */
    const bool entered = c > 0 || a.seg_nofirst;
    ln.noinit = a.seg_nofirst != 0;
    double al[K], be[K];
    double lsa = 0.0, lsb = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        al[k] = (entered && live) ? a.sc_st[p + a.P * (int64_t)(c * K + k)] : 0.0;
        be[k] = 1.0;
        if (fb_base(MODE) != FB_FWD && live)
            be[k] = a.sc_be[p + a.P * (int64_t)(c * K + k)];
    }
    if (entered && live)
        lsa = a.sc_sl[p + a.P * (int64_t)c];
    if (fb_base(MODE) != FB_FWD && live)
        lsb = a.sc_bl[p + a.P * (int64_t)c];
    fb_sweep<MODEL, K, MODE, true>(a, ln, sp, al, lsa, be, lsb);
}

static inline bool model_has_backward(int model)
{
    return model == HHMM_MODEL_HMM_GAUSS || model == HHMM_MODEL_HMM_MULTINOM ||
           model == HHMM_MODEL_HMM_MULTINOM_SEMISUP || model == HHMM_MODEL_TAYAL;
}

static inline bool needs_backward(int model, uint32_t out)
{
    return model_has_backward(model) &&
           (out & (HHMM_OUT_UNBETA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA | HHMM_OUT_FFBS)) != 0;
}

/* ------------------------------------------------------------------ */
/* Launch templates (instantiated per model in hhmm_m_*.hip)            */
/* ------------------------------------------------------------------ */
struct LaunchShape {
    dim3 grid, block;
    size_t lds;
};

/* Probe knob (tools/ab_bench.py --env): a minimum LDS request per workgroup
 * in KiB from the environment variable `name`, which caps how many of the
 * kernel's workgroups share a CU (and so leaves room for the other kernel's). */
static size_t lds_floor(const char *name)
{
    const char *v = probe_env(name);
    return v ? (size_t)atoi(v) * 1024 : 0;
}

static bool shape_for(const DevArgs &a, bool discrete, LaunchShape &s, const char *probe = nullptr)
{
    const int KP = (a.K + 1) / 2;
    size_t per_wave = discrete ? (size_t)a.L * KP * 64 * sizeof(double2) : 0;
    int waves = 4;
    if (probe && probe_env(probe)) /* probe knob (tools/ab_bench.py --env): waves per workgroup, 1..4 */
        waves = std::min(std::max(atoi(probe_env(probe)), 1), 4);
    if (per_wave > 0) {
        while (waves > 0 && per_wave * waves > kLdsLimit)
            --waves;
        if (waves == 0)
            return false;
    }
    const int threads = 64 * waves;
    s.block = dim3(threads);
    s.grid = dim3((unsigned)((a.P + threads - 1) / threads));
    s.lds = per_wave * waves;
    return true;
}

template <int MODEL, int K>
static hhmm_status launch_fb(const DevArgs &a, bool fwd_only, hipStream_t st)
{
    LaunchShape s;
    if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, s, "HHMM_PROBE_FB_WAVES")) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    s.lds = std::max(s.lds, std::min(lds_floor("HHMM_PROBE_FB_LDS_KB"), kLdsLimit));
    const uint32_t extra = HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA | HHMM_OUT_BETA | HHMM_OUT_UNBETA | HHMM_OUT_UNGAMMA;
    const bool ffbs = (a.outputs & HHMM_OUT_FFBS) != 0;
    if (ModelTraits<MODEL>::kGauss && ffbs) /* fb_exp2_lds's table copy */
        s.lds = std::max(s.lds, kExp2TabBytes);
    constexpr bool xchk = !ModelTraits<MODEL>::kAux && ModelTraits<MODEL>::kDiscrete;
    /* every fb_kernel below sweeps x forward over whole series (fb_sweep's inline check) */
    t_data_checked_inline |= xchk && (ffbs || !(a.outputs & (HHMM_OUT_UNALPHA | HHMM_OUT_UNBETA)));
    if (a.outputs & (HHMM_OUT_UNALPHA | HHMM_OUT_UNBETA)) {
        /* log-scale outputs: the log-space recursion; FFBS draws (if any)
         * from the linear filter of the contract in a second launch */
        DevArgs b = a;
        b.outputs &= ~HHMM_OUT_FFBS;
        if (fwd_only)
            hipLaunchKernelGGL((fb_log_kernel<MODEL, K, true>), s.grid, s.block, s.lds, st, b);
        else
            hipLaunchKernelGGL((fb_log_kernel<MODEL, K, false>), s.grid, s.block, s.lds, st, b);
        if (ffbs) {
            DevArgs f = a;
            f.outputs = HHMM_OUT_FFBS;
            f.gamma = nullptr;
            f.loglik = nullptr;
            hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_GAMMA | FB_FFBS>), s.grid, s.block, s.lds, st, f);
        }
    } else if (fwd_only)
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_FWD>), s.grid, s.block, s.lds, st, a);
    else if (MODEL == HHMM_MODEL_HMM_MULTINOM && a.xpk && !(a.outputs & extra) && ffbs)
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_GAMMA | FB_FFBS | FB_PACK>), s.grid, s.block, s.lds, st, a);
    else if (fb_big_ok<MODEL, K>() && a.xpk && !(a.outputs & extra)) {
        constexpr int BIG = fb_big_ok<MODEL, K>() ? FB_GAMMA | FB_PACK | FB_BIG : FB_GAMMA;
        if constexpr (fb_big(BIG))
            (void)hipMemsetAsync(a.rnw, 0, sizeof(int32_t), st); /* the dense-wave list's count */
        hipLaunchKernelGGL((fb_kernel<MODEL, K, BIG>), s.grid, s.block, s.lds, st, a);
        if constexpr (fb_big(BIG)) /* the waves it listed (renorm_sparse_safe) */
            hipLaunchKernelGGL((fb_dense_kernel<MODEL, K, BIG>), dim3(kDenseBlocks), dim3(64),
                               s.lds / (s.block.x / 64), st, a);
    }
    else if (MODEL == HHMM_MODEL_HMM_MULTINOM && a.xpk && !(a.outputs & extra))
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_GAMMA | FB_PACK>), s.grid, s.block, s.lds, st, a);
    else if ((a.outputs & extra) && ffbs)
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_FULL | FB_FFBS>), s.grid, s.block, s.lds, st, a);
    else if (a.outputs & extra)
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_FULL>), s.grid, s.block, s.lds, st, a);
    else if (ffbs)
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_GAMMA | FB_FFBS>), s.grid, s.block, s.lds, st, a);
    else
        hipLaunchKernelGGL((fb_kernel<MODEL, K, FB_GAMMA>), s.grid, s.block, s.lds, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("fb_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* The forward-backward as a parallel scan over T (phases 1-3 above). */
template <int MODEL, int K>
static hhmm_status launch_fb_scan(const DevArgs &a, bool fwd_only, hipStream_t st)
{
    LaunchShape s;
    if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, s)) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const int64_t G = a.P * (int64_t)a.scan_nc;                        /* phase 1 lanes */
    const int64_t G3 = scan_lanes_per_chunk(a.P) * (int64_t)a.scan_nc; /* phase 3 lanes */
    const dim3 gridG((unsigned)((G + s.block.x - 1) / s.block.x));
    const dim3 gridG3((unsigned)((G3 + s.block.x - 1) / s.block.x));
    const uint32_t extra = HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA | HHMM_OUT_BETA | HHMM_OUT_UNBETA | HHMM_OUT_UNGAMMA;
    if (fwd_only) {
        hipLaunchKernelGGL((scan_prod_kernel<MODEL, K, false>), gridG, s.block, s.lds, st, a);
        hipLaunchKernelGGL((scan_bound_kernel<MODEL, K, false>), dim3((unsigned)a.P), dim3(64 * kBoundWaves), 0,
                           st, a);
        hipLaunchKernelGGL((fb_scan_kernel<MODEL, K, FB_FWD>), gridG3, s.block, s.lds, st, a);
    } else {
        hipLaunchKernelGGL((scan_prod_kernel<MODEL, K, true>), gridG, s.block, s.lds, st, a);
        hipLaunchKernelGGL((scan_bound_kernel<MODEL, K, true>), dim3((unsigned)a.P, 2), dim3(64 * kBoundWaves), 0, st,
                           a);
        if (a.outputs & extra)
            hipLaunchKernelGGL((fb_scan_kernel<MODEL, K, FB_FULL>), gridG3, s.block, s.lds, st, a);
        else
            hipLaunchKernelGGL((fb_scan_kernel<MODEL, K, FB_GAMMA>), gridG3, s.block, s.lds, st, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("scan launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* State-parallel decoding for batches too small to hide the per-step
 * latency with other waves (lane-per-pair below ~2 waves per SIMD), or when
 * the caller forces it; K = 2..4 (one lane quad per pair). */
static bool use_vit_states(const DevArgs &a)
{
    if (a.K < 2 || a.K > 4 || (a.flags & HHMM_FLAG_VIT_LANES))
        return false;
    return (a.flags & HHMM_FLAG_VIT_STATES) || a.P < 131072;
}

template <int MODEL, int K>
static hhmm_status launch_viterbi(const DevArgs &a, hipStream_t st, bool packed = false)
{
    if constexpr (K == 2 || K == 4) {
        if (a.vs_nc > 0)
            return launch_vscan<MODEL, K>(a, st);
    }
    if constexpr (K >= 2 && K <= 4) {
        if (use_vit_states(a)) {
            const size_t lds = ((ModelTraits<MODEL>::kDiscrete ? (size_t)a.L : 0) +
                                (ModelTraits<MODEL>::kTayal ? (size_t)3 * K : 0)) * 64 * sizeof(double);
            if (lds > kLdsLimit) {
                set_error("emission column L = %d does not fit in LDS", a.L);
                return HHMM_ERR_UNSUPPORTED;
            }
            const int64_t lanes = 4 * a.P;
            hipLaunchKernelGGL((viterbi_sp_kernel<MODEL, K>), dim3((unsigned)((lanes + 63) / 64)), dim3(64), lds,
                               st, a);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) {
                set_error("viterbi_sp_kernel launch: %s", hipGetErrorString(e));
                return HHMM_ERR_HIP;
            }
            return HHMM_OK;
        }
    }
    LaunchShape s;
    if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, s, "HHMM_PROBE_VIT_WAVES")) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    s.lds = std::max(s.lds, std::min(lds_floor("HHMM_PROBE_VIT_LDS_KB"), kLdsLimit));
    if (packed && fbv_ok<MODEL, K>()) {
        hipLaunchKernelGGL((viterbi_kernel<MODEL, K, fbv_ok<MODEL, K>()>), s.grid, s.block, s.lds, st, a);
    } else {
        /* decodes x itself: viterbi_block's inline check */
        t_data_checked_inline |= !ModelTraits<MODEL>::kAux && ModelTraits<MODEL>::kDiscrete;
        hipLaunchKernelGGL((viterbi_kernel<MODEL, K>), s.grid, s.block, s.lds, st, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("viterbi_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* The fused forward-backward + Viterbi sweep: both emission tables per wave. */
template <int MODEL, int K>
static hhmm_status launch_fbv(const DevArgs &a, hipStream_t st)
{
    const size_t per_wave = 2 * (size_t)a.L * ((K + 1) / 2) * 64 * sizeof(double2);
    int waves = 4;
    while (waves > 0 && per_wave * waves > kLdsLimit)
        --waves;
    if (waves == 0) {
        set_error("emission tables 2*K*L = 2*%d*%d do not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const int threads = 64 * waves;
    hipLaunchKernelGGL((fbv_kernel<MODEL, K>), dim3((unsigned)((a.P + threads - 1) / threads)), dim3(threads),
                       per_wave * waves, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("fbv_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* The phased sweep (HHMM_FLAG_VFB): vfb_kernel, then vfb_dense_kernel over the
 * waves it listed. */
template <int MODEL, int K>
static hhmm_status launch_vfb(const DevArgs &a, hipStream_t st)
{
    LaunchShape s;
    if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, s, "HHMM_PROBE_FB_WAVES")) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    hipError_t e = hipMemsetAsync(a.rnw, 0, sizeof(int32_t), st); /* the dense-wave list's count */
    if (e == hipSuccess) {
        t_data_checked_inline |= !ModelTraits<MODEL>::kAux; /* x (and T) checked in phase 1 */
        hipLaunchKernelGGL((vfb_kernel<MODEL, K>), s.grid, s.block, s.lds, st, a);
        hipLaunchKernelGGL((vfb_dense_kernel<MODEL, K>), dim3(kDenseBlocks), dim3(64), s.lds / (s.block.x / 64), st,
                           a);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        set_error("vfb_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* The split schedule (HHMM_FLAG_FB_SPLIT, C2's profile): the forward sweep
 * alone (x read once: loglik, checkpoints, packed symbols), then the
 * HBM-bound backward sweep on the caller's stream beside the VALU-bound
 * Viterbi on the side stream, which decodes the packed symbols. */
template <int MODEL, int K>
static hhmm_status launch_split(const DevArgs &a, hipStream_t st)
{
    constexpr int MODE = FB_GAMMA | FB_PACK | FB_BIG;
    LaunchShape s;
    if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, s)) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    /* the forward launch sweeps x over whole series (fb_sweep's inline check) */
    t_data_checked_inline |= !ModelTraits<MODEL>::kAux && ModelTraits<MODEL>::kDiscrete;
    hipLaunchKernelGGL((fb_kernel<MODEL, K, MODE, FB_PH_FWD>), s.grid, s.block, s.lds, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("fb_kernel (forward) launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    hipStream_t vs = st;
    hhmm_status r = fork_stream(st, &vs);
    if (r != HHMM_OK)
        return r;
    r = launch_viterbi<MODEL, K>(a, vs, true);
    if (r != HHMM_OK) {
        join_stream(st, vs);
        return r;
    }
    hipLaunchKernelGGL((fb_kernel<MODEL, K, MODE, FB_PH_BWD>), s.grid, s.block, s.lds, st, a);
    e = hipGetLastError();
    if (e != hipSuccess) {
        join_stream(st, vs);
        set_error("fb_kernel (backward) launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return join_stream(st, vs);
}

/* The two calls of a segment window (hhmm_segment; the T-scan of
 * launch_fb_scan split at its exchange point). */
template <int MODEL, int K>
static hhmm_status launch_segment(const DevArgs &a, hipStream_t st)
{
    LaunchShape s;
    if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, s)) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const bool bwd = needs_backward(MODEL, a.outputs);
    if (a.seg_phase == 1) {
        const int64_t G = a.P * (int64_t)a.scan_nc;
        const dim3 gridG((unsigned)((G + s.block.x - 1) / s.block.x));
        const dim3 gridP((unsigned)((a.P + kBlock - 1) / kBlock));
        if (bwd) {
            hipLaunchKernelGGL((scan_prod_kernel<MODEL, K, true>), gridG, s.block, s.lds, st, a);
            hipLaunchKernelGGL((seg_summary_kernel<MODEL, K, true>), gridP, dim3(kBlock), 0, st, a);
        } else {
            hipLaunchKernelGGL((scan_prod_kernel<MODEL, K, false>), gridG, s.block, s.lds, st, a);
            hipLaunchKernelGGL((seg_summary_kernel<MODEL, K, false>), gridP, dim3(kBlock), 0, st, a);
        }
    } else {
        const int64_t G3 = scan_lanes_per_chunk(a.P) * (int64_t)a.scan_nc;
        const dim3 gridG3((unsigned)((G3 + s.block.x - 1) / s.block.x));
        const uint32_t extra = HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA | HHMM_OUT_BETA | HHMM_OUT_UNBETA | HHMM_OUT_UNGAMMA;
        if (bwd) {
            hipLaunchKernelGGL((scan_bound_kernel<MODEL, K, true>), dim3((unsigned)a.P, 2), dim3(64 * kBoundWaves), 0,
                               st, a);
            if (a.outputs & extra)
                hipLaunchKernelGGL((fb_scan_kernel<MODEL, K, FB_FULL>), gridG3, s.block, s.lds, st, a);
            else
                hipLaunchKernelGGL((fb_scan_kernel<MODEL, K, FB_GAMMA>), gridG3, s.block, s.lds, st, a);
        } else {
            hipLaunchKernelGGL((scan_bound_kernel<MODEL, K, false>), dim3((unsigned)a.P), dim3(64 * kBoundWaves), 0,
                               st, a);
            if (a.outputs & (HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA))
                hipLaunchKernelGGL((fb_scan_kernel<MODEL, K, FB_FWD>), gridG3, s.block, s.lds, st, a);
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("segment launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

template <int MODEL, int K>
static hhmm_status run_model_k(const DevArgs &a, const hhmm_request *req, const hhmm_result *res,
                               hipStream_t st)
{
    hhmm_status s = HHMM_OK;
    const uint32_t out = a.outputs;
    if (a.seg_phase) {
        if constexpr (MODEL == HHMM_MODEL_TAYAL_LITE) {
            set_error("segment windows: tayal-lite has no backward pass to split (use hhmm-tayal2009)");
            return HHMM_ERR_UNSUPPORTED;
        } else {
            return launch_segment<MODEL, K>(a, st);
        }
    }
    if (MODEL == HHMM_MODEL_TAYAL_LITE) {
        /* in-sample forward: alpha_tk / unalpha_tk / loglik (hhmm-tayal2009-lite.stan:50-92) */
        if (out & (HHMM_OUT_LOGLIK | HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA)) {
            s = launch_fb<MODEL, K>(a, true, st);
            if (s != HHMM_OK)
                return s;
        }
        /* out-of-sample forward and Viterbi on (x_oos, sign_oos) (:94-158) */
        DevArgs o = a;
        o.Tmax = req->data.T_oos_max;
        o.Tout = req->data.T_oos_max;
        o.T = req->data.T_oos;
        o.x = req->data.x_oos;
        o.sign = req->data.sign_oos;
        o.loglik = nullptr;
        o.alpha = res->alpha_tk_oos;
        o.unalpha = res->unalpha_tk_oos;
        o.outputs = out & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR);
        if (out & HHMM_OUT_ALPHA_OOS)
            o.outputs |= HHMM_OUT_ALPHA;
        if (out & HHMM_OUT_UNALPHA_OOS)
            o.outputs |= HHMM_OUT_UNALPHA;
        if (o.outputs & (HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA)) {
            s = launch_fb<MODEL, K>(o, true, st);
            if (s != HHMM_OK)
                return s;
        }
        if (o.outputs & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR))
            s = launch_viterbi<MODEL, K>(o, st);
        return s;
    }
    const bool any_fwd = (out & (HHMM_OUT_LOGLIK | HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA | HHMM_OUT_BETA |
                                 HHMM_OUT_UNBETA | HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA | HHMM_OUT_FFBS)) != 0;
    /* The Viterbi pass is independent of the forward-backward: it runs on a
     * side stream forked from (and joined back into) the caller's stream, so
     * the VALU-bound decoder's workgroups fill in beside the HBM-bound
     * forward-backward's instead of strictly after them. */
    const bool vit = (out & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR)) != 0;
    /* Both launch shapes are checked before either kernel is enqueued, so an
     * unsupported shape never leaves a kernel running on the side stream
     * while the caller reclaims its buffers. */
    if (any_fwd) {
        LaunchShape chk;
        if (!shape_for(a, ModelTraits<MODEL>::kDiscrete, chk)) {
            set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
            return HHMM_ERR_UNSUPPORTED;
        }
    }
    if constexpr (fbv_ok<MODEL, K>()) {
        /* gamma (+ loglik) and the path in one request, on request: the fused sweep */
        const uint32_t extra = HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA | HHMM_OUT_BETA | HHMM_OUT_UNBETA |
                               HHMM_OUT_UNGAMMA | HHMM_OUT_FFBS;
        if (vit && (out & HHMM_OUT_GAMMA) && !(out & extra) && a.xpk && a.scan_cl == 0 &&
            (a.flags & HHMM_FLAG_FUSED) && !use_vit_states(a))
            return launch_fbv<MODEL, K>(a, st);
        const bool vfb_on = (a.flags & HHMM_FLAG_VFB) ||
                            (HHMM_VFB_DEFAULT && !(a.flags & (HHMM_FLAG_VFB_OFF | HHMM_FLAG_FUSED | HHMM_FLAG_FB_SPLIT |
                                                              HHMM_FLAG_NO_FUSE)));
        if (vit && (out & HHMM_OUT_GAMMA) && (out & HHMM_OUT_ZSTAR) && a.zstar && !(out & extra) && a.xpk &&
            a.rnw && a.scan_cl == 0 && a.vs_nc == 0 && vfb_on && !use_vit_states(a))
            return launch_vfb<MODEL, K>(a, st);
        if (vit && (out & HHMM_OUT_GAMMA) && !(out & extra) && a.xpk && a.scan_cl == 0 && a.vs_nc == 0 &&
            (a.flags & HHMM_FLAG_FB_SPLIT) && !(a.flags & HHMM_FLAG_NO_FUSE) && !use_vit_states(a))
            return launch_split<MODEL, K>(a, st);
    }
    hipStream_t vs = st;
    if (vit && any_fwd && !(a.flags & HHMM_FLAG_NO_FUSE)) {
        s = fork_stream(st, &vs);
        if (s != HHMM_OK)
            return s;
        s = launch_viterbi<MODEL, K>(a, vs);
        if (s != HHMM_OK) {
            join_stream(st, vs);
            return s;
        }
    }
    if (any_fwd) {
        if (a.scan_cl > 0 && !(out & HHMM_OUT_FFBS))
            s = launch_fb_scan<MODEL, K>(a, !needs_backward(MODEL, out), st);
        else
            s = launch_fb<MODEL, K>(a, !needs_backward(MODEL, out), st);
        if (s != HHMM_OK) {
            if (vs != st)
                join_stream(st, vs); /* the caller's stream still orders the running decoder */
            return s;
        }
    }
    if (vs != st)
        return join_stream(st, vs);
    if (vit)
        s = launch_viterbi<MODEL, K>(a, st);
    return s;
}

/* Dispatch on K for the K values [KK, KHI] this translation unit instantiates. */
template <int MODEL, int KK, int KHI>
static hhmm_status run_model_range(const DevArgs &a, const hhmm_request *req, const hhmm_result *res,
                                   hipStream_t st)
{
    if constexpr (KK > KHI) {
        set_error("K = %d not supported by this build of model %d", a.K, MODEL);
        return HHMM_ERR_UNSUPPORTED;
    } else {
        if (a.K == KK)
            return run_model_k<MODEL, KK>(a, req, res, st);
        return run_model_range<MODEL, KK + 1, KHI>(a, req, res, st);
    }
}

} // namespace hhmm
