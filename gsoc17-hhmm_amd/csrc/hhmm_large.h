/*
 * hhmm_large.h -- the HMM family at large K (8 < K <= 32):
 * hmm/stan/hmm.stan and hmm/stan/hmm-multinom.stan with free `int<lower=1> K`
 * (hmm-multinom.stan:9), e.g. the 23-state flattened HHMMs the reference
 * discusses (log.md:657, tayal2009/main.Rmd:310-346).
 *
 * Layout: a GROUP of G lanes owns one (series, draw) pair, lane j state j
 * (lanes j >= K idle): G = 16 for K <= 16 (four pairs per wave), G = 32 above
 * (two).  Idle lanes hold the neutral entry (0 in the filters, -inf in the
 * max-plus recursion), so every loop over states runs a compile-time G.  The K x K transition matrix is
 * split by column and row over the group: lane j keeps column j (forward,
 * Viterbi) and row j (backward) in registers.  Each step the group exchanges
 * its state vector through a per-pair LDS slot -- every lane writes its
 * entry, then reads all K back as broadcast ds_read_b128 -- and reduces
 * across the group with DPP / ds_swizzle butterflies (renormalisation max,
 * gamma sums).
 * The emission table (multinomial: phi[l][j] per pair) sits in LDS so lane
 * j reads its own state's column for the step's symbol.
 *
 * Arithmetic is the lane-per-pair kernels' (hhmm_hmm.h) with the K-vector
 * spread over lanes: the same linear-space scaled filter (K FMAs per state,
 * as four interleaved chains; an exact power-of-two renormalisation per
 * step), the same
 * checkpoint-and-recompute backward sweep, and for the Viterbi the same
 * candidate order (delta + log A) + emission with strict '>' and the Q3 NaN
 * row -- so paths and logp_zstar are bit-identical to the oracle.
 * Back-pointers are one byte per (pair, state, t), [P][K][T_max] (16-byte
 * aligned rows); the backtrack walks them kLBack steps at a time, each lane
 * holding its state's bytes of the chunk and the path state passed by a
 * shuffle per step.
 *
 * Outputs: loglik, alpha_tk, beta_tk, ungamma_tk, gamma_tk, zstar_t,
 * logp_zstar (the log-scale unalpha / unbeta and FFBS stay on K <= 8).
 * Bound: VALU -- K^2 FMAs per pair-step (529 at K = 23) against 8K output
 * bytes; the output stores are 8 B per lane (two pairs per wave).
 */
#pragma once
#include <hip/hip_runtime.h>

#include "hhmm_device.h"

namespace hhmm {

#ifndef HHMM_LK_XCD
#define HHMM_LK_XCD 1 /* build knob: XCD-contiguous pair ranges (lk_group) */
#endif
constexpr int kLChunk = 8;  /* steps per forward checkpoint */
constexpr int kLBack = 16;  /* backtrack steps per back-pointer chunk */
/* The filters renormalise (a group max, an exact power of two) every kLRenorm
 * steps, not every step: the group max is a five-level reduction on the
 * step's dependency chain, and between renormalisations the vectors shrink by
 * the per-step factor only (at least b >= 2^-39 per step below, so >= 2^-312
 * over eight steps), far above the subnormal range; they grow by at most K per
 * step.  A multiple-of-kLRenorm step (every checkpoint step: kLChunk is a
 * multiple) is always renormalised.  Build knob HHMM_LK_RENORM (round 5: 8;
 * rounds 3-4: 4). */
#ifndef HHMM_LK_RENORM
#define HHMM_LK_RENORM 8
#endif
constexpr int kLRenorm = HHMM_LK_RENORM;
static_assert(kLChunk % kLRenorm == 0, "checkpoint steps are renormalisation steps");
/* The cadence is taken only where the pair's parameters bound the shrink:
 * b = phi_min * min(min_i rowmax_i(A), min_i colmax_i(A)) >= 2^-39 (the lane
 * kernels' renorm_sparse_safe argument, hhmm_hmm.h).  Gaussian emissions have
 * no such bound (a density ratio can be anything), and a wave holding an
 * unbounded pair renormalises every step. */
constexpr double kLRenormSafeBound = 0x1p-39;

/* bytes per (pair, state) back-pointer row */
__host__ __device__ constexpr int lk_row_bytes(int Tmax) { return (Tmax + 15) & ~15; }

template <int MODEL>
struct LkTraits {
    static constexpr bool kGauss = (MODEL == HHMM_MODEL_HMM_GAUSS);
};

/* Group reductions over the 32 lanes of a pair (one aligned half of the
 * wave): a butterfly of DPP moves inside each 16-lane row (quad xor 1, quad
 * xor 2, half-row mirror, row mirror) and one ds_swizzle xor 16 across the
 * two rows -- a few cycles per level instead of the LDS crossbar round trip
 * of a ds_bpermute shuffle.  Every level combines two mirror-image partial
 * results, and IEEE addition is commutative, so all lanes end with the same
 * bits. */
template <int CTRL>
__device__ __forceinline__ double lk_dpp(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
/* lane ^ 16 by v_permlane16_swap: a VALU exchange (lane_xor16) instead of a
 * ds_swizzle round trip through the LDS crossbar, on the dependency chain of
 * every group reduction (N1 40.94 against 41.19 ms with ds_swizzle, outputs
 * identical; profiles/r04g_ab_n1.log).  The MFMA chunk-product kernel keeps its
 * ds_bpermute column reductions (__shfl_xor): there the VALU form measured
 * 168.8 against 156.8 ms. */
__device__ __forceinline__ double lk_xor16(double v) { return lane_xor16(v); }
constexpr int kDppXor1 = 0xB1;       /* quad_perm [1,0,3,2] */
constexpr int kDppXor2 = 0x4E;       /* quad_perm [2,3,0,1] */
constexpr int kDppHalfMirror = 0x141;
constexpr int kDppMirror = 0x140;

template <int G>
__device__ __forceinline__ double grp_max(double v)
{
    v = fmax(v, lk_dpp<kDppXor1>(v));
    v = fmax(v, lk_dpp<kDppXor2>(v));
    v = fmax(v, lk_dpp<kDppHalfMirror>(v));
    v = fmax(v, lk_dpp<kDppMirror>(v));
    if constexpr (G == 32)
        v = fmax(v, lk_xor16(v));
    return v;
}
template <int G>
__device__ __forceinline__ double grp_sum(double v)
{
    v = v + lk_dpp<kDppXor1>(v);
    v = v + lk_dpp<kDppXor2>(v);
    v = v + lk_dpp<kDppHalfMirror>(v);
    v = v + lk_dpp<kDppMirror>(v);
    if constexpr (G == 32)
        v = v + lk_xor16(v);
    return v;
}

/* Per-lane state of one pair's group.  KM (<= G, a multiple of 4): the
 * state capacity of the compile-time loops and of the per-lane K-vectors
 * (column / row of A, the exchanged state vector): 24 for 16 < K <= 24 keeps
 * the forward-backward at two waves per SIMD (lanes 24..31 of the group stay
 * idle without a register copy of their neutral entries). */
template <int MODEL, int G, int KM>
struct LkLane {
    int j;          /* this lane's state (>= K: idle) */
    bool on;        /* j < K */
    int64_t p, n, d;
    int Tp, K, L;
    double col[KM]; /* A[i][j] (probabilities; Viterbi: log) */
    double row[KM]; /* A[j][i] (backward) */
    double pj;       /* p_1k[j] */
    double mu, isig, c0, lsig; /* gauss, state j */
    double *xch;     /* this pair's LDS exchange slots: 2 x G doubles */
    const double *tab; /* multinomial: this pair's [L][G] emission table */
    const hhmm_exp2_entry *etab = hhmm_exp2_tab; /* lk_ffbs_kernel (Gaussian): the det exp's LDS copy */
    bool dense;        /* wave-uniform: renormalise every step (kLRenormSafeBound) */
};

/* The group index of this lane's group (workgroup * groups per block + group;
 * lk_group: clamped to nq - 1). */
template <int G>
__device__ __forceinline__ int64_t lk_group_raw()
{
#if HHMM_LK_XCD
    /* a wave holds two or four pairs, so a gamma / alpha row's 128-byte line
     * (16 pairs) spans 4-8 waves of 2 workgroups: keep them on one XCD */
    return xcd_block() * (blockDim.x / G) + threadIdx.x / G;
#else
    return (int64_t)blockIdx.x * (blockDim.x / G) + threadIdx.x / G;
#endif
}
template <int G>
__device__ __forceinline__ int64_t lk_group(int64_t nq)
{
    return min(lk_group_raw<G>(), nq - 1);
}

template <int MODEL, int G, int KM>
__device__ __forceinline__ void lk_setup(LkLane<MODEL, G, KM> &ln, const DevArgs &a, double *lds, bool LOG, int64_t p)
{
    const int tid = threadIdx.x;
    const int g = tid / G;                 /* group in the workgroup */
    const int gpb = blockDim.x / G;        /* groups per workgroup */
    ln.j = tid % G;
    ln.K = a.K;
    ln.L = a.L;
    ln.on = ln.j < a.K;
    ln.p = p;
    pair_coords(a, ln.p, ln.n, ln.d);
    ln.Tp = pair_len(a, ln.n);
    const int jj = ln.on ? ln.j : 0;
    const int64_t S = a.S, d = ln.d;
    double rawc[KM], rawr[KM];
#pragma unroll
    for (int i = 0; i < KM; ++i) {
        rawc[i] = 0.0;
        rawr[i] = 0.0;
        if (i < a.K) {
            rawc[i] = a.A_ij[d + S * ((int64_t)i + (int64_t)a.K * jj)];
            rawr[i] = a.A_ij[d + S * ((int64_t)jj + (int64_t)a.K * i)];
        }
    }
#pragma unroll
    for (int i = 0; i < KM; ++i) {
        ln.col[i] = (LOG && i < a.K) ? dev_cr_log(rawc[i]) : rawc[i];
        ln.row[i] = rawr[i];
    }
    ln.pj = a.p_1k[d + S * jj];
    if constexpr (LkTraits<MODEL>::kGauss) {
        const double sg = a.sigma_k[d + S * jj];
        ln.mu = a.mu_k[d + S * jj];
        ln.isig = 1.0 / sg;
        ln.lsig = dev_cr_log(sg);
        ln.c0 = HHMM_NEG_LOG_SQRT_TWO_PI - ln.lsig;
    }
    /* LDS: [groups][2][G] exchange, then [groups][L][G] tables */
    ln.xch = lds + (size_t)g * 2 * G;
    double *tab = lds + (size_t)gpb * 2 * G + (size_t)g * a.L * G;
    ln.tab = tab;
    double emin = 1.0 / 0.0;
    if constexpr (!LkTraits<MODEL>::kGauss) {
        for (int l0 = 0; l0 < a.L; l0 += 8) {
            double v[8];
#pragma unroll
            for (int r = 0; r < 8; ++r)
                v[r] = a.phi_k[d + S * ((int64_t)jj + (int64_t)a.K * min(l0 + r, a.L - 1))];
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (l0 + r < a.L) {
                    tab[(l0 + r) * G + ln.j] = (LOG && ln.on) ? dev_cr_log(v[r]) : v[r];
                    emin = fmin(emin, v[r]);
                }
        }
    }
    ln.dense = true;
    if (!LOG && !LkTraits<MODEL>::kGauss) {
        double rmax = rawr[0], cmax = rawc[0];
#pragma unroll
        for (int i = 1; i < KM; ++i)
            if (i < a.K) {
                rmax = fmax(rmax, rawr[i]);
                cmax = fmax(cmax, rawc[i]);
            }
        /* group minima of phi and of the row / column maxima (idle lanes +inf;
         * every lane takes part in the butterflies); a NaN parameter anywhere
         * in the pair or an unsafe pair makes the wave dense */
        const double inf = 1.0 / 0.0;
        const double ge = -grp_max<G>(ln.on ? -emin : -inf);
        const double gm = -grp_max<G>(ln.on ? -fmin(rmax, cmax) : -inf);
        const bool bad = !(ge * gm >= kLRenormSafeBound) || (ln.on && !(emin * fmin(rmax, cmax) >= 0.0));
        ln.dense = __builtin_amdgcn_readfirstlane((int)(__ballot(bad) != 0)) != 0;
    }
    __syncthreads();
}

/* Observations come a block of G steps at a time: lane j of the group
 * loads step 32b + j (clamped, unconditional), one load instruction per 32
 * steps, issued a block ahead; step t's symbol is then one shuffle from lane
 * t % 32 of the group. */
template <int MODEL, int G>
struct LkObs {
    int x;
    double xr;
};

template <int MODEL, int G, int KM>
__device__ __forceinline__ LkObs<MODEL, G> lk_block(const LkLane<MODEL, G, KM> &ln, const DevArgs &a, int b)
{
    const int tc = min(max(b * G + ln.j, 0), a.Tmax - 1);
    LkObs<MODEL, G> o;
    o.x = 1;
    o.xr = 0.0;
    if constexpr (LkTraits<MODEL>::kGauss)
        o.xr = a.xr[ln.n + a.N * (int64_t)tc];
    else
        o.x = a.x[ln.n + a.N * (int64_t)tc];
    return o;
}

/* step u of the block: lane u of the group; u is wave-uniform, so two scalar
 * reads (one per group of the wave) and a select replace a shuffle */
template <int G>
__device__ __forceinline__ int lk_pick(int v, int u)
{
    const int a = __builtin_amdgcn_readlane(v, u), b = __builtin_amdgcn_readlane(v, u + G);
    if constexpr (G == 32) {
        return (threadIdx.x & 32) ? b : a;
    } else {
        const int c = __builtin_amdgcn_readlane(v, u + 32), d = __builtin_amdgcn_readlane(v, u + 48);
        const int q = (threadIdx.x >> 4) & 3;
        return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
    }
}

/* step u of the block when u may differ between the wave's two groups (the
 * backward sweep's chunks of pairs with different T): a shuffle */
template <int MODEL, int G>
__device__ __forceinline__ void lk_get_var(const LkObs<MODEL, G> &blk, int u, int &x, double &xr)
{
    x = 1;
    xr = 0.0;
    if constexpr (LkTraits<MODEL>::kGauss)
        xr = __shfl(blk.xr, u, G);
    else
        x = __shfl(blk.x, u, G);
}

/* step u of the block, u the same for the whole wave (the forward sweeps run
 * both groups in lockstep over t) */
template <int MODEL, int G>
__device__ __forceinline__ void lk_get(const LkObs<MODEL, G> &blk, int u, int &x, double &xr)
{
    x = 1;
    xr = 0.0;
    if constexpr (LkTraits<MODEL>::kGauss) {
        const long long b = __double_as_longlong(blk.xr);
        const int lo = lk_pick<G>((int)b, u), hi = lk_pick<G>((int)(b >> 32), u);
        xr = __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
    } else {
        x = lk_pick<G>(blk.x, u);
    }
}

/* Stan's normal_lpdf(y | mu_j, sigma_j), as gauss_lpdf. */
template <int MODEL, int G, int KM>
__device__ __forceinline__ double lk_lpdf(const LkLane<MODEL, G, KM> &ln, double y)
{
    const double z = (y - ln.mu) * ln.isig;
    const double z2 = z * z;
    return ln.c0 + (-0.5 * z2);
}

/* Linear-space emission e_t(j) and its log scale m (gauss: densities over
 * their group max, as emit_prob); idle lanes 0. */
template <int MODEL, int G, int KM>
__device__ __forceinline__ double lk_emit(const LkLane<MODEL, G, KM> &ln, int x, double xr, double &m)
{
    if constexpr (LkTraits<MODEL>::kGauss) {
        const double lp = ln.on ? lk_lpdf<MODEL, G, KM>(ln, xr) : dev_ninf();
        m = grp_max<G>(lp);
        return ln.on ? exp(lp - m) : 0.0;
    } else {
        m = 0.0;
        const int xc = min(max(x, 1), ln.L);
        return ln.on ? ln.tab[(xc - 1) * G + ln.j] : 0.0;
    }
}

/* The group's vector v (this lane's entry) through LDS slot `slot`: w[i] = v
 * of lane i for all G lanes (idle lanes carry the neutral entry). */
template <int G, int KM>
__device__ __forceinline__ void grp_exchange(double *xch, int slot, int j, double v, double (&w)[KM])
{
    double *s = xch + slot * G;
    s[j] = v;
    /* The group is inside one wave, and a wave's LDS instructions execute in
     * order, so its reads see its own write: only the compiler must keep them
     * in order (a fence here would also wait for every outstanding global
     * load and store, i.e. an HBM round trip per step). */
    __asm__ __volatile__("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < KM; i += 2) {
        const double2 q = *reinterpret_cast<const double2 *>(s + i);
        w[i] = q.x;
        w[i + 1] = q.y;
    }
}

/* Power-of-two renormalisation over the group (renorm<K>). */
template <int G>
__device__ __forceinline__ double grp_renorm(double v, int &ex)
{
    const double mx = grp_max<G>(v);
    const int e = __builtin_amdgcn_frexp_exp(mx);
    ex += e;
    return ldexp(v, -e);
}

/* grp_renorm on every kLRenorm-th step t (every step when `dense`, a
 * wave-uniform flag) */
template <int G>
__device__ __forceinline__ double grp_renorm_at(double v, int &ex, int t, bool dense)
{
    return (dense || t % kLRenorm == 0) ? grp_renorm<G>(v, ex) : v;
}

/* sum_i w_i c_i over the G entries (idle ones 0 x 0) as four interleaved fma
 * chains (a quarter of the dependent latency of one chain; the posteriors are
 * tolerance outputs, 1e-9 relative, so the association is free) */
template <int KM>
__device__ __forceinline__ double lk_dot(const double (&w)[KM], const double (&c)[KM])
{
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < KM; ++i)
        acc[i & 3] = fma(w[i], c[i], acc[i & 3]);
    return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

/* alpha_t(j) = e_t(j) * sum_i alpha_{t-1}(i) A(i, j) (fwd_step_raw) */
template <int MODEL, int G, int KM>
__device__ __forceinline__ double lk_fwd(const LkLane<MODEL, G, KM> &ln, const double (&w)[KM], double e)
{
    return ln.on ? lk_dot<KM>(w, ln.col) * e : 0.0;
}

/* beta_{t-1}(j) = sum_i A(j, i) b_i, b_i = e_t(i) beta_t(i) (bwd_step) */
template <int MODEL, int G, int KM>
__device__ __forceinline__ double lk_bwd(const LkLane<MODEL, G, KM> &ln, const double (&w)[KM])
{
    return ln.on ? lk_dot<KM>(w, ln.row) : 0.0;
}

template <int MODEL, int G, int KM>
__device__ __forceinline__ void lk_put(double *out, const DevArgs &a, const LkLane<MODEL, G, KM> &ln, int t, double v)
{
    if (ln.on && out)
        out[ln.p + a.P * ((int64_t)t + (int64_t)a.Tout * ln.j)] = v;
}

/* Forward-backward: loglik, alpha, beta, ungamma, gamma.  One group sweeps a
 * whole series, or -- under the parallel scan over T (a.scan_cl > 0,
 * hhmm_lkscan.h) -- one T-chunk [t0, t1) of a pair (group q = pair + P *
 * chunk), entering with the forward state f_{t0-1} and leaving with beta at
 * t1 - 1 that the scan computed (the log-likelihood is the scan's then). */
template <int MODEL, int G, int KM>
__global__ void __launch_bounds__(kBlock) lk_fb_kernel(const DevArgs a)
{
    HIP_DYNAMIC_SHARED(double, lds)
    const bool scan = a.scan_cl > 0;
    const int64_t nq = scan ? a.P * (int64_t)a.scan_nc : a.P;
    constexpr int KH = KM;
    const int64_t q = lk_group<G>(nq);
    const int64_t pq = scan ? q % a.P : q;
    const int cq = scan ? (int)(q / a.P) : 0;
    LkLane<MODEL, G, KM> ln;
    lk_setup<MODEL, G, KM>(ln, a, lds, false, pq);
    const bool st = ln.on; /* the lane that stores state j's outputs */
    auto fwd = [&](const double (&wv)[KH], double e) -> double {
        const double d = lk_dot<KH>(wv, ln.col);
        return ln.on ? d * e : 0.0;
    };
    auto bwd = [&](const double (&wv)[KH]) -> double {
        const double d = lk_dot<KH>(wv, ln.row);
        return ln.on ? d : 0.0;
    };
    auto xchg = [&](int sl, double v, double (&wv)[KH]) { grp_exchange<G, KM>(ln.xch, sl, ln.j, v, wv); };
    auto put = [&](double *o, int t, double v) {
        if (st && o)
            o[ln.p + a.P * ((int64_t)t + (int64_t)a.Tout * ln.j)] = v;
    };
    const uint32_t out = a.outputs;
    const bool need_bwd = (out & (HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA)) != 0;
    const bool gamma_only = (out & (HHMM_OUT_ALPHA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA)) ==
                            HHMM_OUT_GAMMA && a.gamma;
    /* this group's span (uniform over the group; the wave's two groups may differ) */
    const int t0 = scan ? cq * a.scan_cl : 0;
    const int t1 = scan ? max(min(t0 + a.scan_cl, ln.Tp), t0) : ln.Tp;
    const int K = ln.K;
    const int64_t sbase = ((int64_t)pq * a.scan_nc + cq) * K + (ln.on ? ln.j : 0); /* scan vectors */
    double w[KH];
    int slot = 0;
    auto ckpt = [&](int c) -> double & { return a.ckpt[q + nq * ((int64_t)c * K + (ln.on ? ln.j : 0))]; };

    /* ---- forward: alpha_1 (hmm.stan:30 Q2 / hmm-multinom.stan:31) at t = 0,
     * or the scan's entry state, then the recursion.  Every group of the wave
     * walks t = t0, t0 + 1, ... from a multiple of G (its span's start), so the
     * step's position in the observation block, t % G, is the same for the
     * wave's groups even when they belong to different T-chunks. ---- */
    LkObs<MODEL, G> bcur, bnxt = lk_block<MODEL, G, KM>(ln, a, t0 / G);
    bcur = bnxt;
    double al = 0.0, lsc = 0.0;
    int ex = 0;
    if (t0 > 0 || (scan && a.seg_nofirst)) { /* a segment window's chunk 0 enters too */
        al = (ln.on && t0 < t1) ? a.sc_st[sbase] : 0.0;
        lsc = t0 < t1 ? a.sc_sl[(int64_t)pq * a.scan_nc + cq] : 0.0;
    }
    for (int t = t0; t < t1; ++t) {
        const int u = t % G;
        if (u == 0) { /* group-uniform: next block of observations, prefetch the one after */
            bcur = bnxt;
            bnxt = lk_block<MODEL, G, KM>(ln, a, t / G + 1);
        }
        int x;
        double xr, m;
        lk_get<MODEL, G>(bcur, u, x, xr);
        if (t == 0 && !a.seg_nofirst) {
            if constexpr (LkTraits<MODEL>::kGauss) {
                /* log(p_1k) + SUM_k normal_lpdf(x[1] | mu_k, sigma_k): alpha_1 = p_1k */
                const double z = (xr - ln.mu) * ln.isig;
                const double tk = ln.on ? (HHMM_NEG_LOG_SQRT_TWO_PI - ln.lsig) + (-0.5 * (z * z)) : 0.0;
                lsc += grp_sum<G>(tk);
                al = ln.on ? ln.pj : 0.0;
            } else {
                const double e = lk_emit<MODEL, G, KM>(ln, x, xr, m);
                al = ln.on ? ln.pj * e : 0.0;
            }
            al = grp_renorm<G>(al, ex);
        } else {
            const double e = lk_emit<MODEL, G, KM>(ln, x, xr, m);
            xchg(slot, al, w);
            slot ^= 1;
            lsc += m;
            al = grp_renorm_at<G>(fwd(w, e), ex, t, ln.dense);
        }
        if (!need_bwd) {
            if ((out & HHMM_OUT_ALPHA) && a.alpha)
                put(a.alpha, t, al / grp_sum<G>(al));
        } else if ((t - t0) % kLChunk == 0 && st) {
            ckpt((t - t0) / kLChunk) = al;
        }
    }
    if (!scan) {
        const double sa = grp_sum<G>(al); /* every lane takes part in the shuffle */
        if ((out & HHMM_OUT_LOGLIK) && a.loglik && ln.j == 0)
            a.loglik[ln.p] = log(sa) + (lsc + kLn2 * ex);
    }
    if (!need_bwd || t1 <= t0)
        return;

    /* ---- backward sweep, chunk by chunk from the end: recompute alpha from
     * the checkpoint (prefetched a chunk ahead), then walk the chunk
     * backwards emitting the posteriors and stepping beta (bwd_chunk) ---- */
    double be = ln.on ? (scan ? a.sc_be[sbase] : 1.0) : 0.0; /* unbeta_tk[T] = 1 (Q1): beta_T uniform */
    int bex = 0;
    constexpr int CPB = G / kLChunk; /* chunks per observation block */
    const int nck = (t1 - t0 + kLChunk - 1) / kLChunk;
    const int b0 = t0 / G; /* the span starts on a block boundary */
    int cb = (nck - 1) / CPB;
    LkObs<MODEL, G> ob = lk_block<MODEL, G, KM>(ln, a, b0 + cb), obp = lk_block<MODEL, G, KM>(ln, a, b0 + cb - 1);
    double ck = ckpt(nck - 1), ckn = ckpt(max(nck - 2, 0));
    for (int c = nck - 1; c >= 0; --c) {
        if (c / CPB != cb) { /* group-uniform: step back one observation block */
            cb = c / CPB;
            ob = obp;
            obp = lk_block<MODEL, G, KM>(ln, a, b0 + cb - 1);
        }
        const int tc = t0 + c * kLChunk;
        const int ub = tc % G; /* the chunk's first step inside the block */
        double es[kLChunk];
#pragma unroll
        for (int u = 0; u < kLChunk; ++u) {
            int x;
            double xr, m;
            lk_get_var<MODEL, G>(ob, ub + u, x, xr);
            es[u] = lk_emit<MODEL, G, KM>(ln, x, xr, m);
        }
        double abuf[kLChunk];
        abuf[0] = ln.on ? ck : 0.0;
        ck = ckn;
        ckn = ckpt(max(c - 2, 0));
        int exb = 0;
#pragma unroll
        for (int u = 1; u < kLChunk; ++u) {
            abuf[u] = 0.0;
            if (tc + u < t1) { /* group-uniform */
                xchg(slot, abuf[u - 1], w);
                slot ^= 1;
                abuf[u] = grp_renorm_at<G>(fwd(w, es[u]), exb, tc + u, ln.dense);
            }
        }
        /* gamma-only normaliser: sum_j alpha_t(j) beta_t(j) does not depend on t
         * (alpha_t = e_t .* A' alpha_{t-1} and beta_{t-1} = A (e_t .* beta_t) give
         * sum_i alpha_{t-1}(i) beta_{t-1}(i) = sum_j alpha_t(j) beta_t(j)), so
         * between two renormalisations of the recomputed alpha and of beta --
         * both at steps t with t % kLRenorm == 0, which the walk crosses only
         * after step t's gamma -- the group sum of one step serves the next
         * ones: one five-level sum and one reciprocal per kLRenorm steps instead
         * of per step.  The walk's own rounding moves the sum by a few ulps per
         * step (non-negative terms), far inside gamma's 1e-9 tolerance.  Dense
         * waves renormalise every step and sum every step. */
        double rsg = 0.0;
        bool direct = false, fresh = true;
#pragma unroll
        for (int u = kLChunk - 1; u >= 0; --u) {
            const int t = tc + u;
            if (t >= t1)
                continue;
            const double av = abuf[u];
            if (gamma_only) {
                /* gamma = (alpha .* beta) / sum: the normalisations cancel, one
                 * group sum per step instead of three (emit_posteriors' FB_GAMMA
                 * form); the reference's normalised-vector formula where the
                 * product underflows (group-uniform test) */
                const double ug = av * be;
                if (fresh || ln.dense || (t + 1) % kLRenorm == 0) { /* group-uniform */
                    const double sg = grp_sum<G>(ug);
                    direct = sg > kGammaDirect;
                    /* the refined reciprocal (fast_rcp: within an ulp; gamma is a
                     * tolerance output) instead of an IEEE division per step */
                    rsg = direct ? fast_rcp(sg) : 0.0;
                    fresh = false;
                }
                if (direct) {
                    put(a.gamma, t, ug * rsg);
                } else {
                    const double sa = grp_sum<G>(av), sb = grp_sum<G>(be);
                    const double un = (av / sa) * (be / sb);
                    put(a.gamma, t, un / grp_sum<G>(un));
                }
            } else {
            const double sa = grp_sum<G>(av), sb = grp_sum<G>(be);
            if ((out & HHMM_OUT_ALPHA) && a.alpha)
                put(a.alpha, t, av / sa);
            if ((out & HHMM_OUT_BETA) && a.beta)
                put(a.beta, t, be / sb);
            if (out & (HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA)) {
                /* gamma = normalize(alpha .* beta) from the normalised vectors (hmm.stan:89-96) */
                const double ug = (av / sa) * (be / sb);
                if ((out & HHMM_OUT_UNGAMMA) && a.ungamma)
                    put(a.ungamma, t, ug);
                if ((out & HHMM_OUT_GAMMA) && a.gamma) {
                    const double sg = grp_sum<G>(ug);
                    put(a.gamma, t, ug / sg);
                }
            }
            }
            if (t > t0) {
                xchg(slot, es[u] * be, w);
                slot ^= 1;
                be = grp_renorm_at<G>(bwd(w), bex, t, ln.dense);
            }
        }
    }
}

/* ---- Viterbi (hmm.stan:98-130; hmm-multinom.stan:100-132) ---- */

/* SSE2 maxCoeff order of stan_max_vec for a runtime K (oracle stan_max_vec). */
template <int G>
__device__ __forceinline__ double stan_max_rt(const double (&d)[G], int n) /* G: the array capacity */
{
    if (n < 2)
        return d[0];
    const int aligned = n & ~1, aligned2 = n & ~3;
    double r0a = d[0], r0b = d[1];
    if (aligned > 2) {
        double r1a = d[2], r1b = d[3];
#pragma unroll
        for (int i = 4; i + 4 <= G; i += 4) {
            if (i < aligned2) {
                r0a = sse_max(r0a, d[i]);
                r0b = sse_max(r0b, d[i + 1]);
                r1a = sse_max(r1a, d[i + 2]);
                r1b = sse_max(r1b, d[i + 3]);
            }
        }
        r0a = sse_max(r0a, r1a);
        r0b = sse_max(r0b, r1b);
        if (aligned > aligned2) {
#pragma unroll
            for (int q = 4; q + 2 <= G; q += 4)
                if (q == aligned2) {
                    r0a = sse_max(r0a, d[q]);
                    r0b = sse_max(r0b, d[q + 1]);
                }
        }
    }
    double res = sse_max(r0a, r0b);
#pragma unroll
    for (int i = 2; i < G; ++i)
        if (i >= aligned && i < n)
            res = std_max(res, d[i]);
    return res;
}

template <int MODEL, int G, int KM>
__global__ void __launch_bounds__(kBlock) lk_viterbi_kernel(const DevArgs a)
{
    HIP_DYNAMIC_SHARED(double, lds)
    constexpr int KH = KM;
    LkLane<MODEL, G, KM> ln;
    lk_setup<MODEL, G, KM>(ln, a, lds, true, lk_group<G>(a.P));
    const bool st = ln.on; /* the lane that stores */
    const double (&colh)[KH] = ln.col;
    const int Tp = ln.Tp;
    const int K = ln.K;
    double w[KH];
    int slot = 0;
    auto emit_log = [&](int x, double xr) -> double {
        if constexpr (LkTraits<MODEL>::kGauss)
            return ln.on ? lk_lpdf<MODEL, G, KM>(ln, xr) : 0.0;
        else
            return ln.on ? ln.tab[(min(max(x, 1), ln.L) - 1) * G + ln.j] : 0.0;
    };
    /* back-pointers in blocks of kLBack steps: [P][Tb/16][K][16] bytes (Tb =
     * T_max rounded up to 16).  A lane gathers its state's 16 bytes of a block
     * in registers and stores them with one 16-byte store, so the group's
     * store covers K * 16 contiguous bytes (a byte store per lane and step,
     * into rows T_max apart, moved 20x the bytes: 48 GB per N1 step, PMC
     * profiles/r03d_workloads_pmc.json) */
    const int Tb = lk_row_bytes(a.Tmax), NB = Tb / kLBack;
    uint8_t *bpb = reinterpret_cast<uint8_t *>(a.bp) + (int64_t)ln.p * NB * K * kLBack;
    auto bp_at = [&](int blk) { return bpb + ((int64_t)blk * K + (ln.on ? ln.j : 0)) * kLBack; };

    /* delta_tk[1, K] = emission of state K only (Q3: the others keep NaN) */
    LkObs<MODEL, G> bcur = lk_block<MODEL, G, KM>(ln, a, 0), bnxt = lk_block<MODEL, G, KM>(ln, a, 1);
    int x;
    double xr;
    lk_get<MODEL, G>(bcur, 0, x, xr);
    const double le0 = emit_log(x, xr);
    double dl = !ln.on ? dev_ninf() : ((ln.j == K - 1) ? le0 : dev_nan());
    const int nblk = (wave_max(Tp) + kLBack - 1) / kLBack; /* wave-uniform: the groups walk t together */
    for (int b = 0; b < nblk; ++b) {
        uint32_t wd[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int v = 0; v < kLBack; ++v) {
            const int t = b * kLBack + v;
            if (t == 0)
                continue;
            const int u = t % G;
            if (u == 0) {
                bcur = bnxt;
                bnxt = lk_block<MODEL, G, KM>(ln, a, t / G + 1);
            }
            if (t < Tp) { /* group-uniform */
                lk_get<MODEL, G>(bcur, u, x, xr);
                const double le = emit_log(x, xr);
                grp_exchange<G, KM>(ln.xch, slot, ln.j, dl, w);
                slot ^= 1;
                /* candidate (delta + log A) + emission, strict '>' from -inf; the
                 * running max as fmax (vit_step): NaN never wins, first i on ties */
                double best = dev_ninf();
                int arg = 0;
#pragma unroll
                for (int i = 0; i < KH; ++i) { /* idle i: delta -inf, never greater */
                    const double cand = (w[i] + colh[i]) + le;
                    const bool gt = cand > best;
                    best = fmax(best, cand);
                    arg = gt ? i : arg;
                }
                dl = ln.on ? best : dev_ninf();
                wd[v >> 2] |= (uint32_t)arg << (8 * (v & 3));
            }
        }
        if (st && b * kLBack < Tp)
            *reinterpret_cast<uint4 *>(bp_at(b)) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
    }
    /* logp_zstar = max(delta_T) (SSE2 order); zstar_T = LAST j attaining it */
    double wf[KM];
    grp_exchange<G, KM>(ln.xch, slot, ln.j, dl, wf);
    const double lp = stan_max_rt<KM>(wf, K);
    int z = -1;
#pragma unroll
    for (int j = 0; j < KM; ++j)
        if (j < K && wf[j] == lp)
            z = j;
    const bool invalid = (z < 0) || (Tp >= 2 && lp == dev_ninf());
    if (ln.j == 0) {
        if ((a.outputs & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
            a.logp_zstar[ln.p] = lp;
        if (a.pair_status)
            a.pair_status[ln.p] = invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
    }
    if (!((a.outputs & HHMM_OUT_ZSTAR) && a.zstar))
        return;
    if (invalid) {
        for (int t = ln.j; t < Tp; t += G)
            a.zstar[ln.p + a.P * (int64_t)t] = 0;
        return;
    }
    /* backtrack, kLBack steps at a time: lane s holds state s's bytes of the
     * chunk (one 16-byte load, prefetched two chunks ahead), the path state
     * moves by one shuffle per step, lane u keeps step t0 + u for the store */
    const int nb = (Tp + kLBack - 1) / kLBack;
    auto load = [&](int c) -> uint4 {
        const int cc = min(max(c, 0), NB - 1);
        return *reinterpret_cast<const uint4 *>(bp_at(cc));
    };
    uint4 q0 = load(nb - 1), q1 = load(nb - 2);
    for (int c = nb - 1; c >= 0; --c) {
        const uint4 q2 = load(c - 2);
        const uint32_t wd[4] = {q0.x, q0.y, q0.z, q0.w};
        int mine = 0;
#pragma unroll
        for (int u = kLBack - 1; u >= 0; --u) {
            const int t = c * kLBack + u;
            if (t < Tp) {
                if ((ln.j & (kLBack - 1)) == u)
                    mine = z + 1;
                if (t > 0)
                    z = __shfl((int)((wd[u >> 2] >> (8 * (u & 3))) & 0xffu), z, G);
            }
        }
        const int t = c * kLBack + (ln.j & (kLBack - 1));
        if (ln.j < kLBack && t < Tp)
            a.zstar[ln.p + a.P * (int64_t)t] = mine;
        q0 = q1;
        q1 = q2;
    }
}

/* ---- FFBS at large K (the contract of DESIGN.md §5, oracle
 * ffbs_contract): the filter f_t of the contract -- s_j = f(0) A(0,j), then
 * fma(f(i), A(i,j), s_j) in state order, f_t(j) = s_j e_t(j), an exact
 * power-of-two renormalisation (the frexp exponent of the max) every step --
 * then z_{T-1} = cat(f_{T-1}), z_t = cat(f_t(i) A(i, z_{t+1})) with the
 * caller's uniforms.  Lane j computes s_j with column j of A in registers
 * and the state vector exchanged through LDS (the lk_fb layout), so the
 * sums run in the contract's order and the draws are bit-exact.  Forward
 * checkpoints every kLChunk steps; the backward sampling recomputes each
 * chunk from its checkpoint (the same operations: the same bits). ---- */
template <int KM>
__device__ __forceinline__ int ffbs_cat_rt(const double (&w)[KM], int K, double u)
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
        const bool step = (i < K) & (b == i - 1) & (us > cum);
        b = step ? i : b;
        cum = step ? cum + w[i] : cum;
    }
    return ((sum > 0.0) & __builtin_isfinite(sum)) ? b : -1;
}

template <int MODEL, int G, int KM>
__device__ __forceinline__ double lkf_step(const LkLane<MODEL, G, KM> &ln, const double (&w)[KM], double e)
{
    double s = w[0] * ln.col[0];
#pragma unroll
    for (int i = 1; i < KM; ++i)
        if (i < ln.K)
            s = fma(w[i], ln.col[i], s);
    return ln.on ? s * e : 0.0;
}

/* the contract's emission: phi[j, x] (discrete) or det_exp(lpdf_j - max_j lpdf_j) */
template <int MODEL, int G, int KM>
__device__ __forceinline__ double lkf_emit(const LkLane<MODEL, G, KM> &ln, int x, double xr)
{
    if constexpr (LkTraits<MODEL>::kGauss) {
        const double lp = ln.on ? lk_lpdf<MODEL, G, KM>(ln, xr) : dev_ninf();
        const double m = grp_max<G>(lp);
        return ln.on ? hhmm_det_exp_tab(lp - m, ln.etab) : 0.0;
    } else {
        const int xc = min(max(x, 1), ln.L);
        return ln.on ? ln.tab[(xc - 1) * G + ln.j] : 0.0;
    }
}

template <int MODEL, int G, int KM>
__global__ void __launch_bounds__(kBlock) lk_ffbs_kernel(const DevArgs a)
{
    HIP_DYNAMIC_SHARED(double, lds)
    LkLane<MODEL, G, KM> ln;
    lk_setup<MODEL, G, KM>(ln, a, lds, false, lk_group<G>(a.P));
    if constexpr (LkTraits<MODEL>::kGauss) {
        /* the FFBS contract exp's 2^(j/128) table after the exchange slots (no
         * emission tables here; run_large_model sizes the launch for it) */
        hhmm_exp2_entry *t = reinterpret_cast<hhmm_exp2_entry *>(lds + (size_t)(blockDim.x / G) * 2 * G);
        for (int i = threadIdx.x; i < 128; i += blockDim.x)
            t[i] = hhmm_exp2_tab[i];
        __syncthreads();
        ln.etab = t;
    }
    const int Tp = ln.Tp, K = ln.K;
    double w[KM];
    int slot = 0;
    auto ckpt = [&](int c) -> double & { return a.ckpt[ln.p + a.P * ((int64_t)c * K + (ln.on ? ln.j : 0))]; };
    auto renorm1 = [&](double v) {
        const double mx = grp_max<G>(v);
        return ldexp(v, -__builtin_amdgcn_frexp_exp(mx));
    };
    /* ---- forward filter ---- */
    LkObs<MODEL, G> bcur = lk_block<MODEL, G, KM>(ln, a, 0), bnxt = lk_block<MODEL, G, KM>(ln, a, 1);
    double f;
    {
        int x;
        double xr;
        lk_get<MODEL, G>(bcur, 0, x, xr);
        const double e = lkf_emit<MODEL, G, KM>(ln, x, xr);
        f = !ln.on ? 0.0 : (LkTraits<MODEL>::kGauss ? ln.pj : ln.pj * e); /* hmm.stan: p_1k (Q2) */
        f = renorm1(f);
    }
    if (ln.on)
        ckpt(0) = f;
    for (int t = 1; t < Tp; ++t) {
        const int u = t % G;
        if (u == 0) {
            bcur = bnxt;
            bnxt = lk_block<MODEL, G, KM>(ln, a, t / G + 1);
        }
        int x;
        double xr;
        lk_get<MODEL, G>(bcur, u, x, xr);
        const double e = lkf_emit<MODEL, G, KM>(ln, x, xr);
        grp_exchange<G, KM>(ln.xch, slot, ln.j, f, w);
        slot ^= 1;
        f = renorm1(lkf_step<MODEL, G, KM>(ln, w, e));
        if (t % kLChunk == 0 && ln.on)
            ckpt(t / kLChunk) = f;
    }
    /* ---- backward sampling, chunk by chunk from the end ---- */
    const int nck = (Tp + kLChunk - 1) / kLChunk;
    constexpr int CPB = G / kLChunk;
    int cb = (nck - 1) / CPB;
    LkObs<MODEL, G> ob = lk_block<MODEL, G, KM>(ln, a, cb), obp = lk_block<MODEL, G, KM>(ln, a, cb - 1);
    int z = -2; /* -2: not drawn yet (z_{T-1} comes from f_{T-1} alone) */
    for (int c = nck - 1; c >= 0; --c) {
        if (c / CPB != cb) {
            cb = c / CPB;
            ob = obp;
            obp = lk_block<MODEL, G, KM>(ln, a, cb - 1);
        }
        const int t0 = c * kLChunk, ub = t0 % G;
        double fb[kLChunk];
        fb[0] = ln.on ? ckpt(c) : 0.0;
#pragma unroll
        for (int u = 1; u < kLChunk; ++u) {
            fb[u] = 0.0;
            if (t0 + u < Tp) {
                int x;
                double xr;
                lk_get_var<MODEL, G>(ob, ub + u, x, xr);
                const double e = lkf_emit<MODEL, G, KM>(ln, x, xr);
                grp_exchange<G, KM>(ln.xch, slot, ln.j, fb[u - 1], w);
                slot ^= 1;
                fb[u] = renorm1(lkf_step<MODEL, G, KM>(ln, w, e));
            }
        }
#pragma unroll
        for (int u = kLChunk - 1; u >= 0; --u) {
            const int t = t0 + u;
            if (t >= Tp)
                continue;
            double wt = fb[u];
            if (z >= 0) { /* weight f_t(i) A(i, z_{t+1}): lane i's row, entry z */
                double az = ln.row[0];
#pragma unroll
                for (int k = 1; k < KM; ++k)
                    az = (z == k) ? ln.row[k] : az;
                wt = ln.on ? wt * az : 0.0;
            }
            grp_exchange<G, KM>(ln.xch, slot, ln.j, wt, w);
            slot ^= 1;
            const double uu = a.ffbs_u[ln.p + a.P * (int64_t)t];
            z = (z == -1) ? -1 : ffbs_cat_rt<KM>(w, K, uu);
            if (ln.j == 0)
                a.z_ffbs[ln.p + a.P * (int64_t)t] = z + 1;
        }
    }
}

/* ---- The log-scale profile at large K (unalpha_tk / unbeta_tk requested):
 * the reference's log-space recursion, as fb_log_kernel does at K <= 8 --
 * log A and log phi once per pair, Stan's log_sum_exp per (t, j) over the
 * accumulator (unalpha(t-1, i) + log A(i, j)) + emission (hmm.stan:37,
 * hmm-multinom.stan:39) and (unbeta(t, i) + log A(j, i)) + emission(i)
 * (hmm.stan:79), so a state thousands of nats below the others keeps a
 * finite log value where the linear filter underflows.  Lane j runs state j
 * (K exp and one log per lane-step); unalpha checkpoints every kLChunk steps,
 * recomputed chunk by chunk in the backward sweep; posteriors by the
 * reference's formulas (alpha = softmax(unalpha), beta = softmax(unbeta),
 * ungamma = alpha .* beta, gamma = ungamma / sum: hmm.stan:60-63, 85-96). ---- */
template <int KM>
__device__ __forceinline__ double lk_lse(const double (&acc)[KM], int K)
{
    double mx = dev_ninf();
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K && acc[i] > mx)
            mx = acc[i];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < KM; ++i)
        if (i < K && acc[i] != dev_ninf())
            sum += exp(acc[i] - mx);
    return mx + log(sum);
}

template <int G>
__device__ __forceinline__ double grp_softmax(double v, bool on)
{
    const double m = grp_max<G>(on ? v : dev_ninf());
    const double e = on ? exp(v - m) : 0.0;
    return e / grp_sum<G>(e);
}

template <int MODEL, int G, int KM>
__global__ void __launch_bounds__(kBlock) lk_log_kernel(const DevArgs a)
{
    HIP_DYNAMIC_SHARED(double, lds)
    LkLane<MODEL, G, KM> ln;
    lk_setup<MODEL, G, KM>(ln, a, lds, true, lk_group<G>(a.P)); /* col: log A(i, j); tab: log phi */
    double lrow[KM];                                             /* log A(j, i) */
#pragma unroll
    for (int i = 0; i < KM; ++i)
        lrow[i] = (i < ln.K) ? log(ln.row[i]) : 0.0;
    const uint32_t out = a.outputs;
    const int Tp = ln.Tp, K = ln.K;
    const bool need_bwd = (out & (HHMM_OUT_UNBETA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA)) != 0;
    double w[KM];
    int slot = 0;
    auto ckpt = [&](int c) -> double & { return a.ckpt[ln.p + a.P * ((int64_t)c * K + (ln.on ? ln.j : 0))]; };
    auto le_of = [&](int x, double xr) -> double { /* log emission of state j */
        if constexpr (LkTraits<MODEL>::kGauss)
            return ln.on ? lk_lpdf<MODEL, G, KM>(ln, xr) : 0.0;
        else
            return ln.on ? ln.tab[(min(max(x, 1), ln.L) - 1) * G + ln.j] : 0.0;
    };
    auto fwd = [&](double uprev, double le) { /* unalpha_t(j) */
        grp_exchange<G, KM>(ln.xch, slot, ln.j, uprev, w);
        slot ^= 1;
        double acc[KM];
#pragma unroll
        for (int i = 0; i < KM; ++i)
            acc[i] = (w[i] + ln.col[i]) + le;
        return ln.on ? lk_lse<KM>(acc, K) : dev_ninf();
    };
    auto emit_fwd = [&](int t, double u) {
        if ((out & HHMM_OUT_UNALPHA) && a.unalpha)
            lk_put<MODEL, G, KM>(a.unalpha, a, ln, t, u);
        if ((out & HHMM_OUT_ALPHA) && a.alpha)
            lk_put<MODEL, G, KM>(a.alpha, a, ln, t, grp_softmax<G>(u, ln.on));
    };

    LkObs<MODEL, G> bcur = lk_block<MODEL, G, KM>(ln, a, 0), bnxt = lk_block<MODEL, G, KM>(ln, a, 1);
    double u;
    {
        int x;
        double xr;
        lk_get<MODEL, G>(bcur, 0, x, xr);
        if constexpr (LkTraits<MODEL>::kGauss) {
            /* log(p_1k) + SUM_k normal_lpdf(x[1] | mu_k, sigma_k) (hmm.stan:30, Q2) */
            const double tk = ln.on ? lk_lpdf<MODEL, G, KM>(ln, xr) : 0.0;
            const double s = grp_sum<G>(tk); /* every lane takes part in the butterfly */
            u = ln.on ? log(ln.pj) + s : dev_ninf();
        } else {
            u = ln.on ? log(ln.pj) + le_of(x, xr) : dev_ninf();
        }
    }
    if (need_bwd) {
        if (ln.on)
            ckpt(0) = u;
    } else {
        emit_fwd(0, u);
    }
    for (int t = 1; t < Tp; ++t) {
        const int uu = t % G;
        if (uu == 0) {
            bcur = bnxt;
            bnxt = lk_block<MODEL, G, KM>(ln, a, t / G + 1);
        }
        int x;
        double xr;
        lk_get<MODEL, G>(bcur, uu, x, xr);
        u = fwd(u, le_of(x, xr));
        if (!need_bwd)
            emit_fwd(t, u);
        else if (t % kLChunk == 0 && ln.on)
            ckpt(t / kLChunk) = u;
    }
    {
        /* target += log_sum_exp(unalpha_tk[T]) (hmm.stan:46): every lane holds the group's vector */
        grp_exchange<G, KM>(ln.xch, slot, ln.j, u, w);
        slot ^= 1;
        const double ll = lk_lse<KM>(w, K);
        if ((out & HHMM_OUT_LOGLIK) && a.loglik && ln.j == 0)
            a.loglik[ln.p] = ll;
    }
    if (!need_bwd)
        return;

    /* ---- backward: unbeta_tk[T] = 1 (Q1), chunks from the end ---- */
    double ub = ln.on ? 1.0 : dev_ninf();
    const int nck = (Tp + kLChunk - 1) / kLChunk;
    constexpr int CPB = G / kLChunk;
    int cb = (nck - 1) / CPB;
    LkObs<MODEL, G> ob = lk_block<MODEL, G, KM>(ln, a, cb), obp = lk_block<MODEL, G, KM>(ln, a, cb - 1);
    for (int c = nck - 1; c >= 0; --c) {
        if (c / CPB != cb) {
            cb = c / CPB;
            ob = obp;
            obp = lk_block<MODEL, G, KM>(ln, a, cb - 1);
        }
        const int t0 = c * kLChunk, ub0 = t0 % G;
        double les[kLChunk], ubuf[kLChunk];
#pragma unroll
        for (int v = 0; v < kLChunk; ++v) {
            int x;
            double xr;
            lk_get_var<MODEL, G>(ob, ub0 + v, x, xr);
            les[v] = le_of(x, xr);
        }
        ubuf[0] = ln.on ? ckpt(c) : dev_ninf();
#pragma unroll
        for (int v = 1; v < kLChunk; ++v) {
            ubuf[v] = dev_ninf();
            if (t0 + v < Tp)
                ubuf[v] = fwd(ubuf[v - 1], les[v]);
        }
#pragma unroll
        for (int v = kLChunk - 1; v >= 0; --v) {
            const int t = t0 + v;
            if (t >= Tp)
                continue;
            emit_fwd(t, ubuf[v]);
            if ((out & HHMM_OUT_UNBETA) && a.unbeta)
                lk_put<MODEL, G, KM>(a.unbeta, a, ln, t, ub);
            const double be = grp_softmax<G>(ub, ln.on);
            if ((out & HHMM_OUT_BETA) && a.beta)
                lk_put<MODEL, G, KM>(a.beta, a, ln, t, be);
            if (out & (HHMM_OUT_GAMMA | HHMM_OUT_UNGAMMA)) {
                const double ug = grp_softmax<G>(ubuf[v], ln.on) * be;
                if ((out & HHMM_OUT_UNGAMMA) && a.ungamma)
                    lk_put<MODEL, G, KM>(a.ungamma, a, ln, t, ug);
                if ((out & HHMM_OUT_GAMMA) && a.gamma)
                    lk_put<MODEL, G, KM>(a.gamma, a, ln, t, ug / grp_sum<G>(ug));
            }
            if (t > 0) {
                /* unbeta_{t-1}(j) = LSE_i((unbeta_t(i) + log A(j, i)) + le_t(i)): lane i's
                 * unbeta and emission travel together */
                double wl[KM];
                grp_exchange<G, KM>(ln.xch, slot, ln.j, ub, w);
                slot ^= 1;
                grp_exchange<G, KM>(ln.xch, slot, ln.j, les[v], wl);
                slot ^= 1;
                double acc[KM];
#pragma unroll
                for (int i = 0; i < KM; ++i)
                    acc[i] = (w[i] + lrow[i]) + wl[i];
                ub = ln.on ? lk_lse<KM>(acc, K) : dev_ninf();
            }
        }
    }
}

} // namespace hhmm
