/*
 * hhmm_lkscan.h -- the parallel scan over T at large K (8 < K <= 32; SURVEY.md
 * §8 A16 + N1, the verdict's N2): hmm-multinom -- and hmm.stan's Gaussian
 * emissions, whose per-step shift m_t = max_j lpdf_j travels as each chunk's
 * log scale (sc_bl) -- with few pairs and long series,
 * e.g. a flattened HHMM with 23 states (log.md:657-658) over a tick series of
 * 10^6 zig-zags (tayal2009/main.Rmd:310-346).  The sequential state-parallel
 * kernels (hhmm_large.h) give one 32-lane group per pair: 250 pairs are 125
 * waves on a 1024-SIMD chip, and 10^6 dependent steps each.
 *
 * The forward map is linear, f_t = f_{t-1} F_t with F_t = A diag(e_t), and
 * the backward map uses the same matrices, beta_{t-1} = F_t beta_t
 * (hmm-multinom.stan:36-44 forward, :73-88 backward: no masks in this
 * program).  So ONE chunk product M_c = prod_{t in chunk c} F_t serves both
 * scans:
 *   phase 1  (lks_prod_kernel, MFMA) the chunk products.  Row i of M_c is the
 *            forward filter started from state i at the chunk's entry, i.e.
 *            column i of M_c^T, and v <- diag(e_t) A^T v is a dense K x K by
 *            K x 16 product for 16 such columns that share the pair's A: the
 *            batched K x K contraction the north star reserves the matrix
 *            cores for.  v_mfma_f64_16x16x4_f64 with A^T as the A operand
 *            (fixed in registers for the whole chunk) and the columns as the
 *            B operand; the result registers of one step ARE the next step's
 *            B operand (C/D row (lane>>4) + 4r = B row of k-step r), so the
 *            recursion needs no lane movement.  After every step each column
 *            (one filter) is renormalised by an exact power of two and its
 *            exponent kept: M_c = diag(2^s) M'_c.
 *   phase 2  (lks_bound_kernel, one wave per pair) the forward scan over the
 *            chunks (the filter entering each chunk, its log scale, the
 *            log-likelihood) and the backward scan (beta at each chunk's last
 *            step), with the row exponents folded in exactly.
 *   phase 3  (lk_fb_kernel over (pair, chunk) groups, hhmm_large.h) the
 *            forward-backward sweep of every chunk from those vectors:
 *            alpha, beta, ungamma, gamma.
 * The chunk products' entries are sums of non-negative terms, so they keep
 * their relative precision like the sequential recursion; the outputs are
 * tolerance outputs (1e-9 relative), the Viterbi stays sequential (exact).
 */
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "hhmm_large.h"

namespace hhmm {

typedef double lks_d4 __attribute__((ext_vector_type(4)));

/* v_mfma_f64_16x16x4_f64 operand maps (cdna_hip_programming.md §3, "f64 MFMA
 * does NOT use these maps"): lane l holds A[row l & 15][k l >> 4] and
 * B[k l >> 4][col l & 15]; result register r holds D[row (l >> 4) + 4r][col l & 15]. */
__device__ __forceinline__ lks_d4 lks_mfma(double a, double b, lks_d4 c)
{
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

/* v_mfma_f64_4x4x4_16b_f64 (operand maps measured by tools/mfma_probe.hip,
 * profiles/r05a_mfma_probe.txt): four independent 4 x 4 x 4 blocks b = 0..3;
 * lane 16k + 4b + r holds block b's A[r][k], lane 16k + 4b + c its B[k][c],
 * and the result D[r][c] lands in lane 16r + 4b + c -- the B layout again.
 * 512 FLOP per instruction at a quarter of the 16x16x4 form's cycles (the
 * probe: 71.5 against 49.5 TFLOP/s). */
__device__ __forceinline__ double lks_mfma4(double a, double b, double c)
{
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
/* The chunk products run on v_mfma_f64_4x4x4: with the 4 x 4 blocks the state
 * dimension pads to a multiple of 4 instead of 16 (K = 23: 24 x 24 instead of
 * 32 x 24 per step, VERDICT r4's 1.45x padding; the 16x16x4 form measured
 * slower at N2, round 5). */

/* Columns of M'^T per wave: TPW tiles of 16.  RT row tiles of 16 states, KSM
 * k-steps of 4 states (K <= 16: 1 / 4; K <= 24: 2 / 6; K <= 32: 2 / 8). */
#ifndef HHMM_LKS_TILES
#define HHMM_LKS_TILES 1 /* build knob: 16-column tiles per wave (independent accumulator chains) */
#endif
constexpr int kLksTiles = HHMM_LKS_TILES;
/* Build knob: steps between the chunk products' renormalisations where the
 * pair's parameters bound the shrink (lks_prod_kernel); 1 = every step. */
#ifndef HHMM_LKS_RENORM
#define HHMM_LKS_RENORM 4
#endif
constexpr int kLksRenorm = HHMM_LKS_RENORM;
static_assert(8 % kLksRenorm == 0, "the cadence divides the observation block kB = 8");
/* Build knob: blocks of steps that every column of the wave takes in full run
 * without the per-column step predicates (lks_prod_kernel). */
#ifndef HHMM_LKS_FULLBLK
#define HHMM_LKS_FULLBLK 1
#endif

/* Build knob: registers of lks_prod_kernel capped for this many waves per SIMD
 * where the A operand leaves room (K <= 24, multinomial: 158 registers without
 * a spill at one tile per wave; 0: the compiler's choice everywhere).  N2
 * 188.6 against 195.8 ms with two tiles at two waves (profiles/r05l_ab_n2.log). */
#ifndef HHMM_LKS_WAVES
#define HHMM_LKS_WAVES 3
#endif
template <int KSM, bool GS>
constexpr int lks_waves() { return (HHMM_LKS_WAVES > 0 && KSM <= 6 && !GS) ? HHMM_LKS_WAVES : 1; }
template <int RT, int KSM, bool GS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(lks_waves<KSM, GS>())))
lks_prod_kernel(const DevArgs a)
{
    constexpr int TPW = kLksTiles;
    constexpr int KR = 16 * RT; /* padded rows of the emission table */
    HIP_DYNAMIC_SHARED(double, lds)
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int K = a.K, cl = a.scan_cl, nc = a.scan_nc;
    const int ks = (K + 3) / 4;
    const int ntile = (nc * K + 15) / 16;
    const int wpp = (ntile + TPW - 1) / TPW;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + wv;
    const int64_t p = min(w / wpp, a.P - 1); /* surplus waves redo the last pair's last tiles */
    const int tg = (int)min(w - p * wpp, (int64_t)wpp - 1);
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int64_t S = a.S;

    /* multinomial: the pair's emission table phi[l][j] (rows j >= K zero), one
     * per wave; Gaussian (hmm.stan): mu, 1/sigma and NEG_LOG_SQRT_TWO_PI -
     * log(sigma) of the lane's rows j = 4kk + (lane >> 4) */
    double *tab = lds + (size_t)wv * a.L * KR;
    double gmu[GS ? KSM : 1], gis[GS ? KSM : 1], gc0[GS ? KSM : 1];
    if constexpr (GS) {
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk) {
            const int j = 4 * kk + (lane >> 4);
            const int jc = j < K ? j : 0;
            const double sg = a.sigma_k[d + S * jc];
            gmu[kk] = a.mu_k[d + S * jc];
            gis[kk] = 1.0 / sg;
            gc0[kk] = HHMM_NEG_LOG_SQRT_TWO_PI - dev_cr_log(sg); /* lk_setup's constant */
        }
    } else {
        for (int idx = lane; idx < a.L * KR; idx += 64) {
            const int l = idx / KR, j = idx - l * KR;
            tab[idx] = j < K ? a.phi_k[d + S * ((int64_t)j + (int64_t)K * l)] : 0.0;
        }
    }
    /* A operand of the 4 x 4 blocks: every block takes the same 4 x 4 block of
     * A^T, aop4[so][si] = A^T[4so + r][4si + k] = A(4si + k, 4so + r) with
     * r = lane & 3, k = lane >> 4 */
    double aop4[KSM][KSM];
#pragma unroll
    for (int so = 0; so < KSM; ++so)
#pragma unroll
        for (int si = 0; si < KSM; ++si) {
            const int i = 4 * si + (lane >> 4), j = 4 * so + (lane & 3);
            aop4[so][si] = (i < K && j < K) ? a.A_ij[d + S * ((int64_t)i + (int64_t)K * j)] : 0.0;
        }
    __syncthreads();
    /* Renormalisation cadence: a column is renormalised (its max to [1/2, 1),
     * an exact power of two) every kLksRenorm-th step where the pair bounds the
     * per-step shrink of the max, b = phi_min * min(min_i rowmax_i(A),
     * min_j colmax_j(A)) >= kLRenormSafeBound (lk_setup's test; the growth is at
     * most K per step), else every step ("dense": Gaussian emissions, or a NaN /
     * unsafe draw).  Power-of-two scalings are exact, and every column is
     * renormalised after its last step, so M'_c and its exponents are the same
     * bits at either cadence up to the subnormal floor: between
     * renormalisations the max stays above b^3 >= 2^-117, and only an entry
     * ~2^-900 below it can lose bits sooner than under per-step
     * renormalisation (far below the 1e-250 tolerance floor).  The growth bound
     * needs A and phi entries <= 1, which the test below also requires. */
    bool dense = GS;
    if constexpr (!GS) {
        const int jr = lane < K ? lane : 0; /* lane = state: its phi column, A row and A column */
        double emin = 1.0 / 0.0, emax = 0.0, rmax = 0.0, cmax = 0.0;
        for (int l = 0; l < a.L; ++l) {
            emin = fmin(emin, tab[l * KR + jr]);
            emax = fmax(emax, tab[l * KR + jr]);
        }
        for (int i = 0; i < K; ++i) {
            rmax = fmax(rmax, a.A_ij[d + S * ((int64_t)jr + (int64_t)K * i)]);
            cmax = fmax(cmax, a.A_ij[d + S * ((int64_t)i + (int64_t)K * jr)]);
        }
        const double inf = 1.0 / 0.0;
        double ge = lane < K ? emin : inf, gm = lane < K ? fmin(rmax, cmax) : inf;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            ge = fmin(ge, __shfl_xor(ge, o));
            gm = fmin(gm, __shfl_xor(gm, o));
        }
        /* the growth bound (at most K per step) needs every A and phi entry <= 1 */
        const bool big = lane < K && !(emax <= 1.0 && fmax(rmax, cmax) <= 1.0);
        const bool bad = !(ge * gm >= kLRenormSafeBound) || (lane < K && !(emin * fmin(rmax, cmax) >= 0.0)) || big;
        dense = __builtin_amdgcn_readfirstlane((int)(__ballot(bad) != 0)) != 0;
    }

    /* this lane's column in each tile: (chunk c, initial state i); B operand
     * Q[u][kk] = row 4kk + (lane >> 4) of the column; gls: the chunk's Gaussian
     * log scale (the sum of the steps' emission shifts) */
    double q[TPW][KSM];
    double gls[TPW];
    int ex[TPW], t0[TPW], t1[TPW];
    bool valid[TPW];
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        const int col = (tg * TPW + u) * 16 + (lane & 15);
        valid[u] = col < nc * K;
        const int c = valid[u] ? col / K : 0, i = valid[u] ? col - c * K : 0;
        t0[u] = c * cl;
        t1[u] = valid[u] ? min(t0[u] + cl, Tp) : t0[u];
        ex[u] = 0;
        gls[u] = 0.0;
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            q[u][kk] = (valid[u] && 4 * kk + (lane >> 4) == i) ? 1.0 : 0.0;
    }
    /* the wave's step count: the longest of its columns' chunks */
    int smax = 0;
#pragma unroll
    for (int u = 0; u < TPW; ++u)
        smax = max(smax, t1[u] - t0[u]);
    smax = wave_max(smax);

    /* observations a block of kB steps ahead (clamped, unconditional) */
    constexpr int kB = 8;
    typedef typename std::conditional<GS, double, int>::type ObsT;
    auto ldx = [&](int u, int s) -> ObsT {
        const int t = min(max(t0[u] + s, 0), a.Tmax - 1);
        if constexpr (GS)
            return a.xr[n + a.N * (int64_t)t];
        else
            return a.x[n + a.N * (int64_t)t];
    };
    ObsT xb[TPW][kB], xn[TPW][kB];
#pragma unroll
    for (int u = 0; u < TPW; ++u)
#pragma unroll
        for (int v = 0; v < kB; ++v)
            xb[u][v] = ldx(u, v);
    for (int s0 = 0; s0 < smax; s0 += kB) {
#pragma unroll
        for (int u = 0; u < TPW; ++u)
#pragma unroll
            for (int v = 0; v < kB; ++v)
                xn[u][v] = ldx(u, s0 + kB + v);
        /* a block in which every column of the wave takes all kB steps (the
         * common case) runs without the per-column step predicates */
        bool full = s0 + kB <= smax;
#pragma unroll
        for (int u = 0; u < TPW; ++u)
            full &= (t0[u] + s0 >= 1 || a.seg_nofirst) && t0[u] + s0 + kB <= t1[u];
        full = HHMM_LKS_FULLBLK && __builtin_amdgcn_readfirstlane((int)(__ballot(!full) == 0)) != 0;
        auto block = [&](auto full_c) {
        constexpr bool FULL = decltype(full_c)::value;
#pragma unroll
        for (int v = 0; v < kB; ++v) {
            const int s = s0 + v;
            if (!FULL && s >= smax)
                break;
            /* D = A^T Q for every tile (independent accumulators interleaved);
             * accv(u, kk): state 4kk + (lane >> 4) of the lane's column */
            double acc4[TPW][KSM];
#pragma unroll
            for (int u = 0; u < TPW; ++u)
#pragma unroll
                for (int so = 0; so < KSM; ++so)
                    acc4[u][so] = 0.0;
#pragma unroll
            for (int si = 0; si < KSM; ++si) {
                if (si < ks) {
#pragma unroll
                    for (int so = 0; so < KSM; ++so) {
                        if (so < ks) {
#pragma unroll
                            for (int u = 0; u < TPW; ++u)
                                acc4[u][so] = lks_mfma4(aop4[so][si], q[u][si], acc4[u][so]);
                        }
                    }
                }
            }
            auto accv = [&](int u, int kk) -> double { return acc4[u][kk]; };
            /* emission of the column's step, renormalisation of the column */
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int t = t0[u] + s;
                /* t = 0 is the init (phase 2 applies p_1k .* phi), except in a
                 * segment window that starts inside the series: there every
                 * step is a transition */
                const bool on = FULL || ((t >= 1 || a.seg_nofirst) && t < t1[u]);
                double em[KSM];
                if constexpr (GS) {
                    /* e_t(j) = exp(lpdf_j - m_t), m_t = max_j lpdf_j (emit_prob's
                     * shift; the column's rows sit on lanes l, l ^ 16, l ^ 32, l ^ 48) */
                    double lp[KSM];
                    double m = dev_ninf();
#pragma unroll
                    for (int kk = 0; kk < KSM; ++kk) {
                        const double z = (xb[u][v] - gmu[kk]) * gis[kk];
                        lp[kk] = (4 * kk + (lane >> 4) < K) ? gc0[kk] + (-0.5 * (z * z)) : dev_ninf();
                        m = fmax(m, lp[kk]);
                    }
                    m = fmax(m, __shfl_xor(m, 16));
                    m = fmax(m, __shfl_xor(m, 32));
#pragma unroll
                    for (int kk = 0; kk < KSM; ++kk)
                        em[kk] = exp(lp[kk] - m);
                    gls[u] += on ? m : 0.0;
                } else {
                    const int xc = min(max(xb[u][v], 1), a.L);
                    const double *row = tab + (xc - 1) * KR + (lane >> 4);
#pragma unroll
                    for (int kk = 0; kk < KSM; ++kk)
                        em[kk] = row[4 * kk];
                }
                double nv[KSM];
#pragma unroll
                for (int kk = 0; kk < KSM; ++kk)
                    nv[kk] = accv(u, kk) * em[kk];
                if ((v % kLksRenorm) == kLksRenorm - 1 || dense) { /* v: compile-time; dense: wave-uniform */
                    double mx = 0.0;
#pragma unroll
                    for (int kk = 0; kk < KSM; ++kk)
                        mx = fmax(mx, nv[kk]);
                    mx = fmax(mx, __shfl_xor(mx, 16));
                    mx = fmax(mx, __shfl_xor(mx, 32));
                    const int e2 = __builtin_amdgcn_frexp_exp(mx);
#pragma unroll
                    for (int kk = 0; kk < KSM; ++kk)
                        q[u][kk] = on ? ldexp(nv[kk], -e2) : q[u][kk];
                    ex[u] += on ? e2 : 0;
                } else {
#pragma unroll
                    for (int kk = 0; kk < KSM; ++kk)
                        q[u][kk] = on ? nv[kk] : q[u][kk];
                }
            }
        }
        };
        if (full)
            block(std::true_type{});
        else
            block(std::false_type{});
#pragma unroll
        for (int u = 0; u < TPW; ++u)
#pragma unroll
            for (int v = 0; v < kB; ++v)
                xb[u][v] = xn[u][v];
    }
    /* the renormalisation after each column's last step (a no-op where that
     * step was a renormalised one: its max is already in [1/2, 1)) */
    if (!dense) {
#pragma unroll
        for (int u = 0; u < TPW; ++u) {
            double mx = 0.0;
#pragma unroll
            for (int kk = 0; kk < KSM; ++kk)
                mx = fmax(mx, q[u][kk]);
            mx = fmax(mx, __shfl_xor(mx, 16));
            mx = fmax(mx, __shfl_xor(mx, 32));
            const int e2 = __builtin_amdgcn_frexp_exp(mx);
#pragma unroll
            for (int kk = 0; kk < KSM; ++kk)
                q[u][kk] = ldexp(q[u][kk], -e2);
            ex[u] += e2;
        }
    }
    /* M'_c[i][j] (row i = this column, j = 4kk + (lane >> 4)) and the row
     * exponent (-inf: the filter died, the row is zero) */
#pragma unroll
    for (int u = 0; u < TPW; ++u) {
        if (!valid[u])
            continue;
        const int col = (tg * TPW + u) * 16 + (lane & 15);
        const int c = col / K, i = col - c * K;
        double *m = a.sc_mf + (((int64_t)p * nc + c) * K + i) * K;
        double mx = 0.0;
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk) {
            const int j = 4 * kk + (lane >> 4);
            if (j < K)
                m[j] = q[u][kk];
            mx = fmax(mx, q[u][kk]);
        }
        mx = fmax(mx, __shfl_xor(mx, 16));
        mx = fmax(mx, __shfl_xor(mx, 32));
        if ((lane >> 4) == 0)
            a.sc_mx[((int64_t)p * nc + c) * K + i] = mx > 0.0 ? (double)ex[u] : dev_ninf();
        if (GS && (lane >> 4) == 0 && i == 0) /* every column of the chunk has the same shifts */
            a.sc_bl[(int64_t)p * nc + c] = gls[u];
    }
}

/* Phase 2: one wave per pair, lane j = state j (j < K).  The chunk's M' is
 * staged in LDS (K*K doubles) from a coalesced load that runs one chunk ahead. */
template <int KM>
__device__ __forceinline__ void lks_stage_load(const DevArgs &a, int64_t p, int c, double (&r)[(KM * KM + 63) / 64])
{
    const int K = a.K, nc = a.scan_nc;
    const double *m = a.sc_mf + ((int64_t)p * nc + max(c, 0)) * K * K;
#pragma unroll
    for (int v = 0; v < (KM * KM + 63) / 64; ++v) {
        const int idx = v * 64 + (int)(threadIdx.x & 63);
        r[v] = idx < K * K ? m[idx] : 0.0;
    }
}

/* hmm.stan:30 (Q2): log(p_1k) + SUM_k normal_lpdf(x[1] | mu_k, sigma_k), the
 * sum in state order (fwd_init's), evaluated by every lane */
__device__ __forceinline__ double lks_gauss_init(const DevArgs &a, int64_t n, int64_t d)
{
    const double x1 = a.xr[n];
    double s = 0.0;
    for (int k = 0; k < a.K; ++k) {
        const double sg = a.sigma_k[d + a.S * k];
        const double z = (x1 - a.mu_k[d + a.S * k]) * (1.0 / sg);
        s += HHMM_NEG_LOG_SQRT_TWO_PI;
        s -= dev_cr_log(sg);
        s += -0.5 * (z * z);
    }
    return s;
}

template <int KM, bool GS>
__global__ void __launch_bounds__(64) lks_bound_kernel(const DevArgs a)
{
    __shared__ double mt[KM * KM];
    __shared__ double xv[64];
    constexpr int NV = (KM * KM + 63) / 64;
    const int64_t p = blockIdx.x;
    const int j = threadIdx.x;
    const int K = a.K, nc = a.scan_nc, cl = a.scan_cl;
    const bool on = j < K;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + cl - 1) / cl;
    const int64_t S = a.S;
    const int jj = on ? j : 0;
    auto base = [&](int c) { return ((int64_t)p * nc + c); };
    auto wmax_d = [&](double v) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
            v = fmax(v, __shfl_xor(v, off));
        return v;
    };
    auto wmax_i = [&](int v) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
            v = max(v, __shfl_xor(v, off));
        return v;
    };
    auto wsum_d = [&](double v) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
            v += __shfl_xor(v, off);
        return v;
    };
    /* exponent of a row: frexp exponent of the value + the row's scale; INT_MIN/2 for a zero */
    constexpr int kDead = -(1 << 29);

    /* ---- forward: f_0 = p_1k .* phi[., x_1] (hmm-multinom.stan:31), then f <- f M_c;
     * a segment window that starts inside the series enters from the caller's
     * state (seg_enter: K values up to scale, then their log scale) ---- */
    double f, lsc = 0.0;
    if (!a.seg_nofirst) {
        if constexpr (GS) { /* alpha_1 = p_1k, the summed emission into the log scale (Q2) */
            f = on ? a.p_1k[d + S * jj] : 0.0;
            lsc = lks_gauss_init(a, n, d);
        } else {
            const int x0 = min(max(a.x[n], 1), a.L);
            f = on ? a.p_1k[d + S * jj] * a.phi_k[d + S * ((int64_t)jj + (int64_t)K * (x0 - 1))] : 0.0;
        }
    } else {
        f = on ? a.seg_enter[p + a.P * (int64_t)jj] : 0.0;
        lsc = a.seg_enter[p + a.P * (int64_t)K];
    }
    int fe = __builtin_amdgcn_frexp_exp(wmax_d(f));
    f = ldexp(f, -fe);
    lsc += kLn2 * fe;
    double rb[NV];
    lks_stage_load<KM>(a, p, 0, rb);
    for (int c = 0; c < ncp; ++c) {
        if ((c > 0 || a.seg_nofirst) && on) {
            a.sc_st[base(c) * K + j] = f;
            if (j == 0)
                a.sc_sl[base(c)] = lsc;
        }
        __syncthreads();
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (v * 64 + j < KM * KM)
                mt[v * 64 + j] = rb[v];
        lks_stage_load<KM>(a, p, min(c + 1, ncp - 1), rb);
        const double sr = on ? a.sc_mx[base(c) * K + j] : dev_ninf();
        const int er = (f != 0.0 && sr != dev_ninf()) ? __builtin_amdgcn_frexp_exp(f) + (int)sr : kDead;
        const int em = wmax_i(er);
        xv[j] = (er == kDead || em == kDead) ? 0.0 : ldexp(f, (int)sr - em);
        __syncthreads();
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < KM; ++i)
            if (i < K)
                acc[i & 3] = fma(xv[i], mt[i * K + jj], acc[i & 3]);
        double nf = on ? (acc[0] + acc[1]) + (acc[2] + acc[3]) : 0.0;
        const int e2 = __builtin_amdgcn_frexp_exp(wmax_d(nf));
        f = ldexp(nf, -e2);
        lsc += kLn2 * ((double)(em == kDead ? 0 : em) + e2);
        if constexpr (GS)
            lsc += a.sc_bl[base(c)]; /* the chunk's Gaussian emission shifts */
    }
    const double sf = wsum_d(on ? f : 0.0);
    if (j == 0 && (a.outputs & HHMM_OUT_LOGLIK) && a.loglik && !a.seg_nolast)
        a.loglik[p] = log(sf) + lsc;

    /* ---- backward: beta_T = 1 (unbeta_tk[T] = 1, Q1), or the beta leaving a
     * segment window (the caller's; its scale cancels in the posteriors);
     * b_{c-1} = M_c b_c ---- */
    double b = on ? (a.seg_nolast ? a.seg_leave[p + a.P * (int64_t)jj] : 1.0) : 0.0;
    if (on && ncp > 0)
        a.sc_be[base(ncp - 1) * K + j] = b;
    lks_stage_load<KM>(a, p, ncp - 1, rb);
    for (int c = ncp - 1; c >= 1; --c) {
        __syncthreads();
#pragma unroll
        for (int v = 0; v < NV; ++v)
            if (v * 64 + j < KM * KM)
                mt[v * 64 + j] = rb[v];
        xv[j] = b;
        lks_stage_load<KM>(a, p, c - 1, rb);
        __syncthreads();
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < KM; ++i)
            if (i < K)
                acc[i & 3] = fma(mt[jj * K + i], xv[i], acc[i & 3]);
        const double h = on ? (acc[0] + acc[1]) + (acc[2] + acc[3]) : 0.0;
        const double sr = on ? a.sc_mx[base(c) * K + j] : dev_ninf();
        const int er = (h != 0.0 && sr != dev_ninf()) ? __builtin_amdgcn_frexp_exp(h) + (int)sr : kDead;
        const int em = wmax_i(er);
        b = (er == kDead || em == kDead) ? 0.0 : ldexp(h, (int)sr - em);
        if (on)
            a.sc_be[base(c - 1) * K + j] = b;
    }
}

/* ---- Segment summary at large K (include/hhmm.h hhmm_segment; SURVEY §8e,
 * the flattened-HHMM shape: few pairs, 23 states, T = 10^6 split along T over
 * ranks).  hmm-multinom has no masks, so the window's forward product and its
 * backward product are the same matrix: SF = SQ = M_0 M_1 ... with
 * M_c = diag(2^s) M'_c the chunk products of lks_prod_kernel (row exponents
 * s).  One wave per pair: the running product S (K x K, one power-of-two
 * exponent E) and the chunk's M' sit in LDS; lane l owns column l & 31 of S
 * for the rows of parity l >> 5.  Each chunk scales the columns of S by
 * 2^(s_k - max s) (exact while no entry underflows: rows more than 2^1074
 * below the largest are dropped, as lks_bound_kernel drops them), multiplies
 * by M'_c in state order, and renormalises by the exact power of two of the
 * largest entry.  The first window's rows all hold the state leaving it
 * (p_1k .* phi[., x_1] times S): the layout of the K <= 8 summary
 * (seg_summary_kernel), so hhmm_amd.segment.boundaries chains both. ---- */
template <int KM, bool GS>
__global__ void __launch_bounds__(64) lks_seg_summary_kernel(const DevArgs a)
{
    __shared__ double Sm[KM * KM];
    __shared__ double Mt[KM * KM];
    __shared__ double fk[KM];
    constexpr int RH = (KM + 1) / 2; /* rows per lane */
    constexpr int kDead = -(1 << 29);
    const int64_t p = blockIdx.x;
    const int l = threadIdx.x;
    const int K = a.K, nc = a.scan_nc, cl = a.scan_cl;
    const int col = l & 31, h = l >> 5;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + cl - 1) / cl;
    const int64_t S = a.S;
    auto base = [&](int c) { return ((int64_t)p * nc + c); };
    auto wmax_i = [&](int v) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
            v = max(v, __shfl_xor(v, off));
        return v;
    };
    auto wmax_d = [&](double v) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
            v = fmax(v, __shfl_xor(v, off));
        return v;
    };
    /* the chunk's row exponents: fk[k] = 2^(s_k - smax) (0 for a dead row); returns smax */
    auto stage = [&](int c) {
        for (int idx = l; idx < K * K; idx += 64)
            Mt[idx] = a.sc_mf[base(c) * K * K + idx];
        const double s = l < K ? a.sc_mx[base(c) * K + l] : dev_ninf();
        const int si = (s == dev_ninf()) ? kDead : (int)s;
        const int smax = wmax_i(si);
        if (l < K)
            fk[l] = (si == kDead || smax == kDead) ? 0.0 : ldexp(1.0, si - smax);
        return smax == kDead ? 0 : smax;
    };
    double r[RH];
    int E = 0;
    /* S = M_0 */
    E = stage(0);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < RH; ++q) {
        const int i = 2 * q + h;
        r[q] = (i < K && col < K) ? Mt[i * K + col] * fk[i] : 0.0;
    }
    for (int c = 1; c <= ncp; ++c) {
        /* renormalise the new rows, then publish them */
        double m = 0.0;
#pragma unroll
        for (int q = 0; q < RH; ++q)
            m = fmax(m, r[q]);
        const int e = __builtin_amdgcn_frexp_exp(wmax_d(m));
        E += e;
        __syncthreads(); /* every lane is done reading Sm and Mt */
#pragma unroll
        for (int q = 0; q < RH; ++q) {
            const int i = 2 * q + h;
            if (i < K && col < K)
                Sm[i * K + col] = ldexp(r[q], -e);
        }
        if (c == ncp)
            break;
        E += stage(c);
        __syncthreads();
        /* new S[i][col] = sum_k (S[i][k] 2^(s_k - smax)) M'_c[k][col] */
#pragma unroll
        for (int q = 0; q < RH; ++q) {
            const int i = 2 * q + h;
            double acc = 0.0;
            if (i < K && col < K)
                for (int k = 0; k < K; ++k)
                    acc = fma(Sm[i * K + k] * fk[k], Mt[k * K + col], acc);
            r[q] = acc;
        }
    }
    __syncthreads();
    const int KK = K * K;
    double *out = a.seg_sum;
    for (int idx = l; idx < KK; idx += 64) /* SQ = the product (beta entering = SQ beta leaving) */
        out[p + a.P * (int64_t)(KK + idx)] = Sm[idx];
    int fex = E;
    /* the window's Gaussian log scale: its chunks' emission shifts (hmm.stan) */
    double gl = 0.0;
    if constexpr (GS)
        for (int c = 0; c < ncp; ++c)
            gl += a.sc_bl[base(c)];
    if (!a.seg_nofirst) {
        /* the first window: every row holds p_1k .* phi[., x_1] (hmm-multinom.stan:31) times S;
         * hmm.stan: p_1k, the summed emission of x_1 into the log scale (Q2) */
        double f0;
        if constexpr (GS) {
            f0 = (l < K) ? a.p_1k[d + S * l] : 0.0;
            gl += lks_gauss_init(a, n, d);
        } else {
            const int x0 = min(max(a.x[n], 1), a.L);
            f0 = (l < K) ? a.p_1k[d + S * l] * a.phi_k[d + S * ((int64_t)l + (int64_t)K * (x0 - 1))] : 0.0;
        }
        const int fe = __builtin_amdgcn_frexp_exp(wmax_d(f0));
        if (l < K)
            fk[l] = ldexp(f0, -fe);
        __syncthreads();
        double g = 0.0;
        if (l < K)
            for (int k = 0; k < K; ++k)
                g = fma(fk[k], Sm[k * K + l], g);
        const int e2 = __builtin_amdgcn_frexp_exp(wmax_d(l < K ? g : 0.0));
        g = ldexp(g, -e2);
        fex = E + fe + e2;
        if (l < K)
            for (int i = 0; i < K; ++i)
                out[p + a.P * (int64_t)(i * K + l)] = g;
    } else {
        for (int idx = l; idx < KK; idx += 64)
            out[p + a.P * (int64_t)idx] = Sm[idx];
    }
    if (l == 0) {
        out[p + a.P * (int64_t)(2 * KK + 0)] = (double)fex;
        out[p + a.P * (int64_t)(2 * KK + 1)] = gl; /* the Gaussian log scale (0: hmm-multinom) */
        out[p + a.P * (int64_t)(2 * KK + 2)] = (double)E;
    }
}

/* ---- Many series under one draw (GRID pairing, N >= 16; SURVEY §8 N1 at large
 * K): the forward-backward itself on the matrix cores.  The series evaluated
 * under draw s share its A, so the forward step of 16 of them is the dense
 * product A^T [alpha_1 ... alpha_16] -- one column per series, the same
 * operand layout and register reuse as lks_prod_kernel -- and the backward
 * step is A [e_t .* beta_1 ... e_t .* beta_16].  One wave = (draw s, tile of
 * 16 series), draw-fastest over the grid, so the waves writing the same
 * gamma lines (p = s + S n: consecutive draws) run side by side.
 *   forward   alpha_t column-renormalised by exact powers of two (exponents
 *             summed per column: the log-likelihood), a checkpoint of the
 *             tile every kLmChunk steps (coalesced: register kk of lane l)
 *   backward  chunk by chunk from the end: the chunk's alphas recomputed from
 *             its checkpoint into registers, then gamma_t = alpha .* beta / sum
 *             (the reference's normalised-vector formula where that sum is
 *             below kGammaDirect, as lk_fb_kernel) and the beta step.
 * Outputs: loglik, gamma_tk (the hot profile); ragged T per series. ---- */
constexpr int kLmChunk = 8;

template <int RT, int KSM>
__global__ void __launch_bounds__(256) lkm_fb_kernel(const DevArgs a)
{
    constexpr int KR = 16 * RT;
    constexpr int C = kLmChunk;
    HIP_DYNAMIC_SHARED(double, lds)
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int K = a.K;
    const int ks = (K + 3) / 4;
    const int64_t NT = (a.N + 15) / 16; /* series tiles */
    const int64_t nw = a.S * NT;
    const int64_t w = min((int64_t)blockIdx.x * (blockDim.x >> 6) + wv, nw - 1);
    const int64_t d = w % a.S;        /* the draw */
    const int64_t tile = w / a.S;
    const int64_t n = min(tile * 16 + (lane & 15), a.N - 1);
    const bool col_ok = tile * 16 + (lane & 15) < a.N;
    const int64_t p = d + a.S * n;    /* GRID pair */
    const int Tn = pair_len(a, n);
    const int64_t S = a.S;

    double *tab = lds + (size_t)wv * a.L * KR; /* phi[l][j], rows j >= K zero */
    for (int idx = lane; idx < a.L * KR; idx += 64) {
        const int l = idx / KR, j = idx - l * KR;
        tab[idx] = j < K ? a.phi_k[d + S * ((int64_t)j + (int64_t)K * l)] : 0.0;
    }
    /* A operands: forward A^T[j][i] = A(i, j); backward A[j][i] = A(j, i)
     * (row j = 16rt + (lane & 15), k = i = 4kk + (lane >> 4)) */
    double af[RT][KSM], ab[RT][KSM];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk) {
            const int i = 4 * kk + (lane >> 4), j = 16 * rt + (lane & 15);
            const bool in = i < K && j < K;
            af[rt][kk] = in ? a.A_ij[d + S * ((int64_t)i + (int64_t)K * j)] : 0.0;
            ab[rt][kk] = in ? a.A_ij[d + S * ((int64_t)j + (int64_t)K * i)] : 0.0;
        }
    double pj[KSM];
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk) {
        const int j = 4 * kk + (lane >> 4);
        pj[kk] = j < K ? a.p_1k[d + S * j] : 0.0;
    }
    __syncthreads();

    const int Tw = wave_max(col_ok ? Tn : 1);
    auto xat = [&](int t) -> int { return a.x[n + a.N * (int64_t)min(max(t, 0), a.Tmax - 1)]; };
    /* emission rows j = 4kk + (lane >> 4) of this lane's column at symbol x */
    auto emis = [&](int x, double (&e)[KSM]) {
        const double *row = tab + (min(max(x, 1), a.L) - 1) * KR + (lane >> 4);
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            e[kk] = row[4 * kk];
    };
    /* column reductions over the tile's 4 lane rows (lanes l ^ 16, l ^ 32) */
    auto colmax = [&](double v) {
        v = fmax(v, __shfl_xor(v, 16));
        return fmax(v, __shfl_xor(v, 32));
    };
    auto colsum = [&](double v) {
        v += __shfl_xor(v, 16);
        return v + __shfl_xor(v, 32);
    };
    auto renorm = [&](double (&q)[KSM], int &ex) {
        double mx = q[0];
#pragma unroll
        for (int kk = 1; kk < KSM; ++kk)
            mx = fmax(mx, q[kk]);
        const int e2 = __builtin_amdgcn_frexp_exp(colmax(mx));
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            q[kk] = ldexp(q[kk], -e2);
        ex += e2;
    };
    auto mm = [&](const double (&A)[RT][KSM], const double (&q)[KSM], double (&out)[KSM]) {
        lks_d4 acc[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
            acc[rt] = lks_d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            if (kk < ks) {
#pragma unroll
                for (int rt = 0; rt < RT; ++rt)
                    acc[rt] = lks_mfma(A[rt][kk], q[kk], acc[rt]);
            }
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            out[kk] = acc[kk >> 2][kk & 3];
    };
    /* checkpoints: [wave][chunk][kk][64 lanes] */
    const int nck = (Tw + C - 1) / C;
    double *ck = a.ckpt + (size_t)w * (size_t)((a.Tmax + C - 1) / C) * KSM * 64;
    auto ck_at = [&](int c, int kk) -> double & { return ck[((size_t)c * KSM + kk) * 64 + lane]; };

    /* ---- forward ---- */
    double q[KSM], e[KSM];
    int ex = 0;
    emis(xat(0), e);
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk)
        q[kk] = pj[kk] * e[kk]; /* hmm-multinom.stan:31 */
    renorm(q, ex);
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk)
        ck_at(0, kk) = q[kk];
    /* observations a block of kXb steps ahead (one load per step and lane,
     * issued a block before use: a one-step prefetch waited an HBM round trip
     * per step) */
    constexpr int kXb = 16;
    int xb[kXb], xnb[kXb];
#pragma unroll
    for (int v = 0; v < kXb; ++v)
        xb[v] = xat(v);
    for (int t = 1; t < Tw; ++t) {
        if (t % kXb == 0) { /* wave-uniform */
#pragma unroll
            for (int v = 0; v < kXb; ++v)
                xb[v] = xnb[v];
        }
        if (t % kXb == 1 || t == 1) {
#pragma unroll
            for (int v = 0; v < kXb; ++v)
                xnb[v] = xat((t / kXb + 1) * kXb + v);
        }
        int x = xb[0];
#pragma unroll
        for (int v = 1; v < kXb; ++v)
            x = (t % kXb == v) ? xb[v] : x;
        double dq[KSM];
        mm(af, q, dq);
        emis(x, e);
        const bool on = t < Tn;
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            dq[kk] *= e[kk];
        int e2 = 0;
        renorm(dq, e2);
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            q[kk] = on ? dq[kk] : q[kk];
        ex += on ? e2 : 0;
        if (t % C == 0) {
#pragma unroll
            for (int kk = 0; kk < KSM; ++kk)
                ck_at(t / C, kk) = q[kk];
        }
    }
    {
        double sq = 0.0;
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            sq += q[kk];
        sq = colsum(sq);
        if ((lane >> 4) == 0 && col_ok && (a.outputs & HHMM_OUT_LOGLIK) && a.loglik)
            a.loglik[p] = log(sq) + kLn2 * ex;
    }
    if (!((a.outputs & HHMM_OUT_GAMMA) && a.gamma))
        return;

    /* ---- backward: beta_T = 1 (unbeta_tk[T] = 1, Q1) ---- */
    double be[KSM];
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk)
        be[kk] = (4 * kk + (lane >> 4) < K) ? 1.0 : 0.0;
    int xs[C], xsn[C];
    double ckn[KSM];
#pragma unroll
    for (int u = 0; u < C; ++u)
        xsn[u] = xat((nck - 1) * C + u);
#pragma unroll
    for (int kk = 0; kk < KSM; ++kk)
        ckn[kk] = ck_at(nck - 1, kk);
    for (int c = nck - 1; c >= 0; --c) {
        const int t0 = c * C;
        double al[C][KSM];
#pragma unroll
        for (int u = 0; u < C; ++u)
            xs[u] = xsn[u];
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            al[0][kk] = ckn[kk];
        /* the next chunk's observations and checkpoint, a chunk ahead */
#pragma unroll
        for (int u = 0; u < C; ++u)
            xsn[u] = xat((c - 1) * C + u);
#pragma unroll
        for (int kk = 0; kk < KSM; ++kk)
            ckn[kk] = ck_at(max(c - 1, 0), kk);
#pragma unroll
        for (int u = 1; u < C; ++u) {
            double dq[KSM];
            mm(af, al[u - 1], dq);
            emis(xs[u], e);
#pragma unroll
            for (int kk = 0; kk < KSM; ++kk)
                dq[kk] *= e[kk];
            int e2 = 0;
            renorm(dq, e2);
#pragma unroll
            for (int kk = 0; kk < KSM; ++kk)
                al[u][kk] = dq[kk];
        }
#pragma unroll
        for (int u = C - 1; u >= 0; --u) {
            const int t = t0 + u;
            if (t >= Tw) /* wave-uniform */
                continue;
            const bool on = t < Tn;
            /* gamma_t = alpha .* beta / sum, the normalised-vector form below kGammaDirect */
            double ug[KSM], sg = 0.0;
#pragma unroll
            for (int kk = 0; kk < KSM; ++kk) {
                ug[kk] = al[u][kk] * be[kk];
                sg += ug[kk];
            }
            sg = colsum(sg);
            const bool small = !(sg > kGammaDirect);
            double rg = 1.0 / sg;
            if (__builtin_amdgcn_readfirstlane((int)(__ballot(small) != 0))) { /* rare, wave-uniform */
                double sa = 0.0, sb = 0.0;
#pragma unroll
                for (int kk = 0; kk < KSM; ++kk) {
                    sa += al[u][kk];
                    sb += be[kk];
                }
                sa = colsum(sa);
                sb = colsum(sb);
                double ssum = 0.0;
#pragma unroll
                for (int kk = 0; kk < KSM; ++kk) {
                    ug[kk] = small ? (al[u][kk] / sa) * (be[kk] / sb) : ug[kk];
                    ssum += ug[kk];
                }
                ssum = colsum(ssum);
                rg = small ? 1.0 / ssum : rg;
            }
            if (on && col_ok) {
#pragma unroll
                for (int kk = 0; kk < KSM; ++kk) {
                    const int j = 4 * kk + (lane >> 4);
                    if (j < K)
                        __builtin_nontemporal_store(ug[kk] * rg, a.gamma + p + a.P * ((int64_t)t + (int64_t)a.Tout * j));
                }
            }
            if (t > 0) { /* wave-uniform: the matrix product and the column
                          * reductions run on every lane; columns past their
                          * series' end keep beta_T */
                /* beta_{t-1} = A (e_t .* beta_t) */
                emis(xs[u], e);
                double v[KSM], nb[KSM];
#pragma unroll
                for (int kk = 0; kk < KSM; ++kk)
                    v[kk] = e[kk] * be[kk];
                mm(ab, v, nb);
                int e2 = 0;
                renorm(nb, e2);
#pragma unroll
                for (int kk = 0; kk < KSM; ++kk)
                    be[kk] = on ? nb[kk] : be[kk];
            }
        }
    }
}

/* lkm_fb_kernel's domain: hmm-multinom under GRID pairing with at least 16
 * series per draw, the hot output profile (loglik + gamma_tk), sequential in
 * T (no scan), asked for (HHMM_FLAG_LKM_MFMA, opt-in); hhmm_kernels.hip sizes
 * its checkpoints by the same rule (lkm_plan). */
static inline bool lkm_ok(const DevArgs &a)
{
    return lkm_plan(a.model, a.K, a.N, a.pairing, a.outputs, a.flags, a.scan_cl) != 0;
}

/* LDS bytes of a launch with `threads` lanes: exchange slots + tables. */
template <int G>
static inline size_t lk_lds(const DevArgs &a, int threads, bool discrete)
{
    const size_t groups = (size_t)threads / G;
    return groups * 2 * G * sizeof(double) + (discrete ? groups * (size_t)a.L * G * sizeof(double) : 0);
}

template <int MODEL, int G, int KM>
static hhmm_status run_large_model(const DevArgs &a, hipStream_t st)
{
    constexpr bool discrete = !LkTraits<MODEL>::kGauss;
    const uint32_t out = a.outputs;
    const uint32_t fb = HHMM_OUT_LOGLIK | HHMM_OUT_ALPHA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA;
    const uint32_t vit = HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR;
    const uint32_t ffbs = HHMM_OUT_FFBS;
    if (a.scan_cl > 0 && discrete && a.L * 16 * ((KM + 15) / 16) * 4 * sizeof(double) > 64 * 1024) {
        set_error("K = %d: the parallel scan over T runs hmm-multinom with L <= %d", a.K, 64 * 1024 / (4 * 8 * 16 * ((KM + 15) / 16)));
        return HHMM_ERR_UNSUPPORTED;
    }
    constexpr bool GS = LkTraits<MODEL>::kGauss;
    const size_t plds = discrete ? (size_t)4 * a.L * 16 * ((KM + 15) / 16) * sizeof(double) : 0;
    const uint32_t logs = HHMM_OUT_UNALPHA | HHMM_OUT_UNBETA;
    if (out & ~(fb | vit | ffbs | logs)) {
        set_error("K = %d > %d: the large-K path evaluates loglik, unalpha, alpha, unbeta, beta, ungamma, gamma, "
                  "zstar, logp_zstar and z_ffbs", a.K, kMaxK);
        return HHMM_ERR_UNSUPPORTED;
    }
    int threads = kBlock;
    while (threads > G && lk_lds<G>(a, threads, discrete) > kLdsLimit)
        threads /= 2;
    if (lk_lds<G>(a, threads, discrete) > kLdsLimit) {
        set_error("emission table of L = %d symbols does not fit in LDS", a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const int gpb = threads / G;
    if (a.seg_phase) {
        /* one window of a series split over ranks along T (hhmm_segment):
         * phase 1 + the window's summary, or phases 2 + 3 from the caller's
         * entering state / leaving beta */
        if (a.scan_cl <= 0) {
            set_error("segment windows at K = %d > %d: hmm / hmm-multinom on the T-scan", a.K, kMaxK);
            return HHMM_ERR_UNSUPPORTED;
        }
        constexpr int RT = (KM + 15) / 16, KSM = KM / 4;
        if (a.seg_phase == 1) {
            const int ntile = (a.scan_nc * a.K + 15) / 16;
            const int64_t waves = a.P * (int64_t)((ntile + kLksTiles - 1) / kLksTiles);
            hipLaunchKernelGGL((lks_prod_kernel<RT, KSM, GS>), dim3((unsigned)((waves + 3) / 4)), dim3(256), plds, st,
                               a);
            hipLaunchKernelGGL((lks_seg_summary_kernel<KM, GS>), dim3((unsigned)a.P), dim3(64), 0, st, a);
        } else {
            hipLaunchKernelGGL((lks_bound_kernel<KM, GS>), dim3((unsigned)a.P), dim3(64), 0, st, a);
            const int64_t nq = a.P * (int64_t)a.scan_nc;
            if (out & (fb & ~HHMM_OUT_LOGLIK))
                hipLaunchKernelGGL((lk_fb_kernel<MODEL, G, KM>), dim3((unsigned)((nq + gpb - 1) / gpb)),
                                   dim3(threads), lk_lds<G>(a, threads, discrete), st, a);
        }
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) {
            set_error("large-K segment launch: %s", hipGetErrorString(e));
            return HHMM_ERR_HIP;
        }
        return HHMM_OK;
    }
    const dim3 grid((unsigned)((a.P + gpb - 1) / gpb));
    /* checkpoints use the [rows][K][P] layout of the lane kernels.  With both
     * halves requested the decoder runs on the library's side stream, forked
     * from and joined back into the caller's: the two kernels' registers fit
     * one wave of each per SIMD (K <= 24: 224 + 160), so they overlap */
    hipStream_t vs = st;
    if ((out & fb) && (out & vit) && !(a.flags & HHMM_FLAG_NO_FUSE)) {
        const hhmm_status r = fork_stream(st, &vs);
        if (r != HHMM_OK)
            return r;
    }
    if (out & vit)
        hipLaunchKernelGGL((lk_viterbi_kernel<MODEL, G, KM>), dim3((unsigned)((a.P + gpb - 1) / gpb)), dim3(threads),
                           lk_lds<G>(a, threads, discrete), vs, a);
    hipError_t e = hipGetLastError();
    if ((out & ffbs) && e == hipSuccess) {
        /* the FFBS contract's filter and draws (sequential per pair); its
         * checkpoints share the workspace with lk_fb_kernel's, so it runs
         * first on the caller's stream */
        DevArgs f = a;
        f.outputs = HHMM_OUT_FFBS;
        const size_t tab = discrete ? 0 : 128 * sizeof(hhmm_exp2_entry); /* lk_ffbs_kernel's det-exp table */
        hipLaunchKernelGGL((lk_ffbs_kernel<MODEL, G, KM>), grid, dim3(threads), lk_lds<G>(a, threads, discrete) + tab, st,
                           f);
        e = hipGetLastError();
    }
    const bool mfma_fb = lkm_ok(a);
    if ((out & logs) && e == hipSuccess) {
        /* the log-scale profile: every posterior output of the request from the
         * reference's log-space recursion (as fb_log_kernel at K <= 8) */
        hipLaunchKernelGGL((lk_log_kernel<MODEL, G, KM>), grid, dim3(threads), lk_lds<G>(a, threads, discrete), st, a);
        e = hipGetLastError();
    } else if ((out & fb) && a.scan_cl > 0 && e == hipSuccess) {
        /* parallel scan over T (hhmm_lkscan.h): MFMA chunk products, the scan
         * over chunks, then the chunks' sweeps as groups (pair, chunk) */
        constexpr int RT = (KM + 15) / 16, KSM = KM / 4;
        const int ntile = (a.scan_nc * a.K + 15) / 16;
        const int64_t waves = a.P * (int64_t)((ntile + kLksTiles - 1) / kLksTiles);
        hipLaunchKernelGGL((lks_prod_kernel<RT, KSM, GS>), dim3((unsigned)((waves + 3) / 4)), dim3(256), plds, st, a);
        hipLaunchKernelGGL((lks_bound_kernel<KM, GS>), dim3((unsigned)a.P), dim3(64), 0, st, a);
        const int64_t nq = a.P * (int64_t)a.scan_nc;
        if (out & (fb & ~HHMM_OUT_LOGLIK)) /* the chunks' sweeps: posteriors (the loglik is phase 2's) */
            hipLaunchKernelGGL((lk_fb_kernel<MODEL, G, KM>), dim3((unsigned)((nq + gpb - 1) / gpb)), dim3(threads),
                               lk_lds<G>(a, threads, discrete), st, a);
        e = hipGetLastError();
    } else if ((out & fb) && mfma_fb && e == hipSuccess) {
        /* many series under each draw: the forward-backward on the matrix cores */
        constexpr int RT = (KM + 15) / 16, KSM = KM / 4;
        const int64_t waves = a.S * ((a.N + 15) / 16);
        hipLaunchKernelGGL((lkm_fb_kernel<RT, KSM>), dim3((unsigned)((waves + 3) / 4)), dim3(256), plds, st, a);
        e = hipGetLastError();
    } else if ((out & fb) && e == hipSuccess) {
        hipLaunchKernelGGL((lk_fb_kernel<MODEL, G, KM>), dim3((unsigned)((a.P + gpb - 1) / gpb)), dim3(threads),
                           lk_lds<G>(a, threads, discrete), st, a);
        e = hipGetLastError();
    }
    const hhmm_status j = (vs != st) ? join_stream(st, vs) : HHMM_OK;
    if (e != hipSuccess) {
        set_error("large-K kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return j;
}

} // namespace hhmm
