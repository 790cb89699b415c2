/*
 * hhmm_vscan.h -- T-parallel exact Viterbi for batches of few pairs with long
 * series (SURVEY.md §8 A11 at the C5 shape: 250 pairs x T = 1e6 per GPU, the
 * HMM family at K = 2 and 4).  Included by hhmm_hmm.h; DESIGN.md §3.5.
 *
 * The reference's recursion (hhmm-tayal2009.stan:130-165, hmm.stan:104-117)
 *   delta_t(j) = max_i fl(fl(delta_{t-1}(i) + a) + b)
 * (a, b = log A(i, j) and log phi(j, x_t) in the model's order, strict '>'
 * from -inf) is sequential in t and its rounding depends on the magnitude of
 * delta, which grows like t.  The decoders of hhmm_hmm.h therefore walk T one
 * step at a time; at C5 that leaves 16 waves on a 1024-SIMD chip.
 *
 * What makes T-parallel decoding exact: inside one binade [2^k, 2^(k+1)) of
 * |delta| every double is an integer multiple of u = 2^(k-52), and
 *   fl(n u + a) = (n + rho(a)) u,   rho(a) = rint(a / u)
 * whenever the sum stays in the binade and a / u is not a rounding tie.  So
 * while a chunk of steps keeps every relevant value in one binade, Stan's
 * rounded recursion IS the exact max-plus recursion on the grid values
 * rho(log A), rho(log phi): chunk matrices M_c (K x K max-plus products of the
 * grid step matrices) compose exactly, and delta leaving chunk c is
 * delta_c (x) M_c -- no rounding, no speculation.  (Values below the binade's
 * lower edge are never on a survivor path into an in-binade value: log
 * probabilities are <= 0, so path values only decrease.)
 *
 * Kernels, in stream order (lane = (pair, chunk) unless noted):
 *   vs_prod<GRID=false>  approximate chunk products (plain doubles)
 *   vs_scan0 (wave/pair) chunk 0 exactly (the model's t = 1 row, Q3 NaN step),
 *                        then the approximate scan: the binade k_c expected at
 *                        each chunk's entry
 *   vs_prod<GRID=true>   exact grid products on k_c's grid, tie flags
 *   vs_prod_tie          chunks with a rounding tie (listed by the grid
 *                        pass): products for even and odd entry values
 *                        (round-half-even depends on parity), lane per row
 *   vs_scan1 (wave/pair) the exact scan: delta_c (x) M_c where the checks hold
 *                        (entry max in binade k_c, every finite exit
 *                        value inside the binade), else that chunk decoded
 *                        step by step; one wave per pair, so a chunk crossing
 *                        a binade costs only its own pair
 *   vs_replay            every chunk decoded again from its exact entry vector
 *                        in the reference's arithmetic: back-pointer words in
 *                        the shared layout, the chunk's backtrack map (entry
 *                        state of each exit state), and a bitwise check of its
 *                        exit against the scan (vs_fail on a mismatch)
 *   vs_stitch (lane/pair) logp_zstar, zstar_T, pair_status; the path state at
 *                        every chunk end through the backtrack maps
 *   vs_fill              the path inside each chunk from its end state
 *   viterbi_sp_kernel    restricted to vs_fail pairs (none expected): the
 *                        sequential decoder rewrites their outputs
 * The replay makes correctness independent of the scan's checks: a pair whose
 * chunk exits disagree is decoded sequentially.
 */
#pragma once
#include <type_traits>

namespace hhmm {

constexpr int32_t kVsTie = 1 << 30;     /* vs_k: a grid rounding tie inside the chunk */
/* Tie chunks (round 6).  The grid pass lists every chunk holding a rounding
 * tie (vs_tl) and vs_prod_tie_kernel forms the chunk's two parity products
 * with one lane per (parity, row): 2K lanes per chunk.  At C5, 75 of 488,500
 * chunks hold a tie, but while the tie products ran inline (one lane per chunk,
 * both parities, the whole K x K product) the grid pass needed 293 VGPRs and
 * 31k instructions and took 4.3 ms; listed, it needs 143 VGPRs and takes
 * 1.1 ms, and the row-parallel tie kernel 0.6 ms (C5 8.73 -> 7.71 ms,
 * profiles/r06t_ab_c5_tie_rows.log).  Earlier list versions kept one lane per
 * chunk-parity and lost (rounds 2-3, round 6: 9.67 against 8.71 ms): that
 * lane's 512 steps of the whole product were the critical path.  Leaving tie
 * chunks to the exact scan's step-by-step decode instead costs 4 ms there
 * (a tie persists over a whole binade, so one pair holds dozens of them). */
constexpr int32_t kVsNoGrid = -(1 << 20); /* vs_k: no finite magnitude estimate */
constexpr int32_t kVsSeq = -(1 << 21);    /* vs_k after the exact scan: the chunk was decoded step by step */

/* rho_u(a) = rint(a / u) u (exact: u a power of two); tie when a / u is a
 * half-integer.  -inf maps to -inf (never a tie). */
__device__ __forceinline__ double vs_grid(double a, double iu, double u, bool &tie)
{
    const double s = a * iu;
    const double r = rint(s);
    tie |= (__builtin_fabs(s - r) == 0.5);
    return r * u;
}

/* Binade exponent k of a finite nonzero double: |x| in [2^k, 2^(k+1)). */
__device__ __forceinline__ int vs_binade(double x) { return __builtin_amdgcn_frexp_exp(x) - 1; }

/* lane = (pair, chunk): p fastest so a wave's lanes read one time row. */
struct VsLane {
    int64_t p, n, d;
    int c;
    int Tp;
    int t0, t1; /* the chunk's steps [t0, t1) within the pair's series */
};

__device__ __forceinline__ bool vs_lane(const DevArgs &a, VsLane &v)
{
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    v.p = g % a.P;
    v.c = (int)(g / a.P);
    pair_coords(a, v.p, v.n, v.d);
    v.Tp = pair_len(a, v.n);
    v.t0 = v.c * kVsChunk;
    v.t1 = min(v.t0 + kVsChunk, v.Tp);
    return v.c < a.vs_nc;
}

/* The observation loop of one chunk: STEP(t, obs) for t in [t0, t1), the
 * observations of the next 8 steps in flight. */
template <int MODEL, bool AUX, typename F>
__device__ __forceinline__ void vs_steps(const SeriesPtrs &sp, int t0, int t1, F &&step)
{
    constexpr int C = 8;
    Obs cur[C], nxt[C];
    load_chunk<MODEL, C, AUX>(cur, sp, t0);
    for (int tb = t0; tb < t1; tb += C) {
        load_chunk<MODEL, C, AUX>(nxt, sp, tb + C);
#pragma unroll
        for (int u = 0; u < C; ++u)
            if (tb + u < t1)
                step(tb + u, cur[u]);
#pragma unroll
        for (int u = 0; u < C; ++u)
            cur[u] = nxt[u];
    }
}

/* Rounding ties.  When a / u is a half-integer q + 1/2, fl(n u + a) rounds
 * n + q + 1/2 to the even neighbour: m + (m & 1) with m = n + q, which
 * depends on the parity of n.  Every step map x -> fl(x + a) is still
 * monotone, and along a path the parity of the running value is fixed by the
 * parity of the entry value, so a chunk holding a tie has two exact products:
 * M0 for even entry values and M1 for odd ones (per entry state), and the
 * exit is max_r (delta(r) + M^{parity(delta(r))}[r][j]).  vs_prod_tie_kernel
 * computes both, in units of u (integer-valued doubles), for the chunks the
 * grid pass flagged. */
struct VsTerm {
    double r, q;   /* rint(a/u), floor(a/u) */
    double rp, qp; /* their parities (0 / 1) */
    bool tie;
};

/* The chunk products in HBM, pair-major (round 4): chunk c of pair p is the
 * K*K record at vs_mat, so the scans' lanes (consecutive chunks of one pair)
 * read consecutive lines. */
template <int K>
__device__ __forceinline__ int64_t vs_mat(const DevArgs &a, int64_t p, int c)
{
    return (p * a.vs_nc + c) * (int64_t)(K * K);
}

/* parity (0 or 1) of an integer-valued double */
__device__ __forceinline__ double vs_parity(double x) { return x - 2.0 * floor(x * 0.5); }

__device__ __forceinline__ VsTerm vs_term(double a, double iu)
{
    const double s = a * iu;
    VsTerm t;
    t.r = rint(s);
    t.q = floor(s);
    t.tie = __builtin_fabs(s - t.r) == 0.5;
    t.rp = vs_parity(t.r);
    t.qp = vs_parity(t.q);
    return t;
}

/* o (+) a on the grid (o in units of u; ap = parity of the absolute value):
 * returns the new offset and updates ap.  A tie rounds to the even
 * neighbour: bump = parity(absolute + q), result even.  XOR of 0/1 doubles
 * is |x - y|. */
__device__ __forceinline__ double vs_add(double o, const VsTerm &t, double &ap)
{
    if (!(o > dev_ninf()))
        return o;
    if (t.tie) {
        const double bump = __builtin_fabs(ap - t.qp);
        ap = 0.0;
        return (o + t.q) + bump;
    }
    ap = __builtin_fabs(ap - t.rp);
    return o + t.r;
}

/* Row r of one parity product of a tie chunk (pi = parity of the entry
 * values), into out.  A row of the max-plus product -- the best path sums from
 * entry state r -- evolves on its own, so a chunk's 2K rows (two parities, K
 * entry states) run on 2K lanes: the same operations per row as the whole
 * product, each row's dependent chain a K-th of its length. */
template <int MODEL, int K>
__device__ __forceinline__ void vs_tie_row(const DevArgs &a, const VsLane &v, const PairParams<MODEL, K> &pp,
                                           const double2 *slab, const SeriesPtrs &sp, double iu, double u, double pi,
                                           int r, double *out)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    VsTerm gA[K][K];
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
        for (int i = 0; i < K; ++i)
            gA[i][j] = vs_term(pp.A[i][j], iu);
    double M[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        M[j] = (r == j) ? 0.0 : dev_ninf();
    vs_steps<MODEL, VAUX>(sp, v.t0, v.t1, [&](int, const Obs &o) {
        double le[K];
        emit_log<MODEL, K>(pp, slab, a.L, o, le);
        VsTerm gl[K];
        bool on[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            gl[j] = vs_term(le[j], iu);
            on[j] = true;
            if constexpr (ModelTraits<MODEL>::kTayal)
                on[j] = tayal_pred(o.aux, j);
        }
        double nm[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            double best = dev_ninf();
#pragma unroll
            for (int i = 0; i < K; ++i) {
                double cand;
                const bool t2 = on[j] && gA[i][j].tie;
                if (!gl[j].tie && !t2) { /* no tie in this term: plain grid arithmetic */
                    cand = M[i] + (ModelTraits<MODEL>::kTayal ? (on[j] ? gl[j].r + gA[i][j].r : gl[j].r)
                                                              : gA[i][j].r + gl[j].r);
                } else {
                    double ap = vs_parity(M[i] + pi);
                    if constexpr (ModelTraits<MODEL>::kTayal) {
                        cand = vs_add(M[i], gl[j], ap);
                        if (on[j])
                            cand = vs_add(cand, gA[i][j], ap);
                    } else {
                        cand = vs_add(M[i], gA[i][j], ap);
                        cand = vs_add(cand, gl[j], ap);
                    }
                }
                best = fmax(best, cand);
            }
            nm[j] = best;
        }
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[j] = nm[j];
    });
#pragma unroll
    for (int j = 0; j < K; ++j)
        out[vs_mat<K>(a, v.p, v.c) + r * K + j] = M[j] * u;
}

/* The tie chunks' parity products for the chunks the grid pass listed
 * (kVsTie), one lane per (chunk, parity, row): 2K lanes per chunk. */
constexpr int kVsTieBlocks = 512;
template <int MODEL, int K>
__global__ void __launch_bounds__(kBlock) vs_prod_tie_kernel(const DevArgs a)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    constexpr int KP = (K + 1) / 2;
    HIP_DYNAMIC_SHARED(double2, lds)
    /* work items (listed tie chunk q, parity, row): item i = 2K q + K parity + row;
     * a grid of kVsTieBlocks workgroups walks them */
    const int n = __builtin_amdgcn_readfirstlane(a.vs_tl[0]);
    const int64_t items = 2 * (int64_t)K * n;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x; i0 < items; i0 += stride) {
    const int64_t i = i0 + threadIdx.x;
    const bool live = i < items;
    const int64_t q = live ? i / (2 * K) : 0;
    const int rem = (int)(i - q * 2 * K);
    const int par = rem / K, row = rem % K;
    const int64_t g0 = live ? a.vs_tl[1 + q] : 0;
    VsLane v;
    v.p = g0 % a.P;
    v.c = (int)(g0 / a.P);
    pair_coords(a, v.p, v.n, v.d);
    v.Tp = pair_len(a, v.n);
    v.t0 = v.c * kVsChunk;
    v.t1 = min(v.t0 + kVsChunk, v.Tp);
    const int32_t kw = a.vs_k[v.p + a.P * (int64_t)v.c];
    const bool work = live && !(v.c >= a.vs_nc || v.c == 0 || v.t0 >= v.Tp) &&
                      !(kw == kVsNoGrid || !(kw & kVsTie) || kw < 0);
    const int32_t kc = kw & ~kVsTie;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    if (work) {
        PairParams<MODEL, K> pp;
        load_params<MODEL, K, true>(pp, a, v.d);
        if constexpr (ModelTraits<MODEL>::kDiscrete)
            fill_table<K, true>(slab, a, v.d);
        const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, v.n);
        vs_tie_row<MODEL, K>(a, v, pp, slab, sp, ldexp(1.0, 52 - kc), ldexp(1.0, kc - 52), (double)par, row,
                             par ? a.vs_m1 : a.vs_m);
    }
    }
}

/* A grid-pass lane whose chunk holds a rounding tie: flag it and list it for
 * vs_prod_tie_kernel. */
__device__ __forceinline__ void vs_list_tie(const DevArgs &a, const VsLane &v, int32_t kc)
{
    a.vs_k[v.p + a.P * (int64_t)v.c] = (kc >= 0) ? (kc | kVsTie) : kVsNoGrid;
    if (kc >= 0) {
        const int slot = atomicAdd(&a.vs_tl[0], 1);
        a.vs_tl[1 + slot] = (int32_t)(v.p + a.P * (int64_t)v.c);
    }
}

/* Chunk max-plus product M = S_{t0} (x) ... (x) S_{t1-1}, M[r][j] = best path
 * sum from state r entering the chunk to state j at its last step.  GRID:
 * every term on the grid of the chunk's binade (vs_k), tie flag into vs_k. */
template <int MODEL, int K, bool GRID>
__global__ void __launch_bounds__(kBlock) vs_prod_kernel(const DevArgs a)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    constexpr int KP = (K + 1) / 2;
    HIP_DYNAMIC_SHARED(double2, lds)
    VsLane v;
    if (!vs_lane(a, v) || v.c == 0 || v.t0 >= v.Tp)
        return;
    int32_t kc = 0;
    double u = 0.0, iu = 0.0;
    if constexpr (GRID) {
        kc = a.vs_k[v.p + a.P * (int64_t)v.c];
        if (kc == kVsNoGrid)
            return;
        u = ldexp(1.0, kc - 52);
        iu = ldexp(1.0, 52 - kc);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    PairParams<MODEL, K> pp;
    load_params<MODEL, K, true>(pp, a, v.d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        fill_table<K, true>(slab, a, v.d);
    bool tie = false;
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, v.n);
    if constexpr (GRID && ModelTraits<MODEL>::kDiscrete) {
        /* ties known up front (the log A and log phi tables): the chunk's two
         * parity products right here, so no second pass waits for them */
        bool any = false;
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                any = any || vs_term(pp.A[i][j], iu).tie;
        for (int l = 0; l < a.L; ++l)
#pragma unroll
            for (int kp = 0; kp < KP; ++kp) {
                const double2 e = slab[(l * KP + kp) * 64];
                any = any || vs_term(e.x, iu).tie || (2 * kp + 1 < K && vs_term(e.y, iu).tie);
            }
        if (any) { /* listed: vs_prod_tie_kernel forms its parity products */
            vs_list_tie(a, v, kc);
            return;
        }
    }
    if constexpr (GRID) {
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                pp.A[i][j] = vs_grid(pp.A[i][j], iu, u, tie);
    }
    /* the approximate pass (GRID = false) only predicts the binade of each
     * chunk's entry for the exact pass, which checks it: its products run in
     * float (half the registers; the exact scan decodes a chunk whose entry
     * misses the predicted binade step by step) */
    using V = typename std::conditional<GRID, double, float>::type;
    V Av[K][K];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            Av[i][j] = (V)pp.A[i][j];
    V M[K][K];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[r][j] = (r == j) ? (V)0.0 : (V)dev_ninf();
    if constexpr (GRID && ModelTraits<MODEL>::kDiscrete) {
        /* the emission table on the grid, once (no tie: checked above) */
        for (int l = 0; l < a.L; ++l)
#pragma unroll
            for (int kp = 0; kp < KP; ++kp) {
                double2 &e = slab[(l * KP + kp) * 64];
                e = make_double2(vs_grid(e.x, iu, u, tie), vs_grid(e.y, iu, u, tie));
            }
    }
    /* M'[r][j] = max_i (M[r][i] + log A[i][j]) + log phi_j (the grid sums are
     * exact, so the terms may be regrouped); Tayal steps whose mask is off for
     * j take max_i M[r][i] + log phi_j, the row max shared by those columns */
    vs_steps<MODEL, VAUX>(sp, v.t0, v.t1, [&](int, const Obs &o) {
        double le[K];
        emit_log<MODEL, K>(pp, slab, a.L, o, le);
        V lv[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if constexpr (GRID && ModelTraits<MODEL>::kGauss)
                le[j] = vs_grid(le[j], iu, u, tie);
            lv[j] = (V)le[j];
        }
        /* the Tayal sign class as a constant where the wave shares it */
        tayal_dispatch<MODEL>(o, true, [&](auto sgc) {
        constexpr int SG = decltype(sgc)::value;
        bool on[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            on[j] = true;
            if constexpr (ModelTraits<MODEL>::kTayal)
                on[j] = SG > 0 ? tayal_on(SG, j) : tayal_pred(o.aux, j);
        }
#pragma unroll
        for (int r = 0; r < K; ++r) {
            V nm[K];
            V rm = M[r][0];
            if constexpr (ModelTraits<MODEL>::kTayal) {
#pragma unroll
                for (int i = 1; i < K; ++i)
                    rm = fmax(rm, M[r][i]);
            }
#pragma unroll
            for (int j = 0; j < K; ++j) {
                V best;
                if (ModelTraits<MODEL>::kTayal && !on[j]) {
                    best = rm;
                } else {
                    best = M[r][0] + Av[0][j];
#pragma unroll
                    for (int i = 1; i < K; ++i)
                        if (!(SG > 0 && ModelTraits<MODEL>::kTayal && !tayal_nz(i, j))) /* -inf: no effect */
                            best = fmax(best, M[r][i] + Av[i][j]);
                }
                nm[j] = best + lv[j];
            }
#pragma unroll
            for (int j = 0; j < K; ++j)
                M[r][j] = nm[j];
        }
        });
    });
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            a.vs_m[vs_mat<K>(a, v.p, v.c) + r * K + j] = (double)M[r][j];
    if (GRID && tie) /* a tie met during the pass (Gaussian emissions); kc < 0 (|delta| < 1): decoded step by step */
        vs_list_tie(a, v, kc);
}

template <int K>
__device__ __forceinline__ void vs_store_d(const DevArgs &a, int64_t p, int row, const double (&D)[K])
{
#pragma unroll
    for (int k = 0; k < K; ++k)
        a.vs_d[p + a.P * ((int64_t)row * K + k)] = D[k];
}

template <int K>
__device__ __forceinline__ void vs_load_d(const DevArgs &a, int64_t p, int row, double (&D)[K])
{
#pragma unroll
    for (int k = 0; k < K; ++k)
        D[k] = a.vs_d[p + a.P * ((int64_t)row * K + k)];
}

/* Largest finite entry (-inf if none). */
template <int K>
__device__ __forceinline__ double vs_hi(const double (&D)[K])
{
    double hi = dev_ninf();
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (__builtin_isfinite(D[k]))
            hi = fmax(hi, D[k]);
    return hi;
}

/* One step of the reference's recursion (vit_step's arithmetic) that also
 * returns each state's arg max. */
template <int MODEL, int K, bool NANIN, int SG = -1>
__device__ __forceinline__ void vs_step_sg(double (&dl)[K], const PairParams<MODEL, K> &pp, const double (&le)[K],
                                           const Obs &o, int (&arg)[K])
{
    double nd[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        bool on = true;
        if constexpr (ModelTraits<MODEL>::kTayal)
            on = SG > 0 ? tayal_on(SG, j) : tayal_pred(o.aux, j);
        double best = dev_ninf();
        int am = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
            /* a known-on column's structural zeros (log A = -inf) past i = 0:
             * a -inf / NaN candidate changes neither the max nor the arg max */
            if constexpr (SG > 0 && ModelTraits<MODEL>::kTayal)
                if (i > 0 && on && !tayal_nz(i, j))
                    continue;
            double cand;
            if constexpr (ModelTraits<MODEL>::kTayal) {
                cand = dl[i] + le[j];
                cand = on ? cand + pp.A[i][j] : cand;
            } else {
                cand = (dl[i] + pp.A[i][j]) + le[j];
            }
            if (i == 0) {
                best = NANIN ? fmax(best, cand) : cand;
            } else {
                const bool gt = cand > best;
                best = fmax(best, cand);
                am = gt ? i : am;
            }
        }
        nd[j] = best;
        arg[j] = am;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        dl[j] = nd[j];
}

/* vs_step with the Tayal sign class as a constant where the wave shares it
 * (tayal_dispatch: one series under many draws; the same operations) */
template <int MODEL, int K, bool NANIN>
__device__ __forceinline__ void vs_step(double (&dl)[K], const PairParams<MODEL, K> &pp, const double (&le)[K],
                                        const Obs &o, int (&arg)[K])
{
    tayal_dispatch<MODEL>(o, true, [&](auto sgc) { vs_step_sg<MODEL, K, NANIN, decltype(sgc)::value>(dl, pp, le, o, arg); });
}

/* Chunk 0 from the model's first row: delta_tk[1] has only column K written
 * (Q3), the step after it meets the NaN entries.  ON_STEP(t, arg) sees every
 * step t >= 1. */
template <int MODEL, int K, typename F>
__device__ __forceinline__ void vs_chunk0(const DevArgs &a, const PairParams<MODEL, K> &pp, const double2 *slab,
                                          const SeriesPtrs &sp, int t1, double (&dl)[K], F &&on_step)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    vs_steps<MODEL, VAUX>(sp, 0, t1, [&](int t, const Obs &o) {
        double le[K];
        emit_log<MODEL, K>(pp, slab, a.L, o, le);
        int arg[K];
        if (t == 0) {
#pragma unroll
            for (int k = 0; k < K - 1; ++k)
                dl[k] = dev_nan();
            dl[K - 1] = le[K - 1];
            return;
        }
        if (t == 1)
            vs_step<MODEL, K, true>(dl, pp, le, o, arg);
        else
            vs_step<MODEL, K, false>(dl, pp, le, o, arg);
        on_step(t, arg);
    });
}

/* Chunk c >= 1 from its entry vector. */
template <int MODEL, int K, typename F>
__device__ __forceinline__ void vs_chunk(const DevArgs &a, const PairParams<MODEL, K> &pp, const double2 *slab,
                                         const SeriesPtrs &sp, int t0, int t1, double (&dl)[K], F &&on_step)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    vs_steps<MODEL, VAUX>(sp, t0, t1, [&](int t, const Obs &o) {
        double le[K];
        emit_log<MODEL, K>(pp, slab, a.L, o, le);
        int arg[K];
        vs_step<MODEL, K, false>(dl, pp, le, o, arg);
        on_step(t, arg);
    });
}

/* The scans walk one pair's chunks in order, one wave per pair.  Lane l holds
 * chunk (block + l)'s product and grid word, the next block's 64 chunks in
 * flight while this one is walked; every lane walks the block with the values
 * staged through LDS (uniform-address reads), so the walk neither waits on
 * memory per chunk nor diverges (all lanes compute the same delta; lane 0
 * stores).  A lane-per-pair walk waited one memory round trip per chunk. */
template <int K>
struct VsBlock {
    double m[K][K];
    double m1[K][K]; /* tie chunks: the products for odd entry values */
    int32_t k;
};

template <int K>
__device__ __forceinline__ void vs_fetch(const DevArgs &a, int64_t p, int c0, int ncp, VsBlock<K> &b)
{
    const int c = max(min(c0 + (int)(threadIdx.x & 63), ncp - 1), 0);
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            b.m[r][j] = a.vs_m[vs_mat<K>(a, p, c) + r * K + j];
    b.k = a.vs_k[p + a.P * (int64_t)c];
    const bool tie = b.k >= 0 && (b.k & kVsTie);
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            b.m1[r][j] = tie ? a.vs_m1[vs_mat<K>(a, p, c) + r * K + j] : 0.0;
}

/* The scans' series index as a VGPR value: with one pair per wave every
 * observation address is uniform, and hipcc would fetch x_t / sign_t with
 * scalar loads, which share lgkmcnt with the per-step LDS table reads -- each
 * step's LDS wait then also waited for the prefetched observations. */
__device__ __forceinline__ int64_t vs_vector_index(int64_t n)
{
    uint32_t v = (uint32_t)n;
    asm volatile("" : "+v"(v));
    return v;
}

/* The block in LDS, one row of 18 doubles per chunk (K*K products, the grid
 * word): the walk then reads chunk i with uniform-address LDS loads instead
 * of K*K*2 readlanes per chunk. */
constexpr int kVsRow = 34; /* K*K products, K*K odd-entry products, the grid word */

template <int K>
__device__ __forceinline__ void vs_stage(const VsBlock<K> &b, double *blk)
{
    double *r = blk + (threadIdx.x & 63) * kVsRow;
#pragma unroll
    for (int rr = 0; rr < K; ++rr)
#pragma unroll
        for (int j = 0; j < K; ++j)
            r[rr * K + j] = b.m[rr][j];
#pragma unroll
    for (int rr = 0; rr < K; ++rr)
#pragma unroll
        for (int j = 0; j < K; ++j)
            r[16 + rr * K + j] = b.m1[rr][j];
    r[32] = __longlong_as_double((long long)b.k);
}

template <int K>
__device__ __forceinline__ int32_t vs_apply_lds(const double *blk, int i, const double (&D)[K], double (&out)[K])
{
    const double *r = blk + i * kVsRow;
    const int32_t kw = (int32_t)__double_as_longlong(r[32]);
    int off[K];
#pragma unroll
    for (int rr = 0; rr < K; ++rr)
        off[rr] = rr * K;
    if (kw >= 0 && (kw & kVsTie)) { /* M^{parity(delta(r))} per entry state */
        const double iu = ldexp(1.0, 52 - (kw & ~kVsTie));
#pragma unroll
        for (int rr = 0; rr < K; ++rr)
            off[rr] = (vs_parity(D[rr] * iu) == 1.0) ? 16 + rr * K : rr * K;
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double best = D[0] + r[off[0] + j];
#pragma unroll
        for (int rr = 1; rr < K; ++rr)
            best = fmax(best, D[rr] + r[off[rr] + j]);
        out[j] = best;
    }
    return kw;
}

/* Step-by-step decoding inside the scans (chunk 0, and chunks that fail the
 * grid checks), one lane per (state, quad) as viterbi_sp_kernel does: every
 * quad of the wave runs the same pair, lane j of a quad holds delta(j) and
 * forms its K candidates from the quad's delta by DPP broadcasts, with
 * vit_step's arithmetic (the two decoders are bit-identical).  A lane walking
 * all K states alone took ~1200 cycles per step on a wave with nothing else
 * to hide its latency; the quad form has a K-times shorter chain per lane. */
template <int MODEL, int K>
__device__ __forceinline__ void vs_sp_setup(const DevArgs &a, int64_t d, double *ldsd, SpLane<MODEL, K> &ln)
{
    const int lane = threadIdx.x & 63;
    ln.j = lane & 3;
    ln.js = min(ln.j, K - 1);
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
}

/* Steps [t0, t1) from the quad's delta (FIRST: t0 = 0, the model's first row).
 * The emission column entry and the masked log A row of step t+1 are read
 * while step t computes, so the per-step chain is the DPP broadcast, two adds
 * and the max. */
template <int MODEL, int K, bool FIRST>
__device__ __forceinline__ void vs_sp_steps(const DevArgs &a, const SpLane<MODEL, K> &ln, const SeriesPtrs &sp,
                                            int t0, int t1, double (&D)[K])
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    constexpr int C = 16;
    double dl = D[0];
#pragma unroll
    for (int k = 1; k < K; ++k)
        dl = (ln.js == k) ? D[k] : dl;
    Obs cur[C], nxt[C];
    load_chunk<MODEL, C, VAUX>(cur, sp, t0);
    double le = sp_emit<MODEL, K>(ln, cur[0], a.L);
    double ar[K];
#pragma unroll
    for (int i = 0; i < K; ++i)
        ar[i] = 0.0;
    if constexpr (ModelTraits<MODEL>::kTayal)
        sp_arow<MODEL, K>(ln, cur[0].aux, ar);
    for (int tb = t0; tb < t1; tb += C) {
        load_chunk<MODEL, C, VAUX>(nxt, sp, tb + C);
#pragma unroll
        for (int u = 0; u < C; ++u) {
            const int t = tb + u;
            const Obs &on1 = (u + 1 < C) ? cur[u + 1 < C ? u + 1 : 0] : nxt[0];
            const double lnx = sp_emit<MODEL, K>(ln, on1, a.L);
            double arx[K];
#pragma unroll
            for (int i = 0; i < K; ++i)
                arx[i] = 0.0;
            if constexpr (ModelTraits<MODEL>::kTayal)
                sp_arow<MODEL, K>(ln, on1.aux, arx);
            if (t < t1) {
                if (FIRST && t == 0) { /* Q3: only column K of delta_tk[1] is written */
                    dl = (ln.js == K - 1) ? le : dev_nan();
                } else {
                    double d[K];
                    quad_gather<K>(dl, d);
                    double best = dev_ninf();
#pragma unroll
                    for (int i = 0; i < K; ++i) {
                        double cand;
                        if constexpr (ModelTraits<MODEL>::kTayal)
                            cand = (d[i] + le) + ar[i]; /* (delta + log phi) [+ log A] */
                        else
                            cand = (d[i] + ln.colA[i]) + le; /* (delta + log A) + emission */
                        best = fmax(best, cand);
                    }
                    dl = best;
                }
            }
            le = lnx;
#pragma unroll
            for (int i = 0; i < K; ++i)
                ar[i] = arx[i];
        }
#pragma unroll
        for (int u = 0; u < C; ++u)
            cur[u] = nxt[u];
    }
    quad_gather<K>(dl, D);
}

/* LDS of the scans: the state-parallel columns (log phi, Tayal masked log A rows). */
template <int MODEL, int K>
constexpr size_t vs_sp_lds(int L)
{
    return ((ModelTraits<MODEL>::kDiscrete ? (size_t)L : 0) + (ModelTraits<MODEL>::kTayal ? (size_t)3 * K : 0)) *
           64 * sizeof(double);
}

/* Max-plus product of two K x K matrices, C = A (x) B (approximate scan). */
template <int K>
__device__ __forceinline__ void vs_mp_mul(const double (&A)[K][K], const double (&B)[K][K], double (&C)[K][K])
{
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j) {
            double b = A[i][0] + B[0][j];
#pragma unroll
            for (int k = 1; k < K; ++k)
                b = fmax(b, A[i][k] + B[k][j]);
            C[i][j] = b;
        }
}

template <int K>
__device__ __forceinline__ void vs_mp_shfl_up(const double (&A)[K][K], int d, double (&Q)[K][K])
{
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            Q[i][j] = __shfl_up(A[i][j], d, 64);
}

/* One block of the approximate scan with the wave's lanes in parallel: lane l
 * holds chunk cb + l's approximate product (identity past the pair's last
 * chunk); a Hillis-Steele max-plus prefix over the 64 lanes gives every lane
 * the delta entering its chunk from the block's entry `dl` (uniform), whose
 * binade it stores; `dl` leaves as the block's exit.  The approximate scan
 * only predicts each chunk's grid (the exact scan checks every prediction),
 * so the reassociated sums are harmless; the serial walk spent ~1,200 cycles
 * of dependent latency per chunk on its one wave. */
template <int K>
__device__ __forceinline__ void vs_scan0_block(const DevArgs &a, int64_t p, int cb, int ncp, const VsBlock<K> &b,
                                               double (&dl)[K])
{
    const int lane = threadIdx.x & 63;
    const bool live = cb + lane < ncp;
    double P[K][K];
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            P[i][j] = live ? b.m[i][j] : (i == j ? 0.0 : dev_ninf());
#pragma unroll
    for (int d = 1; d < 64; d *= 2) {
        double Q[K][K], R[K][K];
        vs_mp_shfl_up<K>(P, d, Q);
        vs_mp_mul<K>(Q, P, R);
        if (lane >= d) {
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int j = 0; j < K; ++j)
                    P[i][j] = R[i][j];
        }
    }
    /* exclusive prefix: the product of the chunks before this lane's */
    double E[K][K];
    vs_mp_shfl_up<K>(P, 1, E);
    double din[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (lane == 0) {
            din[j] = dl[j];
        } else {
            double v = dl[0] + E[0][j];
#pragma unroll
            for (int r = 1; r < K; ++r)
                v = fmax(v, dl[r] + E[r][j]);
            din[j] = v;
        }
    }
    if (live) {
        const double hi = vs_hi<K>(din);
        a.vs_k[p + a.P * (int64_t)(cb + lane)] = (hi > dev_ninf() && hi != 0.0) ? vs_binade(hi) : kVsNoGrid;
    }
    /* the block's exit: dl (x) the inclusive prefix of lane 63 (identity past ncp) */
    double out[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double v = dl[0] + __shfl(P[0][j], 63, 64);
#pragma unroll
        for (int r = 1; r < K; ++r)
            v = fmax(v, dl[r] + __shfl(P[r][j], 63, 64));
        out[j] = v;
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        dl[j] = out[j];
}

/* One wave per pair: chunk 0 exactly (row 1 of vs_d), then the approximate
 * scan over the approximate chunk products: k_c = binade of the largest
 * finite delta entering chunk c.  PAR: the lane-parallel prefix per block of
 * 64 chunks (vs_scan0_block); else the serial walk. */
template <int MODEL, int K, bool PAR>
__global__ void __launch_bounds__(64) vs_scan0_kernel(const DevArgs a)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    HIP_DYNAMIC_SHARED(double, ldsd)
    const int64_t p = blockIdx.x;
    const bool l0 = threadIdx.x == 0;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + kVsChunk - 1) / kVsChunk;
    SpLane<MODEL, K> ln;
    vs_sp_setup<MODEL, K>(a, d, ldsd, ln);
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, vs_vector_index(n));
    double *blk = ldsd + vs_sp_lds<MODEL, K>(a.L) / sizeof(double);
    VsBlock<K> nxt;
    vs_fetch<K>(a, p, 1, ncp, nxt);
    double dl[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
        dl[k] = 0.0;
    vs_sp_steps<MODEL, K, true>(a, ln, sp, 0, min(kVsChunk, Tp), dl);
    if (l0)
        vs_store_d<K>(a, p, 1, dl);
    if constexpr (PAR) {
        for (int cb = 1; cb < ncp; cb += 64) {
            const VsBlock<K> cur = nxt;
            vs_fetch<K>(a, p, cb + 64, ncp, nxt);
            vs_scan0_block<K>(a, p, cb, ncp, cur, dl);
        }
        return;
    }
    for (int cb = 1; cb < ncp; cb += 64) {
        vs_stage<K>(nxt, blk);
        __syncthreads();
        vs_fetch<K>(a, p, cb + 64, ncp, nxt);
        for (int i = 0; i < 64 && cb + i < ncp; ++i) {
            const double hi = vs_hi<K>(dl);
            if (l0)
                a.vs_k[p + a.P * (int64_t)(cb + i)] = (hi > dev_ninf() && hi != 0.0) ? vs_binade(hi) : kVsNoGrid;
            double nx[K];
            (void)vs_apply_lds<K>(blk, i, dl, nx);
#pragma unroll
            for (int k = 0; k < K; ++k)
                dl[k] = nx[k];
        }
        __syncthreads();
    }
}

/* A chunk the exact scan cannot take whole -- its values cross into the next
 * binade (11 chunks per pair at C5, each 512 steps decoded step by step at
 * ~370 cycles a step on the pair's one wave), or a check failed -- in
 * kVsSub sub-chunks (round 4, discrete emissions): lane g kVsSub + s forms
 * sub-chunk s's max-plus product on the grid of the entry's binade kb + g
 * (g = 0, 1: the chunk's values start in kb and cross into kb + 1), then the
 * wave walks the sub-chunks from the exact entry with the chunk checks at the
 * sub-chunk's own binade: a sub-chunk that passes takes its product (exact,
 * the grid argument), the one the crossing falls in (or a rounding tie) is
 * decoded step by step.  The replay still checks the chunk's exit bit for
 * bit. */
constexpr int kVsSub = 8;

template <int MODEL, int K>
__device__ __forceinline__ void vs_cross_chunk(const DevArgs &a, const SpLane<MODEL, K> &ln,
                                                         const SeriesPtrs &sp, const double *ldsd, int t0, int t1,
                                                         double (&dl)[K])
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    constexpr int SL = kVsChunk / kVsSub;
    const int lane = threadIdx.x & 63;
    const double hi0 = vs_hi<K>(dl);
    if (!(hi0 > dev_ninf() && hi0 != 0.0)) {
        vs_sp_steps<MODEL, K, false>(a, ln, sp, t0, t1, dl);
        return;
    }
    const int kb0 = vs_binade(hi0);
    const int sub = lane % kVsSub, g = min(lane / kVsSub, 1);
    const double u = ldexp(1.0, kb0 + g - 52), iu = ldexp(1.0, 52 - (kb0 + g));
    bool tie = false;
    double gA[K][K]; /* log A[i][j] on the grid: column j from quad lane j (non-Tayal) */
#pragma unroll
    for (int i = 0; i < K; ++i)
#pragma unroll
        for (int j = 0; j < K; ++j)
            gA[i][j] = vs_grid(__shfl(ln.colA[i], j, 64), iu, u, tie);
    double M[K][K];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[r][j] = (r == j) ? 0.0 : dev_ninf();
    const int s0 = t0 + sub * SL, s1 = min(s0 + SL, t1);
    for (int t = s0; t < s1; ++t) {
        Obs o[1];
        load_chunk<MODEL, 1, VAUX>(o, sp, t);
        const int xr = min(max(o[0].x, 1), a.L) - 1;
        double le[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            le[j] = vs_grid(ldsd[xr * 64 + j], iu, u, tie); /* log phi[j][x_t]: quad lane j's column */
        double aij[K][K];
        if constexpr (ModelTraits<MODEL>::kTayal) {
            /* the masked column of quad lane j for this step's sign (-0.0 where off) */
            const int rr = (o[0].aux == 1) ? 0 : (o[0].aux == 2 ? 1 : 2);
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int j = 0; j < K; ++j)
                    aij[i][j] = vs_grid(ldsd[(size_t)(a.L + rr * K + i) * 64 + j], iu, u, tie);
        } else {
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int j = 0; j < K; ++j)
                    aij[i][j] = gA[i][j];
        }
#pragma unroll
        for (int r = 0; r < K; ++r) {
            double nm[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                double best = M[r][0] + aij[0][j];
#pragma unroll
                for (int i = 1; i < K; ++i)
                    best = fmax(best, M[r][i] + aij[i][j]);
                nm[j] = best + le[j];
            }
#pragma unroll
            for (int j = 0; j < K; ++j)
                M[r][j] = nm[j];
        }
    }
    const uint64_t ties = __ballot(tie && lane < 2 * kVsSub);
    for (int sb = 0; sb < kVsSub; ++sb) {
        const int a0 = t0 + sb * SL;
        if (a0 >= t1)
            break;
        const int a1 = min(a0 + SL, t1);
        const double hi = vs_hi<K>(dl);
        bool ok = hi > dev_ninf() && hi != 0.0;
        const int kd = ok ? vs_binade(hi) : kb0;
        const int gg = kd - kb0;
        ok = ok && (gg == 0 || gg == 1);
        const int src = (ok ? gg : 0) * kVsSub + sb;
        ok = ok && !((ties >> src) & 1);
        double nx[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            double best = dl[0] + __shfl(M[0][j], src, 64);
#pragma unroll
            for (int r = 1; r < K; ++r)
                best = fmax(best, dl[r] + __shfl(M[r][j], src, 64));
            nx[j] = best;
        }
        const double edge = -ldexp(1.0 - 0x1p-40, kd + 1);
#pragma unroll
        for (int k = 0; k < K; ++k)
            ok = ok && (nx[k] == dev_ninf() || nx[k] > edge);
        if (ok) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                dl[k] = nx[k];
        } else {
            vs_sp_steps<MODEL, K, false>(a, ln, sp, a0, a1, dl);
        }
    }
}

/* One chunk of the exact scan from the exact entry dl (wave-uniform): the
 * grid product where the checks hold (a tie chunk through M0 / M1 by the
 * entry values' parities), else in sub-chunks (vs_cross_chunk; step by step
 * for Gaussian emissions).  Row c + 1 of vs_d. */
template <int MODEL, int K>
__device__ __forceinline__ void vs_exact_chunk(const DevArgs &a, int64_t p, const SpLane<MODEL, K> &ln,
                                               const SeriesPtrs &sp, const double *blk, const double *ldsd, int i,
                                               int c, int Tp, double (&dl)[K])
{
    const bool l0 = (threadIdx.x & 63) == 0;
    const double hi = vs_hi<K>(dl);
    double nx[K];
    const int32_t kc = vs_apply_lds<K>(blk, i, dl, nx);
    const int32_t kb = (kc >= 0) ? (kc & ~kVsTie) : kc; /* ties are exact through M0 / M1 */
    bool ok = kc != kVsNoGrid && hi > dev_ninf() && hi != 0.0 && vs_binade(hi) == kb;
    /* every finite exit value inside the binade, 2^-40 of its width clear of the edge */
    const double edge = -ldexp(1.0 - 0x1p-40, kb + 1);
#pragma unroll
    for (int k = 0; k < K; ++k)
        ok = ok && (nx[k] == dev_ninf() || nx[k] > edge);
    if (ok) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            dl[k] = nx[k];
    } else {
        const int t0 = c * kVsChunk;
        if constexpr (ModelTraits<MODEL>::kDiscrete)
            vs_cross_chunk<MODEL, K>(a, ln, sp, ldsd, t0, min(t0 + kVsChunk, Tp), dl);
        else
            vs_sp_steps<MODEL, K, false>(a, ln, sp, t0, min(t0 + kVsChunk, Tp), dl);
        if (l0)
            a.vs_k[p + a.P * (int64_t)c] = kVsSeq;
    }
    if (l0)
        vs_store_d<K>(a, p, c + 1, dl);
}

/* One wave per pair: the exact scan over the grid products, chunks failing
 * the checks decoded step by step.  Rows 2..ncp of vs_d.
 * Lane-parallel per block of 64 chunks (round 4): a max-plus Hillis-Steele
 * prefix of the grid products from lane s on gives every lane a candidate
 * entry, every lane applies its own chunk to it and makes the serial walk's
 * checks, and a lane's candidate counts only if it is bit for bit the exit of
 * the lane before it: so every committed exit is the serial walk's own
 * arithmetic from a verified entry, whatever the reassociated prefix did.
 * (Within one binade the grid sums are exact, so the candidates do match; a
 * tie chunk, a binade crossing or a failed check ends the run.)  The first
 * lane f that fails is walked exactly as before, then the prefix restarts at
 * f + 1.  At C5 the serial walk took 2.4 ms, ~1,900 cycles per chunk on one
 * wave per pair. */
template <int MODEL, int K>
__global__ void __launch_bounds__(64) vs_scan1_kernel(const DevArgs a)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    HIP_DYNAMIC_SHARED(double, ldsd)
    const int64_t p = blockIdx.x;
    const int lane = threadIdx.x & 63;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + kVsChunk - 1) / kVsChunk;
    if (ncp < 2)
        return;
    SpLane<MODEL, K> ln;
    vs_sp_setup<MODEL, K>(a, d, ldsd, ln);
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, vs_vector_index(n));
    double *blk = ldsd + vs_sp_lds<MODEL, K>(a.L) / sizeof(double);
    VsBlock<K> nxt;
    vs_fetch<K>(a, p, 1, ncp, nxt);
    double dl[K];
    vs_load_d<K>(a, p, 1, dl);
    for (int cb = 1; cb < ncp; cb += 64) {
        const VsBlock<K> cur = nxt;
        vs_stage<K>(cur, blk);
        __syncthreads();
        vs_fetch<K>(a, p, cb + 64, ncp, nxt);
        const int nb = min(ncp - cb, 64);
        const int32_t kc = cur.k;
        const bool tie = kc >= 0 && (kc & kVsTie);
        const int32_t kb = (kc >= 0) ? (kc & ~kVsTie) : kc;
        const double edge = -ldexp(1.0 - 0x1p-40, kb + 1);
        int s = 0; /* the first lane of the run; dl enters its chunk */
        while (s < nb) {
            const bool in = lane >= s && lane < nb;
            double P[K][K];
#pragma unroll
            for (int i = 0; i < K; ++i)
#pragma unroll
                for (int j = 0; j < K; ++j)
                    P[i][j] = in ? cur.m[i][j] : (i == j ? 0.0 : dev_ninf());
#pragma unroll
            for (int dd = 1; dd < 64; dd *= 2) {
                double Q[K][K], R[K][K];
                vs_mp_shfl_up<K>(P, dd, Q);
                vs_mp_mul<K>(Q, P, R);
                if (lane >= dd) {
#pragma unroll
                    for (int i = 0; i < K; ++i)
#pragma unroll
                        for (int j = 0; j < K; ++j)
                            P[i][j] = R[i][j];
                }
            }
            /* candidate entry: dl (x) the product of the run's chunks before this lane's */
            double E[K][K];
            vs_mp_shfl_up<K>(P, 1, E);
            double din[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                double v = dl[0] + E[0][j];
#pragma unroll
                for (int r = 1; r < K; ++r)
                    v = fmax(v, dl[r] + E[r][j]);
                din[j] = (lane == s) ? dl[j] : v;
            }
            /* the lane's own chunk from its candidate, in vs_apply_lds's order */
            double nx[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                double best = din[0] + cur.m[0][j];
#pragma unroll
                for (int r = 1; r < K; ++r)
                    best = fmax(best, din[r] + cur.m[r][j]);
                nx[j] = best;
            }
            const double hi = vs_hi<K>(din);
            bool ok = in && !tie && kc != kVsNoGrid && hi > dev_ninf() && hi != 0.0 && vs_binade(hi) == kb;
#pragma unroll
            for (int k = 0; k < K; ++k)
                ok = ok && (nx[k] == dev_ninf() || nx[k] > edge);
            /* the candidate must be the previous lane's exit, bit for bit */
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const double prev = __shfl_up(nx[k], 1, 64);
                ok = ok && (lane == s || __double_as_longlong(prev) == __double_as_longlong(din[k]));
            }
            const uint64_t bad = __ballot(in && !ok);
            const int f = __builtin_amdgcn_readfirstlane(bad ? __ffsll((unsigned long long)bad) - 1 : nb);
            if (lane >= s && lane < f)
                vs_store_d<K>(a, p, cb + lane + 1, nx);
            /* the exact entry of lane f: the exit of lane f - 1 (or dl) */
            if (f > s) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    dl[k] = __shfl(nx[k], f - 1, 64);
            }
            if (f == nb)
                break;
            vs_exact_chunk<MODEL, K>(a, p, ln, sp, blk, ldsd, f, cb + f, Tp, dl);
            s = f + 1;
        }
        __syncthreads();
    }
}

/* Each chunk again from its exact entry in the reference's arithmetic:
 * back-pointer words (the layout of hhmm_hmm.h's decoders), the backtrack map
 * and the bitwise check of the exit against the scan. */
template <int MODEL, int K>
__global__ void __launch_bounds__(kBlock) vs_replay_kernel(const DevArgs a)
{
    constexpr int KP = (K + 1) / 2;
    constexpr int BITS = bp_bits(K);
    constexpr int STEPB = K * BITS;
    constexpr int SPW = bp_steps_per_word(K);
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    static_assert(kVsChunk % SPW == 0, "V-chunks hold whole back-pointer words");
    HIP_DYNAMIC_SHARED(double2, lds)
    VsLane v;
    if (!vs_lane(a, v) || v.t0 >= v.Tp)
        return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double2 *slab = lds + (size_t)wave * a.L * KP * 64 + lane;
    PairParams<MODEL, K> pp;
    load_params<MODEL, K, true>(pp, a, v.d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        fill_table<K, true>(slab, a, v.d);
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, v.n);
    double dl[K];
    uint32_t word = 0;
    uint32_t org = 0; /* byte j: entry state of the survivor ending in j */
#pragma unroll
    for (int j = 0; j < K; ++j)
        org |= (uint32_t)j << (8 * j);
    auto on_step = [&](int t, const int (&arg)[K]) {
        uint32_t no = 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            word |= (uint32_t)arg[j] << ((t % SPW) * STEPB + j * BITS);
            no |= ((org >> (8 * arg[j])) & 0xffu) << (8 * j);
        }
        org = no;
        if (t % SPW == SPW - 1 || t == v.t1 - 1) {
            put_tmp(a.bp + a.P * (int64_t)(t / SPW), (uint32_t)v.p * 4u, word);
            word = 0;
        }
    };
    if (v.c == 0) {
        vs_chunk0<MODEL, K>(a, pp, slab, sp, v.t1, dl, on_step);
        if (v.t1 == 1) /* T = 1: no step, the lone word of t = 0 */
            put_tmp(a.bp, (uint32_t)v.p * 4u, 0u);
    } else {
        vs_load_d<K>(a, v.p, v.c, dl);
        vs_chunk<MODEL, K>(a, pp, slab, sp, v.t0, v.t1, dl, on_step);
    }
    a.vs_e[v.p + a.P * (int64_t)v.c] = org;
    double want[K];
    vs_load_d<K>(a, v.p, v.c + 1, want);
    bool same = true;
#pragma unroll
    for (int k = 0; k < K; ++k)
        same = same && (__double_as_longlong(want[k]) == __double_as_longlong(dl[k]));
    if (!same)
        a.vs_fail[v.p] = 1;
}

/* Composition of two backtrack maps (byte j: the entry state of the survivor
 * ending in j): (g o h)(j) = g(h(j)). */
__device__ __forceinline__ uint32_t vs_map_compose(uint32_t g, uint32_t h, int K)
{
    uint32_t r = 0;
    for (int j = 0; j < K; ++j)
        r |= ((g >> (8 * ((h >> (8 * j)) & 0xffu))) & 0xffu) << (8 * j);
    return r;
}

/* One wave per pair: logp_zstar, zstar_T and pair_status (viterbi_epilogue's
 * rules), then the path state at the end of every chunk through the backtrack
 * maps, 64 chunks at a time from the top: lane l holds chunk top - l's map, a
 * Hillis-Steele prefix of the compositions over the lanes gives every lane the
 * map from the block's top state to its chunk's end state (round 4; a lane per
 * pair walking 1,954 chunks took 0.42 ms at C5). */
template <int K>
__global__ void __launch_bounds__(64) vs_stitch_kernel(const DevArgs a)
{
    const int64_t p = blockIdx.x;
    const int lane = threadIdx.x & 63;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + kVsChunk - 1) / kVsChunk;
    double dl[K];
    vs_load_d<K>(a, p, ncp, dl);
    const double lp = stan_max_vec<K>(dl);
    int z = -1;
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (dl[j] == lp)
            z = j;
    const bool invalid = (z < 0) || (Tp >= 2 && lp == dev_ninf());
    if (lane == 0) {
        if ((a.outputs & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
            a.logp_zstar[p] = lp;
        if (a.pair_status)
            a.pair_status[p] = invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
    }
    if (!((a.outputs & HHMM_OUT_ZSTAR) && a.zstar))
        return;
    if (invalid)
        z = -1;
    uint32_t ident = 0;
#pragma unroll
    for (int j = 0; j < K; ++j)
        ident |= (uint32_t)j << (8 * j);
    for (int top = ncp - 1; top >= 0; top -= 64) {
        const int cc = top - lane;
        /* lane l: the map of chunk top - l + 1 (the one applied to reach chunk
         * top - l's end state); lane 0: the identity (the block's top state) */
        uint32_t m = (lane > 0 && cc >= 0) ? a.vs_e[p + a.P * (int64_t)(cc + 1)] : ident;
#pragma unroll
        for (int dd = 1; dd < 64; dd *= 2) {
            const uint32_t q = __shfl_up(m, dd, 64);
            const uint32_t r = vs_map_compose(m, q, K);
            m = lane >= dd ? r : m;
        }
        /* m: the map from the top state to chunk cc's end state */
        const int zc = z < 0 ? -1 : (int)((m >> (8 * z)) & 0xffu);
        if (cc >= 0)
            a.vs_z[p + a.P * (int64_t)cc] = zc;
        /* the next block's top state: chunk top - 64's end state */
        const int last = min(top, 63);
        int zn = __shfl(zc, last, 64);
        if (top - 64 >= 0 && zn >= 0)
            zn = (int)((a.vs_e[p + a.P * (int64_t)(top - 63)] >> (8 * zn)) & 0xffu);
        z = zn;
    }
}

/* The path inside each chunk, walked back from the chunk's end state. */
template <int K>
__global__ void __launch_bounds__(kBlock) vs_fill_kernel(const DevArgs a)
{
    constexpr int BITS = bp_bits(K);
    constexpr int STEPB = K * BITS;
    constexpr int SPW = bp_steps_per_word(K);
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    constexpr int G = 8; /* words in flight */
    VsLane v;
    if (!vs_lane(a, v) || v.t0 >= v.Tp)
        return;
    int z = a.vs_z[v.p + a.P * (int64_t)v.c];
    const int w0 = v.t0 / SPW, w1 = (v.t1 - 1) / SPW; /* the chunk's words */
    uint32_t w[G], wn[G];
    const int gl = (w1 - w0) / G;
#pragma unroll
    for (int i = 0; i < G; ++i)
        w[i] = get_tmp(a.bp + a.P * (int64_t)min(w0 + gl * G + i, w1), (uint32_t)v.p * 4u);
    for (int g = gl; g >= 0; --g) {
#pragma unroll
        for (int i = 0; i < G; ++i)
            wn[i] = get_tmp(a.bp + a.P * (int64_t)max(min(w0 + (g - 1) * G + i, w1), w0), (uint32_t)v.p * 4u);
#pragma unroll
        for (int i = G - 1; i >= 0; --i) {
            const int wi = w0 + g * G + i;
            if (wi > w1)
                continue;
#pragma unroll
            for (int s = SPW - 1; s >= 0; --s) {
                const int t = wi * SPW + s;
                if (t < v.t0 || t >= v.t1)
                    continue;
                put_out(a.zstar + a.P * (int64_t)t, (uint32_t)v.p * 4u, z + 1);
                if (z >= 0 && t > 0)
                    z = (int)((w[i] >> (s * STEPB + z * BITS)) & MASK);
            }
        }
#pragma unroll
        for (int i = 0; i < G; ++i)
            w[i] = wn[i];
    }
}

template <int MODEL, int K>
static hhmm_status launch_vscan(const DevArgs &a, hipStream_t st)
{
    constexpr int KP = (K + 1) / 2;
    const size_t slab = ModelTraits<MODEL>::kDiscrete ? (size_t)a.L * KP * 64 * sizeof(double2) : 0;
    if (slab * (kBlock / 64) > kLdsLimit) {
        set_error("emission table K*L = %d*%d does not fit in LDS", a.K, a.L);
        return HHMM_ERR_UNSUPPORTED;
    }
    const int64_t lanes = a.P * a.vs_nc;
    const dim3 gc((unsigned)((lanes + kBlock - 1) / kBlock)), bc(kBlock);
    const dim3 gp((unsigned)((a.P + 63) / 64)), b64(64);
    const size_t lds_c = slab * (kBlock / 64), lds_s = vs_sp_lds<MODEL, K>(a.L) + 64 * kVsRow * sizeof(double);
    hipError_t e = hipMemsetAsync(a.vs_fail, 0, (size_t)a.P * sizeof(int32_t), st);
    if (e == hipSuccess)
        e = hipMemsetAsync(a.vs_tl, 0, sizeof(int32_t), st); /* the tie list's count */
    if (e == hipSuccess) {
        hipLaunchKernelGGL((vs_prod_kernel<MODEL, K, false>), gc, bc, lds_c, st, a);
        if (probe_env("HHMM_PROBE_VS_SCAN0_SERIAL")) /* probe knob: the serial approximate walk */
            hipLaunchKernelGGL((vs_scan0_kernel<MODEL, K, false>), dim3((unsigned)a.P), b64, lds_s, st, a);
        else
            hipLaunchKernelGGL((vs_scan0_kernel<MODEL, K, true>), dim3((unsigned)a.P), b64, lds_s, st, a);
        hipLaunchKernelGGL((vs_prod_kernel<MODEL, K, true>), gc, bc, lds_c, st, a);
        /* the listed tie chunks */
        hipLaunchKernelGGL((vs_prod_tie_kernel<MODEL, K>), dim3(kVsTieBlocks), bc, lds_c, st, a);
        hipLaunchKernelGGL((vs_scan1_kernel<MODEL, K>), dim3((unsigned)a.P), b64, lds_s, st, a);
        hipLaunchKernelGGL((vs_replay_kernel<MODEL, K>), gc, bc, lds_c, st, a);
        hipLaunchKernelGGL((vs_stitch_kernel<K>), dim3((unsigned)a.P), b64, 0, st, a);
        if ((a.outputs & HHMM_OUT_ZSTAR) && a.zstar)
            hipLaunchKernelGGL((vs_fill_kernel<K>), gc, bc, 0, st, a);
        /* pairs whose replay disagreed with the scan: the sequential decoder */
        DevArgs r = a;
        r.vs_redo = a.vs_fail;
        const size_t lds = ((ModelTraits<MODEL>::kDiscrete ? (size_t)a.L : 0) +
                            (ModelTraits<MODEL>::kTayal ? (size_t)3 * K : 0)) * 64 * sizeof(double);
        hipLaunchKernelGGL((viterbi_sp_kernel<MODEL, K>), dim3((unsigned)((4 * a.P + 63) / 64)), dim3(64), lds, st, r);
        e = hipGetLastError();
    }
    if (e == hipSuccess && probe_env("HHMM_PROBE_VS_STATS")) {
        /* probe: chunks the exact scan decoded step by step, and replay failures */
        std::vector<int32_t> k((size_t)a.P * a.vs_nc), f((size_t)a.P);
        e = hipStreamSynchronize(st);
        if (e == hipSuccess)
            e = hipMemcpy(k.data(), a.vs_k, k.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
        if (e == hipSuccess)
            e = hipMemcpy(f.data(), a.vs_fail, f.size() * sizeof(int32_t), hipMemcpyDeviceToHost);
        int64_t seq = 0, fail = 0, worst = 0, first = -1;
        for (int64_t q = 0; q < a.P; ++q) {
            int64_t n = 0;
            for (int c = 1; c < a.vs_nc; ++c)
                if (k[(size_t)q + (size_t)a.P * c] == kVsSeq) {
                    ++n;
                    if (q == 0 && first < 0)
                        first = c;
                }
            seq += n;
            worst = std::max(worst, n);
        }
        for (int32_t v : f)
            fail += v != 0;
        fprintf(stderr,
                "[vscan] pairs %lld chunks/pair %d sequential chunks %lld (%.2f per pair, worst pair %lld) "
                "replay failures %lld; pair 0:",
                (long long)a.P, a.vs_nc, (long long)seq, (double)seq / (double)a.P, (long long)worst, (long long)fail);
        for (int c = 1; c < a.vs_nc; ++c)
            if (k[(size_t)a.P * c] == kVsSeq)
                fprintf(stderr, " %d", c);
        int64_t wq = 0, wn = -1;
        for (int64_t q = 0; q < a.P; ++q) {
            int64_t n = 0;
            for (int c = 1; c < a.vs_nc; ++c)
                n += k[(size_t)q + (size_t)a.P * c] == kVsSeq;
            if (n > wn) {
                wn = n;
                wq = q;
            }
        }
        fprintf(stderr, "; worst pair %lld:", (long long)wq);
        for (int c = 1; c < a.vs_nc; ++c)
            if (k[(size_t)wq + (size_t)a.P * c] == kVsSeq)
                fprintf(stderr, " %d", c);
        int64_t ties = 0;
        for (int32_t v : k)
            ties += v >= 0 && (v & kVsTie);
        fprintf(stderr, "; tie chunks %lld of %lld\n", (long long)ties, (long long)k.size());
    }
    if (e != hipSuccess) {
        set_error("T-parallel Viterbi launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

} // namespace hhmm
