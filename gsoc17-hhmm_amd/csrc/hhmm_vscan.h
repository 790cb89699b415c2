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
 *   vs_scan0 (lane/pair) chunk 0 exactly (the model's t = 1 row, Q3 NaN step),
 *                        then the approximate scan: the binade k_c expected at
 *                        each chunk's entry
 *   vs_prod<GRID=true>   exact grid products on k_c's grid, tie flags
 *   vs_scan1 (wave/pair) the exact scan: delta_c (x) M_c where the checks hold
 *                        (entry max in binade k_c, no tie, every finite exit
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

namespace hhmm {

constexpr int32_t kVsTie = 1 << 30;     /* vs_k: a grid rounding tie inside the chunk */
constexpr int32_t kVsNoGrid = -(1 << 20); /* vs_k: no finite magnitude estimate */

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

/* Candidate of (i -> j) relative to delta_{t-1}(i), the model's two terms. */
template <int MODEL>
__device__ __forceinline__ double vs_rel(double la, double le, bool on)
{
    if constexpr (ModelTraits<MODEL>::kTayal)
        return on ? le + la : le; /* (delta + log phi) [+ log A] (hhmm-tayal2009.stan:143-146) */
    else
        return la + le; /* (delta + log A) + emission (hmm.stan:111) */
}

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
    if constexpr (GRID) {
#pragma unroll
        for (int i = 0; i < K; ++i)
#pragma unroll
            for (int j = 0; j < K; ++j)
                pp.A[i][j] = vs_grid(pp.A[i][j], iu, u, tie);
    }
    double M[K][K];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[r][j] = (r == j) ? 0.0 : dev_ninf();
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, v.n);
    vs_steps<MODEL, VAUX>(sp, v.t0, v.t1, [&](int, const Obs &o) {
        double le[K];
        emit_log<MODEL, K>(pp, slab, a.L, o, le);
        bool on[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            if constexpr (GRID)
                le[j] = vs_grid(le[j], iu, u, tie);
            on[j] = true;
            if constexpr (ModelTraits<MODEL>::kTayal)
                on[j] = tayal_pred(o.aux, j);
        }
#pragma unroll
        for (int r = 0; r < K; ++r) {
            double nm[K];
#pragma unroll
            for (int j = 0; j < K; ++j) {
                double best = M[r][0] + vs_rel<MODEL>(pp.A[0][j], le[j], on[j]);
#pragma unroll
                for (int i = 1; i < K; ++i)
                    best = fmax(best, M[r][i] + vs_rel<MODEL>(pp.A[i][j], le[j], on[j]));
                nm[j] = best;
            }
#pragma unroll
            for (int j = 0; j < K; ++j)
                M[r][j] = nm[j];
        }
    });
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            a.vs_m[v.p + a.P * ((int64_t)v.c * K * K + r * K + j)] = M[r][j];
    if (GRID && tie)
        a.vs_k[v.p + a.P * (int64_t)v.c] = kc | kVsTie;
}

/* delta (x) M for chunk c (rows of vs_m). */
template <int K>
__device__ __forceinline__ void vs_apply(const DevArgs &a, int64_t p, int c, const double (&D)[K], double (&out)[K])
{
    double M[K][K];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
        for (int j = 0; j < K; ++j)
            M[r][j] = a.vs_m[p + a.P * ((int64_t)c * K * K + r * K + j)];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        double best = D[0] + M[0][j];
#pragma unroll
        for (int r = 1; r < K; ++r)
            best = fmax(best, D[r] + M[r][j]);
        out[j] = best;
    }
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
template <int MODEL, int K, bool NANIN>
__device__ __forceinline__ void vs_step(double (&dl)[K], const PairParams<MODEL, K> &pp, const double (&le)[K],
                                        const Obs &o, int (&arg)[K])
{
    double nd[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        bool on = true;
        if constexpr (ModelTraits<MODEL>::kTayal)
            on = tayal_pred(o.aux, j);
        double best = dev_ninf();
        int am = 0;
#pragma unroll
        for (int i = 0; i < K; ++i) {
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

/* lane = pair: chunk 0 exactly (row 1 of vs_d), then the approximate scan
 * over the approximate chunk products: k_c = binade of the largest finite
 * delta entering chunk c. */
template <int MODEL, int K>
__global__ void __launch_bounds__(64) vs_scan0_kernel(const DevArgs a)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    HIP_DYNAMIC_SHARED(double2, lds)
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= a.P)
        return;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + kVsChunk - 1) / kVsChunk;
    double2 *slab = lds + threadIdx.x;
    PairParams<MODEL, K> pp;
    load_params<MODEL, K, true>(pp, a, d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        fill_table<K, true>(slab, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, n);
    double dl[K];
    vs_chunk0<MODEL, K>(a, pp, slab, sp, min(kVsChunk, Tp), dl, [](int, const int (&)[K]) {});
    vs_store_d<K>(a, p, 1, dl);
    for (int c = 1; c < ncp; ++c) {
        const double hi = vs_hi<K>(dl);
        a.vs_k[p + a.P * (int64_t)c] = (hi > dev_ninf() && hi != 0.0) ? vs_binade(hi) : kVsNoGrid;
        double nx[K];
        vs_apply<K>(a, p, c, dl, nx);
#pragma unroll
        for (int k = 0; k < K; ++k)
            dl[k] = nx[k];
    }
}

/* One wave per pair (lane 0 works): the exact scan over the grid products,
 * chunks failing the checks decoded step by step.  Rows 2..ncp of vs_d. */
template <int MODEL, int K>
__global__ void __launch_bounds__(64) vs_scan1_kernel(const DevArgs a)
{
    constexpr bool VAUX = ModelTraits<MODEL>::kTayal;
    HIP_DYNAMIC_SHARED(double2, lds)
    if (threadIdx.x != 0)
        return;
    const int64_t p = blockIdx.x;
    int64_t n, d;
    pair_coords(a, p, n, d);
    const int Tp = pair_len(a, n);
    const int ncp = (Tp + kVsChunk - 1) / kVsChunk;
    if (ncp < 2)
        return;
    double2 *slab = lds;
    PairParams<MODEL, K> pp;
    load_params<MODEL, K, true>(pp, a, d);
    if constexpr (ModelTraits<MODEL>::kDiscrete)
        fill_table<K, true>(slab, a, d);
    const SeriesPtrs sp = series_ptrs<MODEL, VAUX>(a, n);
    double dl[K];
    vs_load_d<K>(a, p, 1, dl);
    for (int c = 1; c < ncp; ++c) {
        const int32_t kc = a.vs_k[p + a.P * (int64_t)c];
        const double hi = vs_hi<K>(dl);
        bool ok = kc != kVsNoGrid && !(kc & kVsTie) && hi > dev_ninf() && hi != 0.0 && vs_binade(hi) == kc;
        double nx[K];
        if (ok) {
            vs_apply<K>(a, p, c, dl, nx);
            /* every finite exit value inside the binade, 2^-40 of its width clear of the edge */
            const double edge = -ldexp(1.0 - 0x1p-40, kc + 1);
#pragma unroll
            for (int k = 0; k < K; ++k)
                ok = ok && (nx[k] == dev_ninf() || nx[k] > edge);
        }
        if (ok) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                dl[k] = nx[k];
        } else {
            const int t0 = c * kVsChunk;
            vs_chunk<MODEL, K>(a, pp, slab, sp, t0, min(t0 + kVsChunk, Tp), dl, [](int, const int (&)[K]) {});
        }
        vs_store_d<K>(a, p, c + 1, dl);
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

/* lane = pair: logp_zstar, zstar_T and pair_status (viterbi_epilogue's rules),
 * then the path state at the end of every chunk through the backtrack maps. */
template <int K>
__global__ void __launch_bounds__(64) vs_stitch_kernel(const DevArgs a)
{
    const int64_t p = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (p >= a.P)
        return;
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
    if ((a.outputs & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
        a.logp_zstar[p] = lp;
    if (a.pair_status)
        a.pair_status[p] = invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
    if (!((a.outputs & HHMM_OUT_ZSTAR) && a.zstar))
        return;
    if (invalid)
        z = -1;
    /* maps prefetched G chunks at a time: the walk itself is a byte extract per chunk */
    constexpr int G = 16;
    uint32_t e[G], en[G];
    int c = ncp - 1;
    const int gl = c / G;
#pragma unroll
    for (int i = 0; i < G; ++i)
        e[i] = a.vs_e[p + a.P * (int64_t)min(gl * G + i, ncp - 1)];
    for (int g = gl; g >= 0; --g) {
#pragma unroll
        for (int i = 0; i < G; ++i)
            en[i] = a.vs_e[p + a.P * (int64_t)max(min((g - 1) * G + i, ncp - 1), 0)];
#pragma unroll
        for (int i = G - 1; i >= 0; --i) {
            const int cc = g * G + i;
            if (cc <= c) {
                a.vs_z[p + a.P * (int64_t)cc] = z;
                if (z >= 0)
                    z = (int)((e[i] >> (8 * z)) & 0xffu);
            }
        }
#pragma unroll
        for (int i = 0; i < G; ++i)
            e[i] = en[i];
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
    const size_t lds_c = slab * (kBlock / 64), lds_p = slab;
    hipError_t e = hipMemsetAsync(a.vs_fail, 0, (size_t)a.P * sizeof(int32_t), st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL((vs_prod_kernel<MODEL, K, false>), gc, bc, lds_c, st, a);
        hipLaunchKernelGGL((vs_scan0_kernel<MODEL, K>), gp, b64, lds_p, st, a);
        hipLaunchKernelGGL((vs_prod_kernel<MODEL, K, true>), gc, bc, lds_c, st, a);
        hipLaunchKernelGGL((vs_scan1_kernel<MODEL, K>), dim3((unsigned)a.P), b64, lds_p, st, a);
        hipLaunchKernelGGL((vs_replay_kernel<MODEL, K>), gc, bc, lds_c, st, a);
        hipLaunchKernelGGL((vs_stitch_kernel<K>), gp, b64, 0, st, a);
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
    if (e != hipSuccess) {
        set_error("T-parallel Viterbi launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

} // namespace hhmm
