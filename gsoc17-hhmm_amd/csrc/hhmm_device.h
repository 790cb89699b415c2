/*
 * hhmm_device.h -- device helpers shared by the gfx950 kernels
 * (hhmm_kernels.hip: HMM / semisup / Tayal; hhmm_iohmm.hip: IOHMM).
 * Not part of the public ABI.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "hhmm_internal.h"

#ifndef HHMM_MATH_FN
#define HHMM_MATH_FN static __device__ __forceinline__
#define HHMM_MATH_COLD static __device__ __attribute__((noinline))
#define HHMM_MATH_TABLE static __constant__
#endif
#include "hhmm_crmath.h"
/* hhmm_detmath.h's coefficients through a scalar-register-class hint (an
 * empty asm: no instruction, value unchanged) */
static __device__ __forceinline__ double hhmm_det_sgpr(double c)
{
    __asm__("" : "+s"(c));
    return c;
}
#define HHMM_DET_K(c) hhmm_det_sgpr(c)
#include "hhmm_detmath.h"

namespace hhmm {

constexpr double kLn2 = 0x1.62e42fefa39efp-1;

/* ------------------------------------------------------------------ */
/* Correctly rounded exp / log for hot loops                            */
/* ------------------------------------------------------------------ */

/* hhmm_cr_exp / hhmm_cr_log as a kernel's inner loop wants them: the quick
 * phase runs on every lane unconditionally (special arguments replaced by a
 * harmless one, the rounding test as selects), and ONE divergent branch sends
 * the lanes whose argument is special or whose rounding test fails (~2^-15 of
 * arguments) to the full function.  The same double as hhmm_cr_exp /
 * hhmm_cr_log for every argument: the full functions take exactly this quick
 * branch when its conditions hold.  Written out as nested branches, the full
 * functions cost ~4 exec-mask regions per call in every loop iteration. */
__device__ __attribute__((noinline)) static double cr_exp_cold(double x) { return hhmm_cr_exp(x); }
__device__ __attribute__((noinline)) static double cr_log_cold(double x) { return hhmm_cr_log(x); }

__device__ __forceinline__ bool cr_round_safe(double v, double w, double err)
{
    const uint64_t b = hhmm_double_to_bits(v);
    const uint64_t eb = b & 0x7ff0000000000000ULL;
    const double hu0 = hhmm_bits_to_double(eb) * 0x1p-53;
    const double hu = (b & 0x000fffffffffffffULL) == 0 ? hu0 * 0.5 : hu0;
    return (eb != 0) & (eb != 0x7ff0000000000000ULL) & (__builtin_fabs(w) + err < hu);
}

/* The quick phases' rounding test on the device: hhmm_round_ziv (one fma and
 * one compare; hhmm_crmath.h states the bound) instead of cr_round_safe's
 * ~10 VALU -- the round tests were 154 static VALU of the C3 sweep. */
__device__ __forceinline__ bool cr_fast_ok(double hi, double lo, double c) { return hhmm_round_ziv(hi, lo, c); }
constexpr double kCrExpC = HHMM_CR_EXP_ZIV;
constexpr double kCrLogC = HHMM_CR_LOG_ZIV;

__device__ __forceinline__ double dev_cr_exp(double x)
{
    const bool in = (x > -707.0) & (x < 693.0); /* NaN: false */
    int e;
    const hhmm_dd f = hhmm_cr_exp_quick_dd(in ? x : 0.0, &e);
    const bool ok = in & cr_fast_ok(f.hi, f.lo, kCrExpC); /* f.hi in [0.99, 2.01): normal */
    double r = f.hi * hhmm_bits_to_double((uint64_t)(e + 1023) << 52);
    if (!ok)
        r = cr_exp_cold(x);
    return r;
}

__device__ __forceinline__ double dev_cr_log(double x)
{
    const bool in = (x >= 0x1p-1022) & (x < __builtin_inf()) & (x != 1.0); /* NaN: false */
    const hhmm_dd f = hhmm_cr_log_quick_dd(in ? x : 2.0);
    const bool ok = in & cr_fast_ok(f.hi, f.lo, kCrLogC); /* x normal, != 1: |f.hi| >= 2^-54, normal */
    double r = f.hi;
    if (!ok)
        r = cr_log_cold(x);
    return r;
}

/* ------------------------------------------------------------------ */
/* Small device helpers                                                  */
/* ------------------------------------------------------------------ */

__device__ __forceinline__ double dev_nan() { return __builtin_nan(""); }
__device__ __forceinline__ double dev_ninf() { return -__builtin_inf(); }

/* max(std::vector<double>) of Stan Math on x86-64 (Eigen SSE2 maxCoeff):
 * identical to stan_max_vec in oracle/hhmm_oracle.c.  NaN-aware order. */
__device__ __forceinline__ double sse_max(double a, double b) { return a > b ? a : b; }
__device__ __forceinline__ double std_max(double a, double b) { return a < b ? b : a; }
template <int K>
__device__ __forceinline__ double stan_max_vec(const double (&d)[K])
{
    if constexpr (K < 2) {
        return d[0];
    } else {
        constexpr int aligned = K & ~1, aligned2 = K & ~3;
        double r0a = d[0], r0b = d[1];
        if constexpr (aligned > 2) {
            double r1a = d[2], r1b = d[3];
#pragma unroll
            for (int i = 4; i < aligned2; i += 4) {
                r0a = sse_max(r0a, d[i]);
                r0b = sse_max(r0b, d[i + 1]);
                r1a = sse_max(r1a, d[i + 2]);
                r1b = sse_max(r1b, d[i + 3]);
            }
            r0a = sse_max(r0a, r1a);
            r0b = sse_max(r0b, r1b);
            if constexpr (aligned > aligned2) {
                r0a = sse_max(r0a, d[aligned2]);
                r0b = sse_max(r0b, d[aligned2 + 1]);
            }
        }
        double res = sse_max(r0a, r0b);
#pragma unroll
        for (int i = aligned; i < K; ++i)
            res = std_max(res, d[i]);
        return res;
    }
}

/* Lane-quad exchanges (DPP quad_perm) of the state-parallel decoders. */
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}

/* v of lane ^ 16 through the gfx950 half-exchange v_permlane16_swap (both
 * operands v: the first result holds the lower 16-lane row of each pair of
 * rows in both rows, the second the upper) -- VALU moves instead of a
 * ds_swizzle round trip through the LDS crossbar. */
__device__ __forceinline__ double lane_xor16(double v)
{
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const bool up = (threadIdx.x & 16) != 0;
    const int l = up ? lo[0] : lo[1];
    const int h = up ? hi[0] : hi[1];
    return __longlong_as_double((long long)(((unsigned long long)(unsigned)h << 32) | (unsigned)l));
}
/* d[i] = v of lane i of this lane's quad. */
template <int K>
__device__ __forceinline__ void quad_gather(double v, double (&d)[K])
{
    d[0] = dpp_f64<0x00>(v);
    if constexpr (K > 1)
        d[1] = dpp_f64<0x55>(v);
    if constexpr (K > 2)
        d[2] = dpp_f64<0xAA>(v);
    if constexpr (K > 3)
        d[3] = dpp_f64<0xFF>(v);
}

/* OR of w over this lane's quad. */
__device__ __forceinline__ uint32_t quad_or(uint32_t w)
{
    w |= (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0xB1, 0xF, 0xF, false); /* quad_perm(1,0,3,2) */
    w |= (uint32_t)__builtin_amdgcn_mov_dpp((int)w, 0x4E, 0xF, 0xF, false); /* quad_perm(2,3,0,1) */
    return w;
}

/* Element of a row addressed as (uniform row pointer) + (32-bit lane byte
 * offset): lets hipcc emit SGPR-base + VGPR-offset global memory ops. */
template <typename T>
__device__ __forceinline__ T &at(T *row, uint32_t byte_off)
{
    return *reinterpret_cast<T *>(reinterpret_cast<char *>(row) + byte_off);
}
template <typename T>
__device__ __forceinline__ const T &at(const T *row, uint32_t byte_off)
{
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(row) + byte_off);
}

/* Store of a write-once output element (gamma, zstar): no kernel re-reads it,
 * so it is a nontemporal (streaming) store -- 3 % off both the forward-backward
 * and the Viterbi at C2 (tools/ab_bench.py, one box, interleaved). */
template <typename T>
__device__ __forceinline__ void put_out(T *row, uint32_t byte_off, T v)
{
    __builtin_nontemporal_store(v, reinterpret_cast<T *>(reinterpret_cast<char *>(row) + byte_off));
}

/* Scratch written by one sweep and read back once by the next (alpha
 * checkpoints, Viterbi back-pointer words): plain stores and loads.  Streaming
 * hints on both sides cost the forward-backward 6.5 % at C2 (7.97 against 7.48
 * ms: the checkpoints are re-read out of the caches) and left the Viterbi
 * unchanged. */
template <typename T>
__device__ __forceinline__ void put_tmp(T *row, uint32_t byte_off, T v)
{
    at(row, byte_off) = v;
}
template <typename T>
__device__ __forceinline__ T get_tmp(const T *row, uint32_t byte_off)
{
    return at(row, byte_off);
}

/* Power-of-two renormalisation of a K-vector after every step: the largest
 * entry is brought into [0.5, 1) by an exact ldexp and the removed exponent
 * is accumulated in `ex`.  Keeping the max near 1 (rather than letting it
 * drift) keeps every component down to 1e-300 of the max a NORMAL double, so
 * posteriors down to the 1e-250 tolerance floor keep full precision.
 * mx == 0 / inf / NaN: frexp_exp returns 0 and v is unchanged. */
template <int K>
__device__ __forceinline__ void renorm(double (&v)[K], int &ex)
{
    double mx = v[0];
#pragma unroll
    for (int k = 1; k < K; ++k)
        mx = fmax(mx, v[k]);
    const int e = __builtin_amdgcn_frexp_exp(mx);
#pragma unroll
    for (int k = 0; k < K; ++k)
        v[k] = ldexp(v[k], -e);
    ex += e;
}

/* Wave-wide min / max, returned through readfirstlane so that hipcc knows
 * the result is uniform: every time index derived from it (row pointers of
 * the per-step loads and stores) is then computed on the scalar unit. */
__device__ __forceinline__ int wave_min(int v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v = min(v, __shfl_xor(v, off));
    return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v = max(v, __shfl_xor(v, off));
    return __builtin_amdgcn_readfirstlane(v);
}

/* XCD-aware workgroup order (cdna_hip_programming.md T1; speed only, never
 * correctness): workgroups are dealt round-robin over the 8 XCDs, so blocks b
 * and b + 8 share an L2.  This bijection gives each XCD a contiguous range of
 * logical blocks, so neighbouring pairs -- whose 8-byte output stores share
 * 128-byte lines when a group of lanes owns a pair -- are written through one
 * L2 and leave it as whole lines. */
__device__ __forceinline__ int64_t xcd_block()
{
    const int64_t nb = gridDim.x, b = blockIdx.x;
    const int64_t x = b & 7, q = nb >> 3, r = nb & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

__device__ __forceinline__ void pair_coords(const DevArgs &a, int64_t p, int64_t &n, int64_t &d)
{
    if (a.pairing == HHMM_PAIR_ZIP) {
        n = p;
        d = p;
    } else if (a.pairing == HHMM_PAIR_BLOCK) { /* series n's own block of S / N draws */
        n = p / (a.S / a.N);
        d = p;
    } else {
        n = p / a.S;
        d = p - n * a.S;
    }
}

__device__ __forceinline__ int pair_len(const DevArgs &a, int64_t n)
{
    int Tp = a.T ? a.T[n] : a.Tmax;
    return min(max(Tp, 1), a.Tmax);
}

/* out[p, t, k] for k = 0..K-1: uniform row pointer out + P*(t + Tout*k)
 * (SGPR base) plus the lane's 32-bit pair index (P < 2^29 per launch). */
template <int K>
__device__ __forceinline__ void store_tk(double *out, const DevArgs &a, int64_t p, int t, const double (&v)[K])
{
#pragma unroll
    for (int k = 0; k < K; ++k)
        put_out(out + a.P * ((int64_t)t + (int64_t)a.Tout * k), (uint32_t)p * 8u, v[k]);
}

/* 1/x to ~1 ulp: v_rcp_f64 + two Newton steps (tolerance 1e-9 outputs only);
 * IEEE division for x below 2^-1000 where the reciprocal would overflow. */
__device__ __forceinline__ double fast_rcp(double x)
{
    if (__builtin_expect(!(x > 0x1p-1000), 0))
        return 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    r = fma(fma(-x, r, 1.0), r, r);
    return r;
}

template <int K>
__device__ __forceinline__ double vsum(const double (&v)[K])
{
    double s = v[0];
#pragma unroll
    for (int k = 1; k < K; ++k)
        s += v[k];
    return s;
}

/* cat(w, u): Stan's categorical_rng(w / sum(w)) with the caller's uniform u
 * (Stan Math: cumulative_sum of theta, `while (c > cum[b]) b++`), bounded to
 * K - 1, with the comparison scaled by the sum instead of dividing every
 * weight: us = u * sum against the running sum of w.  Returns the 0-based
 * state, or -1 when sum(w) is not a positive finite number.  FFBS contract,
 * DESIGN.md §5 (oracle ffbs_cat). */
template <int K>
__device__ __forceinline__ int ffbs_cat(const double (&w)[K], double u)
{
    double sum = w[0];
#pragma unroll
    for (int i = 1; i < K; ++i)
        sum = sum + w[i];
    const double us = u * sum;
    int b = 0;
    double cum = w[0];
#pragma unroll
    for (int i = 1; i < K; ++i) {
        const bool step = (b == i - 1) & (us > cum);
        b = step ? i : b;
        cum = step ? cum + w[i] : cum;
    }
    return ((sum > 0.0) & __builtin_isfinite(sum)) ? b : -1;
}

/* Viterbi chunk length: a multiple of the back-pointer steps per word so
 * that every word boundary falls on a static unrolled slot. */
constexpr int vit_chunk(int K)
{
    return bp_steps_per_word(K) >= 8 ? bp_steps_per_word(K)
                                      : (8 % bp_steps_per_word(K) == 0 ? 8 : 2 * bp_steps_per_word(K));
}

/* Backtrack over chunk c (descending): zb[u] = zstar[t0 + u] (1-based) for
 * the chunk's steps inside the series, stepping z; the stores are issued
 * later (vit_back_flush), after the next chunk's word loads, so that waiting
 * for those loads never waits for stores as well (vmcnt counts both on gfx9). */
template <int K, int CV, bool FULLC>
__device__ __forceinline__ void vit_back_chunk(int Tp, int c, const uint32_t (&w)[CV / bp_steps_per_word(K)],
                                               int &z, int (&zb)[CV])
{
    constexpr int BITS = bp_bits(K);
    constexpr int SPW = bp_steps_per_word(K);
    constexpr int STEPB = K * BITS;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    const int t0 = c * CV;
#pragma unroll
    for (int u = CV - 1; u >= 0; --u) {
        const int t = t0 + u;
        if (FULLC || t < Tp) {
            zb[u] = z + 1;
            if (t > 0)
                z = (int)((w[u / SPW] >> ((u % SPW) * STEPB + z * BITS)) & MASK);
        }
    }
}

/* Stores chunk c's zstar values.  QUAD (one lane quad per pair, all four
 * holding the same zb): lane j of the quad stores steps u = j, j+4, ... so a
 * chunk takes CV/4 store instructions instead of CV. */
template <int CV, bool QUAD>
__device__ __forceinline__ void vit_back_flush(const DevArgs &a, int64_t p, int Tp, int c, const int (&zb)[CV])
{
    const int t0 = c * CV;
    if constexpr (QUAD) {
        static_assert(CV % 4 == 0, "quad flush needs whole quads of steps");
        const int j = (int)(threadIdx.x & 3);
#pragma unroll
        for (int m = 0; m < CV / 4; ++m) {
            /* masked OR, not a select chain: LLVM folds selects of array
             * elements into a dynamically indexed load, i.e. scratch */
            const int v = (zb[4 * m] & -(int)(j == 0)) | (zb[4 * m + 1] & -(int)(j == 1)) |
                          (zb[4 * m + 2] & -(int)(j == 2)) | (zb[4 * m + 3] & -(int)(j == 3));
            const int t = t0 + 4 * m + j;
            if (t < Tp)
                put_out(a.zstar + a.P * (int64_t)t, (uint32_t)p * 4u, v);
        }
    } else {
#pragma unroll
        for (int u = 0; u < CV; ++u) {
            const int t = t0 + u;
            if (t < Tp)
                put_out(a.zstar + a.P * (int64_t)t, (uint32_t)p * 4u, zb[u]);
        }
    }
}

/* Viterbi epilogue shared by every Viterbi pass: flushes the partial last
 * back-pointer word, logp_zstar = max(delta_T) with Eigen's SSE2 maxCoeff NaN
 * rule, zstar_T = the LAST j attaining it (e.g. hmm/stan/hmm.stan:120-124),
 * pair_status, then the backtrack chunk by chunk with the words prefetched a
 * group of chunks ahead (hmm.stan:126-128).  QUAD: the state-parallel decoder's lane
 * quads (every lane of a quad holds the same delta_T and word). */
template <int K, bool QUAD = false>
__device__ __forceinline__ void viterbi_epilogue(const DevArgs &a, int64_t p, int Tp, int Tw_min, int Tw_max,
                                                 const double (&dl)[K], uint32_t word)
{
    constexpr int SPW = bp_steps_per_word(K);
    constexpr int CV = QUAD ? 2 * vit_chunk(K) : vit_chunk(K);
    constexpr int WPC = CV / SPW; /* words per chunk */
    const int nfull = Tw_min / CV;
    const int nchunk = (Tw_max + CV - 1) / CV;
    if ((Tp - 1) % SPW != SPW - 1) /* partial last word */
        put_tmp(a.bp + a.P * (int64_t)((Tp - 1) / SPW), (uint32_t)p * 4u, word);

    /* logp_zstar = max(delta_tk[T]); zstar[T] = LAST j attaining it (hmm.stan:120-124). */
    const double lp = stan_max_vec<K>(dl);
    int z = -1;
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (dl[j] == lp)
            z = j;
    /* Backtracking reads an unset back-pointer exactly when zstar[T] is unset
     * (NaN row at T = 1) or every delta_T is -inf. */
    const bool invalid = (z < 0) || (Tp >= 2 && lp == dev_ninf());
    if ((a.outputs & HHMM_OUT_LOGP_ZSTAR) && a.logp_zstar)
        a.logp_zstar[p] = lp;
    if (a.pair_status)
        a.pair_status[p] = invalid ? HHMM_PAIR_INVALID_BACKPOINTER : HHMM_PAIR_OK;
    if (!((a.outputs & HHMM_OUT_ZSTAR) && a.zstar))
        return;
    if (invalid) {
        for (int t = 0; t < Tp; ++t)
            a.zstar[p + a.P * (int64_t)t] = 0;
        return;
    }
    /* backtrack, chunk by chunk; word rows are wave-uniform, clamped to the
     * allocation (a short lane's extra rows are never consumed) */
    const int wmax = a.Tmax / SPW;
    int zb[CV];
    const int clast = nchunk - 1;
    {
        /* The words come in groups of G chunks, the next group prefetched
         * while this one runs: one chunk of backtrack (CV steps of dependent
         * shifts) is far shorter than an HBM round trip, so a one-chunk
         * prefetch leaves the wave waiting on every chunk (C5: one wave per
         * SIMD and nothing else to hide it; C2: the lane decoder's backtrack
         * phase, T/CV round trips per pair). */
        constexpr int G = 8;
        uint32_t w[G * WPC], wn[G * WPC];
        const int glast = clast / G;
#pragma unroll
        for (int i = 0; i < G * WPC; ++i)
            w[i] = get_tmp(a.bp + a.P * (int64_t)min(max(glast * G * WPC + i, 0), wmax), (uint32_t)p * 4u);
        for (int g = glast; g >= 0; --g) {
#pragma unroll
            for (int i = 0; i < G * WPC; ++i)
                wn[i] = get_tmp(a.bp + a.P * (int64_t)min(max((g - 1) * G * WPC + i, 0), wmax), (uint32_t)p * 4u);
#pragma unroll
            for (int cc = G - 1; cc >= 0; --cc) {
                const int c = g * G + cc;
                if (c > clast)
                    continue;
                if (c < clast)
                    vit_back_flush<CV, QUAD>(a, p, Tp, c + 1, zb);
                uint32_t wc[WPC];
#pragma unroll
                for (int i = 0; i < WPC; ++i)
                    wc[i] = w[cc * WPC + i];
                if (c < nfull)
                    vit_back_chunk<K, CV, true>(Tp, c, wc, z, zb);
                else
                    vit_back_chunk<K, CV, false>(Tp, c, wc, z, zb);
            }
#pragma unroll
            for (int i = 0; i < G * WPC; ++i)
                w[i] = wn[i];
        }
        if (clast >= 0)
            vit_back_flush<CV, QUAD>(a, p, Tp, 0, zb);
    }
}

} // namespace hhmm
