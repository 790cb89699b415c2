/*
 * hhmm_detmath.h -- deterministic exp / log, shared verbatim by the CPU oracle
 * (gcc, oracle/hhmm_oracle.c) and the gfx950 kernels (hipcc).
 *
 * Why: the FFBS draws (the contract of DESIGN.md §5) are
 * compared index-for-index with the oracle, so every transcendental the
 * contract consumes must be the same double on both sides.  It does NOT have
 * to be Stan's (the reference's draws come from Stan's RNG and are not
 * reproducible at all), so instead of the correctly rounded hhmm_cr_exp /
 * hhmm_cr_log (table lookups, a rounding test, a rarely taken accurate phase)
 * the contract uses these: a fixed sequence of IEEE-754 operations -- +, -, *,
 * /, explicit fma, rint, bit moves, one read of a fixed table -- each exactly
 * rounded in round-to-nearest on both sides, so the result is bit-identical
 * wherever it is evaluated.  No branch (selects only), about 20 (exp) / 35
 * (log) instructions.  Accuracy: about one ulp (well inside the 1e-9
 * tolerance of the float outputs computed from them).
 *
 *   hhmm_det_exp (round 5): x = k ln2/128 + r (ln2/128 in two parts, k*HI
 *     exact for |k| < 2^18), |r| <= ln2/256; exp(r) - 1 = r (1 + r/2 + r^2/6 +
 *     r^3/24 + r^4/120) by Horner (truncation < 2^-60); times 2^(j/128) from
 *     the double-double table hhmm_exp2_tab of hhmm_crmath.h (j = k mod 128):
 *     T.hi + fma(T.hi, q, T.lo), within ~0.51 ulp; times 2^(k >> 7) by ldexp
 *     (one rounding, also for subnormal results).  5 fma instead of the
 *     degree-13 Taylor sum over |r| <= ln2/2 of rounds 2-4 (35 %
 *     of C4's VALU).  hhmm_det_exp_tab takes the table's address, so a
 *     kernel can read a copy staged in LDS (a global read on each exp's
 *     dependency chain cost more than the 8 fma it saves: C4 32.0 vs 30.0 ms,
 *     profiles/r05c_ab_c4.log); the entries, and so the results, are the same.
 *   hhmm_det_log: x = 2^e m, m in [sqrt(1/2), sqrt(2)); s = (m - 1) / (m + 1),
 *     log m = 2 s + s^3 (2/3 + 2/5 s^2 + ... + 2/21 s^18) (truncation < 2^-60),
 *     + e ln2 (two parts).
 *
 * The includer defines HHMM_MATH_FN (see hhmm_crmath.h).  Both sides compile
 * with -ffp-contract=off, so no multiply-add is fused behind our back.
 */
#pragma once
#include <stdint.h>

#define HHMM_DET_LN2_HI 0x1.62e42feep-1 /* 32 significant bits */
#define HHMM_DET_LN2_LO 0x1.a39ef35793c76p-33
#define HHMM_DET_SQRT2 0x1.6a09e667f3bcdp+0

HHMM_MATH_FN double hhmm_det_bits(uint64_t u)
{
    union { uint64_t u; double d; } v;
    v.u = u;
    return v.d;
}

HHMM_MATH_FN uint64_t hhmm_det_ubits(double d)
{
    union { uint64_t u; double d; } v;
    v.d = d;
    return v.u;
}

/* 2^k for k in [-1022, 1023]. */
HHMM_MATH_FN double hhmm_det_pow2(int k)
{
    return hhmm_det_bits((uint64_t)(k + 1023) << 52);
}

/* HHMM_DET_K(c): a polynomial coefficient.  The device build defines it as a
 * register-class hint that keeps the double in a scalar register pair, so
 * each Horner step is one fma with a scalar operand instead of two 32-bit
 * literal moves and an fma; the value (and so every result) is unchanged. */
#ifndef HHMM_DET_K
#define HHMM_DET_K(c) (c)
#endif

HHMM_MATH_FN double hhmm_det_exp_tab(double x, const hhmm_exp2_entry *tab)
{
    /* clamp into [-746, 710]: below, exp rounds to 0; above, to +inf -- the
     * clamped argument still gives exactly that (fmax / fmin take a NaN to a
     * bound; NaN is selected at the end) */
    const double xc = __builtin_fmin(__builtin_fmax(x, -746.0), 710.0);
    const double kd = __builtin_rint(xc * HHMM_EXP_INV_L2); /* 128 / ln2 */
    double r = __builtin_fma(-kd, HHMM_EXP_L2_HI, xc);      /* exact: HI has 35 bits, |k| < 2^18 */
    r = __builtin_fma(-kd, HHMM_EXP_L2_MID, r);
    const int k = (int)kd;
    double p = 0x1.1111111111111p-7;                           /* 1/120 */
    p = __builtin_fma(p, r, HHMM_DET_K(0x1.5555555555555p-5)); /* 1/24 */
    p = __builtin_fma(p, r, HHMM_DET_K(0x1.5555555555555p-3)); /* 1/6 */
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    const double q = p * r; /* exp(r) - 1 */
    const hhmm_exp2_entry t = tab[k & 127]; /* 2^(j/128), double-double */
    const double y0 = t.hi + __builtin_fma(t.hi, q, t.lo);
    /* times 2^(k >> 7) (floor division), rounded once: ldexp is exactly
     * RN(y0 2^m) on both sides (v_ldexp_f64; C's ldexp) */
    const double y = __builtin_ldexp(y0, k >> 7);
    return x != x ? x + x : y;
}

HHMM_MATH_FN double hhmm_det_exp(double x)
{
    return hhmm_det_exp_tab(x, hhmm_exp2_tab);
}

HHMM_MATH_FN double hhmm_det_log(double x)
{
    const int sub = x < 0x1p-1022;
    const uint64_t u = hhmm_det_ubits(sub ? x * 0x1p54 : x);
    const double m0 = hhmm_det_bits((u & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL); /* [1, 2) */
    const int hi = m0 > HHMM_DET_SQRT2;
    const double m = hi ? m0 * 0.5 : m0; /* [sqrt(1/2), sqrt(2)), exact */
    const int e = (int)((u >> 52) & 0x7ff) - 1023 - (sub ? 54 : 0) + hi;
    const double s = (m - 1.0) / (m + 1.0); /* m - 1 exact */
    const double s2 = s * s;
    double q = 0x1.8618618618618p-4;
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.af286bca1af28p-4));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.e1e1e1e1e1e1ep-4));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.1111111111111p-3));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.3b13b13b13b14p-3));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.745d1745d1746p-3));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.c71c71c71c71cp-3));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.2492492492492p-2));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.999999999999ap-2));
    q = __builtin_fma(q, s2, HHMM_DET_K(0x1.5555555555555p-1));
    const double lm = __builtin_fma(s * s2, q, 2.0 * s);
    const double E = (double)e;
    const double y = __builtin_fma(E, HHMM_DET_LN2_HI, __builtin_fma(E, HHMM_DET_LN2_LO, lm));
    /* log(+0) = -inf, log(x < 0) = log(NaN) = NaN, log(+inf) = +inf */
    const double special = x == 0.0 ? -__builtin_inf() : (x == __builtin_inf() ? x : hhmm_det_bits(0x7ff8000000000000ULL));
    return (x > 0.0 && x < __builtin_inf()) ? y : special;
}
