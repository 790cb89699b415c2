/*
 * features_oracle.c -- CPU ORACLE for the tick -> zig-zag -> leg feature
 * extractor.
 *
 * TEST INFRASTRUCTURE ONLY (same rule as hhmm_oracle.c): only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.  The
 * product path is hhmm_features.hip in libhhmm.so.
 *
 * A sequential restatement of `extract_features(tdata, alpha)`,
 * tayal2009/R/feature-extraction.R:8-133, with R's semantics spelled out:
 *   * lag() on an xts shifts by one row (first row NA); ifelse(NA) is NA;
 *   * `x[cond] <- v` with a logical cond assigns only where cond is TRUE
 *     (an NA in cond leaves the element unchanged);
 *   * difftime(t1, t0) picks its units from |t1 - t0| (< 60 s: secs, < 3600:
 *     mins, < 86400: hours, else days) and divides; as.numeric(units="secs")
 *     multiplies back (R base `difftime` / `units<-.difftime`);
 *   * sum() of doubles accumulates in long double (R's rsum); the result is
 *     rounded to double once.
 * Constants from tayal2009/R/constants.R:2-14 (up = 1, lt = 0, dn = -1;
 * extrema max = 1, min = -1).
 *
 * Parity status: unpinned against R outputs (R is absent here and on the GPU
 * box; the reference stores no extracted features).  Pinned by an
 * independent pure-Python transcription (tests/test_features.py) and by
 * hand-built known-answer tick series.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "hhmm_features.h"

/* ifelse(ratio - 1 > alpha, 1, ifelse(1 - ratio > alpha, -1, 0)); NA -> 2
 * (feature-extraction.R:77-79).  A ratio is NA when a lag is missing or
 * it is NaN (0 / 0). */
#define NA_CODE 2
static int discretize(double ratio, int avail, double alpha)
{
    if (!avail || isnan(ratio))
        return NA_CODE;
    if (ratio - 1 > alpha)
        return 1;
    if (1 - ratio > alpha)
        return -1;
    return 0;
}

/* as.numeric(difftime(t1, t0), units = "secs") */
static double difftime_secs(double t1, double t0)
{
    const double z = t1 - t0;
    const double az = fabs(z);
    double f = 1.0;
    if (!isfinite(az) || az < 60)
        f = 1.0;
    else if (az < 3600)
        f = 60.0;
    else if (az < 86400)
        f = 3600.0;
    else
        f = 86400.0;
    return (z / f) * (f / 1.0);
}

/* legs table, feature-extraction.R:92-110: (f0, f1, f2) -> code. */
static int leg_code(int f0, int f1, int f2)
{
    static const int legs[18][4] = {
        {1, 1, 1, 1},    {1, -1, 1, 2},   {1, 1, 0, 3},    {1, 0, 1, 4},    {1, 0, 0, 5},   {1, 0, -1, 6},
        {1, -1, 0, 7},   {1, 1, -1, 8},   {1, -1, -1, 9},  {-1, 1, -1, 10}, {-1, -1, -1, 11}, {-1, 1, 0, 12},
        {-1, 0, -1, 13}, {-1, 0, 0, 14},  {-1, 0, 1, 15},  {-1, -1, 0, 16}, {-1, 1, 1, 17},  {-1, -1, 1, 18}};
    for (int i = 0; i < 18; ++i) /* find_leg (:113-121) */
        if (legs[i][0] == f0 && legs[i][1] == f1 && legs[i][2] == f2)
            return legs[i][3];
    return 0; /* "Not a valid leg" (unreachable: every combination is listed) */
}

/* Returns 0 on success, -1 on bad input / fewer than 2 legs, 1 when the
 * capacity is too small (legs->n_legs = rows needed). */
int hhmm_oracle_extract_features(const hhmm_ticks *tk, hhmm_legs *lg)
{
    const int64_t n = tk->n;
    if (n < 3 || !tk->price || !tk->size || !tk->time)
        return -1;
    const double *price = tk->price;
    /* 3. zig-zag (:20-24, :26-27): direction and its change points */
    int8_t *dir = malloc((size_t)n);
    int64_t *chg = malloc(sizeof(int64_t) * (size_t)n); /* 1-based tick indices */
    int64_t m = 0;
    dir[0] = 0;
    for (int64_t t = 1; t < n; ++t)
        dir[t] = price[t] > price[t - 1] ? 1 : (price[t] < price[t - 1] ? -1 : 0);
    for (int64_t t = 1; t < n; ++t)
        if (dir[t] != 0 && dir[t] != dir[t - 1])
            chg[m++] = t + 1;
    free(dir);
    lg->n_legs = m;
    if (m < 2) {
        free(chg);
        return -1;
    }
    if (m > lg->capacity) {
        free(chg);
        return 1;
    }
    double *lp = malloc(sizeof(double) * (size_t)m), *sav = malloc(sizeof(double) * (size_t)m);
    for (int64_t r = 0; r < m; ++r) {
        /* zigzag <- price[which(direction.chg) - 1, ] (:30) */
        lp[r] = price[chg[r] - 2];
        /* start <- c(1, head(chg, -1)); end <- lag(start, -1) - 1; end[m] <- n (:33-36) */
        const int64_t s = (r == 0) ? 1 : chg[r - 1];
        const int64_t e = (r == m - 1) ? n : chg[r] - 1;
        /* size.av (:41-47): sum(size[s:e]) / (secs(index[e] - index[s]) + 1) */
        long double acc = 0.0L;
        for (int64_t i = s - 1; i < e; ++i)
            acc += (long double)tk->size[i];
        sav[r] = (double)acc / (difftime_secs(tk->time[e - 1], tk->time[s - 1]) + 1);
        if (lg->price) lg->price[r] = lp[r];
        if (lg->start) lg->start[r] = (int32_t)s;
        if (lg->end) lg->end[r] = (int32_t)e;
        if (lg->size_av) lg->size_av[r] = sav[r];
    }
    for (int64_t r = 0; r < m; ++r) {
        /* 4. f0 (:50-51) */
        int f0;
        if (r == 0)
            f0 = (lp[0] < lp[1]) ? -1 : 1; /* f0[1] <- if (f0[2] == max) min else max */
        else
            f0 = (lp[r - 1] < lp[r]) ? 1 : -1;
        /* 5. f1 (:55-70) */
        int f1 = 0;
        if (r >= 4) {
            const double *e = &lp[r - 4];
            if (e[0] < e[2] && e[2] < e[4] && e[1] < e[3])
                f1 = 1;
            else if (e[0] > e[2] && e[2] > e[4] && e[1] > e[3])
                f1 = -1;
        }
        /* 6. f2 (:73-89) */
        int f2 = 0;
        if (r >= 2) {
            const int s1 = discretize(sav[r] / sav[r - 1], 1, tk->alpha);
            const int s2 = discretize(sav[r] / sav[r - 2], 1, tk->alpha);
            const int s3 = discretize(sav[r - 1] / sav[r - 2], 1, tk->alpha);
            const int ok = s1 != NA_CODE && s2 != NA_CODE && s3 != NA_CODE;
            if (ok && s1 == 1 && s2 > -1 && s3 < 1)
                f2 = 1;
            if (ok && s1 == -1 && s2 < 1 && s3 > -1)
                f2 = -1;
        }
        /* 7. feature (:123-125), 8. trend (:128-130) */
        const int code = leg_code(f0, f1, f2);
        int trend = 1;
        if ((code >= 6 && code <= 9) || (code >= 15 && code <= 18))
            trend = -1;
        else if (code == 5 || code == 14)
            trend = 0;
        if (lg->f0) lg->f0[r] = f0;
        if (lg->f1) lg->f1[r] = f1;
        if (lg->f2) lg->f2[r] = f2;
        if (lg->feature) lg->feature[r] = code;
        if (lg->trend) lg->trend[r] = trend;
        /* tayal2009/main.R:85-89 */
        if (lg->sign) lg->sign[r] = code < 10 ? 1 : 2;
        if (lg->x) lg->x[r] = code < 10 ? code : code - 9;
    }
    free(lp);
    free(sav);
    free(chg);
    return 0;
}
