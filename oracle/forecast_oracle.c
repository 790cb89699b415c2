/*
 * forecast_oracle.c -- CPU ORACLE for the nearest-neighbour forecast
 * (SURVEY.md §8 F3).  TEST INFRASTRUCTURE ONLY (same rule as hhmm_oracle.c).
 *
 * Restates neighbouring_forecast(x, oblik_t, h, threshold),
 * hassan2005/R/forecast.R:1-31, per draw, in R's semantics:
 *   find_closest (:9-16): which(abs(target - cand) < abs(target) * threshold),
 *     else which(abs(target - cand) == min(abs(target - cand))) -- min() is NA
 *     when any distance is NaN, and then no index matches;
 *   d = abs(target - oblik_t[n, closests]); w = exp(d) (:24-25);
 *   forecast = x[T] + sum((x[closests + h] - x[closests]) * w) / sum(w) (:27),
 *     each sum() accumulated in long double (R's rsum) and rounded once.
 * exp is the host libm's (R's).  Parity with R: unpinned (no R here).
 */
#include <math.h>
#include <stdint.h>

#include "hhmm_forecast.h"

int hhmm_oracle_neighbouring_forecast(const hhmm_forecast_request *r, double *out)
{
    if (!r || !out || r->T <= r->h || r->h < 1)
        return -1;
    const int64_t N = r->n_series, S = r->n_draws, P = N * S;
    const int T = r->T, h = r->h, nc = T - h;
    for (int64_t p = 0; p < P; ++p) {
        const int64_t n = p / S;
        const double tgt = r->oblik_t[p + P * (int64_t)(T - 1)];
        const double thr = fabs(tgt) * r->threshold;
        int cnt = 0, nan_seen = 0;
        double mn = INFINITY;
        for (int c = 0; c < nc; ++c) {
            const double d = fabs(tgt - r->oblik_t[p + P * (int64_t)c]);
            if (d < thr)
                ++cnt;
            if (isnan(d))
                nan_seen = 1;
            else if (d < mn)
                mn = d;
        }
        if (cnt == 0 && nan_seen) {
            out[p] = NAN;
            continue;
        }
        long double num = 0.0L, den = 0.0L;
        for (int c = 0; c < nc; ++c) {
            const double d = fabs(tgt - r->oblik_t[p + P * (int64_t)c]);
            if (cnt > 0 ? (d < thr) : (d == mn)) {
                const double w = exp(d);
                num += (long double)((r->x[n + N * (int64_t)(c + h)] - r->x[n + N * (int64_t)c]) * w);
                den += (long double)w;
            }
        }
        out[p] = r->x[n + N * (int64_t)(T - 1)] + (double)num / (double)den;
    }
    return 0;
}
