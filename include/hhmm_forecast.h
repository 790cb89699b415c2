/*
 * hhmm_forecast.h -- C ABI of the nearest-neighbour forecast over the
 * one-step observation likelihood oblik_t, part of
 * libhhmm.so.
 *
 * Replaces the reference's
 *     neighbouring_forecast(x, oblik_t, h = 1, threshold = 0.05)
 * (hassan2005/R/forecast.R:1-31; called at hassan2005/main.R:138 and inside
 * the walk-forward loop of hassan2005/R/wf-forecast.R) on the `oblik_t`
 * [S, T] array that rstan::extract returns for iohmm-hmix(-lite)
 * (hassan2005/main.R:94) -- here the engine's HHMM_OUT_OBLIK_T output.
 *
 * Per draw s of series n (pair p = s + S*n, the engine's GRID order), with
 * target = oblik_t[p, T-1] and candidates c = 0 .. T-1-h (0-based):
 *     closest = { c : |target - oblik_t[p, c]| < |target| * threshold },
 *               or, if empty, every c attaining min_c |target - oblik_t[p, c]|
 *     w_c     = exp(|target - oblik_t[p, c]|)            (forecast.R:24-25)
 *     forecast[p] = x[n, T-1] + sum_c (x[n, c+h] - x[n, c]) * w_c / sum_c w_c   (:27)
 * The set selection is exact (the same double comparisons as R).  R sums in
 * 80-bit long double; the engine sums in double in R's order (ascending c),
 * so forecasts agree with R to a few ulps (the tests use 1e-12 relative).
 *
 * Layouts are R column-major as in hhmm.h: x[n + N*t], oblik_t[p + P*t].
 */
#ifndef HHMM_FORECAST_H
#define HHMM_FORECAST_H

#include "hhmm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hhmm_forecast_request {
    int64_t n_series;      /* N */
    int64_t n_draws;       /* S; pairs P = N * S, p = s + S*n */
    int32_t T;             /* series length (= dim(oblik_t)[2]); needs T > h */
    int32_t h;             /* forecast horizon (reference default 1) */
    double threshold;      /* relative neighbourhood (reference default 0.05) */
    const double *x;       /* [N, T] observed series */
    const double *oblik_t; /* [P, T] */
} hhmm_forecast_request;

/* Host pointers: uploads, runs on `device` (-1 = current), downloads forecast [P]. */
hhmm_status hhmm_neighbouring_forecast(const hhmm_forecast_request *req, double *forecast, int device);

/* Device pointers on the current device, enqueued on `stream` (no synchronisation). */
hhmm_status hhmm_neighbouring_forecast_device(const hhmm_forecast_request *req, double *forecast, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HHMM_FORECAST_H */
