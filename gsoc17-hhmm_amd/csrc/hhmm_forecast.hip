/*
 * hhmm_forecast.hip -- gfx950 nearest-neighbour forecast over oblik_t
 * (C ABI in include/hhmm_forecast.h).
 *
 * Reference: neighbouring_forecast(x, oblik_t, h, threshold),
 * hassan2005/R/forecast.R:1-31, the consumer of iohmm-hmix(-lite)'s
 * one-step observation likelihood (iohmm-hmix.stan:118-121).
 *
 * One lane per (series, draw) pair, p = s + S*n: oblik_t[p + P*t] is read
 * pair-fastest, so every step is one coalesced wave load, and x[n + N*t] is a
 * broadcast within a wave (GRID order keeps a series' draws together).  Two
 * sweeps over the candidates (count / minimum, then the weighted sums in R's
 * ascending order); HBM-bound at 2 x 8 B per (pair, t) of oblik_t.
 */
#include <hip/hip_runtime.h>
#include <math.h>

#include "hhmm_forecast.h"
#include "hhmm_internal.h"

#ifndef HHMM_MATH_FN
#define HHMM_MATH_FN static __device__ __forceinline__
#define HHMM_MATH_TABLE static __constant__
#endif
#include "hhmm_crmath.h"

namespace hhmm {

__global__ void __launch_bounds__(256) forecast_kernel(const hhmm_forecast_request r, double *out)
{
    const int64_t P = r.n_series * r.n_draws;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P)
        return;
    const int64_t n = p / r.n_draws;
    const int T = r.T, h = r.h;
    const int nc = T - h;              /* oblik_cand <- oblik_t[n, 1:(T.length - h)] (:21) */
    const double *ob = r.oblik_t + p;
    const double tgt = ob[P * (int64_t)(T - 1)]; /* oblik_target (:20) */
    const double thr = fabs(tgt) * r.threshold;
    /* find_closest (:9-16): which(|target - cand| < |target| * threshold), else the minimisers */
    int cnt = 0;
    bool nan_seen = false;
    double mn = __builtin_inf();
    for (int c = 0; c < nc; ++c) {
        const double d = fabs(tgt - ob[P * (int64_t)c]);
        cnt += (d < thr) ? 1 : 0;
        nan_seen |= isnan(d);
        mn = fmin(mn, d);
    }
    const double *x = r.x + n;
    const int64_t N = r.n_series;
    double res;
    if (cnt == 0 && nan_seen) {
        res = __builtin_nan(""); /* min() is NA: no index equals it, 0/0 */
    } else {
        double num = 0.0, den = 0.0;
        for (int c = 0; c < nc; ++c) {
            const double d = fabs(tgt - ob[P * (int64_t)c]); /* d <- abs(target - oblik_t[n, closests]) (:24) */
            const bool sel = cnt > 0 ? (d < thr) : (d == mn);
            if (sel) {
                const double w = hhmm_cr_exp(d);         /* w <- exp(d) (:25) */
                num += (x[N * (int64_t)(c + h)] - x[N * (int64_t)c]) * w;
                den += w;
            }
        }
        res = x[N * (int64_t)(T - 1)] + num / den; /* (:27) */
    }
    out[p] = res;
}

static hhmm_status check_forecast(const hhmm_forecast_request *r, const double *out)
{
    if (!r || !out || !r->x || !r->oblik_t) {
        set_error("NULL forecast argument");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (r->n_series < 1 || r->n_draws < 1 || r->h < 1 || r->T <= r->h) {
        set_error("forecast needs N, S >= 1, h >= 1 and T > h (got N=%lld S=%lld T=%d h=%d)",
                  (long long)r->n_series, (long long)r->n_draws, r->T, r->h);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    return HHMM_OK;
}

static hhmm_status launch_forecast(const hhmm_forecast_request *r, double *out, hipStream_t st)
{
    const int64_t P = r->n_series * r->n_draws;
    hipLaunchKernelGGL(forecast_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, *r, out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("forecast_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

} // namespace hhmm

using namespace hhmm;

extern "C" {

hhmm_status hhmm_neighbouring_forecast_device(const hhmm_forecast_request *req, double *forecast, void *stream)
{
    hhmm_status s = check_forecast(req, forecast);
    if (s != HHMM_OK)
        return s;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        (void)hipGetLastError();
        set_error("no HIP device visible: libhhmm has no CPU path (gfx950 required)");
        return HHMM_ERR_NO_DEVICE;
    }
    return launch_forecast(req, forecast, (hipStream_t)stream);
}

hhmm_status hhmm_neighbouring_forecast(const hhmm_forecast_request *req, double *forecast, int device)
{
    hhmm_status s = check_forecast(req, forecast);
    if (s != HHMM_OK)
        return s;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        (void)hipGetLastError();
        set_error("no HIP device visible: libhhmm has no CPU path (gfx950 required)");
        return HHMM_ERR_NO_DEVICE;
    }
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice(%d) failed", device);
        return HHMM_ERR_HIP;
    }
    const int64_t P = req->n_series * req->n_draws;
    const size_t bx = sizeof(double) * (size_t)req->n_series * req->T;
    const size_t bo = sizeof(double) * (size_t)P * req->T;
    double *dx = nullptr, *dob = nullptr, *dout = nullptr;
    hipError_t e = hipMalloc(&dx, bx);
    if (e == hipSuccess)
        e = hipMalloc(&dob, bo);
    if (e == hipSuccess)
        e = hipMalloc(&dout, sizeof(double) * (size_t)P);
    if (e == hipSuccess)
        e = hipMemcpy(dx, req->x, bx, hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipMemcpy(dob, req->oblik_t, bo, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hhmm_forecast_request dr = *req;
        dr.x = dx;
        dr.oblik_t = dob;
        s = launch_forecast(&dr, dout, nullptr);
        if (s == HHMM_OK)
            e = hipMemcpy(forecast, dout, sizeof(double) * (size_t)P, hipMemcpyDeviceToHost);
    }
    (void)hipFree(dx);
    (void)hipFree(dob);
    (void)hipFree(dout);
    if (e != hipSuccess) {
        set_error("forecast: %s", hipGetErrorString(e));
        return (e == hipErrorOutOfMemory) ? HHMM_ERR_OUT_OF_MEMORY : HHMM_ERR_HIP;
    }
    return s;
}

} // extern "C"
