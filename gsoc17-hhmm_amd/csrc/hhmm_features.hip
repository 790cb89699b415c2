/*
 * hhmm_features.hip -- gfx950 tick -> zig-zag -> leg feature extractor
 * (C ABI in include/hhmm_features.h).
 *
 * Reference: extract_features(tdata, alpha), tayal2009/R/feature-extraction.R:8-133
 * (called at tayal2009/main.R:61 and tayal2009/R/wf-trade.R:58).  The R code
 * walks the ticks with vectorised xts ops and then row-by-row sapply /
 * rollapply calls (:41-47, :55-70, :123-125 -- "This function is the
 * bottleneck", :112).  Here it is a stream compaction plus two per-leg maps,
 * all HBM-bound integer / byte work (no MFMA):
 *
 *   1. leg_count_kernel    tile of kTile ticks per workgroup: direction
 *                          (:20-24) and change flags (:26-27), count per tile;
 *   2. leg_scan_kernel     one workgroup: exclusive scan of the tile counts;
 *   3. leg_scatter_kernel  the change-point tick indices in tick order (wave
 *                          ballot + popcount prefix, LDS wave offsets);
 *   4. leg_kernel          lane per leg: start / end / closing price (:30-36),
 *                          size.av (:41-47) with R's difftime unit round trip,
 *                          kept in LDS with a 4 + 1 leg halo; then f0 (:50-51),
 *                          f1 (:55-70), f2 (:73-89), leg code (:92-125), trend
 *                          (:128-130) and the Tayal coding x / sign
 *                          (tayal2009/main.R:85-89).
 *
 * Bytes per tick (algorithmic): price 8 + size 8 (+ time 16 per leg and
 * 64 B of leg columns per leg).  The change flags need price[t-1], price[t-2]:
 * neighbouring lanes' loads, served from L1/L2, so price crosses HBM twice
 * (count + scatter).  A single-pass decoupled look-back variant (ticketed
 * tiles, wave-parallel look-back over 64 predecessors) was measured at
 * 5.2 ms against 1.69 ms for this three-kernel form on 10^8 ticks: the
 * look-back chain through L2 dominates at 24k tiles.
 */
#include <hip/hip_runtime.h>
#include <math.h>

#include "hhmm_features.h"
#include "hhmm_internal.h"

namespace hhmm {

constexpr int kFeatBlock = 256;
constexpr int kFeatRows = 16;                       /* ticks per lane per tile */
constexpr int kTile = kFeatBlock * kFeatRows;       /* ticks per workgroup */

/* direction of tick t (0-based): sign(price[t] - price[t-1]); tick 0 is
 * direction.lt (feature-extraction.R:24). */
__device__ __forceinline__ int tick_dir(const double *price, int64_t t)
{
    if (t <= 0)
        return 0;
    const double a = price[t], b = price[t - 1];
    return a > b ? 1 : (a < b ? -1 : 0);
}

/* direction.chg[t] = direction != lt & direction != lag(direction) (:27). */
__device__ __forceinline__ bool tick_chg(const double *price, int64_t n, int64_t t)
{
    if (t < 1 || t >= n)
        return false;
    const int d = tick_dir(price, t);
    return d != 0 && d != tick_dir(price, t - 1);
}

__device__ __forceinline__ int block_sum(int v, int *red)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        v += __shfl_xor(v, off);
    if (lane == 0)
        red[wave] = v;
    __syncthreads();
    int s = 0;
#pragma unroll
    for (int w = 0; w < kFeatBlock / 64; ++w)
        s += red[w];
    __syncthreads();
    return s;
}

__global__ void __launch_bounds__(kFeatBlock) leg_count_kernel(const double *price, int64_t n, int32_t *counts)
{
    __shared__ int red[kFeatBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kTile;
    int c = 0;
#pragma unroll 4
    for (int i = 0; i < kFeatRows; ++i)
        c += tick_chg(price, n, base + i * kFeatBlock + threadIdx.x) ? 1 : 0;
    c = block_sum(c, red);
    if (threadIdx.x == 0)
        counts[blockIdx.x] = c;
}

/* Exclusive scan of counts[0..nt) in place; counts[nt] = total. */
__global__ void __launch_bounds__(1024) leg_scan_kernel(int32_t *counts, int64_t nt)
{
    __shared__ int wsum[16];
    __shared__ int carry_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0)
        carry_s = 0;
    __syncthreads();
    for (int64_t b = 0; b < nt; b += 1024) {
        const int64_t i = b + threadIdx.x;
        const int v = i < nt ? counts[i] : 0;
        int x = v; /* inclusive wave scan */
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(x, off);
            if (lane >= off)
                x += y;
        }
        if (lane == 63)
            wsum[wave] = x;
        __syncthreads();
        int wo = 0;
        for (int w = 0; w < wave; ++w)
            wo += wsum[w];
        const int carry = carry_s;
        if (i < nt)
            counts[i] = carry + wo + x - v;
        __syncthreads();
        if (threadIdx.x == 1023)
            carry_s = carry + wo + x;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        counts[nt] = carry_s;
}

/* chg[k] = 1-based tick index of the k-th change point, in tick order. */
__global__ void __launch_bounds__(kFeatBlock) leg_scatter_kernel(const double *price, int64_t n,
                                                                 const int32_t *offsets, int32_t *chg)
{
    __shared__ int wcnt[kFeatBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kTile;
    int run = offsets[blockIdx.x];
    for (int i = 0; i < kFeatRows; ++i) {
        const int64_t t = base + i * kFeatBlock + threadIdx.x;
        const bool f = tick_chg(price, n, t);
        const uint64_t bal = __ballot(f);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0)
            wcnt[wave] = __popcll(bal);
        __syncthreads();
        int wo = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kFeatBlock / 64; ++w) {
            wo += (w < wave) ? wcnt[w] : 0;
            tot += wcnt[w];
        }
        if (f)
            chg[run + wo + below] = (int32_t)(t + 1);
        run += tot;
        __syncthreads();
    }
}

/* as.numeric(difftime(t1, t0), units = "secs"): R picks the units from |z|
 * and multiplies back (base R difftime / `units<-.difftime`). */
__device__ __forceinline__ double difftime_secs(double t1, double t0)
{
    const double z = t1 - t0;
    const double az = fabs(z);
    double f = 1.0;
    if (!isfinite(az) || az < 60.0)
        f = 1.0;
    else if (az < 3600.0)
        f = 60.0;
    else if (az < 86400.0)
        f = 3600.0;
    else
        f = 86400.0;
    return (z / f) * f;
}

struct LegArgs {
    const double *price, *size, *time;
    int64_t n;
    double alpha;
    const int32_t *chg;
    const int32_t *total; /* device: number of legs */
    double *o_price, *o_size_av;
    int32_t *o_start, *o_end, *o_f0, *o_f1, *o_f2, *o_feature, *o_trend, *o_x, *o_sign;
};

/* Row r of the zig-zag (0 <= r < m): closing price and size.av. */
__device__ __forceinline__ void leg_row(const LegArgs &a, int64_t m, int64_t r, double &p, double &sav, int64_t &s,
                                        int64_t &e)
{
    const int64_t cr = a.chg[r];
    p = a.price[cr - 2];                    /* price[which(direction.chg) - 1] (:30) */
    s = (r == 0) ? 1 : a.chg[r - 1];        /* start (:33) */
    e = (r == m - 1) ? a.n : cr - 1;        /* end (:35-36) */
    double acc = 0.0;
    for (int64_t i = s - 1; i < e; ++i)
        acc += a.size[i];
    sav = acc / (difftime_secs(a.time[e - 1], a.time[s - 1]) + 1.0); /* size.av (:41-47) */
}

/* ifelse(ratio - 1 > alpha, 1, ifelse(1 - ratio > alpha, -1, 0)), NA (NaN) -> 2 (:77-79). */
__device__ __forceinline__ int discretize(double ratio, double alpha)
{
    if (isnan(ratio))
        return 2;
    return (ratio - 1.0 > alpha) ? 1 : ((1.0 - ratio > alpha) ? -1 : 0);
}

/* legs table (:92-110) as a lookup: code = table[f0 up/down][f1 + 1][f2 + 1]. */
__constant__ int8_t kLegCode[2][3][3] = {
    /* f0 = +1 (up legs):   f2 = -1, 0, +1 */
    {{9, 7, 2},   /* f1 = -1 */
     {6, 5, 4},   /* f1 =  0 */
     {8, 3, 1}},  /* f1 = +1 */
    /* f0 = -1 (down legs) */
    {{11, 16, 18},
     {13, 14, 15},
     {10, 12, 17}}};

/* One workgroup = legs [r0, r0 + kFeatBlock): every lane forms its own row
 * (start / end / price / size.av) into LDS, plus a halo of 4 legs before and
 * 1 after (the f0 / f1 / ratio stencils), then the features -- the per-leg
 * state never leaves the CU. */
constexpr int kHaloLo = 4, kHaloHi = 1;

__global__ void __launch_bounds__(kFeatBlock) leg_kernel(const LegArgs a)
{
    __shared__ double s_lp[kFeatBlock + kHaloLo + kHaloHi];
    __shared__ double s_sav[kFeatBlock + kHaloLo + kHaloHi];
    const int64_t m = *a.total;
    const int64_t r0 = (int64_t)blockIdx.x * kFeatBlock;
    for (int k = threadIdx.x; k < kFeatBlock + kHaloLo + kHaloHi; k += kFeatBlock) {
        const int64_t r = r0 - kHaloLo + k;
        double p = 0.0, sav = 0.0;
        if (r >= 0 && r < m) {
            int64_t st, en;
            leg_row(a, m, r, p, sav, st, en);
            if (k >= kHaloLo && k < kHaloLo + kFeatBlock) {
                if (a.o_price) a.o_price[r] = p;
                if (a.o_start) a.o_start[r] = (int32_t)st;
                if (a.o_end) a.o_end[r] = (int32_t)en;
                if (a.o_size_av) a.o_size_av[r] = sav;
            }
        }
        s_lp[k] = p;
        s_sav[k] = sav;
    }
    __syncthreads();
    const int64_t r = r0 + threadIdx.x;
    if (r >= m)
        return;
    const double *lp = s_lp + kHaloLo + threadIdx.x;  /* lp[j] = price of leg r + j */
    const double *sv = s_sav + kHaloLo + threadIdx.x;
    /* f0 (:50-51): lag(price) < price ? max : min; f0[1] = opposite of f0[2] */
    const int f0 = (r == 0) ? ((lp[0] < lp[1]) ? -1 : 1) : ((lp[-1] < lp[0]) ? 1 : -1);
    /* f1 (:55-70) */
    int f1 = 0;
    if (r >= 4) {
        const double e0 = lp[-4], e1 = lp[-3], e2 = lp[-2], e3 = lp[-1], e4 = lp[0];
        if (e0 < e2 && e2 < e4 && e1 < e3)
            f1 = 1;
        else if (e0 > e2 && e2 > e4 && e1 > e3)
            f1 = -1;
    }
    /* f2 (:73-89): assignments only where every comparison is TRUE (NA never assigns) */
    int f2 = 0;
    if (r >= 2) {
        const double v0 = sv[0], v1 = sv[-1], v2 = sv[-2];
        const int s1 = discretize(v0 / v1, a.alpha), s2 = discretize(v0 / v2, a.alpha),
                  s3 = discretize(v1 / v2, a.alpha);
        const bool ok = s1 != 2 && s2 != 2 && s3 != 2;
        if (ok && s1 == 1 && s2 > -1 && s3 < 1)
            f2 = 1;
        if (ok && s1 == -1 && s2 < 1 && s3 > -1)
            f2 = -1;
    }
    const int code = kLegCode[f0 > 0 ? 0 : 1][f1 + 1][f2 + 1];
    const int trend = ((code >= 6 && code <= 9) || code >= 15) ? -1 : ((code == 5 || code == 14) ? 0 : 1);
    if (a.o_f0) a.o_f0[r] = f0;
    if (a.o_f1) a.o_f1[r] = f1;
    if (a.o_f2) a.o_f2[r] = f2;
    if (a.o_feature) a.o_feature[r] = code;
    if (a.o_trend) a.o_trend[r] = trend;
    if (a.o_sign) a.o_sign[r] = code < 10 ? 1 : 2;   /* tayal2009/main.R:87 */
    if (a.o_x) a.o_x[r] = code < 10 ? code : code - 9; /* tayal2009/main.R:88 */
}

static int64_t feat_tiles(int64_t n) { return (n + kTile - 1) / kTile; }

static size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

size_t features_workspace_bytes(int64_t n)
{
    return align256(sizeof(int32_t) * (size_t)(feat_tiles(n) + 1)) + align256(sizeof(int32_t) * (size_t)n);
}

/* Enqueues the pipeline on `st` (device pointers); returns the leg count via
 * a synchronising 4-byte read after the scan. */
hhmm_status features_run_device(const hhmm_ticks *tk, hhmm_legs *lg, void *ws, size_t ws_bytes, hipStream_t st)
{
    const int64_t n = tk->n;
    if (ws_bytes < features_workspace_bytes(n)) {
        set_error("features workspace %zu B < %zu B needed", ws_bytes, features_workspace_bytes(n));
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    const int64_t nt = feat_tiles(n);
    char *w = static_cast<char *>(ws);
    int32_t *counts = reinterpret_cast<int32_t *>(w);
    w += align256(sizeof(int32_t) * (size_t)(nt + 1));
    int32_t *chg = reinterpret_cast<int32_t *>(w);

    hipLaunchKernelGGL(leg_count_kernel, dim3((unsigned)nt), dim3(kFeatBlock), 0, st, tk->price, n, counts);
    hipLaunchKernelGGL(leg_scan_kernel, dim3(1), dim3(1024), 0, st, counts, nt);
    hipLaunchKernelGGL(leg_scatter_kernel, dim3((unsigned)nt), dim3(kFeatBlock), 0, st, tk->price, n,
                       (const int32_t *)counts, chg);
    int32_t m = 0;
    hipError_t e = hipMemcpyAsync(&m, counts + nt, sizeof(int32_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess)
        e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
        set_error("feature extraction (change points): %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    lg->n_legs = m;
    if (m < 2) {
        set_error("the ticks form %d zig-zag leg(s); the reference needs at least 2 (feature-extraction.R:51)", m);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (m > lg->capacity) {
        set_error("%d legs do not fit in capacity %lld (n_legs holds the rows needed)", m,
                  (long long)lg->capacity);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    LegArgs a;
    a.price = tk->price;
    a.size = tk->size;
    a.time = tk->time;
    a.n = n;
    a.alpha = tk->alpha;
    a.chg = chg;
    a.total = counts + nt;
    a.o_price = lg->price;
    a.o_size_av = lg->size_av;
    a.o_start = lg->start;
    a.o_end = lg->end;
    a.o_f0 = lg->f0;
    a.o_f1 = lg->f1;
    a.o_f2 = lg->f2;
    a.o_feature = lg->feature;
    a.o_trend = lg->trend;
    a.o_x = lg->x;
    a.o_sign = lg->sign;
    const dim3 grid((unsigned)((m + kFeatBlock - 1) / kFeatBlock));
    hipLaunchKernelGGL(leg_kernel, grid, dim3(kFeatBlock), 0, st, a);
    e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("feature extraction launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

} // namespace hhmm
