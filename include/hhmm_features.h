/*
 * hhmm_features.h -- C ABI of the tick -> zig-zag -> leg feature extractor
 * (SURVEY.md §8 F1), part of libhhmm.so.
 *
 * Replaces the reference's `extract_features(tdata, alpha)`
 * (tayal2009/R/feature-extraction.R:8-133, called at tayal2009/main.R:61 and tayal2009/R/wf-trade.R:58 as
 * `zig <- extract_features(tdata, features.alpha)`), whose output feeds the
 * Tayal HHMM through the Q11 coding of tayal2009/main.R:85-89
 * (sign = feature <= 9 ? 1 : 2, x = feature <= 9 ? feature : feature - 9).
 *
 * Input: one tick series (an xts of PRICE and SIZE in the reference) as three
 * parallel arrays: price, size and the POSIXct index in seconds.  Output: one
 * row per zig-zag leg, the columns of the reference's `zigzag` xts:
 *   price    the extreme price closing the leg      (feature-extraction.R:30)
 *   start    first tick of the leg (1-based)        (:33)
 *   end      last tick of the leg (1-based)         (:35-36)
 *   size_av  sum(size[start..end]) / (secs(end - start) + 1)  (:41-47)
 *   f0       local extremum: +1 max, -1 min         (:50-51)
 *   f1       trend: +1 up, 0 none, -1 down          (:55-70)
 *   f2       volume strength: +1 / 0 / -1           (:73-89)
 *   feature  leg code 1..18 (legs table)            (:92-125)
 *   trend    +1 / 0 / -1 by leg code                (:128-130)
 *   x, sign  the Tayal data-block coding of feature (tayal2009/main.R:85-89)
 *
 * Semantics follow R exactly, including: direction of tick 1 = 0; a leg
 * boundary where the direction is non-zero and differs from the previous
 * tick's; the last leg's price is the tick before the last boundary while its
 * end is the last tick; difftime's automatic units (secs / mins / hours /
 * days) and the conversion back to seconds; NA size ratios never setting f2.
 * size_av is bit-exact with R when the partial sums of size are exact doubles
 * (integer volumes below 2^53); R accumulates sum() in 80-bit long double.
 *
 * Errors: HHMM_ERR_INVALID_ARGUMENT for n < 3, NULL pointers, or fewer than
 * two legs (the reference fails there: f0[2] does not exist); capacity too
 * small is reported with the number of legs needed in n_legs.
 */
#ifndef HHMM_FEATURES_H
#define HHMM_FEATURES_H

#include "hhmm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hhmm_ticks {
    int64_t n;             /* ticks */
    const double *price;   /* [n] tdata$PRICE */
    const double *size;    /* [n] tdata$SIZE */
    const double *time;    /* [n] index(tdata) as POSIXct seconds, non-decreasing */
    double alpha;          /* volume-strength threshold (features.alpha; reference default 0.25) */
} hhmm_ticks;

typedef struct hhmm_legs {
    int64_t capacity;      /* rows allocated in every output array below */
    int64_t n_legs;        /* out: zig-zag rows written (or needed, if > capacity) */
    double  *price;        /* [capacity] */
    int32_t *start;        /* [capacity] 1-based tick index */
    int32_t *end;          /* [capacity] 1-based tick index */
    double  *size_av;      /* [capacity] */
    int32_t *f0, *f1, *f2; /* [capacity] */
    int32_t *feature;      /* [capacity] 1..18 */
    int32_t *trend;        /* [capacity] */
    int32_t *x;            /* [capacity] 1..9  (feature folded, tayal2009/main.R:88) */
    int32_t *sign;         /* [capacity] 1 up leg, 2 down leg (tayal2009/main.R:87) */
} hhmm_legs;

/* Host pointers: uploads the ticks, runs the extractor on device `device`
 * (-1 = current), downloads the legs, synchronises.  Any output pointer may be
 * NULL (not materialised). */
hhmm_status hhmm_extract_features(const hhmm_ticks *ticks, hhmm_legs *legs, int device);

/* Device pointers (every array in ticks / legs lives on the current device):
 * enqueues on `stream`, then synchronises it once to read the leg count. */
hhmm_status hhmm_features_workspace_size(int64_t n, size_t *bytes);
hhmm_status hhmm_extract_features_device(const hhmm_ticks *ticks, hhmm_legs *legs, void *workspace,
                                         size_t workspace_bytes, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HHMM_FEATURES_H */
