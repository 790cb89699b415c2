/*
 * hhmm_internal.h -- declarations shared by the host API (hhmm_api.cpp) and
 * the gfx950 kernels (hhmm_kernels.hip).  Not part of the public ABI.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "hhmm.h"
#include "hhmm_features.h"

namespace hhmm {

/* Probe knobs (HHMM_PROBE_* environment variables: launch shapes, stream
 * priority, the V-scan statistics) exist only in a build with -DHHMM_PROBES
 * (tools/build_variant.sh); a release libhhmm.so never reads the environment,
 * so a stray variable cannot change its schedule or synchronise it. */
#ifdef HHMM_PROBES
static inline const char *probe_env(const char *name) { return getenv(name); }
#else
static inline const char *probe_env(const char *) { return nullptr; }
#endif

/* Everything one launch needs, by value in the kernel argument segment.
 * All pointers are device pointers; layouts as in include/hhmm.h. */
struct DevArgs {
    int64_t P;          /* pairs */
    int64_t N;          /* series */
    int64_t S;          /* draws */
    int32_t pairing;    /* HHMM_PAIR_GRID / ZIP / BLOCK */
    int32_t model;
    int32_t K, L, M;
    int32_t Tmax;       /* padded extent of the time axis of the data arrays in use */
    int32_t Tout;       /* padded extent of the time axis of the [P,T,K] outputs in use */
    uint32_t outputs;
    /* series data (already switched to the OOS arrays for a tayal-lite OOS pass) */
    const int32_t *T;
    const int32_t *x;
    const double *xr;
    const int32_t *g;
    const int32_t *sign;
    const double *u;
    /* draws */
    const double *p_1k, *A_ij, *phi_k, *mu_k, *sigma_k;
    const double *w_km, *b_km, *s_k, *lambda_kl, *mu_kl, *s_kl;
    const double *p_11, *A_row;
    /* outputs */
    double *loglik;
    double *unalpha, *alpha, *unbeta, *beta, *ungamma, *gamma;
    int32_t *zstar;
    double *logp_zstar;
    int32_t *pair_status;
    double *oblik;      /* [P, Tout, K] oblik_tk */
    double *oblik_t;    /* [P, Tout]    oblik_t */
    double *logA;       /* [P, Tout, K] A_ij (reg / mix) or logA_ij (hmix / lite) */
    int32_t *z_ffbs;    /* [P, Tout]    FFBS draw */
    const double *ffbs_u; /* [P, Tmax]  caller uniforms */
    /* fitted-output GQ draws */
    double *hatpi;        /* [P, Tout, K] */
    int32_t *hatz, *hatl; /* [P, Tout] 1-based */
    double *hatx;         /* [P, Tout] */
    const double *hat_rand; /* [P, Tmax, 3] caller uniforms / normal deviates */
    /* workspace */
    double *ckpt;       /* [nchunk][K][P] forward checkpoints */
    double *ckpt_ls;    /* [nchunk][P]    log scale at each checkpoint */
    uint32_t *bp;       /* [nword][P]     packed Viterbi back-pointers */
    double *lam;        /* [Tmax][P]      IOHMM: running sum of log c_t (unbeta pass) */
    uint32_t *xpk;      /* [nchunk][P]    packed symbols of each checkpoint chunk (multinom, L <= 16) */
    int32_t *rnw;       /* [waves]        FB_BIG: the wave renormalises every step (fb_dense_kernel) */
    int32_t *io_redo;   /* [1 + P]        IOHMM: pairs whose linear filter underflowed (count, then ids) */
    /* parallel scan over T; scan_cl = 0: sequential sweeps */
    uint32_t flags;     /* hhmm_request.flags */
    int32_t scan_cl;    /* steps per T-chunk (multiple of fb_chunk(K)) */
    int32_t scan_nc;    /* T-chunks per pair (of T_max) */
    double *sc_mf;      /* [nc][K][K][P] forward chunk products (chunk 0: row 0 = f at its end) */
    double *sc_qb;      /* [nc][K][K][P] backward chunk products */
    double *sc_mx;      /* [nc][3][P]    per chunk: forward exponent, log scale, backward exponent */
    double *sc_st;      /* [nc][K][P]    forward state entering each chunk */
    double *sc_sl;      /* [nc][P]       its log scale */
    double *sc_be;      /* [nc][K][P]    beta at each chunk's last step */
    double *sc_bl;      /* [nc][P]       its log scale; large K: [P][nc] the chunk products' Gaussian log scales */
    /* T-parallel exact Viterbi (hhmm_vscan.h); vs_nc = 0: sequential decoders */
    int32_t vs_nc;      /* V-chunks of kVsChunk steps per pair (of the Viterbi's T_max) */
    double *vs_m;       /* [nc][K*K][P] chunk max-plus products (approximate, then on the grid) */
    double *vs_m1;      /* [nc][K*K][P] chunks with a rounding tie: the products for odd entry values */
    double *vs_d;       /* [nc+1][K][P] delta leaving chunk c - 1 (row c); row ncp: delta_T */
    int32_t *vs_k;      /* [nc][P]      binary exponent of the chunk's grid (| kVsTie) */
    uint32_t *vs_e;     /* [nc][P]      chunk backtrack map: byte s = entry state of exit state s */
    int32_t *vs_z;      /* [nc][P]      path state at each chunk's last step (-1: no path) */
    int32_t *vs_fail;   /* [P]          a replayed chunk disagreed: decode again sequentially */
    int32_t *vs_tl;     /* [1 + P*nc]   chunks with a grid rounding tie: count, then p + P c */
    const int32_t *vs_redo; /* state-parallel decoder: only pairs with vs_redo[p] != 0 (null: all) */
    int32_t *dc_flag;       /* [N] device entry: series breaking a data-block constraint (null: host-validated) */
    /* one time window of a series split over ranks (hhmm_segment; 0: a whole series) */
    int32_t seg_phase;      /* 1: summary call, 2: finish call */
    int32_t seg_nofirst;    /* the window does not start at t = 1: chunk 0 enters from seg_enter */
    int32_t seg_nolast;     /* the window does not end at T: beta leaves as seg_leave, no loglik */
    double *seg_sum;        /* [2K^2 + 3][P] */
    const double *seg_enter;/* [K + 1][P] */
    const double *seg_leave;/* [K + 1][P] */
};

/* Phase-3 lanes of the T-scan per T-chunk: P rounded up to whole waves. */
constexpr int64_t scan_lanes_per_chunk(int64_t P) { return (P + 63) & ~(int64_t)63; }

/* Parallel-scan plan of one request: T-chunk length and count (cl = 0: off). */
struct ScanPlan {
    int cl;
    int nc;
};
ScanPlan scan_plan(int model, int K, int Tmax, int64_t P, uint32_t outputs, uint32_t flags);

/* T-parallel exact Viterbi (hhmm_vscan.h): V-chunks of kVsChunk steps (a whole
 * number of back-pointer words at K = 2 and 4); returns the chunk count per
 * pair of a Viterbi over Tv steps, 0 when the sequential decoders run. */
#ifndef HHMM_VS_CHUNK
#define HHMM_VS_CHUNK 512 /* build knob: steps per V-chunk */
#endif
constexpr int kVsChunk = HHMM_VS_CHUNK;
int vscan_chunks(int model, int K, int Tv, int64_t P, uint32_t outputs, uint32_t flags);

/* Large K under GRID pairing (hhmm_lkscan.h lkm_fb_kernel): the k-steps of
 * its state capacity when it runs the forward-backward, else 0. */
int lkm_plan(int model, int K, int64_t N, int pairing, uint32_t outputs, uint32_t flags, int scan_cl);

/* Time steps between forward checkpoints kept for the backward sweep. */
constexpr int fb_chunk(int K) { return K <= 4 ? 8 : 4; }

/* Viterbi back-pointer packing: bits per state, bits per step, steps per word. */
constexpr int bp_bits(int K) { return K <= 2 ? 1 : (K <= 4 ? 2 : (K <= 8 ? 3 : 4)); }
constexpr int bp_steps_per_word(int K) { return 32 / (K * bp_bits(K)); }

constexpr int kMaxK = 8;       /* lane-per-pair kernels (hhmm_hmm.h, hhmm_iohmm.h) */
constexpr int kMaxKLarge = 32; /* state-parallel HMM-family kernels (hhmm_large.h) */
constexpr int kBlock = 256;
constexpr size_t kLdsLimit = 160 * 1024;

/* Bytes of workspace the kernels need for this launch shape. */
size_t workspace_bytes(int model, int K, int L, int Tmax, int Toos, int64_t P, uint32_t outputs, uint32_t flags,
                       int64_t N, int pairing);

/* Carves the workspace into DevArgs pointers. */
void bind_workspace(DevArgs &a, void *ws, int Tmax, int Toos, uint32_t flags);

/* Launches every kernel the request needs on `stream` (device pointers).
 * check_data: the data arrays were not validated on the host (the device
 * entry): flag pairs whose series breaks a data-block constraint
 * (HHMM_PAIR_INVALID_DATA) after the model's kernels. */
hhmm_status launch_all(const hhmm_request *req, const hhmm_result *res, int64_t P, void *ws, hipStream_t st,
                       const hhmm_segment *seg = nullptr, int seg_phase = 0, bool check_data = false);
/* Set by a launcher whose kernel checks the data-block constraints inline
 * (the phased sweep, launch_vfb): launch_all then skips its separate pass. */
extern thread_local bool t_data_checked_inline;

/* HMM family, one translation unit per model / K range (hhmm_m_*.hip). */
hhmm_status run_gauss_lo(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_gauss_hi(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_multinom_lo(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_multinom_hi(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_semisup_lo(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_semisup_hi(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_tayal(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
hhmm_status run_tayal_lite(const DevArgs &a, const hhmm_request *req, const hhmm_result *res, hipStream_t st);
/* hmm / hmm-multinom at kMaxK < K <= kMaxKLarge (hhmm_m_large.hip) */
hhmm_status run_large(const DevArgs &a, hipStream_t st);
/* the IOHMM programs at kMaxK < K <= kMaxKLarge (hhmm_io_large.hip) */
hhmm_status run_large_iohmm(const DevArgs &a, hipStream_t st);

/* IOHMM family (iohmm-reg / -mix / -hmix / -hmix-lite), hhmm_iohmm.hip. */
hhmm_status launch_iohmm(const DevArgs &a, hipStream_t stream);
/* The outputs the IOHMM linear-space filter produces; a pair whose filter
 * drops below kIoWeak is listed in a.io_redo and re-run in log space by
 * launch_iohmm_log (hhmm_iolog.hip). */
constexpr uint32_t kIoFilt = HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_ALPHA | HHMM_OUT_UNBETA | HHMM_OUT_BETA |
                             HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA | HHMM_OUT_OBLIK_T;
constexpr uint32_t kIoBack = HHMM_OUT_UNBETA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA;
constexpr double kIoWeak = 0x1p-960;
/* t = 0: f_0 = p .* e_0 keeps every component above 2^-1074, i.e. down to
 * 2^-834 (below the 1e-250 tolerance floor) of a max of at least 2^-240 */
constexpr double kIoWeak0 = 0x1p-240;
/* gamma = (alpha .* beta) * (1 / sum) straight from the scaled vectors while
 * the sum sg exceeds kGammaDirect; below it the reference's normalised-vector
 * form.  A product alpha_j beta_j = gamma_j sg that falls into the subnormal
 * range is off by at most 2^-1075, i.e. gamma_j by 2^-1075 / sg < 2^-835 --
 * under the 1e-250 absolute floor of the tolerance -- exactly when sg >
 * 2^-240 (round 5; rounds 1-4 took 2^-960, which let gamma_j below ~2^-114
 * of the sum flush: tests/test_gpu_large_k.py::test_gamma_only_large_K_disjoint_filters
 * at lk_fb_kernel's 8-step renormalisation cadence). */
constexpr double kGammaDirect = 0x1p-240;
hhmm_status launch_iohmm_log(const DevArgs &a, hipStream_t stream);
/* Fitted-output draws hatpi / hatz / hatl / hatx (hhmm_fitted.hip). */
hhmm_status launch_fitted(const DevArgs &a, hipStream_t stream);
hhmm_status run_io_reg_lo(const DevArgs &a, hipStream_t st);
hhmm_status run_io_reg_hi(const DevArgs &a, hipStream_t st);
hhmm_status run_io_mix_lo(const DevArgs &a, hipStream_t st);
hhmm_status run_io_mix_hi(const DevArgs &a, hipStream_t st);
bool iohmm_supported(int K, int M, int L, char *why, size_t why_len);

/* Side stream of the calling thread's current device for an independent
 * pass: fork_stream makes *side wait for everything enqueued on `st` so far;
 * join_stream makes `st` wait for everything enqueued on `side`. */
hhmm_status fork_stream(hipStream_t st, hipStream_t *side);
hhmm_status join_stream(hipStream_t st, hipStream_t side);

/* Device self-test of the correctly rounded log (which = 0) / exp (1), host arrays. */
hhmm_status selftest_cr_math(const double *in, double *out, int64_t n, int which);

void set_error(const char *fmt, ...);

/* Tick -> zig-zag -> leg feature extractor (hhmm_features.hip). */
size_t features_workspace_bytes(int64_t n);
hhmm_status features_run_device(const hhmm_ticks *tk, hhmm_legs *lg, void *ws, size_t ws_bytes, hipStream_t st);

} // namespace hhmm
