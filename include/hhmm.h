/*
 * hhmm.h -- C ABI of the MI355X batched HMM-family engine (libhhmm.so).
 *
 * Drop-in boundary.  The reference evaluates its hot path inside one Stan
 * program per fit: R hands the model's `data` block to
 *     rstan::stan(file, data = list(...))          (hmm/main.R:49-54,
 *                                                   tayal2009/main.R:103-108)
 * and reads the transformed parameters / generated quantities back with
 *     rstan::extract(fit, pars = '<name>')          (hmm/main.R:67-68,98;
 *                                                   hassan2005/main.R:90-95).
 * Per saved draw, stanc's `write_array(params -> TP + GQ)` recomputes the
 * forward filter, backward pass, smoothed posteriors and Viterbi decoding
 * (e.g. hmm/stan/hmm.stan:24-130).  This library replaces that per-draw
 * evaluation for a whole batch of (series x posterior draw) PAIRS at once:
 *
 *   inputs  = the `data` block of the Stan program, batched over series
 *             (hhmm_data), and the `parameters` block as rstan::extract()
 *             returns it for S draws (hhmm_draws);
 *   outputs = the TP / GQ arrays with the names and shapes extract() gives
 *             (hhmm_result), plus the model-block log-likelihood and FFBS.
 *
 * Layout convention: every array is R column-major with its FIRST index
 * fastest, exactly the memory of the R array (zero-copy from .Call):
 *   series arrays  [N, T_max]      x[n + N*t]
 *                  [N, T_max, M]   u[n + N*(t + T_max*m)]
 *   draw arrays    [S, K]          p_1k[s + S*k]
 *                  [S, K, K]       A_ij[s + S*(i + K*j)]   (row i = from, col j = to)
 *                  [S, K, L]       phi_k[s + S*(k + K*l)]
 *   pair outputs   [P]             loglik[p]
 *                  [P, T_max]      zstar_t[p + P*t]
 *                  [P, T_max, K]   gamma_tk[p + P*(t + T_max*k)]
 * Indices in and out are 1-based as in Stan/R (x in 1..L, sign in 1..2,
 * g in 1..G, zstar in 1..K).  Time steps t >= T[n] of a padded series are
 * neither read nor written.
 *
 * Pairing: HHMM_PAIR_GRID evaluates every series under every draw,
 * P = N*S, pair p = s + S*n (draw fastest: a batch of draws of one series is
 * rstan's [S, ...] slab).  HHMM_PAIR_ZIP pairs series n with draw n (N == S).
 * HHMM_PAIR_BLOCK gives every series its own block of B = S / N draws (one
 * fit per series, as the reference's walk-forward runs one stan() per window,
 * tayal2009/R/wf-trade.R:30-100): P = S pairs, pair p = b + B*n evaluates
 * series n under draw p.
 *
 * Errors: every entry point returns hhmm_status; the message of the last
 * failure on the calling thread is hhmm_last_error().  No C++ exception or
 * longjmp crosses this ABI.  Where Stan would throw inside write_array
 * (a Viterbi backtrack through an unset back-pointer: the Q3 initialisation
 * quirk of SURVEY.md App. A, or all delta_T = -inf), the pair's zstar_t is
 * filled with 0, pair_status[p] = HHMM_PAIR_INVALID_BACKPOINTER and the call
 * returns HHMM_WARN_PAIR_FAILURES after completing every other pair.
 *
 * Ownership: the caller owns every input and output buffer; the library never
 * retains a caller pointer after return.  The library owns its device pool,
 * released by hhmm_shutdown().
 */
#ifndef HHMM_H
#define HHMM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HHMM_ABI_VERSION 2u

typedef enum hhmm_status {
    HHMM_OK = 0,
    HHMM_WARN_PAIR_FAILURES = 1,       /* completed; some pair_status != 0 */
    HHMM_ERR_INVALID_ARGUMENT = -1,
    HHMM_ERR_OUT_OF_MEMORY = -2,
    HHMM_ERR_HIP = -3,
    HHMM_ERR_UNSUPPORTED = -4,
    HHMM_ERR_NO_DEVICE = -5
} hhmm_status;

/* Per-pair status codes (hhmm_result.pair_status). */
#define HHMM_PAIR_OK 0
#define HHMM_PAIR_INVALID_BACKPOINTER 1
/* hhmm_run_device only (hhmm_run rejects the whole request instead, as Stan
 * rejects the data block): the pair's series breaks a data-block constraint --
 * x outside 1..L (int<lower=1,upper=L> x[T], hmm-multinom.stan:11), sign outside
 * 1..2 (hhmm-tayal2009.stan:11-12), g outside 1..G, T[n] outside 1..T_max, or
 * the same for the tayal-lite out-of-sample arrays.  The pair's outputs are
 * unspecified; every other pair is computed as usual. */
#define HHMM_PAIR_INVALID_DATA 2

/* One id per Stan program on the path. */
typedef enum hhmm_model {
    HHMM_MODEL_HMM_GAUSS = 1,            /* hmm/stan/hmm.stan */
    HHMM_MODEL_HMM_MULTINOM = 2,         /* hmm/stan/hmm-multinom.stan */
    HHMM_MODEL_HMM_MULTINOM_SEMISUP = 3, /* hmm/stan/hmm-multinom-semisup.stan */
    HHMM_MODEL_IOHMM_REG = 4,            /* iohmm-reg/stan/iohmm-reg.stan */
    HHMM_MODEL_IOHMM_MIX = 5,            /* iohmm-mix/stan/iohmm-mix.stan */
    HHMM_MODEL_IOHMM_HMIX = 6,           /* iohmm-mix/stan/iohmm-hmix.stan */
    HHMM_MODEL_IOHMM_HMIX_LITE = 7,      /* iohmm-mix/stan/iohmm-hmix-lite.stan */
    HHMM_MODEL_TAYAL = 8,                /* tayal2009/stan/hhmm-tayal2009.stan */
    HHMM_MODEL_TAYAL_LITE = 9            /* tayal2009/stan/hhmm-tayal2009-lite.stan */
} hhmm_model;

typedef enum hhmm_pairing {
    HHMM_PAIR_GRID = 0,
    HHMM_PAIR_ZIP = 1,
    HHMM_PAIR_BLOCK = 2
} hhmm_pairing;

/* Output selection bitmask (hhmm_request.outputs).  Names are the Stan names. */
#define HHMM_OUT_LOGLIK        (1u << 0)  /* target += log_sum_exp(unalpha_tk[T])   [P] */
#define HHMM_OUT_UNALPHA       (1u << 1)  /* unalpha_tk                             [P,T,K] */
#define HHMM_OUT_ALPHA         (1u << 2)  /* alpha_tk                               [P,T,K] */
#define HHMM_OUT_UNBETA        (1u << 3)  /* unbeta_tk                              [P,T,K] */
#define HHMM_OUT_BETA          (1u << 4)  /* beta_tk                                [P,T,K] */
#define HHMM_OUT_UNGAMMA       (1u << 5)  /* ungamma_tk                             [P,T,K] */
#define HHMM_OUT_GAMMA         (1u << 6)  /* gamma_tk                               [P,T,K] */
#define HHMM_OUT_ZSTAR         (1u << 7)  /* zstar_t (Viterbi path, 1-based)        [P,T] */
#define HHMM_OUT_LOGP_ZSTAR    (1u << 8)  /* logp_zstar_t / logp_zstar              [P] */
#define HHMM_OUT_OBLIK_TK      (1u << 9)  /* oblik_tk (IOHMM emission log-density)  [P,T,K] */
#define HHMM_OUT_OBLIK_T       (1u << 10) /* oblik_t  (iohmm-hmix[-lite])           [P,T] */
#define HHMM_OUT_FFBS          (1u << 11) /* FFBS state draw (needs ffbs_u)          [P,T] */
#define HHMM_OUT_ALPHA_OOS     (1u << 12) /* tayal-lite alpha_tk_oos                [P,T_oos,K] */
#define HHMM_OUT_UNALPHA_OOS   (1u << 13) /* tayal-lite unalpha_tk_oos              [P,T_oos,K] */
#define HHMM_OUT_LOGA          (1u << 14) /* IOHMM A_ij / logA_ij per t             [P,T,K] */
/* Fitted-output draws of the IOHMM generated quantities:
 * iohmm-reg.stan:124-148, iohmm-mix.stan:133-161, iohmm-hmix.stan:137-157.
 * Stan draws them with its own RNG; here the caller supplies the randomness
 * (hhmm_request.hat_rand), so draws are reproducible bit for bit:
 *   hatpi_tk[t] = softmax(u_t' w_j)                         (reg, mix)
 *   hatz_t[t]   = categorical_rng(hatpi_tk[t])  with uniform hat_rand[p,t,0]
 *   hatl_t[t]   = categorical_rng(lambda_kl[hatz]) with uniform hat_rand[p,t,1] (mix, hmix)
 *   hatx_t[t]   = normal_rng(mu, sigma) = z * sigma + mu with the standard
 *                 normal deviate z = hat_rand[p,t,2] (boost's normal_distribution
 *                 form); mu, sigma = u_t' b_km[hatz], s_k[hatz] (reg) or
 *                 mu_kl, s_kl[hatz][hatl] (mix, hmix)
 * categorical_rng(theta, u) = Stan's inverse CDF: c = theta[1], b = 1;
 * while (b < K && u > c) c += theta[++b]; returns b. */
#define HHMM_OUT_HATPI         (1u << 15) /* hatpi_tk                               [P,T,K] */
#define HHMM_OUT_HATZ          (1u << 16) /* hatz_t (1-based)                       [P,T] */
#define HHMM_OUT_HATL          (1u << 17) /* hatl_t (1-based)                       [P,T] */
#define HHMM_OUT_HATX          (1u << 18) /* hatx_t                                 [P,T] */

/* The Stan `data` block, batched over N series (series fastest). */
typedef struct hhmm_data {
    int64_t n_series;          /* N */
    int32_t T_max;             /* padded time extent of every [N, T_max] array */
    int32_t K;                 /* hidden states */
    int32_t L;                 /* outputs per state (multinom/tayal) or mixture components (iohmm-mix) */
    int32_t M;                 /* input dimension (iohmm) */
    int32_t G;                 /* feature sets (semisup) */
    int32_t T_oos_max;         /* tayal-lite: padded out-of-sample extent */
    const int32_t *T;          /* [N] lengths 1..T_max; NULL: every series has T_max */
    const int32_t *x_int;      /* [N, T_max] int<lower=1,upper=L> x[T] */
    const double  *x_real;     /* [N, T_max] real x[T] / x_t[T] */
    const int32_t *g;          /* [N, T_max] semisup group 1..G */
    const int32_t *sign;       /* [N, T_max] tayal sign 1 = up, 2 = down */
    const double  *u;          /* [N, T_max, M] iohmm inputs u_tm */
    const int32_t *T_oos;      /* [N] tayal-lite out-of-sample lengths; NULL: T_oos_max */
    const int32_t *x_oos;      /* [N, T_oos_max] */
    const int32_t *sign_oos;   /* [N, T_oos_max] */
    const double  *hyperparams;/* [9] iohmm-hmix priors: read by no path output (model block only) */
} hhmm_data;

/* The `parameters` block for S draws, as rstan::extract() returns it (S fastest). */
typedef struct hhmm_draws {
    int64_t n_draws;           /* S */
    const double *p_1k;        /* [S, K] simplex */
    const double *A_ij;        /* [S, K, K] A_ij[i][j] = p(z_t = j | z_{t-1} = i) */
    const double *phi_k;       /* [S, K, L] simplex rows */
    const double *mu_k;        /* [S, K] hmm.stan */
    const double *sigma_k;     /* [S, K] hmm.stan */
    const double *w_km;        /* [S, K, M] iohmm state regressors */
    const double *b_km;        /* [S, K, M] iohmm-reg mean regressors */
    const double *s_k;         /* [S, K] iohmm-reg residual sd */
    const double *lambda_kl;   /* [S, K, L] iohmm-mix component weights */
    const double *mu_kl;       /* [S, K, L] iohmm-mix component means */
    const double *s_kl;        /* [S, K, L] iohmm-mix component sds */
    const double *p_11;        /* [S] tayal */
    const double *A_row;       /* [S, 2, 2] tayal A_row[r][c] at s + S*(r + 2*c) */
} hhmm_draws;

/* Request flags (hhmm_request.flags).  Forward/backward over long series with
 * few pairs runs as a parallel scan over T (T-chunks per pair: chunk transfer
 * products, a scan over chunk boundaries, then per-chunk sweeps).  AUTO picks
 * it when the batch has too few pairs to fill the GPU; FFBS always runs
 * sequentially (the draws chain across the whole series). */
#define HHMM_FLAG_SCAN_AUTO 0u
#define HHMM_FLAG_SCAN_FORCE (1u << 0)
#define HHMM_FLAG_SCAN_OFF (1u << 1)
#define HHMM_FLAG_SCAN_CHUNK_LOG2(n) ((uint32_t)(n) << 8) /* T-chunk length 2^n (0 = automatic) */
/* With the forward-backward and Viterbi outputs both requested, the Viterbi
 * pass runs on a library side stream forked from the caller's stream and
 * joined back into it (the call's semantics are unchanged); this flag runs
 * both passes on the caller's stream, one after the other. */
#define HHMM_FLAG_NO_FUSE (1u << 2)
/* Layout of the per-pair recursions at K = 2..4: by default batches below
 * 131072 pairs run one lane per (pair, state), larger ones one lane per pair;
 * results are bit-identical either way.  These force one or the other.  They
 * apply to the HMM-family Viterbi and to the IOHMM sweep's loglik / alpha /
 * gamma / FFBS profile. */
#define HHMM_FLAG_VIT_LANES (1u << 3)
#define HHMM_FLAG_VIT_STATES (1u << 4)
/* hmm-multinom at K = 4 with gamma_tk (+ loglik) and zstar_t / logp_zstar in one
 * request (the C2 profile, lane decoder): run both halves as ONE fused sweep
 * over a single pass of x instead of two concurrent kernels (identical
 * results).  Measured slower on MI355X (C2: 11.3 against 10.4 ms; both
 * emission tables in LDS hold the fused kernel at one wave per SIMD), so the
 * two-kernel schedule is the default. */
#define HHMM_FLAG_FUSED (1u << 5)
/* Viterbi over T in parallel (HMM family, K = 2 or 4): a batch
 * of few pairs with long series decodes T-chunks in parallel and stays
 * bit-identical to the sequential decoders -- inside a chunk whose values keep
 * one binary exponent, Stan's rounded max-plus recursion is exact integer
 * max-plus on that exponent's grid, so chunk products compose exactly; the
 * chunks that cross an exponent are decoded sequentially, and every chunk is
 * replayed from its exact entry vector and checked (a pair failing the check
 * is decoded again by the sequential decoder).  AUTO picks it below 2048
 * pairs with T >= 16384; VIT_SCAN forces it, VIT_SCAN_OFF forbids it. */
#define HHMM_FLAG_VIT_SCAN (1u << 6)
#define HHMM_FLAG_VIT_SCAN_OFF (1u << 7)
/* The C2 profile (hmm-multinom, K = 4, gamma_tk (+ loglik) with zstar_t /
 * logp_zstar, lane decoder) as three launches: the forward sweep, then the
 * backward sweep beside a Viterbi that reads the forward sweep's packed
 * symbols instead of x (identical results). */
#define HHMM_FLAG_FB_SPLIT (1u << 16)
/* Opt-in: K > 8 under GRID pairing with at least 16 series per draw
 * (hmm-multinom, loglik / gamma_tk): the forward-backward on the matrix cores
 * (the series under one draw share its A, so a step of 16 of them is a dense
 * product).  Measured 3x slower than the state-parallel VALU
 * kernels at N1 (117 vs 41 ms): a wave's 16 series write gamma at a stride of
 * S pairs, so every store is a partial line.  Off by default. */
#define HHMM_FLAG_LKM_MFMA (1u << 17)
/* The C2 profile (hmm-multinom, K = 4, gamma_tk (+ loglik) with zstar_t, lane
 * decoder) as one phased sweep per pair: the Viterbi over x (packing the
 * symbols), then the forward-backward over the packed symbols with the
 * backtrack in its backward sweep (identical results). */
#define HHMM_FLAG_VFB (1u << 18)
/* Forbids the phased sweep where it is the default (the C2 request then runs
 * fb_kernel beside viterbi_kernel on the library's side stream). */
#define HHMM_FLAG_VFB_OFF (1u << 19)
/* hhmm_run only (host arrays): the number of chunks its host pipeline splits a
 * device's share of the request into (0 = automatic: about 512 MB of staged
 * traffic per chunk, at least 16384 pairs each).  Chunk i+1's upload and
 * kernels overlap chunk i's download through pinned staging buffers.  The
 * pipeline chunks only a request that runs no parallel scan over T (it then
 * pins SCAN_OFF / VIT_SCAN_OFF on the chunks), so the outputs are those of one
 * device call on the whole request. */
#define HHMM_FLAG_HOST_CHUNKS(n) ((uint32_t)((n) & 0xff) << 20)

typedef struct hhmm_request {
    uint32_t abi_version;      /* HHMM_ABI_VERSION */
    int32_t model;             /* hhmm_model */
    int32_t pairing;           /* hhmm_pairing */
    uint32_t outputs;          /* HHMM_OUT_* */
    hhmm_data data;
    hhmm_draws draws;
    const double *ffbs_u;      /* [P, T_max] uniforms in (0,1) for HHMM_OUT_FFBS */
    int32_t device;            /* HIP device ordinal for hhmm_run; -1 = current; HHMM_DEVICE_SET = the set */
    int32_t flags;             /* HHMM_FLAG_* (0 = defaults) */
    const double *hat_rand;    /* [P, T_max, 3] for HHMM_OUT_HATZ/HATL/HATX: uniform (hatz),
                                * uniform (hatl), standard normal (hatx) at p + P*(t + T_max*c) */
} hhmm_request;

/* Caller-allocated outputs; a pointer may be NULL when its bit is not requested. */
typedef struct hhmm_result {
    double  *loglik;           /* [P] */
    double  *unalpha_tk;       /* [P, T_max, K] */
    double  *alpha_tk;         /* [P, T_max, K] */
    double  *unbeta_tk;        /* [P, T_max, K] */
    double  *beta_tk;          /* [P, T_max, K] */
    double  *ungamma_tk;       /* [P, T_max, K] */
    double  *gamma_tk;         /* [P, T_max, K] */
    int32_t *zstar_t;          /* [P, T_max]; tayal-lite: [P, T_oos_max] */
    double  *logp_zstar;       /* [P] */
    double  *oblik_tk;         /* [P, T_max, K] */
    double  *oblik_t;          /* [P, T_max] */
    int32_t *z_ffbs;           /* [P, T_max] */
    double  *alpha_tk_oos;     /* [P, T_oos_max, K] */
    double  *unalpha_tk_oos;   /* [P, T_oos_max, K] */
    double  *logA_ij;          /* [P, T_max, K] */
    int32_t *pair_status;      /* [P] optional */
    double  *hatpi_tk;         /* [P, T_max, K] */
    int32_t *hatz_t;           /* [P, T_max] */
    int32_t *hatl_t;           /* [P, T_max] */
    double  *hatx_t;           /* [P, T_max] */
} hhmm_result;

/* Library identity, e.g. "hhmm-mi355x 0.1.0 gfx950 abi 1". */
const char *hhmm_version(void);

/* Message of the last non-OK status returned on this thread ("" if none). */
const char *hhmm_last_error(void);

/* Number of pairs the request describes (N*S for GRID, N for ZIP), or -1. */
int64_t hhmm_num_pairs(const hhmm_request *req);

/* Checks a request (dims, pointers for the requested outputs, index ranges on
 * host data).  hhmm_run calls it; exposed for the R shim and tests. */
hhmm_status hhmm_validate(const hhmm_request *req, const hhmm_result *res, int host_pointers);

/* hhmm_request.device: shard the request over the device set, one host thread
 * per device; each writes its slice of the caller's outputs (hhmm_run only). */
#define HHMM_DEVICE_SET (-2)

/* Explicit init: verifies that ndev gfx950 devices are visible and makes
 * devices 0 .. ndev-1 the device set. */
hhmm_status hhmm_init(int ndev);

/* The device set as explicit ordinals (a device may repeat: two shards on one
 * GPU run in two threads).  Replaces the set hhmm_init made. */
hhmm_status hhmm_init_devices(const int32_t *ordinals, int n);

/* Writes up to `capacity` ordinals of the device set; returns its size. */
int hhmm_device_set(int32_t *ordinals, int capacity);

/* Releases the device pool (R finaliser / process exit). */
hhmm_status hhmm_shutdown(void);

/* Host-pointer entry (the R .Call path): uploads, runs on request->device,
 * downloads, synchronises.  Replaces rstan write_array over all pairs. */
hhmm_status hhmm_run(const hhmm_request *req, hhmm_result *res);

/* Device-resident entry: every pointer in req/res is a device pointer on the
 * current HIP device; enqueues on `stream` (hipStream_t, NULL = default) and
 * returns without synchronising.  `workspace` must hold
 * hhmm_workspace_size() bytes.  Per-pair failures land in res->pair_status,
 * among them the data-block bounds hhmm_run checks on the host: a pair whose
 * series breaks one is flagged HHMM_PAIR_INVALID_DATA (when pair_status is
 * given), every other pair is unaffected. */
hhmm_status hhmm_workspace_size(const hhmm_request *req, size_t *bytes);
hhmm_status hhmm_run_device(const hhmm_request *req, hhmm_result *res,
                            void *workspace, size_t workspace_bytes, void *stream);

/* ---- One series split over ranks along T -----------------
 * A rank holds one time window [t0, t1) of every pair's series: the request's
 * data arrays hold the window's steps only ([N, T_window], T = NULL: every
 * series spans the whole window), and its scan runs in two calls on the same
 * workspace (hhmm_segment_workspace_size) and stream:
 *   hhmm_segment_summary_device  the window's chunk products (the T-scan's
 *       phase 1) and their ordered products: per pair the forward product SF
 *       (K x K, row vector times SF maps the state entering the window to the
 *       state leaving it; the first window's rows all hold the state leaving
 *       it), the backward product SQ (SQ times beta leaving the window is
 *       beta entering it), their power-of-two exponents and the Gaussian log
 *       scale: summary[p + P*f], f = 0 .. 2K^2 + 2 in the order
 *       SF (row-major), SQ (row-major), SF exponent, log scale, SQ exponent.
 *   hhmm_segment_finish_device  given the forward state entering the window
 *       (`enter`, [P, K + 1]: K probabilities up to scale, then their log
 *       scale; unused for the first window) and beta leaving it (`leave`,
 *       likewise; unused for the last window), the scan's phases 2 and 3:
 *       loglik (last window only), alpha_tk, beta_tk, ungamma_tk, gamma_tk of
 *       the window's steps.
 * The caller all-gathers the ranks' summaries (K x K per pair: 2K^2 + 3
 * doubles) and chains them (hhmm_amd.segment.boundaries; dist.gqs_tsplit).
 * HMM family at K <= 8 (hmm, hmm-multinom, semisup, tayal) and hmm /
 * hmm-multinom at 8 < K <= 32 (the flattened-HHMM state spaces: SF = SQ, its
 * chunk products on the matrix cores); the Viterbi and FFBS stay sequential
 * per pair (no segment form). */
typedef struct hhmm_segment {
    int32_t first;           /* the window starts at the series' first step */
    int32_t last;            /* the window ends at the series' last step */
    double *summary;         /* summary call: [P, 2K^2 + 3] out */
    const double *enter;     /* finish call, first = 0: [P, K + 1] */
    const double *leave;     /* finish call, last = 0: [P, K + 1] */
} hhmm_segment;

hhmm_status hhmm_segment_workspace_size(const hhmm_request *req, size_t *bytes);
hhmm_status hhmm_segment_summary_device(const hhmm_request *req, const hhmm_segment *seg, void *workspace,
                                        size_t workspace_bytes, void *stream);
hhmm_status hhmm_segment_finish_device(const hhmm_request *req, hhmm_result *res, const hhmm_segment *seg,
                                       void *workspace, size_t workspace_bytes, void *stream);

/* Self-test hooks: the device's correctly rounded log / exp over n host
 * doubles (the transcendentals every exact Viterbi input goes through), and
 * the deterministic log / exp of the FFBS contract (hhmm_detmath.h). */
hhmm_status hhmm_selftest_cr_log(const double *in, double *out, int64_t n);
hhmm_status hhmm_selftest_cr_exp(const double *in, double *out, int64_t n);
hhmm_status hhmm_selftest_det_log(const double *in, double *out, int64_t n);
hhmm_status hhmm_selftest_det_exp(const double *in, double *out, int64_t n);

/* Host-only self-test of the device-set sharding (HHMM_DEVICE_SET; no GPU
 * used): splits the request over `nshards` shards exactly as hhmm_run does,
 * moves every input array's slices into packed shard buffers and back, and
 * adds 1 to every element of every requested output through the same slice
 * copies.  A caller that zero-fills the outputs then finds each element equal
 * to 1 iff the shards cover every output element exactly once (driven under
 * host ASan / UBSan by tools/sanitize.sh). */
hhmm_status hhmm_selftest_shards(const hhmm_request *req, hhmm_result *res, int nshards);

/* Host-only self-test of hhmm_run's host pipeline (no GPU used): every
 * device shard split into `nchunks` chunks exactly as hhmm_run splits it, each
 * chunk staged through a host "slot" with the pipeline's own layout and
 * copies (the gather checked byte for byte against a row-by-row pack), every
 * output element + 1 and every pair status 1 in the slot, then scattered into
 * the caller's arrays.  Zero-filled outputs end at 1 iff the chunks cover
 * every element exactly once. */
hhmm_status hhmm_selftest_pipeline(const hhmm_request *req, hhmm_result *res, int nshards, int nchunks);

#ifdef __cplusplus
}
#endif

#endif /* HHMM_H */
