/*
 * hhmm_kernels.hip -- host-side launch plumbing of libhhmm.so: workspace
 * sizing and carving, request -> DevArgs, per-model dispatch to the
 * translation units that instantiate the kernels (hhmm_m_*.hip for the HMM
 * family, hhmm_iohmm*.hip for the IOHMM family), and the device self-test of
 * the correctly rounded log.
 */
#include <hip/hip_runtime.h>
#include <string.h>

#include <stdio.h>

#include "hhmm_device.h"

namespace hhmm {

constexpr int kIoLmax = 8; /* mixture components per state on the IOHMM device path (hhmm_iohmm.h) */

bool iohmm_supported(int K, int M, int L, char *why, size_t why_len)
{
    if (K < 1 || K > kMaxK) {
        snprintf(why, why_len, "IOHMM device path supports K = 1..%d (got %d)", kMaxK, K);
        return false;
    }
    if (M < 1 || M > 8) {
        snprintf(why, why_len, "IOHMM device path supports M = 1..8 (got %d)", M);
        return false;
    }
    if (L > kIoLmax) {
        snprintf(why, why_len, "IOHMM mixture device path supports L <= %d (got %d)", kIoLmax, L);
        return false;
    }
    return true;
}

hhmm_status launch_iohmm(const DevArgs &a, hipStream_t st)
{
    char why[160];
    if (!iohmm_supported(a.K, a.M, a.model == HHMM_MODEL_IOHMM_REG ? 1 : a.L, why, sizeof(why))) {
        set_error("%s", why);
        return HHMM_ERR_UNSUPPORTED;
    }
    const bool lo = a.K <= 4;
    if (a.model == HHMM_MODEL_IOHMM_REG)
        return lo ? run_io_reg_lo(a, st) : run_io_reg_hi(a, st);
    return lo ? run_io_mix_lo(a, st) : run_io_mix_hi(a, st);
}


/* ------------------------------------------------------------------ */
/* Self-test kernel                                                       */
/* ------------------------------------------------------------------ */
__global__ void cr_math_kernel(const double *in, double *out, int64_t n, int which)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = which == 0 ? dev_cr_log(in[i])
                 : which == 1 ? dev_cr_exp(in[i])
                 : which == 2 ? hhmm_det_log(in[i])
                              : hhmm_det_exp(in[i]);
}


/* ------------------------------------------------------------------ */
/* Workspace                                                              */
/* ------------------------------------------------------------------ */


static bool needs_ckpt(int model, uint32_t out)
{
    const bool hmm_bwd = model == HHMM_MODEL_HMM_GAUSS || model == HHMM_MODEL_HMM_MULTINOM ||
                         model == HHMM_MODEL_HMM_MULTINOM_SEMISUP || model == HHMM_MODEL_TAYAL;
    return hmm_bwd &&
           (out & (HHMM_OUT_UNBETA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA | HHMM_OUT_FFBS)) != 0;
}

static bool is_iohmm_model(int model)
{
    return model == HHMM_MODEL_IOHMM_REG || model == HHMM_MODEL_IOHMM_MIX || model == HHMM_MODEL_IOHMM_HMIX ||
           model == HHMM_MODEL_IOHMM_HMIX_LITE;
}

static int nchunk_of(int K, int T) { return (T + fb_chunk(K) - 1) / fb_chunk(K); }
static int nword_of(int K, int T) { return T / bp_steps_per_word(K) + 1; }

/* K > kMaxK (hhmm_large.h): 8-step checkpoints [rows][K][P], one back-pointer
 * byte per (pair, state, t) in rows of T_max rounded up to 16 */
static bool large_k(int K) { return K > kMaxK; }

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

/* Parallel scan over T for the HMM-family forward-backward:
 * used when a batch has too few pairs to fill the chip with one lane per
 * pair.  The T-chunk length targets ~512k (pair, chunk) lanes. */
ScanPlan scan_plan(int model, int K, int Tmax, int64_t P, uint32_t outputs, uint32_t flags)
{
    ScanPlan sp{0, 0};
    const bool family = model == HHMM_MODEL_HMM_GAUSS || model == HHMM_MODEL_HMM_MULTINOM ||
                        model == HHMM_MODEL_HMM_MULTINOM_SEMISUP || model == HHMM_MODEL_TAYAL;
    const uint32_t fb_out = HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_ALPHA | HHMM_OUT_UNBETA | HHMM_OUT_BETA |
                            HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA;
    /* the log-scale outputs run the sequential log-space recursion (hhmm_hmm.h) */
    if (!family || (flags & HHMM_FLAG_SCAN_OFF) ||
        (outputs & (HHMM_OUT_FFBS | HHMM_OUT_UNALPHA | HHMM_OUT_UNBETA)) || !(outputs & fb_out))
        return sp;
    const int log2cl = (int)((flags >> 8) & 0xffu);
    if (K > kMaxK) {
        /* large K (hhmm_lkscan.h): hmm-multinom and hmm; chunks a multiple of the
         * 32-step observation blocks; automatic when the batch is under 4096
         * pairs (2048 waves of two groups: two per SIMD) and long, with about
         * 128k (pair, chunk) groups for the chunks' sweeps.  At N2 (250 pairs x
         * T = 10^6) that is 2048-step chunks: 223.4 ms against 228.2 for 4096
         * and 226.0 for 1024, and lk_fb_kernel writes 55.7 GB against 68.1
         * (1024: 53.6) for 46 GB of gamma + 5.75 GB of checkpoints: a 128-byte
         * line of a gamma row is written by several waves, whose stores meet in
         * L2 less often the longer the chunks (profiles/r04r_n2_chunks.txt) */
        if ((model != HHMM_MODEL_HMM_MULTINOM && model != HHMM_MODEL_HMM_GAUSS) || K > kMaxKLarge)
            return sp;
        if (!(flags & HHMM_FLAG_SCAN_FORCE) && !(P < 4096 && Tmax >= 8192))
            return sp;
        int cl = 256;
        if (log2cl > 0) {
            cl = max(32, 1 << log2cl);
        } else {
            while ((int64_t)P * ((Tmax + cl - 1) / cl) > 131072 && cl < (1 << 20))
                cl *= 2;
        }
        cl = (cl + 31) & ~31;
        sp.cl = cl;
        sp.nc = (Tmax + cl - 1) / cl;
        return sp;
    }
    const int C = fb_chunk(K);
    /* a batch of under 16384 pairs (256 waves: a quarter of the chip's SIMDs)
     * is latency-bound on its T sequential steps already at T of a few hundred:
     * chunks of 4 C steps (C1, 1000 pairs x T = 500: 0.32 -> 0.10 ms), grown
     * until about 512k (pair, chunk) lanes.  At C5 (250 pairs x T = 10^6, the
     * V-scan on the high-priority side stream) that is 512-step chunks: once
     * the V-scan's tie chunks left its grid pass (round 6) the forward-backward
     * chain was the longer one, and 512 measured 6.85 / 7.50 ms against 7.96 /
     * 7.94 for 128, 7.19 for 256, 8.18 for 1024 (two boxes,
     * profiles/r06w_ab_c5_fb_chunks*.log).  Before it, 128 had been best
     * (9.80 ms against 10.22 for 256, profiles/r04l_ab_c5_rn4_chunks.log). */
    const bool small = P < 16384 && Tmax >= 256;
    int cl;
    if (log2cl > 0) {
        cl = 1 << log2cl;
    } else if (small) {
        cl = 4 * C;
        while ((int64_t)P * ((Tmax + cl - 1) / cl) > 524288 && cl < 65536)
            cl *= 2;
    } else {
        const int64_t want = (int64_t)Tmax * P / 524288;
        cl = 8 * C;
        while (cl < want && cl < 65536)
            cl *= 2;
    }
    if (cl < C)
        cl = C;
    cl -= cl % C;
    const int nc = (Tmax + cl - 1) / cl;
    if (!(flags & HHMM_FLAG_SCAN_FORCE) && !small && (P >= 131072 || Tmax < 16384 || nc < 4))
        return sp;
    if (!(flags & HHMM_FLAG_SCAN_FORCE) && nc < 4)
        return sp;
    if (scan_lanes_per_chunk(P) * nc >= (int64_t(1) << 29)) /* checkpoint columns are 32-bit byte offsets */
        return sp;
    sp.cl = cl;
    sp.nc = nc;
    return sp;
}

int lkm_plan(int model, int K, int64_t N, int pairing, uint32_t outputs, uint32_t flags, int scan_cl)
{
    const uint32_t fb = HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_ALPHA | HHMM_OUT_UNBETA | HHMM_OUT_BETA |
                        HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA;
    if (model != HHMM_MODEL_HMM_MULTINOM || K <= kMaxK || K > kMaxKLarge || pairing != HHMM_PAIR_GRID || N < 16 ||
        scan_cl > 0 || !(flags & HHMM_FLAG_LKM_MFMA) || !(outputs & fb) ||
        (outputs & fb & ~(HHMM_OUT_LOGLIK | HHMM_OUT_GAMMA)))
        return 0;
    return K <= 16 ? 4 : (K <= 24 ? 6 : 8);
}

int vscan_chunks(int model, int K, int Tv, int64_t P, uint32_t outputs, uint32_t flags)
{
    const bool family = model == HHMM_MODEL_HMM_GAUSS || model == HHMM_MODEL_HMM_MULTINOM ||
                        model == HHMM_MODEL_HMM_MULTINOM_SEMISUP || model == HHMM_MODEL_TAYAL ||
                        model == HHMM_MODEL_TAYAL_LITE;
    if (!family || !(K == 2 || K == 4) || !(outputs & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR)) ||
        (flags & (HHMM_FLAG_VIT_SCAN_OFF | HHMM_FLAG_VIT_LANES | HHMM_FLAG_VIT_STATES)))
        return 0;
    if (!(flags & HHMM_FLAG_VIT_SCAN) && (P >= 2048 || Tv < 16384))
        return 0;
    const int64_t nc = (Tv + kVsChunk - 1) / kVsChunk;
    if (nc * P * K * K >= (int64_t(1) << 31)) /* 32-bit element offsets of the chunk products */
        return 0;
    return (int)nc;
}

/* Offsets of every workspace region (SIZE_MAX = unused) and the total. */
struct WsLayout {
    size_t ckpt, ckpt_ls, xpk, rnw, bp, lam, ior, mf, qb, mx, st, sl, be, bl, total;
    size_t vm, vm1, vd, vk, ve, vz, vf, vt;
    size_t dc; /* [N] int32 data-check flags (the device entry) */
    int vnc;
    ScanPlan sp;
};

static WsLayout ws_layout(int model, int K, int L, int Tmax, int Toos, int64_t P, uint32_t outputs, uint32_t flags,
                          int64_t N, int pairing)
{
    WsLayout w;
    const size_t NONE = SIZE_MAX;
    w.ckpt = w.ckpt_ls = w.xpk = w.rnw = w.bp = w.lam = w.ior = w.mf = w.qb = w.mx = w.st = w.sl = w.be = w.bl = NONE;
    w.vm = w.vm1 = w.vd = w.vk = w.ve = w.vz = w.vf = w.vt = NONE;
    w.vnc = 0;
    w.dc = NONE;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align256(bytes);
        return o;
    };
    const size_t d = sizeof(double);
    w.sp = scan_plan(model, K, Tmax, P, outputs, flags);
    if (large_k(K)) {
        if (w.sp.cl > 0) {
            /* hhmm_lkscan.h: chunk products [P][nc][K][K] and row exponents
             * [P][nc][K]; entry states, their log scales and exit betas per
             * (pair, chunk); the chunks' sweeps' checkpoints [rows][K][P * nc] */
            const size_t nc = (size_t)w.sp.nc, Q = (size_t)P * nc;
            w.mf = take(Q * K * K * d);
            w.mx = take(Q * K * d);
            w.st = take(Q * K * d);
            w.sl = take(Q * d);
            w.be = take(Q * K * d);
            w.bl = take(Q * d); /* hmm.stan: each chunk's Gaussian log scale */
            if (needs_ckpt(model, outputs))
                w.ckpt = take((size_t)((w.sp.cl + 7) / 8) * K * Q * d);
        } else if (lkm_plan(model, K, N, pairing, outputs, flags, 0) && needs_ckpt(model, outputs)) {
            /* lkm_fb_kernel: [wave][chunk][KSM][64] per (draw, 16-series tile) */
            const size_t ksm = (size_t)lkm_plan(model, K, N, pairing, outputs, flags, 0);
            w.ckpt = take((size_t)(P / N) * (size_t)((N + 15) / 16) * ((Tmax + 7) / 8) * ksm * 64 * d);
        } else if (needs_ckpt(model, outputs)) {
            w.ckpt = take((size_t)((Tmax + 7) / 8) * K * P * d);
        }
        if (outputs & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR))
            w.bp = take((size_t)P * K * (size_t)((Tmax + 15) & ~15));
        if (is_iohmm_model(model) && (outputs & HHMM_OUT_UNBETA))
            w.lam = take((size_t)Tmax * P * d);
        if (is_iohmm_model(model) && (outputs & kIoFilt))
            w.ior = take((size_t)(1 + P) * sizeof(int32_t));
        w.dc = take((size_t)N * sizeof(int32_t));
        w.total = off + 256;
        return w;
    }
    if (w.sp.cl > 0) {
        /* phase-3 checkpoint columns: one per (pair rounded up to whole waves, chunk) */
        const size_t nc = (size_t)w.sp.nc, G = (size_t)scan_lanes_per_chunk(P) * nc,
                     rows = (size_t)(w.sp.cl / fb_chunk(K));
        w.ckpt = take(rows * K * G * d);
        w.ckpt_ls = take(rows * G * d);
        w.mf = take(nc * K * K * P * d);
        w.qb = take(nc * K * K * P * d);
        w.mx = take(nc * 3 * P * d);
        w.st = take(nc * K * P * d);
        w.sl = take(nc * P * d);
        w.be = take(nc * K * P * d);
        w.bl = take(nc * P * d);
    } else if (needs_ckpt(model, outputs)) {
        w.ckpt = take((size_t)nchunk_of(K, Tmax) * K * P * d);
        w.ckpt_ls = take((size_t)nchunk_of(K, Tmax) * P * d);
        /* hot profile of hmm-multinom: symbols repacked 4 bits each for the backward sweep */
        const uint32_t extra = HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA | HHMM_OUT_BETA | HHMM_OUT_UNBETA | HHMM_OUT_UNGAMMA;
        if (model == HHMM_MODEL_HMM_MULTINOM && L <= 16 && !(outputs & extra))
            /* ceil(T/8) words (8-step chunks, 1 word each) or ceil(T/32) * 4
             * (32-step chunks of the two-level recompute): at most T/8 + 4 */
        {
            w.xpk = take(((size_t)nchunk_of(K, Tmax) + 4) * P * sizeof(uint32_t));
            w.rnw = take(((size_t)P / 64 + 64) * sizeof(int32_t)); /* one flag per fb_kernel wave */
        }
    }
    if (outputs & (HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR)) {
        const int Tv = (model == HHMM_MODEL_TAYAL_LITE) ? Toos : Tmax;
        w.bp = take((size_t)nword_of(K, Tv) * P * sizeof(uint32_t));
        w.vnc = vscan_chunks(model, K, Tv, P, outputs, flags);
        if (w.vnc > 0) {
            const size_t nc = (size_t)w.vnc;
            w.vm = take(nc * K * K * P * d);
            w.vm1 = take(nc * K * K * P * d);
            w.vd = take((nc + 1) * K * P * d);
            w.vk = take(nc * P * sizeof(int32_t));
            w.ve = take(nc * P * sizeof(uint32_t));
            w.vz = take(nc * P * sizeof(int32_t));
            w.vf = take(P * sizeof(int32_t));
            w.vt = take((1 + nc * P) * sizeof(int32_t));
        }
    }
    if (is_iohmm_model(model) && (outputs & HHMM_OUT_UNBETA))
        w.lam = take((size_t)Tmax * P * d);
    if (is_iohmm_model(model) && (outputs & kIoFilt))
        w.ior = take((size_t)(1 + P) * sizeof(int32_t));
    w.dc = take((size_t)N * sizeof(int32_t));
    w.total = off + 256;
    return w;
}

size_t workspace_bytes(int model, int K, int L, int Tmax, int Toos, int64_t P, uint32_t outputs, uint32_t flags,
                       int64_t N, int pairing)
{
    return ws_layout(model, K, L, Tmax, Toos, P, outputs, flags, N, pairing).total;
}

void bind_workspace(DevArgs &a, void *ws, int Tmax, int Toos, uint32_t flags)
{
    char *b = (char *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    const WsLayout w = ws_layout(a.model, a.K, a.L, Tmax, Toos, a.P, a.outputs, flags, a.N, a.pairing);
    auto at_off = [&](size_t o) -> void * { return o == SIZE_MAX ? nullptr : (void *)(b + o); };
    a.ckpt = (double *)at_off(w.ckpt);
    a.ckpt_ls = (double *)at_off(w.ckpt_ls);
    a.xpk = (uint32_t *)at_off(w.xpk);
    a.rnw = (int32_t *)at_off(w.rnw);
    a.bp = (uint32_t *)at_off(w.bp);
    a.lam = (double *)at_off(w.lam);
    a.io_redo = (int32_t *)at_off(w.ior);
    a.scan_cl = w.sp.cl;
    a.scan_nc = w.sp.nc;
    a.sc_mf = (double *)at_off(w.mf);
    a.sc_qb = (double *)at_off(w.qb);
    a.sc_mx = (double *)at_off(w.mx);
    a.sc_st = (double *)at_off(w.st);
    a.sc_sl = (double *)at_off(w.sl);
    a.sc_be = (double *)at_off(w.be);
    a.sc_bl = (double *)at_off(w.bl);
    a.vs_nc = w.vnc;
    a.vs_m = (double *)at_off(w.vm);
    a.vs_m1 = (double *)at_off(w.vm1);
    a.vs_d = (double *)at_off(w.vd);
    a.vs_k = (int32_t *)at_off(w.vk);
    a.vs_e = (uint32_t *)at_off(w.ve);
    a.vs_z = (int32_t *)at_off(w.vz);
    a.vs_fail = (int32_t *)at_off(w.vf);
    a.vs_tl = (int32_t *)at_off(w.vt);
    a.dc_flag = (int32_t *)at_off(w.dc);
}

DevArgs make_args(const hhmm_request *req, const hhmm_result *res, int64_t P)
{
    DevArgs a;
    memset(&a, 0, sizeof(a));
    const hhmm_data &d = req->data;
    const hhmm_draws &w = req->draws;
    a.P = P;
    a.N = d.n_series;
    a.S = w.n_draws;
    a.pairing = req->pairing;
    a.model = req->model;
    a.K = d.K;
    a.L = d.L > 0 ? d.L : 1;
    a.M = d.M;
    a.Tmax = d.T_max;
    a.Tout = d.T_max;
    a.outputs = req->outputs;
    a.flags = (uint32_t)req->flags;
    a.T = d.T;
    a.x = d.x_int;
    a.xr = d.x_real;
    a.g = d.g;
    a.sign = d.sign;
    a.u = d.u;
    a.p_1k = w.p_1k;
    a.A_ij = w.A_ij;
    a.phi_k = w.phi_k;
    a.mu_k = w.mu_k;
    a.sigma_k = w.sigma_k;
    a.w_km = w.w_km;
    a.b_km = w.b_km;
    a.s_k = w.s_k;
    a.lambda_kl = w.lambda_kl;
    a.mu_kl = w.mu_kl;
    a.s_kl = w.s_kl;
    a.p_11 = w.p_11;
    a.A_row = w.A_row;
    a.loglik = res->loglik;
    a.unalpha = res->unalpha_tk;
    a.alpha = res->alpha_tk;
    a.unbeta = res->unbeta_tk;
    a.beta = res->beta_tk;
    a.ungamma = res->ungamma_tk;
    a.gamma = res->gamma_tk;
    a.zstar = res->zstar_t;
    a.logp_zstar = res->logp_zstar;
    a.pair_status = res->pair_status;
    a.oblik = res->oblik_tk;
    a.oblik_t = res->oblik_t;
    a.logA = res->logA_ij;
    a.z_ffbs = res->z_ffbs;
    a.ffbs_u = req->ffbs_u;
    a.hatpi = res->hatpi_tk;
    a.hatz = res->hatz_t;
    a.hatl = res->hatl_t;
    a.hatx = res->hatx_t;
    a.hat_rand = req->hat_rand;
    return a;
}

/* ------------------------------------------------------------------ */
/* Data-block constraints on the device entry (HHMM_PAIR_INVALID_DATA)   */
/* ------------------------------------------------------------------ */
thread_local bool t_data_checked_inline = false;

constexpr int kDcSteps = 64; /* time steps per thread of data_check_kernel (per strip) */
constexpr unsigned kDcMaxStrips = 32768; /* grid.y cap: longer series loop over strips */
constexpr int kDcSeries = 4; /* series per thread (one 16-byte load per step) */

/* Flags series n when one of its steps t < T[n] breaks an int<lower=1,
 * upper=hi> bound: v (x, 1..L), w (sign 1..2 / g 1..G; null: none).  A
 * thread takes kDcSeries consecutive series (the fastest index: a wave reads
 * 1 KB of each row), strips of kDcSteps steps (strip blockIdx.y, then every
 * gridDim.y-th strip: grid.y is capped at kDcMaxStrips), 8 steps of independent
 * loads in flight (HBM-bound: the pass reads each element once).  Steps at or
 * past a series' own length are read (inside the T_max x N block) and masked.
 * A flag is a plain vector store of 1 (every writer stores the same value). */
__global__ void __launch_bounds__(256) data_check_kernel(const int32_t *v, int vhi, const int32_t *w, int whi,
                                                         const int32_t *T, int64_t N, int Tmax, int32_t *flag)
{
    const int64_t n0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kDcSeries;
    if (n0 >= N)
        return;
    const int nk = (int)min<int64_t>(kDcSeries, N - n0);
    int Tn[kDcSeries];
#pragma unroll
    for (int j = 0; j < kDcSeries; ++j) /* a length outside 1..T_max: data_mark_kernel */
        Tn[j] = j < nk ? (T ? min(max(T[n0 + j], 1), Tmax) : Tmax) : 0;
    const bool vec = nk == kDcSeries && (N % kDcSeries) == 0 && ((uintptr_t)v % 16) == 0 &&
                     (!w || ((uintptr_t)w % 16) == 0);
    bool bad[kDcSeries] = {};
    auto test = [&](int hi, int t, int j, int val) {
        bad[j] |= (t < Tn[j]) & ((uint32_t)(val - 1) >= (uint32_t)hi);
    };
    for (int64_t s0 = (int64_t)blockIdx.y * kDcSteps; s0 < Tmax; s0 += (int64_t)gridDim.y * kDcSteps) {
    const int t0 = (int)s0;
    const int t1 = min(t0 + kDcSteps, Tmax);
    if (vec) {
        auto pass = [&](const int32_t *u, int hi) {
            int t = t0;
            for (; t + 8 <= t1; t += 8) {
                int4 q[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    q[i] = *reinterpret_cast<const int4 *>(u + n0 + N * (int64_t)(t + i));
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    test(hi, t + i, 0, q[i].x);
                    test(hi, t + i, 1, q[i].y);
                    test(hi, t + i, 2, q[i].z);
                    test(hi, t + i, 3, q[i].w);
                }
            }
            for (; t < t1; ++t) {
                const int4 q = *reinterpret_cast<const int4 *>(u + n0 + N * (int64_t)t);
                test(hi, t, 0, q.x);
                test(hi, t, 1, q.y);
                test(hi, t, 2, q.z);
                test(hi, t, 3, q.w);
            }
        };
        pass(v, vhi);
        if (w)
            pass(w, whi);
    } else {
        for (int j = 0; j < nk; ++j)
            for (int t = t0; t < min(t1, Tn[j]); ++t) {
                const int64_t i = n0 + j + N * (int64_t)t;
                test(vhi, t, j, v[i]);
                if (w)
                    test(whi, t, j, w[i]);
            }
    }
    }
#pragma unroll
    for (int j = 0; j < kDcSeries; ++j)
        if (bad[j])
            flag[n0 + j] = 1;
}

/* pair_status[p] = HHMM_PAIR_INVALID_DATA for the pairs of flagged series and
 * of series whose T[n] / T_oos[n] lies outside 1..T_max / 1..T_oos_max.
 * Segment windows: the summary call has no pair_status, so a bad
 * pair's summary carries a NaN log scale (field 2K^2 + 1) instead; every rank
 * that chains it (hhmm_amd.segment.boundaries) then receives a NaN in the
 * entering state or the leaving beta, and the finish call flags the pair. */
__global__ void __launch_bounds__(256) data_mark_kernel(const DevArgs a, const int32_t *T_oos, int Toos_max)
{
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.P)
        return;
    int64_t n, d;
    pair_coords(a, p, n, d);
    bool bad = a.dc_flag[n] != 0;
    if (a.T)
        bad |= a.T[n] < 1 || a.T[n] > a.Tmax;
    if (T_oos)
        bad |= T_oos[n] < 1 || T_oos[n] > Toos_max;
    if (a.seg_phase == 1) {
        if (bad && a.seg_sum)
            a.seg_sum[p + a.P * (int64_t)(2 * a.K * a.K + 1)] = __builtin_nan("");
        return;
    }
    if (a.seg_phase == 2) {
        for (int f = 0; f <= a.K; ++f) {
            if (a.seg_nofirst && a.seg_enter)
                bad |= isnan(a.seg_enter[p + a.P * (int64_t)f]);
            if (a.seg_nolast && a.seg_leave)
                bad |= isnan(a.seg_leave[p + a.P * (int64_t)f]);
        }
    }
    if (bad)
        a.pair_status[p] = HHMM_PAIR_INVALID_DATA;
}

static hhmm_status launch_data_check(const DevArgs &a, const hhmm_request *req, hipStream_t st, bool inline_checked)
{
    const hhmm_data &d = req->data;
    const int m = req->model;
    const bool discrete = m == HHMM_MODEL_HMM_MULTINOM || m == HHMM_MODEL_HMM_MULTINOM_SEMISUP ||
                          m == HHMM_MODEL_TAYAL || m == HHMM_MODEL_TAYAL_LITE;
    const bool tayal = m == HHMM_MODEL_TAYAL || m == HHMM_MODEL_TAYAL_LITE;
    hipError_t e = hipSuccess; /* a.dc_flag cleared by launch_all before the model's kernels */
    auto check = [&](const int32_t *v, int vhi, const int32_t *w, int whi, const int32_t *T, int Tmax) {
        const int64_t thr = (d.n_series + kDcSeries - 1) / kDcSeries;
        const dim3 grid((unsigned)((thr + 255) / 256),
                        std::min((unsigned)((Tmax + kDcSteps - 1) / kDcSteps), kDcMaxStrips));
        hipLaunchKernelGGL(data_check_kernel, grid, dim3(256), 0, st, v, vhi, w, whi, T, (int64_t)d.n_series, Tmax,
                           a.dc_flag);
    };
    /* the summary call's sweeps are not the ones that check x inline */
    if (e == hipSuccess && discrete && (!inline_checked || a.seg_phase == 1))
        check(d.x_int, d.L, tayal ? d.sign : (m == HHMM_MODEL_HMM_MULTINOM_SEMISUP ? d.g : nullptr),
              tayal ? 2 : d.G, d.T, d.T_max);
    if (e == hipSuccess && m == HHMM_MODEL_TAYAL_LITE)
        check(d.x_oos, d.L, d.sign_oos, 2, d.T_oos, d.T_oos_max);
    if (e == hipSuccess)
        hipLaunchKernelGGL(data_mark_kernel, dim3((unsigned)((a.P + 255) / 256)), dim3(256), 0, st, a,
                           m == HHMM_MODEL_TAYAL_LITE ? d.T_oos : nullptr, d.T_oos_max);
    if (e == hipSuccess)
        e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("data check: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* An IOHMM sweep with its log-space fallback: the list of underflowed pairs
 * is cleared, the sweep lists them, launch_iohmm_log re-runs them (all on `st`). */
static hhmm_status run_iohmm_filtered(const DevArgs &a, hipStream_t st, hhmm_status (*sweep)(const DevArgs &, hipStream_t))
{
    if (a.io_redo && (a.outputs & kIoFilt)) {
        const hipError_t e = hipMemsetAsync(a.io_redo, 0, sizeof(int32_t), st);
        if (e != hipSuccess) {
            set_error("hipMemsetAsync: %s", hipGetErrorString(e));
            return HHMM_ERR_HIP;
        }
    }
    const hhmm_status s = sweep(a, st);
    if (s != HHMM_OK)
        return s;
    return launch_iohmm_log(a, st);
}

/* The IOHMM sweep (with its log-space fallback) for every output but the
 * fitted draws, then the fitted draws (hatpi / hatz / hatl / hatx). */
static hhmm_status run_iohmm_hat(const DevArgs &a, hipStream_t st, hhmm_status (*sweep)(const DevArgs &, hipStream_t))
{
    constexpr uint32_t kHat = HHMM_OUT_HATPI | HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX;
    hhmm_status s = HHMM_OK;
    if (a.outputs & ~kHat) {
        DevArgs b = a;
        b.outputs &= ~kHat;
        s = run_iohmm_filtered(b, st, sweep);
    }
    if (s == HHMM_OK && (a.outputs & kHat))
        s = launch_fitted(a, st);
    return s;
}

static hhmm_status launch_model(const hhmm_request *req, const DevArgs &a, const hhmm_result *res, hipStream_t st);

hhmm_status launch_all(const hhmm_request *req, const hhmm_result *res, int64_t P, void *ws, hipStream_t st,
                       const hhmm_segment *seg, int seg_phase, bool check_data)
{
    DevArgs a = make_args(req, res, P);
    bind_workspace(a, ws, req->data.T_max, req->data.T_oos_max, (uint32_t)req->flags);
    const bool check = check_data && a.dc_flag && (a.pair_status || (seg && seg_phase == 1 && seg->summary));
    if (!check)
        a.dc_flag = nullptr;
    if (seg) {
        a.seg_phase = seg_phase;
        a.seg_nofirst = !seg->first;
        a.seg_nolast = !seg->last;
        a.seg_sum = seg->summary;
        a.seg_enter = seg->enter;
        a.seg_leave = seg->leave;
        if (a.scan_cl <= 0) {
            set_error("segment: the request has no T-scan plan (HMM family, K <= 8, probability-space outputs)");
            return HHMM_ERR_UNSUPPORTED;
        }
    }
    t_data_checked_inline = false;
    if (check) { /* series flags: the inline checks of the model's sweeps, then data_check_kernel */
        const hipError_t e = hipMemsetAsync(a.dc_flag, 0, (size_t)req->data.n_series * sizeof(int32_t), st);
        if (e != hipSuccess) {
            set_error("data check: %s", hipGetErrorString(e));
            return HHMM_ERR_HIP;
        }
    }
    hhmm_status s = launch_model(req, a, res, st);
    if (s != HHMM_OK || !check)
        return s;
    return launch_data_check(a, req, st, t_data_checked_inline);
}

static hhmm_status launch_model(const hhmm_request *req, const DevArgs &a, const hhmm_result *res, hipStream_t st)
{
    const bool lo = a.K <= 4;
    if (a.K > kMaxK) {
        if (a.K > kMaxKLarge) {
            set_error("K = %d: the device path supports K <= %d", a.K, kMaxKLarge);
            return HHMM_ERR_UNSUPPORTED;
        }
        if (is_iohmm_model(req->model))
            return run_iohmm_hat(a, st, run_large_iohmm);
        if (req->model != HHMM_MODEL_HMM_GAUSS && req->model != HHMM_MODEL_HMM_MULTINOM) {
            set_error("K = %d: the device path of model %d supports K <= %d", a.K, req->model, kMaxK);
            return HHMM_ERR_UNSUPPORTED;
        }
        return run_large(a, st);
    }
    switch (req->model) {
    case HHMM_MODEL_HMM_GAUSS: return lo ? run_gauss_lo(a, req, res, st) : run_gauss_hi(a, req, res, st);
    case HHMM_MODEL_HMM_MULTINOM: return lo ? run_multinom_lo(a, req, res, st) : run_multinom_hi(a, req, res, st);
    case HHMM_MODEL_HMM_MULTINOM_SEMISUP:
        return lo ? run_semisup_lo(a, req, res, st) : run_semisup_hi(a, req, res, st);
    case HHMM_MODEL_TAYAL: return run_tayal(a, req, res, st);
    case HHMM_MODEL_TAYAL_LITE: return run_tayal_lite(a, req, res, st);
    case HHMM_MODEL_IOHMM_REG:
    case HHMM_MODEL_IOHMM_MIX:
    case HHMM_MODEL_IOHMM_HMIX:
    case HHMM_MODEL_IOHMM_HMIX_LITE:
        return run_iohmm_hat(a, st, launch_iohmm);
    default:
        set_error("model %d has no device path in this build", req->model);
        return HHMM_ERR_UNSUPPORTED;
    }
}

hhmm_status selftest_cr_math(const double *in, double *out, int64_t n, int which)
{
    double *din = nullptr, *dout = nullptr;
    const size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(double);
    if (hipMalloc(&din, bytes) != hipSuccess || hipMalloc(&dout, bytes) != hipSuccess) {
        (void)hipFree(din);
        set_error("hipMalloc failed in selftest");
        return HHMM_ERR_OUT_OF_MEMORY;
    }
    hipError_t e = hipMemcpy(din, in, (size_t)n * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess && n > 0) {
        hipLaunchKernelGGL(cr_math_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, din, dout, n, which);
        e = hipGetLastError();
    }
    if (e == hipSuccess)
        e = hipMemcpy(out, dout, (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    (void)hipFree(din);
    (void)hipFree(dout);
    if (e != hipSuccess) {
        set_error("selftest: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

} // namespace hhmm
