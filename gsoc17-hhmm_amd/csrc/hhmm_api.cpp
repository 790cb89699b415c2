/*
 * hhmm_api.cpp -- the C ABI of libhhmm.so (include/hhmm.h).
 *
 * Host side of the drop-in boundary: validates a request the way Stan's data
 * block and parameter constraints would (declared bounds such as
 * `int<lower=1, upper=L> x[T]`, hmm/stan/hmm-multinom.stan:12), sizes the
 * workspace, moves host arrays to and from the device for the R path
 * (hhmm_run), and launches the gfx950 kernels (hhmm_kernels.hip).  There is
 * no CPU compute path: without a gfx950 device every entry point fails with
 * HHMM_ERR_NO_DEVICE.
 */
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>
#include <emmintrin.h>

#include "hhmm_internal.h"
#include "build_id.h" /* HHMM_SOURCE_HASH (Makefile) */

namespace hhmm {

static thread_local std::string g_last_error;

void set_error(const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

/* ---------------- device pool (per device, size-bucketed) ---------------- */
struct Pool {
    std::mutex mu;
    std::map<int, std::multimap<size_t, void *>> free_blocks;
    std::map<void *, std::pair<int, size_t>> live;
};
static Pool &pool()
{
    static Pool p;
    return p;
}

static void *pool_get(int dev, size_t bytes)
{
    if (bytes == 0)
        bytes = 256;
    bytes = (bytes + 4095) & ~(size_t)4095;
    Pool &p = pool();
    {
        std::lock_guard<std::mutex> g(p.mu);
        auto &fb = p.free_blocks[dev];
        auto it = fb.lower_bound(bytes);
        if (it != fb.end() && it->first <= bytes + bytes / 4) {
            void *ptr = it->second;
            p.live[ptr] = {dev, it->first};
            fb.erase(it);
            return ptr;
        }
    }
    void *ptr = nullptr;
    if (hipMalloc(&ptr, bytes) != hipSuccess) {
        /* release cached blocks of this device and retry once */
        std::vector<void *> drop;
        {
            std::lock_guard<std::mutex> g(p.mu);
            for (auto &kv : p.free_blocks[dev])
                drop.push_back(kv.second);
            p.free_blocks[dev].clear();
        }
        for (void *q : drop)
            (void)hipFree(q);
        (void)hipGetLastError();
        if (hipMalloc(&ptr, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    }
    std::lock_guard<std::mutex> g(p.mu);
    p.live[ptr] = {dev, bytes};
    return ptr;
}

static void pool_put(void *ptr)
{
    if (!ptr)
        return;
    Pool &p = pool();
    std::lock_guard<std::mutex> g(p.mu);
    auto it = p.live.find(ptr);
    if (it == p.live.end())
        return;
    p.free_blocks[it->second.first].emplace(it->second.second, ptr);
    p.live.erase(it);
}

/* ---------------- side streams (one per device) ---------------- */
struct SideStreams {
    std::mutex mu;
    std::map<int, std::pair<hipStream_t, hipEvent_t>> by_dev; /* key dev * 2 + high priority: stream, fork event */
    std::map<int, hipEvent_t> join_ev;
};
static SideStreams &side_streams()
{
    static SideStreams s;
    return s;
}

hhmm_status fork_stream(hipStream_t st, hipStream_t *side)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        set_error("hipGetDevice failed");
        return HHMM_ERR_HIP;
    }
    SideStreams &ss = side_streams();
    /* The side pass (the decoder beside the forward-backward) runs on a
     * high-priority stream: at C5 its chain of V-scan kernels is the critical
     * path, and the forward-backward scan's waves fill in around it (13.37 ->
     * 12.71 ms interleaved on one box, profiles/r03s_ab_c5_side_prio.log).
     * Probe knob HHMM_PROBE_SIDE_PRIO=0: a normal-priority side stream. */
    const char *pk = probe_env("HHMM_PROBE_SIDE_PRIO");
    const int hi = (pk && pk[0] == '0') ? 0 : 1;
    const int key = dev * 2 + hi;
    std::lock_guard<std::mutex> g(ss.mu);
    auto it = ss.by_dev.find(key);
    if (it == ss.by_dev.end()) {
        hipStream_t s2 = nullptr;
        hipEvent_t ev = nullptr, ej = nullptr;
        int lo_p = 0, hi_p = 0;
        if (hi)
            (void)hipDeviceGetStreamPriorityRange(&lo_p, &hi_p);
        if (hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, hi ? hi_p : 0) != hipSuccess ||
            hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&ej, hipEventDisableTiming) != hipSuccess) {
            set_error("side stream creation failed");
            return HHMM_ERR_HIP;
        }
        it = ss.by_dev.emplace(key, std::make_pair(s2, ev)).first;
        ss.join_ev[key] = ej;
    }
    if (hipEventRecord(it->second.second, st) != hipSuccess ||
        hipStreamWaitEvent(it->second.first, it->second.second, 0) != hipSuccess) {
        set_error("stream fork failed");
        return HHMM_ERR_HIP;
    }
    *side = it->second.first;
    return HHMM_OK;
}

hhmm_status join_stream(hipStream_t st, hipStream_t side)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        set_error("hipGetDevice failed");
        return HHMM_ERR_HIP;
    }
    SideStreams &ss = side_streams();
    std::lock_guard<std::mutex> g(ss.mu);
    hipEvent_t ej = nullptr;
    for (int hi = 0; hi < 2 && !ej; ++hi) /* the side stream is the one `side` names */
        if (ss.by_dev.count(dev * 2 + hi) && ss.by_dev[dev * 2 + hi].first == side)
            ej = ss.join_ev[dev * 2 + hi];
    if (!ej || hipEventRecord(ej, side) != hipSuccess || hipStreamWaitEvent(st, ej, 0) != hipSuccess) {
        set_error("stream join failed");
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

/* Waits for a request's work: its own stream and, when this device has one,
 * the library's side stream (a failed launch can leave a forked kernel there
 * unjoined).  Other streams -- other threads' requests -- are not waited on. */
static hipError_t sync_request(hipStream_t st)
{
    hipError_t e = hipStreamSynchronize(st);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return e;
    SideStreams &ss = side_streams();
    for (int hi = 0; hi < 2; ++hi) {
        hipStream_t side = nullptr;
        {
            std::lock_guard<std::mutex> g(ss.mu);
            auto it = ss.by_dev.find(dev * 2 + hi);
            if (it != ss.by_dev.end())
                side = it->second.first;
        }
        if (side) {
            hipError_t e2 = hipStreamSynchronize(side);
            if (e == hipSuccess)
                e = e2;
        }
    }
    return e;
}

static void pool_release_all()
{
    Pool &p = pool();
    std::lock_guard<std::mutex> g(p.mu);
    for (auto &dv : p.free_blocks) {
        (void)hipSetDevice(dv.first);
        for (auto &kv : dv.second)
            (void)hipFree(kv.second);
    }
    p.free_blocks.clear();
}

/* ---------------- request description ---------------- */

static bool is_iohmm(int m)
{
    return m == HHMM_MODEL_IOHMM_REG || m == HHMM_MODEL_IOHMM_MIX || m == HHMM_MODEL_IOHMM_HMIX ||
           m == HHMM_MODEL_IOHMM_HMIX_LITE;
}
static bool is_discrete(int m)
{
    return m == HHMM_MODEL_HMM_MULTINOM || m == HHMM_MODEL_HMM_MULTINOM_SEMISUP || m == HHMM_MODEL_TAYAL ||
           m == HHMM_MODEL_TAYAL_LITE;
}

/* Outputs each Stan program declares (TP / GQ names), SURVEY.md §2.3. */
static uint32_t available_outputs(int m)
{
    const uint32_t fb = HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_ALPHA | HHMM_OUT_UNBETA | HHMM_OUT_BETA |
                        HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA | HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR;
    /* FFBS (the engine's contract, §8 A14) is offered wherever the program has
     * a forward filter over the full series and a backward pass */
    switch (m) {
    case HHMM_MODEL_HMM_GAUSS:
    case HHMM_MODEL_HMM_MULTINOM:
    case HHMM_MODEL_HMM_MULTINOM_SEMISUP:
    case HHMM_MODEL_TAYAL:
        return fb | HHMM_OUT_FFBS;
    case HHMM_MODEL_IOHMM_REG:
    case HHMM_MODEL_IOHMM_MIX:
        /* + the fitted-output GQ draws (iohmm-reg.stan:124-148; iohmm-mix.stan:133-161) */
        return fb | HHMM_OUT_OBLIK_TK | HHMM_OUT_LOGA | HHMM_OUT_FFBS | HHMM_OUT_HATPI | HHMM_OUT_HATZ |
               HHMM_OUT_HATX | (m == HHMM_MODEL_IOHMM_MIX ? HHMM_OUT_HATL : 0u);
    case HHMM_MODEL_IOHMM_HMIX: /* hatpi_tk is a local there (iohmm-hmix.stan:147) */
        return HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_ALPHA | HHMM_OUT_BETA | HHMM_OUT_GAMMA |
               HHMM_OUT_OBLIK_TK | HHMM_OUT_OBLIK_T | HHMM_OUT_LOGA | HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR |
               HHMM_OUT_FFBS | HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX;
    case HHMM_MODEL_IOHMM_HMIX_LITE:
        return HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_OBLIK_TK | HHMM_OUT_OBLIK_T | HHMM_OUT_LOGA;
    case HHMM_MODEL_TAYAL_LITE:
        return HHMM_OUT_LOGLIK | HHMM_OUT_UNALPHA | HHMM_OUT_ALPHA | HHMM_OUT_UNALPHA_OOS | HHMM_OUT_ALPHA_OOS |
               HHMM_OUT_ZSTAR | HHMM_OUT_LOGP_ZSTAR;
    default:
        return 0;
    }
}

/* Models with a gfx950 path in this build. */
static bool device_supported(int m)
{
    return m >= HHMM_MODEL_HMM_GAUSS && m <= HHMM_MODEL_TAYAL_LITE;
}

static int64_t npairs(const hhmm_request *r)
{
    if (!r)
        return -1;
    if (r->data.n_series < 1 || r->draws.n_draws < 1)
        return -1;
    if (r->pairing == HHMM_PAIR_ZIP)
        return r->data.n_series == r->draws.n_draws ? r->data.n_series : -1;
    if (r->pairing == HHMM_PAIR_GRID)
        return r->data.n_series * r->draws.n_draws;
    if (r->pairing == HHMM_PAIR_BLOCK)
        return r->draws.n_draws % r->data.n_series == 0 ? r->draws.n_draws : -1;
    return -1;
}

/* One array of the request: where it lives and how many elements. */
enum ArrayClass { SERIES = 0, DRAWS = 1, PAIRS = 2 }; /* leading (fastest) dimension N, S or P */
struct ArrayDesc {
    const void *host;
    void **dev_slot; /* field in the device copy of the request/result */
    size_t elems;
    size_t esize;
    bool output;
    int cls;         /* ArrayClass */
};

#define REQUIRE(cond, ...)                                                                          \
    do {                                                                                            \
        if (!(cond)) {                                                                              \
            set_error(__VA_ARGS__);                                                                 \
            return HHMM_ERR_INVALID_ARGUMENT;                                                       \
        }                                                                                           \
    } while (0)

/* 1 when some element v[n + N t] with t < T[n] (T null: every t < Tm) lies
 * outside [lo, hi].  Time-major, so each thread streams contiguous rows (the
 * n-major loop that names the first offender in the error message strides by
 * N and took ~0.2 s at C2-host's 2e8 symbols); threads over time ranges for
 * large arrays. */
static bool any_out_of_range(const int32_t *v, int64_t N, int Tm, const int32_t *T, int32_t lo, int32_t hi)
{
    const uint32_t span = (uint32_t)(hi - lo);
    auto rows = [&](int t0, int t1) {
        bool bad = false;
        for (int t = t0; t < t1 && !bad; ++t) {
            const int32_t *r = v + N * (int64_t)t;
            if (!T) {
                uint32_t acc = 0;
                for (int64_t n = 0; n < N; ++n)
                    acc |= (uint32_t)((uint32_t)(r[n] - lo) > span);
                bad = acc != 0;
            } else {
                for (int64_t n = 0; n < N; ++n)
                    bad |= (t < T[n]) & ((uint32_t)(r[n] - lo) > span);
            }
        }
        return bad;
    };
    const int64_t total = N * (int64_t)Tm;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nt = total < (int64_t(1) << 22) ? 1 : (int)std::min<int64_t>(std::min(16u, hw), Tm);
    if (nt <= 1)
        return rows(0, Tm);
    std::vector<char> res((size_t)nt, 0);
    auto part = [&](int i) { res[(size_t)i] = rows((int)((int64_t)Tm * i / nt), (int)((int64_t)Tm * (i + 1) / nt)); };
    std::vector<std::thread> th;
    std::vector<int> mine{0};
    for (int i = 1; i < nt; ++i) {
        try {
            th.emplace_back(part, i);
        } catch (...) { /* no exception crosses the C ABI: this thread takes the share */
            mine.push_back(i);
        }
    }
    for (int i : mine)
        part(i);
    for (auto &x : th)
        x.join();
    for (char c : res)
        if (c)
            return true;
    return false;
}

/* o == nullptr: the request side only (the segment summary call has no result). */
static hhmm_status validate_impl(const hhmm_request *r, const hhmm_result *o, bool host)
{
    REQUIRE(r, "request must be non-NULL");
    REQUIRE(r->abi_version == HHMM_ABI_VERSION, "abi_version %u != %u", r->abi_version, HHMM_ABI_VERSION);
    REQUIRE(r->model >= 1 && r->model <= 9, "unknown model id %d", r->model);
    REQUIRE(r->pairing == HHMM_PAIR_GRID || r->pairing == HHMM_PAIR_ZIP || r->pairing == HHMM_PAIR_BLOCK,
            "unknown pairing %d", r->pairing);
    const hhmm_data &d = r->data;
    const hhmm_draws &w = r->draws;
    REQUIRE(d.n_series >= 1, "n_series must be >= 1");
    REQUIRE(w.n_draws >= 1, "n_draws must be >= 1");
    REQUIRE(npairs(r) >= 1, "%s pairing needs %s (n_series %lld, n_draws %lld)",
            r->pairing == HHMM_PAIR_ZIP ? "ZIP" : "BLOCK",
            r->pairing == HHMM_PAIR_ZIP ? "n_series == n_draws" : "n_draws a multiple of n_series",
            (long long)d.n_series, (long long)w.n_draws);
    REQUIRE(d.T_max >= 1, "T_max must be >= 1 (int<lower=1> T)");
    /* kernels address rows as uniform base + 32-bit lane offset (8-byte elements) */
    REQUIRE(npairs(r) <= (int64_t(1) << 28) && d.n_series <= (int64_t(1) << 28) && w.n_draws <= (int64_t(1) << 28),
            "at most 2^28 pairs / series / draws per call (split larger batches)");
    REQUIRE(d.K >= 1, "K must be >= 1 (int<lower=1> K)");
    const int m = r->model;
    if (is_discrete(m))
        REQUIRE(d.L >= 1 && d.x_int, "model %d needs L >= 1 and x_int", m);
    if (m == HHMM_MODEL_HMM_GAUSS || is_iohmm(m))
        REQUIRE(d.x_real, "model %d needs x_real", m);
    if (is_iohmm(m))
        REQUIRE(d.M >= 1 && d.u, "IOHMM needs M >= 1 and u_tm");
    if (m == HHMM_MODEL_HMM_MULTINOM_SEMISUP)
        REQUIRE(d.G >= 1 && d.g, "semisup needs G >= 1 and g");
    if (m == HHMM_MODEL_TAYAL || m == HHMM_MODEL_TAYAL_LITE) {
        REQUIRE(d.K == 4, "the Tayal model is the K = 4 flattened HHMM (got K = %d)", d.K);
        REQUIRE(d.sign && w.p_11 && w.A_row && w.phi_k, "tayal needs sign, p_11, A_row, phi_k");
    }
    if (m == HHMM_MODEL_TAYAL_LITE)
        REQUIRE(d.T_oos_max >= 1 && d.x_oos && d.sign_oos, "tayal-lite needs T_oos_max, x_oos, sign_oos");
    if (m == HHMM_MODEL_HMM_GAUSS)
        REQUIRE(w.p_1k && w.A_ij && w.mu_k && w.sigma_k, "hmm-gauss needs p_1k, A_ij, mu_k, sigma_k");
    if (m == HHMM_MODEL_HMM_MULTINOM || m == HHMM_MODEL_HMM_MULTINOM_SEMISUP)
        REQUIRE(w.p_1k && w.A_ij && w.phi_k, "multinomial HMM needs p_1k, A_ij, phi_k");
    if (m == HHMM_MODEL_IOHMM_REG)
        REQUIRE(w.p_1k && w.w_km && w.b_km && w.s_k, "iohmm-reg needs p_1k, w_km, b_km, s_k");
    if (m == HHMM_MODEL_IOHMM_MIX || m == HHMM_MODEL_IOHMM_HMIX || m == HHMM_MODEL_IOHMM_HMIX_LITE)
        REQUIRE(d.L >= 1 && w.p_1k && w.w_km && w.lambda_kl && w.mu_kl && w.s_kl,
                "iohmm-mix needs L, p_1k, w_km, lambda_kl, mu_kl, s_kl");

    const uint32_t avail = available_outputs(m);
    REQUIRE((r->outputs & ~avail) == 0, "outputs 0x%x not declared by model %d (available 0x%x)",
            r->outputs & ~avail, m, avail);
    REQUIRE(r->outputs != 0, "no outputs requested");
    static const hhmm_result none{};
    const hhmm_result *oo = o ? o : &none;
    struct {
        uint32_t bit;
        const void *ptr;
        const char *name;
    } outs[] = {{HHMM_OUT_LOGLIK, oo->loglik, "loglik"},
                {HHMM_OUT_UNALPHA, oo->unalpha_tk, "unalpha_tk"},
                {HHMM_OUT_ALPHA, oo->alpha_tk, "alpha_tk"},
                {HHMM_OUT_UNBETA, oo->unbeta_tk, "unbeta_tk"},
                {HHMM_OUT_BETA, oo->beta_tk, "beta_tk"},
                {HHMM_OUT_UNGAMMA, oo->ungamma_tk, "ungamma_tk"},
                {HHMM_OUT_GAMMA, oo->gamma_tk, "gamma_tk"},
                {HHMM_OUT_ZSTAR, oo->zstar_t, "zstar_t"},
                {HHMM_OUT_LOGP_ZSTAR, oo->logp_zstar, "logp_zstar"},
                {HHMM_OUT_OBLIK_TK, oo->oblik_tk, "oblik_tk"},
                {HHMM_OUT_OBLIK_T, oo->oblik_t, "oblik_t"},
                {HHMM_OUT_FFBS, oo->z_ffbs, "z_ffbs"},
                {HHMM_OUT_ALPHA_OOS, oo->alpha_tk_oos, "alpha_tk_oos"},
                {HHMM_OUT_UNALPHA_OOS, oo->unalpha_tk_oos, "unalpha_tk_oos"},
                {HHMM_OUT_LOGA, oo->logA_ij, "logA_ij"},
                {HHMM_OUT_HATPI, oo->hatpi_tk, "hatpi_tk"},
                {HHMM_OUT_HATZ, oo->hatz_t, "hatz_t"},
                {HHMM_OUT_HATL, oo->hatl_t, "hatl_t"},
                {HHMM_OUT_HATX, oo->hatx_t, "hatx_t"}};
    if (o)
        for (auto &e : outs)
            REQUIRE(!(r->outputs & e.bit) || e.ptr, "output %s requested but its pointer is NULL", e.name);
    if (r->outputs & HHMM_OUT_FFBS)
        REQUIRE(r->ffbs_u, "FFBS needs ffbs_u");
    if (r->outputs & (HHMM_OUT_HATZ | HHMM_OUT_HATL | HHMM_OUT_HATX))
        REQUIRE(r->hat_rand, "hatz_t / hatl_t / hatx_t need hat_rand");

    if (host) {
        const int64_t N = d.n_series;
        const int Tm = d.T_max;
        if (d.T)
            for (int64_t n = 0; n < N; ++n)
                REQUIRE(d.T[n] >= 1 && d.T[n] <= Tm, "T[%lld] = %d outside 1..T_max=%d", (long long)n, d.T[n], Tm);
        auto len = [&](int64_t n) { return d.T ? d.T[n] : Tm; };
        /* the fast time-major scan first; the n-major loops below only run to
         * name the first offender when it found one */
        if (is_discrete(m) && any_out_of_range(d.x_int, N, Tm, d.T, 1, d.L))
            for (int64_t n = 0; n < N; ++n)
                for (int t = 0; t < len(n); ++t) {
                    const int32_t v = d.x_int[n + N * (int64_t)t];
                    REQUIRE(v >= 1 && v <= d.L, "x[%lld, %d] = %d outside 1..L=%d", (long long)n, t + 1, v, d.L);
                }
        if (m == HHMM_MODEL_HMM_MULTINOM_SEMISUP && any_out_of_range(d.g, N, Tm, d.T, 1, d.G))
            for (int64_t n = 0; n < N; ++n)
                for (int t = 0; t < len(n); ++t) {
                    const int32_t v = d.g[n + N * (int64_t)t];
                    REQUIRE(v >= 1 && v <= d.G, "g[%lld, %d] = %d outside 1..G=%d", (long long)n, t + 1, v, d.G);
                }
        if ((m == HHMM_MODEL_TAYAL || m == HHMM_MODEL_TAYAL_LITE) && any_out_of_range(d.sign, N, Tm, d.T, 1, 2))
            for (int64_t n = 0; n < N; ++n)
                for (int t = 0; t < len(n); ++t) {
                    const int32_t v = d.sign[n + N * (int64_t)t];
                    REQUIRE(v == 1 || v == 2, "sign[%lld, %d] = %d outside 1..2", (long long)n, t + 1, v);
                }
        if (m == HHMM_MODEL_TAYAL_LITE) {
            for (int64_t n = 0; n < N; ++n) {
                const int To = d.T_oos ? d.T_oos[n] : d.T_oos_max;
                REQUIRE(To >= 1 && To <= d.T_oos_max, "T_oos[%lld] = %d outside 1..T_oos_max", (long long)n, To);
                for (int t = 0; t < To; ++t) {
                    const int32_t v = d.x_oos[n + N * (int64_t)t];
                    const int32_t sg = d.sign_oos[n + N * (int64_t)t];
                    REQUIRE(v >= 1 && v <= d.L, "x_oos[%lld, %d] = %d outside 1..L", (long long)n, t + 1, v);
                    REQUIRE(sg == 1 || sg == 2, "sign_oos[%lld, %d] = %d outside 1..2", (long long)n, t + 1, sg);
                }
            }
        }
        if (m == HHMM_MODEL_HMM_GAUSS)
            for (int64_t i = 0; i < w.n_draws * d.K; ++i)
                REQUIRE(w.sigma_k[i] > 0.0, "sigma_k must be > 0 (real<lower=0.0001>)");
    }
    return HHMM_OK;
}

static hhmm_status validate(const hhmm_request *r, const hhmm_result *o, bool host)
{
    REQUIRE(r && o, "request and result must be non-NULL");
    return validate_impl(r, o, host);
}

/* Element counts of every input / output array the request uses. */
static void describe(const hhmm_request *r, const hhmm_result *o, hhmm_request *dr, hhmm_result *dq,
                     std::vector<ArrayDesc> &v)
{
    const hhmm_data &d = r->data;
    const hhmm_draws &w = r->draws;
    const size_t N = (size_t)d.n_series, S = (size_t)w.n_draws, Tm = (size_t)d.T_max;
    const size_t To = (size_t)(d.T_oos_max > 0 ? d.T_oos_max : 0);
    const size_t K = (size_t)d.K, L = (size_t)(d.L > 0 ? d.L : 0), M = (size_t)(d.M > 0 ? d.M : 0);
    const size_t P = (size_t)npairs(r);
    const uint32_t out = r->outputs;
    /* the class follows from the leading dimension of the element count */
    auto cls_of = [&](size_t lead) { return lead == 0 ? (int)SERIES : lead == 1 ? (int)DRAWS : (int)PAIRS; };
    auto in = [&](const void *h, const void **slot, size_t n, size_t es, int lead) {
        if (h)
            v.push_back({h, (void **)slot, n, es, false, cls_of((size_t)lead)});
    };
    auto ou = [&](uint32_t bit, void *h, void **slot, size_t n, size_t es) {
        if ((out & bit) && h)
            v.push_back({h, slot, n, es, true, PAIRS});
        else
            *slot = nullptr;
    };
    in(d.T, (const void **)&dr->data.T, N, 4, 0);
    in(d.x_int, (const void **)&dr->data.x_int, N * Tm, 4, 0);
    in(d.x_real, (const void **)&dr->data.x_real, N * Tm, 8, 0);
    in(d.g, (const void **)&dr->data.g, N * Tm, 4, 0);
    in(d.sign, (const void **)&dr->data.sign, N * Tm, 4, 0);
    in(d.u, (const void **)&dr->data.u, N * Tm * M, 8, 0);
    in(d.T_oos, (const void **)&dr->data.T_oos, N, 4, 0);
    in(d.x_oos, (const void **)&dr->data.x_oos, N * To, 4, 0);
    in(d.sign_oos, (const void **)&dr->data.sign_oos, N * To, 4, 0);
    dr->data.hyperparams = nullptr;
    in(w.p_1k, (const void **)&dr->draws.p_1k, S * K, 8, 1);
    in(w.A_ij, (const void **)&dr->draws.A_ij, S * K * K, 8, 1);
    in(w.phi_k, (const void **)&dr->draws.phi_k, S * K * L, 8, 1);
    in(w.mu_k, (const void **)&dr->draws.mu_k, S * K, 8, 1);
    in(w.sigma_k, (const void **)&dr->draws.sigma_k, S * K, 8, 1);
    in(w.w_km, (const void **)&dr->draws.w_km, S * K * M, 8, 1);
    in(w.b_km, (const void **)&dr->draws.b_km, S * K * M, 8, 1);
    in(w.s_k, (const void **)&dr->draws.s_k, S * K, 8, 1);
    in(w.lambda_kl, (const void **)&dr->draws.lambda_kl, S * K * L, 8, 1);
    in(w.mu_kl, (const void **)&dr->draws.mu_kl, S * K * L, 8, 1);
    in(w.s_kl, (const void **)&dr->draws.s_kl, S * K * L, 8, 1);
    in(w.p_11, (const void **)&dr->draws.p_11, S, 8, 1);
    in(w.A_row, (const void **)&dr->draws.A_row, S * 4, 8, 1);
    in(r->ffbs_u, (const void **)&dr->ffbs_u, P * Tm, 8, 2);
    in(r->hat_rand, (const void **)&dr->hat_rand, P * Tm * 3, 8, 2);
    const size_t Tz = (r->model == HHMM_MODEL_TAYAL_LITE) ? To : Tm;
    ou(HHMM_OUT_LOGLIK, o->loglik, (void **)&dq->loglik, P, 8);
    ou(HHMM_OUT_UNALPHA, o->unalpha_tk, (void **)&dq->unalpha_tk, P * Tm * K, 8);
    ou(HHMM_OUT_ALPHA, o->alpha_tk, (void **)&dq->alpha_tk, P * Tm * K, 8);
    ou(HHMM_OUT_UNBETA, o->unbeta_tk, (void **)&dq->unbeta_tk, P * Tm * K, 8);
    ou(HHMM_OUT_BETA, o->beta_tk, (void **)&dq->beta_tk, P * Tm * K, 8);
    ou(HHMM_OUT_UNGAMMA, o->ungamma_tk, (void **)&dq->ungamma_tk, P * Tm * K, 8);
    ou(HHMM_OUT_GAMMA, o->gamma_tk, (void **)&dq->gamma_tk, P * Tm * K, 8);
    ou(HHMM_OUT_ZSTAR, o->zstar_t, (void **)&dq->zstar_t, P * Tz, 4);
    ou(HHMM_OUT_LOGP_ZSTAR, o->logp_zstar, (void **)&dq->logp_zstar, P, 8);
    ou(HHMM_OUT_OBLIK_TK, o->oblik_tk, (void **)&dq->oblik_tk, P * Tm * K, 8);
    ou(HHMM_OUT_OBLIK_T, o->oblik_t, (void **)&dq->oblik_t, P * Tm, 8);
    ou(HHMM_OUT_FFBS, o->z_ffbs, (void **)&dq->z_ffbs, P * Tm, 4);
    ou(HHMM_OUT_ALPHA_OOS, o->alpha_tk_oos, (void **)&dq->alpha_tk_oos, P * To * K, 8);
    ou(HHMM_OUT_UNALPHA_OOS, o->unalpha_tk_oos, (void **)&dq->unalpha_tk_oos, P * To * K, 8);
    ou(HHMM_OUT_LOGA, o->logA_ij, (void **)&dq->logA_ij, P * Tm * K, 8);
    ou(HHMM_OUT_HATPI, o->hatpi_tk, (void **)&dq->hatpi_tk, P * Tm * K, 8);
    ou(HHMM_OUT_HATZ, o->hatz_t, (void **)&dq->hatz_t, P * Tm, 4);
    ou(HHMM_OUT_HATL, o->hatl_t, (void **)&dq->hatl_t, P * Tm, 4);
    ou(HHMM_OUT_HATX, o->hatx_t, (void **)&dq->hatx_t, P * Tm, 8);
}

static hhmm_status hip_fail(hipError_t e, const char *what)
{
    set_error("%s: %s", what, hipGetErrorString(e));
    return (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) ? HHMM_ERR_OUT_OF_MEMORY : HHMM_ERR_HIP;
}

static hhmm_status check_device()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1) {
        (void)hipGetLastError();
        set_error("no HIP device visible: libhhmm has no CPU path (gfx950 required)");
        return HHMM_ERR_NO_DEVICE;
    }
    return HHMM_OK;
}

static hhmm_status check_arch(int dev)
{
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return hip_fail(hipGetLastError(), "hipGetDeviceProperties");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device %d is %s, this build targets gfx950", dev, prop.gcnArchName);
        return HHMM_ERR_NO_DEVICE;
    }
    return HHMM_OK;
}

/* ---------------- device set (hhmm_init / hhmm_init_devices) ---------------- */
struct DevSet {
    std::mutex mu;
    std::vector<int> devs; /* ordinals HHMM_DEVICE_SET shards over (repeats allowed); empty: {0} */
};
static DevSet &devset()
{
    static DevSet d;
    return d;
}

/* One shard of a host request: per array class (series, draws, pairs) the
 * first element, the element count and the caller's leading extent.  An
 * array of class c with e elements is then `e / lead` rows of `cnt` elements,
 * at a pitch of `lead` in the caller's buffer and packed in the shard's
 * device copy -- which is exactly the [N', ...] / [S', ...] / [P', ...]
 * layout of the sub-request (every array is series-, draw- or pair-fastest). */
struct Shard {
    int64_t off[3], cnt[3], lead[3];
};

static Shard whole_shard(const hhmm_request *r)
{
    const int64_t N = r->data.n_series, S = r->draws.n_draws, P = npairs(r);
    return Shard{{0, 0, 0}, {N, S, P}, {N, S, P}};
}

/* Splits a request over `n` shards: contiguous series ranges (ZIP / BLOCK take
 * the series' own draws, GRID all draws); a GRID request with fewer series
 * than shards splits its draws instead (pairs p = s + S*n with s in the
 * range: rows of S' pairs at a pitch of S). */
static std::vector<Shard> make_shards(const hhmm_request *r, int n)
{
    const int64_t N = r->data.n_series, S = r->draws.n_draws, P = npairs(r);
    std::vector<Shard> v;
    const bool by_draws = r->pairing == HHMM_PAIR_GRID && N < n;
    const int64_t units = by_draws ? S : N;
    const int64_t ns = std::min<int64_t>(n, units);
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t a = units * i / ns, b = units * (i + 1) / ns;
        Shard sh;
        if (by_draws) {
            sh = Shard{{0, a, a}, {N, b - a, b - a}, {N, S, S}};
        } else if (r->pairing == HHMM_PAIR_ZIP) {
            sh = Shard{{a, a, a}, {b - a, b - a, b - a}, {N, S, P}};
        } else if (r->pairing == HHMM_PAIR_BLOCK) {
            const int64_t B = S / N;
            sh = Shard{{a, B * a, B * a}, {b - a, B * (b - a), B * (b - a)}, {N, S, P}};
        } else { /* GRID by series */
            sh = Shard{{a, 0, S * a}, {b - a, S, S * (b - a)}, {N, S, P}};
        }
        v.push_back(sh);
    }
    return v;
}

/* One array's shard in the caller's buffer: `rows` rows of `width` bytes at a
 * pitch of `pitch` bytes from `base`; packed (pitch = width) in the shard's copy. */
struct ShardRows {
    char *base;
    size_t rows, width, pitch;
};
static ShardRows shard_rows(const void *host, const ArrayDesc &a, const Shard &sh)
{
    const size_t es = a.esize, lead = (size_t)sh.lead[a.cls], cnt = (size_t)sh.cnt[a.cls];
    return ShardRows{(char *)host + (size_t)sh.off[a.cls] * es, a.elems / lead, cnt * es, lead * es};
}

/* A shard's rows packed / unpacked on the host for hhmm_selftest_shards (memcpy per row). */
static void copy_shard_host(void *packed, const void *host, const ArrayDesc &a, const Shard &sh, bool to_packed)
{
    const ShardRows r = shard_rows(host, a, sh);
    for (size_t i = 0; i < r.rows; ++i) {
        char *h = r.base + i * r.pitch, *q = (char *)packed + i * r.width;
        if (to_packed)
            memcpy(q, h, r.width);
        else
            memcpy(h, q, r.width);
    }
}

/* ---------------- the R path: a pipelined host request ----------------
 * hhmm_run's caller hands over pageable host arrays (R's REAL() buffers,
 * SURVEY §8b).  A device's shard is split into chunks of series (or draws),
 * and chunk i's upload and kernels overlap chunk i-1's download: per device
 * three non-blocking streams (upload, compute, download), two slots of
 * device buffers and two pinned staging slots per direction.  The host thread
 * gathers chunk i's input rows into a pinned slot (threads over rows), the
 * upload stream DMAs the slot to the device in one copy, the compute stream
 * runs the chunk's sub-request, the download stream DMAs its outputs and
 * pair_status into the other pinned slot in one copy, and the host thread
 * scatters chunk i-1's rows into the caller's arrays meanwhile.  Every array
 * of a chunk sits at the same offset in its device slot and its pinned slot,
 * so each direction is one DMA per chunk. */

struct HostPool { /* pinned staging blocks, reused across calls (hhmm_shutdown frees them) */
    std::mutex mu;
    std::multimap<size_t, void *> free_blocks;
    std::map<void *, size_t> live;
};
static HostPool &host_pool()
{
    static HostPool p;
    return p;
}
static void *host_get(size_t bytes)
{
    bytes = (std::max<size_t>(bytes, 4096) + 4095) & ~(size_t)4095;
    HostPool &p = host_pool();
    {
        std::lock_guard<std::mutex> g(p.mu);
        auto it = p.free_blocks.lower_bound(bytes);
        if (it != p.free_blocks.end() && it->first <= bytes + bytes / 4) {
            void *ptr = it->second;
            p.live[ptr] = it->first;
            p.free_blocks.erase(it);
            return ptr;
        }
    }
    void *ptr = nullptr;
    if (hipHostMalloc(&ptr, bytes, hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::lock_guard<std::mutex> g(p.mu);
    p.live[ptr] = bytes;
    return ptr;
}
static void host_put(void *ptr)
{
    if (!ptr)
        return;
    HostPool &p = host_pool();
    std::lock_guard<std::mutex> g(p.mu);
    auto it = p.live.find(ptr);
    if (it == p.live.end())
        return;
    p.free_blocks.emplace(it->second, ptr);
    p.live.erase(it);
}
static void host_release_all()
{
    HostPool &p = host_pool();
    std::lock_guard<std::mutex> g(p.mu);
    for (auto &kv : p.free_blocks)
        (void)hipHostFree(kv.second);
    p.free_blocks.clear();
}

struct PipeStreams {
    std::mutex mu;
    std::map<int, std::vector<hipStream_t>> by_dev; /* upload, compute, download */
};
static PipeStreams &pipe_streams()
{
    static PipeStreams s;
    return s;
}
static hhmm_status get_pipe_streams(int dev, hipStream_t (&st)[3])
{
    PipeStreams &ps = pipe_streams();
    std::lock_guard<std::mutex> g(ps.mu);
    auto it = ps.by_dev.find(dev);
    if (it == ps.by_dev.end()) {
        std::vector<hipStream_t> v(3, nullptr);
        for (auto &x : v)
            if (hipStreamCreateWithFlags(&x, hipStreamNonBlocking) != hipSuccess) {
                set_error("device %d: stream creation failed", dev);
                return HHMM_ERR_HIP;
            }
        it = ps.by_dev.emplace(dev, v).first;
    }
    for (int i = 0; i < 3; ++i)
        st[i] = it->second[(size_t)i];
    return HHMM_OK;
}

/* One row of a staging copy.  Large rows leave the cache alone: the
 * destination is written with streaming stores (no read-for-ownership of the
 * caller's lines, which would double the DRAM traffic of the scatter into R's
 * arrays), 16 bytes at a time once it is 16-byte aligned. */
static void copy_row(char *dst, const char *src, size_t n)
{
    if (n < 4096) {
        memcpy(dst, src, n);
        return;
    }
    const size_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    const size_t m = n & ~(size_t)63;
    for (size_t i = 0; i < m; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(src + i));
        const __m128i b = _mm_loadu_si128((const __m128i *)(src + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i *)(src + i + 32));
        const __m128i d = _mm_loadu_si128((const __m128i *)(src + i + 48));
        _mm_stream_si128((__m128i *)(dst + i), a);
        _mm_stream_si128((__m128i *)(dst + i + 16), b);
        _mm_stream_si128((__m128i *)(dst + i + 32), c);
        _mm_stream_si128((__m128i *)(dst + i + 48), d);
    }
    memcpy(dst + m, src + m, n - m);
}

/* rows x width bytes between pitched buffers, split over host threads when
 * the copy is large (the staging copies run beside the GPU's DMA; up to 16
 * threads, the CPU share of one GPU on an 8-GPU node) */
static void par_copy_rows(char *dst, size_t dpitch, const char *src, size_t spitch, size_t width, size_t rows)
{
    if (rows == 0 || width == 0)
        return;
    if (dpitch == width && spitch == width) { /* contiguous: one long row, split in pieces */
        width *= rows;
        rows = 1;
        dpitch = spitch = width;
    }
    const size_t total = width * rows;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t nt = total < ((size_t)4 << 20) ? 1 : std::min<size_t>(16u, hw);
    /* work item i: a range of rows, or of bytes of the single row */
    auto run = [&](size_t i) {
        if (rows >= nt) {
            const size_t r0 = rows * i / nt, r1 = rows * (i + 1) / nt;
            for (size_t r = r0; r < r1; ++r)
                copy_row(dst + r * dpitch, src + r * spitch, width);
        } else {
            for (size_t r = 0; r < rows; ++r) {
                const size_t b0 = (width * i / nt) & ~(size_t)63, b1 = i + 1 == nt ? width : (width * (i + 1) / nt) & ~(size_t)63;
                copy_row(dst + r * dpitch + b0, src + r * spitch + b0, b1 - b0);
            }
        }
        _mm_sfence(); /* this thread's streaming stores, before the join */
    };
    if (nt <= 1) {
        run(0);
        return;
    }
    /* a thread that cannot be started leaves its share to this one (no
     * exception crosses the C ABI) */
    std::vector<std::thread> th;
    std::vector<size_t> mine{0};
    for (size_t i = 1; i < nt; ++i) {
        try {
            th.emplace_back(run, i);
        } catch (...) {
            mine.push_back(i);
        }
    }
    for (size_t i : mine)
        run(i);
    for (auto &t : th)
        t.join();
}

/* A chunk: its shard, its sub-request, and where each array sits in the slot. */
struct ChunkLayout {
    Shard sh;
    std::vector<size_t> off;   /* per array of `arrays`, bytes from the slot base */
    size_t status_off = 0;
    size_t in_end = 0;         /* [0, in_end): uploaded */
    size_t out_begin = 0;      /* [out_begin, total): downloaded */
    size_t total = 0;
    int64_t P = 0;
};

static size_t shard_bytes(const ArrayDesc &a, const Shard &sh)
{
    return a.elems / (size_t)sh.lead[a.cls] * (size_t)sh.cnt[a.cls] * a.esize;
}

static ChunkLayout chunk_layout(const hhmm_request *req, const std::vector<ArrayDesc> &arrays, const Shard &sh,
                                bool ragged)
{
    ChunkLayout L;
    L.sh = sh;
    hhmm_request r = *req;
    r.data.n_series = sh.cnt[SERIES];
    r.draws.n_draws = sh.cnt[DRAWS];
    L.P = npairs(&r);
    L.off.assign(arrays.size(), 0);
    size_t o = 0;
    auto place = [&](size_t bytes) {
        const size_t at = o;
        o += (bytes + 255) & ~(size_t)255;
        return at;
    };
    for (size_t i = 0; i < arrays.size(); ++i) /* inputs first */
        if (!arrays[i].output)
            L.off[i] = place(shard_bytes(arrays[i], sh));
    const size_t outs = o;
    for (size_t i = 0; i < arrays.size(); ++i)
        if (arrays[i].output)
            L.off[i] = place(shard_bytes(arrays[i], sh));
    L.status_off = place((size_t)L.P * sizeof(int32_t));
    L.total = o;
    /* outputs travel up too where padded steps must round-trip untouched */
    L.in_end = ragged ? L.status_off : outs;
    L.out_begin = outs;
    return L;
}

/* Sub-shards of a device shard: `n` contiguous ranges of its units (series,
 * or draws for a GRID request split by draws), each a Shard of the request. */
static std::vector<Shard> split_shard(const hhmm_request *r, const Shard &sh, int64_t n)
{
    const int64_t S = r->draws.n_draws;
    /* a GRID shard holding every series splits by draws (rows of the chunk's
     * draws at a pitch of S pairs) when it is a draws shard already or has
     * fewer series than chunks; every other shard splits by series */
    const bool all_series = sh.cnt[SERIES] == r->data.n_series;
    const bool draws_shard = sh.lead[PAIRS] == S && sh.cnt[DRAWS] < S;
    const bool by_draws = r->pairing == HHMM_PAIR_GRID && all_series && (draws_shard || sh.cnt[SERIES] < n);
    const int64_t u0 = by_draws ? sh.off[DRAWS] : sh.off[SERIES];
    const int64_t units = by_draws ? sh.cnt[DRAWS] : sh.cnt[SERIES];
    const int64_t ns = std::max<int64_t>(1, std::min(n, units));
    std::vector<Shard> v;
    for (int64_t i = 0; i < ns; ++i) {
        const int64_t a = u0 + units * i / ns, b = u0 + units * (i + 1) / ns;
        Shard c = sh;
        if (by_draws) {
            c.lead[PAIRS] = S;
            c.off[DRAWS] = c.off[PAIRS] = a;
            c.cnt[DRAWS] = c.cnt[PAIRS] = b - a;
        } else {
            const int64_t per = sh.cnt[SERIES] > 0 ? sh.cnt[PAIRS] / sh.cnt[SERIES] : 0; /* pairs per series */
            const int64_t dper = sh.cnt[SERIES] > 0 ? sh.cnt[DRAWS] / sh.cnt[SERIES] : 0;
            c.off[SERIES] = a;
            c.cnt[SERIES] = b - a;
            c.off[PAIRS] = sh.off[PAIRS] + (a - u0) * per;
            c.cnt[PAIRS] = (b - a) * per;
            if (r->pairing != HHMM_PAIR_GRID) { /* ZIP / BLOCK: the series' own draws */
                c.off[DRAWS] = sh.off[DRAWS] + (a - u0) * dper;
                c.cnt[DRAWS] = (b - a) * dper;
            }
        }
        v.push_back(c);
    }
    return v;
}

/* Chunks of a device shard: about kChunkBytes of staged traffic each, with at
 * least kChunkMinPairs pairs (256 waves) so a chunk's kernels still fill the
 * chip, and only where the whole request runs no parallel scan over T: the
 * chunks then take the same sequential recursions (SCAN_OFF / VIT_SCAN_OFF
 * pin it) and the outputs are bit-identical to one device call.
 * HHMM_FLAG_HOST_CHUNKS(n) asks for n chunks. */
constexpr size_t kChunkBytes = (size_t)512 << 20;
constexpr int64_t kChunkMinPairs = 16384;

static int64_t choose_chunks(const hhmm_request *req, const std::vector<ArrayDesc> &arrays, const Shard &sh,
                             bool ragged, bool &pin_flags)
{
    pin_flags = false;
    const hhmm_data &d = req->data;
    const int64_t Pw = npairs(req);
    const bool seq = scan_plan(req->model, d.K, d.T_max, Pw, req->outputs, (uint32_t)req->flags).cl == 0 &&
                     vscan_chunks(req->model, d.K, req->model == HHMM_MODEL_TAYAL_LITE ? d.T_oos_max : d.T_max, Pw,
                                  req->outputs, (uint32_t)req->flags) == 0;
    if (!seq)
        return 1;
    const int64_t forced = (int64_t)(((uint32_t)req->flags >> 20) & 0xffu);
    size_t bytes = 0; /* staged bytes of the shard, both directions */
    for (const ArrayDesc &a : arrays)
        bytes += shard_bytes(a, sh) * ((a.output && ragged) ? 2 : 1);
    const int64_t P = sh.cnt[PAIRS];
    int64_t n = forced > 0 ? forced : (int64_t)((bytes + kChunkBytes - 1) / kChunkBytes);
    if (forced == 0)
        n = std::min<int64_t>(n, std::max<int64_t>(1, P / kChunkMinPairs));
    n = std::max<int64_t>(1, n);
    pin_flags = n > 1;
    return n;
}

/* Runs one shard of a host request on the current device (the pipeline
 * above).  status: the caller's [P] host array, written at the shard's pairs;
 * *failures counts them. */
static hhmm_status run_on_device(const hhmm_request *req, hhmm_result *res, const Shard &sh, int32_t *status,
                                 int64_t *failures)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess)
        return hip_fail(e, "hipGetDevice");
    hhmm_request dreq = *req;
    hhmm_result dres = *res;
    dres.pair_status = nullptr;
    std::vector<ArrayDesc> arrays;
    describe(req, res, &dreq, &dres, arrays);
    const bool ragged = req->data.T != nullptr || req->data.T_oos != nullptr;
    bool pin = false;
    const int64_t nch = choose_chunks(req, arrays, sh, ragged, pin);
    const std::vector<Shard> chunks = split_shard(req, sh, nch);
    std::vector<ChunkLayout> lay;
    size_t slot_bytes = 0, in_bytes = 0, out_bytes = 0, wsb = 0;
    for (const Shard &c : chunks) {
        lay.push_back(chunk_layout(req, arrays, c, ragged));
        const ChunkLayout &L = lay.back();
        if (L.P < 1) {
            set_error("internal: shard describes no pairs");
            return HHMM_ERR_INVALID_ARGUMENT;
        }
        slot_bytes = std::max(slot_bytes, L.total);
        in_bytes = std::max(in_bytes, L.in_end);
        out_bytes = std::max(out_bytes, L.total - L.out_begin);
        wsb = std::max(wsb, workspace_bytes(dreq.model, dreq.data.K, dreq.data.L, dreq.data.T_max,
                                            dreq.data.T_oos_max, L.P, dreq.outputs, (uint32_t)dreq.flags,
                                            c.cnt[SERIES], dreq.pairing));
    }
    if (pin)
        dreq.flags |= (int32_t)(HHMM_FLAG_SCAN_OFF | HHMM_FLAG_VIT_SCAN_OFF);
    const int nslot = chunks.size() > 1 ? 2 : 1;
    hipStream_t st[3];
    hhmm_status s = get_pipe_streams(dev, st);
    if (s != HHMM_OK)
        return s;
    void *dslot[2] = {nullptr, nullptr}, *hin[2] = {nullptr, nullptr}, *hout[2] = {nullptr, nullptr};
    void *ws = nullptr;
    hipEvent_t ev[3][2] = {}; /* uploaded, computed, downloaded -- per slot */
    auto cleanup = [&]() {
        for (int k = 0; k < 2; ++k) {
            pool_put(dslot[k]);
            host_put(hin[k]);
            host_put(hout[k]);
            for (int j = 0; j < 3; ++j)
                if (ev[j][k])
                    (void)hipEventDestroy(ev[j][k]);
        }
        pool_put(ws);
    };
    auto drain = [&]() { /* every stream of this request, the side stream included */
        hipError_t r = hipSuccess;
        for (int j = 0; j < 3; ++j) {
            const hipError_t q = (j == 1) ? sync_request(st[1]) : hipStreamSynchronize(st[j]);
            if (r == hipSuccess)
                r = q;
        }
        return r;
    };
    for (int k = 0; k < nslot; ++k) {
        dslot[k] = pool_get(dev, slot_bytes);
        hin[k] = host_get(in_bytes);
        hout[k] = host_get(out_bytes);
        for (int j = 0; j < 3; ++j)
            if (hipEventCreateWithFlags(&ev[j][k], hipEventDisableTiming) != hipSuccess)
                ev[j][k] = nullptr;
        if (!dslot[k] || !hin[k] || !hout[k] || !ev[0][k] || !ev[1][k] || !ev[2][k]) {
            cleanup();
            set_error("device %d: allocation of the host pipeline's buffers failed (%zu device, %zu + %zu pinned bytes)",
                      dev, slot_bytes, in_bytes, out_bytes);
            return HHMM_ERR_OUT_OF_MEMORY;
        }
    }
    ws = pool_get(dev, wsb);
    if (!ws) {
        cleanup();
        set_error("device %d: workspace allocation of %zu bytes failed", dev, wsb);
        return HHMM_ERR_OUT_OF_MEMORY;
    }

    auto bind = [&](const ChunkLayout &L, int k, hhmm_request &cr, hhmm_result &cq) {
        cr = dreq;
        cq = dres;
        cr.data.n_series = L.sh.cnt[SERIES];
        cr.draws.n_draws = L.sh.cnt[DRAWS];
        /* the device copies of the request's arrays: describe() recorded where
         * each pointer lives in dreq / dres; the same field of cr / cq */
        for (size_t i = 0; i < arrays.size(); ++i) {
            const char *slot_base = (const char *)arrays[i].dev_slot;
            void **f = nullptr;
            if (slot_base >= (const char *)&dreq && slot_base < (const char *)(&dreq + 1))
                f = (void **)((char *)&cr + (slot_base - (const char *)&dreq));
            else
                f = (void **)((char *)&cq + (slot_base - (const char *)&dres));
            *f = (char *)dslot[k] + L.off[i];
        }
        cq.pair_status = (int32_t *)((char *)dslot[k] + L.status_off);
    };
    auto gather = [&](const ChunkLayout &L, int k) {
        for (size_t i = 0; i < arrays.size(); ++i) {
            const ArrayDesc &a = arrays[i];
            if (L.off[i] >= L.in_end)
                continue;
            const ShardRows r = shard_rows(a.host, a, L.sh);
            par_copy_rows((char *)hin[k] + L.off[i], r.width, r.base, r.pitch, r.width, r.rows);
        }
    };
    int64_t fails = 0;
    auto scatter = [&](const ChunkLayout &L, int k) {
        for (size_t i = 0; i < arrays.size(); ++i) {
            const ArrayDesc &a = arrays[i];
            if (!a.output)
                continue;
            const ShardRows r = shard_rows(a.host, a, L.sh);
            par_copy_rows(r.base, r.pitch, (const char *)hout[k] + (L.off[i] - L.out_begin), r.width, r.width,
                          r.rows);
        }
        /* pair_status: [P] in the caller's layout (a PAIRS array of P elements) */
        const ArrayDesc sa{status, nullptr, (size_t)npairs(req), sizeof(int32_t), true, PAIRS};
        const ShardRows r = shard_rows(status, sa, L.sh);
        const char *src = (const char *)hout[k] + (L.status_off - L.out_begin);
        par_copy_rows(r.base, r.pitch, src, r.width, r.width, r.rows);
        const int32_t *q = (const int32_t *)src;
        for (int64_t p = 0; p < L.P; ++p)
            fails += q[p] != 0;
    };

    hhmm_status ls = HHMM_OK;
    const size_t n = chunks.size();
    for (size_t i = 0; i < n && ls == HHMM_OK; ++i) {
        const int k = (int)(i % (size_t)nslot);
        const ChunkLayout &L = lay[i];
        if (i >= (size_t)nslot && (e = hipEventSynchronize(ev[0][k])) != hipSuccess) /* pinned in-slot free */
            break;
        gather(L, k);
        if (i >= (size_t)nslot && (e = hipStreamWaitEvent(st[0], ev[2][k], 0)) != hipSuccess) /* device slot free */
            break;
        if ((e = hipMemcpyAsync(dslot[k], hin[k], L.in_end, hipMemcpyHostToDevice, st[0])) != hipSuccess ||
            (e = hipEventRecord(ev[0][k], st[0])) != hipSuccess || (e = hipStreamWaitEvent(st[1], ev[0][k], 0)) !=
                                                                         hipSuccess ||
            (e = hipMemsetAsync((char *)dslot[k] + L.status_off, 0, (size_t)L.P * sizeof(int32_t), st[1])) !=
                hipSuccess)
            break;
        hhmm_request cr;
        hhmm_result cq;
        bind(L, k, cr, cq);
        ls = launch_all(&cr, &cq, L.P, ws, st[1]);
        if (ls != HHMM_OK)
            break;
        if ((e = hipEventRecord(ev[1][k], st[1])) != hipSuccess || (e = hipStreamWaitEvent(st[2], ev[1][k], 0)) !=
                                                                        hipSuccess ||
            (e = hipMemcpyAsync(hout[k], (char *)dslot[k] + L.out_begin, L.total - L.out_begin,
                                hipMemcpyDeviceToHost, st[2])) != hipSuccess ||
            (e = hipEventRecord(ev[2][k], st[2])) != hipSuccess)
            break;
        if (i >= 1) { /* the previous chunk's outputs, while this one uploads and runs */
            const int kp = (int)((i - 1) % (size_t)nslot);
            if ((e = hipEventSynchronize(ev[2][kp])) != hipSuccess)
                break;
            scatter(lay[i - 1], kp);
        }
    }
    if (ls != HHMM_OK || e != hipSuccess) {
        /* a failed launch may follow one that is still running: drain this
         * request's streams before its pooled buffers can be handed to another
         * request; a sticky device error from an earlier fault is reported
         * beside the launch error instead of being buried under it */
        const std::string first = hhmm_last_error();
        const hipError_t d = drain();
        cleanup();
        if (ls == HHMM_OK)
            return hip_fail(e, "host pipeline (copy or kernel execution)");
        if (d != hipSuccess)
            set_error("%s; draining the request's streams then failed: %s", first.c_str(), hipGetErrorString(d));
        return ls;
    }
    e = drain();
    if (e != hipSuccess) {
        cleanup();
        return hip_fail(e, "kernel execution");
    }
    scatter(lay[n - 1], (int)((n - 1) % (size_t)nslot));
    cleanup();
    *failures = fails;
    return HHMM_OK;
}

/* HHMM_DEVICE_SET: one host thread per shard, each on its device of the set
 * (hhmm_init / hhmm_init_devices), writing its slices of the caller's
 * outputs; the first failing shard's error is returned (device
 * set {GPU 0..7}, one host thread per GPU; §8e: contiguous series ranges). */
static hhmm_status run_sharded(const hhmm_request *req, hhmm_result *res)
{
    std::vector<int> devs;
    {
        std::lock_guard<std::mutex> g(devset().mu);
        devs = devset().devs.empty() ? std::vector<int>{0} : devset().devs;
    }
    const std::vector<Shard> shards = make_shards(req, (int)devs.size());
    const int64_t P = npairs(req);
    std::vector<int32_t> status((size_t)P, 0);
    std::vector<hhmm_status> st(shards.size(), HHMM_OK);
    std::vector<std::string> msg(shards.size());
    std::vector<int64_t> fails(shards.size(), 0);
    auto work = [&](size_t i) {
        hipError_t e = hipSetDevice(devs[i]);
        if (e != hipSuccess) {
            st[i] = hip_fail(e, "hipSetDevice");
        } else {
            st[i] = run_on_device(req, res, shards[i], status.data(), &fails[i]);
        }
        if (st[i] != HHMM_OK)
            msg[i] = hhmm_last_error(); /* thread-local: carried to the caller's thread */
    };
    std::vector<std::thread> th;
    std::vector<size_t> mine{0};
    for (size_t i = 1; i < shards.size(); ++i) {
        try {
            th.emplace_back(work, i);
        } catch (...) { /* no exception crosses the C ABI: this thread runs that shard too */
            mine.push_back(i);
        }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (size_t i : mine)
        work(i);
    for (auto &t : th)
        t.join();
    (void)hipSetDevice(cur);
    for (size_t i = 0; i < shards.size(); ++i)
        if (st[i] != HHMM_OK) {
            set_error("shard %zu (device %d): %s", i, devs[i], msg[i].c_str());
            return st[i];
        }
    if (res->pair_status)
        memcpy(res->pair_status, status.data(), (size_t)P * sizeof(int32_t));
    int64_t failures = 0;
    for (int64_t f : fails)
        failures += f;
    if (failures) {
        set_error("%lld pair(s) hit an unset Viterbi back-pointer (Stan would throw)", (long long)failures);
        return HHMM_WARN_PAIR_FAILURES;
    }
    return HHMM_OK;
}

} // namespace hhmm

using namespace hhmm;

extern "C" {

const char *hhmm_version(void) { return "hhmm-mi355x 0.3.0 gfx950 abi 2 src " HHMM_SOURCE_HASH; }

const char *hhmm_last_error(void) { return g_last_error.c_str(); }

int64_t hhmm_num_pairs(const hhmm_request *req) { return npairs(req); }

hhmm_status hhmm_validate(const hhmm_request *req, const hhmm_result *res, int host_pointers)
{
    return validate(req, res, host_pointers != 0);
}

hhmm_status hhmm_init(int ndev)
{
    hhmm_status s = check_device();
    if (s != HHMM_OK)
        return s;
    int n = 0;
    (void)hipGetDeviceCount(&n);
    if (ndev > n) {
        set_error("%d devices requested, %d visible", ndev, n);
        return HHMM_ERR_NO_DEVICE;
    }
    std::vector<int> d;
    for (int i = 0; i < (ndev > 0 ? ndev : 1); ++i) {
        if ((s = check_arch(i)) != HHMM_OK)
            return s;
        d.push_back(i);
    }
    std::lock_guard<std::mutex> g(devset().mu);
    devset().devs = d; /* HHMM_DEVICE_SET shards over devices 0 .. ndev-1 */
    return HHMM_OK;
}

hhmm_status hhmm_shutdown(void)
{
    pool_release_all();
    host_release_all();
    return HHMM_OK;
}

hhmm_status hhmm_workspace_size(const hhmm_request *req, size_t *bytes)
{
    if (!req || !bytes) {
        set_error("NULL argument");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    const int64_t P = npairs(req);
    if (P < 1) {
        set_error("request describes no pairs");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    *bytes = workspace_bytes(req->model, req->data.K, req->data.L, req->data.T_max, req->data.T_oos_max, P, req->outputs,
                            (uint32_t)req->flags, req->data.n_series, req->pairing);
    return HHMM_OK;
}

hhmm_status hhmm_run_device(const hhmm_request *req, hhmm_result *res, void *workspace, size_t workspace_bytes_,
                            void *stream)
{
    hhmm_status s = validate(req, res, false);
    if (s != HHMM_OK)
        return s;
    if (!device_supported(req->model)) {
        set_error("model %d has no gfx950 path in this build", req->model);
        return HHMM_ERR_UNSUPPORTED;
    }
    if ((s = check_device()) != HHMM_OK)
        return s;
    size_t need = 0;
    hhmm_workspace_size(req, &need);
    if (workspace_bytes_ < need || (!workspace && need > 256)) {
        set_error("workspace of %zu bytes < %zu required", workspace_bytes_, need);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    /* the data arrays are device memory: their data-block bounds are checked on
     * the device, pair by pair (HHMM_PAIR_INVALID_DATA) */
    return launch_all(req, res, npairs(req), workspace, (hipStream_t)stream, nullptr, 0, true);
}

hhmm_status hhmm_run(const hhmm_request *req, hhmm_result *res)
{
    hhmm_status s = validate(req, res, true);
    if (s != HHMM_OK)
        return s;
    if (!device_supported(req->model)) {
        set_error("model %d has no gfx950 path in this build", req->model);
        return HHMM_ERR_UNSUPPORTED;
    }
    if ((s = check_device()) != HHMM_OK)
        return s;
    if (req->device == HHMM_DEVICE_SET)
        return run_sharded(req, res);
    int dev = req->device;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess)
            return hip_fail(hipGetLastError(), "hipGetDevice");
    }
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess)
        return hip_fail(e, "hipSetDevice");
    const int64_t P = npairs(req);
    std::vector<int32_t> status((size_t)P, 0);
    int64_t failures = 0;
    s = run_on_device(req, res, whole_shard(req), status.data(), &failures);
    if (s != HHMM_OK)
        return s;
    if (res->pair_status)
        memcpy(res->pair_status, status.data(), (size_t)P * sizeof(int32_t));
    if (failures) {
        set_error("%lld pair(s) hit an unset Viterbi back-pointer (Stan would throw)", (long long)failures);
        return HHMM_WARN_PAIR_FAILURES;
    }
    return HHMM_OK;
}

int hhmm_device_set(int32_t *ordinals, int capacity)
{
    std::lock_guard<std::mutex> g(devset().mu);
    const std::vector<int> d = devset().devs.empty() ? std::vector<int>{0} : devset().devs;
    for (int i = 0; i < (int)d.size() && i < capacity; ++i)
        if (ordinals)
            ordinals[i] = d[(size_t)i];
    return (int)d.size();
}

hhmm_status hhmm_init_devices(const int32_t *ordinals, int n)
{
    hhmm_status s = check_device();
    if (s != HHMM_OK)
        return s;
    if (!ordinals || n < 1) {
        set_error("hhmm_init_devices needs n >= 1 ordinals");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    int vis = 0;
    (void)hipGetDeviceCount(&vis);
    std::vector<int> d;
    for (int i = 0; i < n; ++i) {
        if (ordinals[i] < 0 || ordinals[i] >= vis) {
            set_error("device ordinal %d not visible (%d devices)", ordinals[i], vis);
            return HHMM_ERR_NO_DEVICE;
        }
        if ((s = check_arch(ordinals[i])) != HHMM_OK)
            return s;
        d.push_back(ordinals[i]);
    }
    std::lock_guard<std::mutex> g(devset().mu);
    devset().devs = d;
    return HHMM_OK;
}

/* ---- one series split over ranks along T (include/hhmm.h hhmm_segment) ---- */
static hhmm_status segment_check(const hhmm_request *req, const hhmm_segment *seg, hhmm_request &r2)
{
    if (!req || !seg) {
        set_error("NULL argument");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    const int m = req->model;
    if (!(m == HHMM_MODEL_HMM_GAUSS || m == HHMM_MODEL_HMM_MULTINOM || m == HHMM_MODEL_HMM_MULTINOM_SEMISUP ||
          m == HHMM_MODEL_TAYAL) ||
        req->data.K > kMaxKLarge ||
        (req->data.K > kMaxK && m != HHMM_MODEL_HMM_MULTINOM && m != HHMM_MODEL_HMM_GAUSS)) {
        set_error("segment windows: the HMM family at K <= %d (hmm, hmm-multinom, semisup, tayal), "
                  "hmm and hmm-multinom at K <= %d", kMaxK, kMaxKLarge);
        return HHMM_ERR_UNSUPPORTED;
    }
    const uint32_t ok = HHMM_OUT_LOGLIK | HHMM_OUT_ALPHA | HHMM_OUT_BETA | HHMM_OUT_UNGAMMA | HHMM_OUT_GAMMA;
    if (req->outputs & ~ok) {
        set_error("segment windows: outputs 0x%x have no segment form (loglik, alpha_tk, beta_tk, ungamma_tk, "
                  "gamma_tk only; the Viterbi and FFBS stay sequential per pair)", req->outputs & ~ok);
        return HHMM_ERR_UNSUPPORTED;
    }
    if (req->data.T) {
        set_error("segment windows: every series spans the whole window (data.T must be NULL)");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (req->abi_version != HHMM_ABI_VERSION || npairs(req) < 1 || req->data.T_max < 1 || req->data.K < 1 ||
        (is_discrete(m) && (req->data.L < 1 || !req->data.x_int)) || (m == HHMM_MODEL_HMM_GAUSS && !req->data.x_real)) {
        set_error("segment windows: malformed request (abi, pairs, T_max, K, L or observations)");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    r2 = *req;
    r2.flags = (req->flags & ~(int32_t)HHMM_FLAG_SCAN_OFF) | (int32_t)HHMM_FLAG_SCAN_FORCE;
    return HHMM_OK;
}

hhmm_status hhmm_segment_workspace_size(const hhmm_request *req, size_t *bytes)
{
    hhmm_segment dummy{1, 1, nullptr, nullptr, nullptr};
    hhmm_request r2;
    hhmm_status s = segment_check(req, &dummy, r2);
    if (s != HHMM_OK)
        return s;
    return hhmm_workspace_size(&r2, bytes);
}

static hhmm_status segment_run(const hhmm_request *req, hhmm_result *res, const hhmm_segment *seg, void *ws,
                               size_t wsb, void *stream, int phase)
{
    hhmm_request r2;
    hhmm_status s = segment_check(req, seg, r2);
    if (s != HHMM_OK)
        return s;
    hhmm_result empty;
    memset(&empty, 0, sizeof(empty));
    hhmm_result *rr = res ? res : &empty;
    if (phase == 1) {
        if (!seg->summary) {
            set_error("segment summary: seg->summary is NULL");
            return HHMM_ERR_INVALID_ARGUMENT;
        }
        /* the request side (draw and data pointers) before any launch */
        if ((s = validate_impl(&r2, nullptr, false)) != HHMM_OK)
            return s;
    } else {
        if ((!seg->first && !seg->enter) || (!seg->last && !seg->leave)) {
            set_error("segment finish: a window that is not first needs enter, one that is not last needs leave");
            return HHMM_ERR_INVALID_ARGUMENT;
        }
        if ((s = validate(&r2, rr, false)) != HHMM_OK)
            return s;
    }
    if ((s = check_device()) != HHMM_OK)
        return s;
    size_t need = 0;
    hhmm_workspace_size(&r2, &need);
    if (wsb < need || !ws) {
        set_error("workspace of %zu bytes < %zu required (hhmm_segment_workspace_size)", wsb, need);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    /* both calls check the window's data: the summary marks a bad pair's record
     * (NaN log scale) so that every rank chaining it flags the pair */
    return launch_all(&r2, rr, npairs(&r2), ws, (hipStream_t)stream, seg, phase, true);
}

hhmm_status hhmm_segment_summary_device(const hhmm_request *req, const hhmm_segment *seg, void *workspace,
                                        size_t workspace_bytes_, void *stream)
{
    return segment_run(req, nullptr, seg, workspace, workspace_bytes_, stream, 1);
}

hhmm_status hhmm_segment_finish_device(const hhmm_request *req, hhmm_result *res, const hhmm_segment *seg,
                                       void *workspace, size_t workspace_bytes_, void *stream)
{
    return segment_run(req, res, seg, workspace, workspace_bytes_, stream, 2);
}

hhmm_status hhmm_selftest_shards(const hhmm_request *req, hhmm_result *res, int nshards)
{
    hhmm_status s = validate(req, res, true);
    if (s != HHMM_OK)
        return s;
    if (nshards < 1) {
        set_error("nshards must be >= 1");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    hhmm_request dreq = *req;
    hhmm_result dres = *res;
    std::vector<ArrayDesc> arrays;
    describe(req, res, &dreq, &dres, arrays);
    for (const Shard &sh : make_shards(req, nshards)) {
        for (const ArrayDesc &a : arrays) {
            const ShardRows r = shard_rows(a.host, a, sh);
            std::vector<char> packed(r.rows * r.width);
            copy_shard_host(packed.data(), a.host, a, sh, true);
            if (!a.output) /* inputs only travel host -> shard: back into a scratch twin */
                continue;
            const size_t n = packed.size() / a.esize;
            for (size_t i = 0; i < n; ++i) {
                if (a.esize == sizeof(double)) {
                    double v;
                    memcpy(&v, &packed[i * 8], 8);
                    v += 1.0;
                    memcpy(&packed[i * 8], &v, 8);
                } else {
                    int32_t v;
                    memcpy(&v, &packed[i * 4], 4);
                    v += 1;
                    memcpy(&packed[i * 4], &v, 4);
                }
            }
            copy_shard_host(packed.data(), a.host, a, sh, false);
        }
    }
    return HHMM_OK;
}

hhmm_status hhmm_selftest_pipeline(const hhmm_request *req, hhmm_result *res, int nshards, int nchunks)
{
    hhmm_status s = validate(req, res, true);
    if (s != HHMM_OK)
        return s;
    if (nshards < 1 || nchunks < 1) {
        set_error("nshards and nchunks must be >= 1");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    hhmm_request dreq = *req;
    hhmm_result dres = *res;
    std::vector<ArrayDesc> arrays;
    describe(req, res, &dreq, &dres, arrays);
    const bool ragged = req->data.T != nullptr || req->data.T_oos != nullptr;
    for (const Shard &sh : make_shards(req, nshards)) {
        for (const Shard &c : split_shard(req, sh, nchunks)) {
            const ChunkLayout L = chunk_layout(req, arrays, c, ragged);
            std::vector<char> slot(L.total, 0);
            /* the gather, as run_on_device stages it, checked byte for byte
             * against a row-by-row pack of the same slice */
            for (size_t i = 0; i < arrays.size(); ++i) {
                const ArrayDesc &a = arrays[i];
                if (L.off[i] >= L.in_end)
                    continue;
                const ShardRows r = shard_rows(a.host, a, L.sh);
                par_copy_rows(slot.data() + L.off[i], r.width, r.base, r.pitch, r.width, r.rows);
                std::vector<char> ref(r.rows * r.width);
                copy_shard_host(ref.data(), a.host, a, L.sh, true);
                if (memcmp(ref.data(), slot.data() + L.off[i], ref.size()) != 0) {
                    set_error("pipeline self-test: the staged slice of an input differs");
                    return HHMM_ERR_INVALID_ARGUMENT;
                }
            }
            /* the "kernel": every output element + 1, every pair status 1 */
            for (size_t i = 0; i < arrays.size(); ++i) {
                const ArrayDesc &a = arrays[i];
                if (!a.output)
                    continue;
                const size_t n = shard_bytes(a, L.sh) / a.esize;
                for (size_t k = 0; k < n; ++k) {
                    char *e = slot.data() + L.off[i] + k * a.esize;
                    if (a.esize == sizeof(double)) {
                        double v;
                        memcpy(&v, e, 8);
                        v += 1.0;
                        memcpy(e, &v, 8);
                    } else {
                        int32_t v;
                        memcpy(&v, e, 4);
                        v += 1;
                        memcpy(e, &v, 4);
                    }
                }
            }
            for (int64_t q = 0; q < L.P; ++q) {
                const int32_t one = 1;
                memcpy(slot.data() + L.status_off + (size_t)q * 4, &one, 4);
            }
            /* the scatter of the downloaded region, as run_on_device runs it */
            const char *down = slot.data() + L.out_begin;
            for (size_t i = 0; i < arrays.size(); ++i) {
                const ArrayDesc &a = arrays[i];
                if (!a.output)
                    continue;
                const ShardRows r = shard_rows(a.host, a, L.sh);
                par_copy_rows(r.base, r.pitch, down + (L.off[i] - L.out_begin), r.width, r.width, r.rows);
            }
            if (res->pair_status) {
                const ArrayDesc sa{res->pair_status, nullptr, (size_t)npairs(req), sizeof(int32_t), true, PAIRS};
                const ShardRows r = shard_rows(res->pair_status, sa, L.sh);
                par_copy_rows(r.base, r.pitch, down + (L.status_off - L.out_begin), r.width, r.width, r.rows);
            }
        }
    }
    return HHMM_OK;
}

hhmm_status hhmm_selftest_cr_log(const double *in, double *out, int64_t n)
{
    hhmm_status s = check_device();
    if (s != HHMM_OK)
        return s;
    return selftest_cr_math(in, out, n, 0);
}

hhmm_status hhmm_selftest_cr_exp(const double *in, double *out, int64_t n)
{
    hhmm_status s = check_device();
    if (s != HHMM_OK)
        return s;
    return selftest_cr_math(in, out, n, 1);
}

hhmm_status hhmm_selftest_det_log(const double *in, double *out, int64_t n)
{
    hhmm_status s = check_device();
    if (s != HHMM_OK)
        return s;
    return selftest_cr_math(in, out, n, 2);
}

hhmm_status hhmm_selftest_det_exp(const double *in, double *out, int64_t n)
{
    hhmm_status s = check_device();
    if (s != HHMM_OK)
        return s;
    return selftest_cr_math(in, out, n, 3);
}

} /* extern "C" */

/* ------------------------------------------------------------------ */
/* Feature extractor entry points (include/hhmm_features.h)            */
/* ------------------------------------------------------------------ */

extern "C" {

static hhmm_status check_ticks(const hhmm_ticks *tk, const hhmm_legs *lg)
{
    if (!tk || !lg) {
        set_error("NULL ticks / legs");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (tk->n < 3 || tk->n > 0x7fffffffLL) {
        set_error("n = %lld ticks outside 3..2^31-1", (long long)tk->n);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (!tk->price || !tk->size || !tk->time) {
        set_error("price, size and time are required");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (lg->capacity < 0) {
        set_error("negative leg capacity");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    return HHMM_OK;
}

hhmm_status hhmm_features_workspace_size(int64_t n, size_t *bytes)
{
    if (!bytes || n < 0) {
        set_error("bad argument");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    *bytes = features_workspace_bytes(n);
    return HHMM_OK;
}

hhmm_status hhmm_extract_features_device(const hhmm_ticks *ticks, hhmm_legs *legs, void *workspace,
                                         size_t workspace_bytes_, void *stream)
{
    hhmm_status s = check_ticks(ticks, legs);
    if (s != HHMM_OK)
        return s;
    if ((s = check_device()) != HHMM_OK)
        return s;
    return features_run_device(ticks, legs, workspace, workspace_bytes_, (hipStream_t)stream);
}

hhmm_status hhmm_extract_features(const hhmm_ticks *ticks, hhmm_legs *legs, int device)
{
    hhmm_status s = check_ticks(ticks, legs);
    if (s != HHMM_OK)
        return s;
    if ((s = check_device()) != HHMM_OK)
        return s;
    int dev = device;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess)
        return hip_fail(hipGetLastError(), "hipGetDevice");
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess)
        return hip_fail(e, "hipSetDevice");
    const int64_t n = ticks->n;
    const int64_t cap = legs->capacity;
    std::vector<void *> owned;
    auto cleanup = [&]() {
        for (void *p : owned)
            pool_put(p);
    };
    auto get = [&](size_t bytes) -> void * {
        void *p = pool_get(dev, bytes ? bytes : 8);
        if (p)
            owned.push_back(p);
        return p;
    };
    hhmm_ticks dt = *ticks;
    const double *hin[3] = {ticks->price, ticks->size, ticks->time};
    const double **din[3] = {&dt.price, &dt.size, &dt.time};
    for (int i = 0; i < 3; ++i) {
        void *p = get(sizeof(double) * (size_t)n);
        if (!p) {
            cleanup();
            set_error("device allocation failed (ticks)");
            return HHMM_ERR_OUT_OF_MEMORY;
        }
        e = hipMemcpy(p, hin[i], sizeof(double) * (size_t)n, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            cleanup();
            return hip_fail(e, "hipMemcpy H2D (ticks)");
        }
        *din[i] = (const double *)p;
    }
    hhmm_legs dl = *legs;
    struct Col {
        void *host;
        void **dev;
        size_t es;
    } cols[] = {{legs->price, (void **)&dl.price, 8},     {legs->start, (void **)&dl.start, 4},
                {legs->end, (void **)&dl.end, 4},         {legs->size_av, (void **)&dl.size_av, 8},
                {legs->f0, (void **)&dl.f0, 4},           {legs->f1, (void **)&dl.f1, 4},
                {legs->f2, (void **)&dl.f2, 4},           {legs->feature, (void **)&dl.feature, 4},
                {legs->trend, (void **)&dl.trend, 4},     {legs->x, (void **)&dl.x, 4},
                {legs->sign, (void **)&dl.sign, 4}};
    for (auto &c : cols) {
        if (!c.host || cap == 0) {
            *c.dev = nullptr;
            continue;
        }
        void *p = get(c.es * (size_t)cap);
        if (!p) {
            cleanup();
            set_error("device allocation failed (legs)");
            return HHMM_ERR_OUT_OF_MEMORY;
        }
        *c.dev = p;
    }
    const size_t wsb = features_workspace_bytes(n);
    void *ws = get(wsb);
    if (!ws) {
        cleanup();
        set_error("workspace allocation of %zu bytes failed", wsb);
        return HHMM_ERR_OUT_OF_MEMORY;
    }
    s = features_run_device(&dt, &dl, ws, wsb, nullptr);
    legs->n_legs = dl.n_legs;
    if (s == HHMM_OK) {
        for (auto &c : cols) {
            if (!*c.dev)
                continue;
            e = hipMemcpy(c.host, *c.dev, c.es * (size_t)dl.n_legs, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                cleanup();
                return hip_fail(e, "hipMemcpy D2H (legs)");
            }
        }
    }
    cleanup();
    return s;
}

} // extern "C"
