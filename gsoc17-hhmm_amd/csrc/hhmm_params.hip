/*
 * hhmm_params.hip -- gfx950 parameter-draw ingestion (C ABI
 * in include/hhmm_params.h): Stan's constraining transforms for a batch of
 * unconstrained draws, written straight into the hhmm_draws layouts.
 *
 * One lane per draw; theta [S, n_unc] and every output [S, ...] are draw
 * fastest, so each element is one coalesced wave access.  A model is a short
 * table of segments (declaration order of its parameters block, e.g.
 * hmm/stan/hmm.stan:13-22); each segment is `count` array elements of a
 * length-n vector of one constraint kind, stored at out[s + S*(a + count*v)]
 * -- the [S, K, L] / [S, K, K] / [S, K] layouts of include/hhmm.h.
 */
#include <hip/hip_runtime.h>
#include <math.h>

#include <vector>

#include "hhmm_internal.h"
#include "hhmm_params.h"

#ifndef HHMM_MATH_FN
#define HHMM_MATH_FN static __device__ __forceinline__
#define HHMM_MATH_TABLE static __constant__
#endif
#include "hhmm_crmath.h"

namespace hhmm {

enum SegKind { SEG_SIMPLEX = 0, SEG_ORDERED = 1, SEG_LB = 2, SEG_LUB01 = 3, SEG_IDENT = 4 };

struct Seg {
    int kind, count, n;
    double lb;
    double *out;
};

constexpr int kMaxSeg = 8;

struct ParamPlan {
    int nseg;
    int64_t S, n_unc;
    Seg seg[kMaxSeg];
};

/* Stan Math inv_logit (stable form): exp(a) below log(epsilon),
 * exp(a) / (1 + exp(a)) for a < 0, 1 / (1 + exp(-a)) otherwise. */
__device__ __forceinline__ double stan_inv_logit(double a)
{
    if (a < 0) {
        const double ea = hhmm_cr_exp(a);
        if (a < -36.04365338911715) /* LOG_EPSILON = log(2^-52) */
            return ea;
        return ea / (1 + ea);
    }
    return 1.0 / (1 + hhmm_cr_exp(-a));
}

/* lub_constrain(x, 0, 1) (Stan Math): inv_logit with the 1 - 1e-15 / 1e-15
 * clamps, then lb + (ub - lb) * inv_logit_x. */
__device__ __forceinline__ double stan_lub01(double x)
{
    double il;
    if (x > 0) {
        const double em = hhmm_cr_exp(-x);
        il = 1.0 / (1.0 + em);
        if (x < __builtin_inf() && il == 1)
            il = 1 - 1e-15;
    } else {
        const double ex = hhmm_cr_exp(x);
        il = 1.0 - 1.0 / (1.0 + ex);
        if (x > -__builtin_inf() && il == 0)
            il = 1e-15;
    }
    return 0.0 + (1.0 - 0.0) * il;
}

__global__ void __launch_bounds__(256) constrain_kernel(const ParamPlan pl, const double *theta)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= pl.S)
        return;
    const int64_t S = pl.S;
    int64_t i = 0; /* position in the unconstrained vector */
    for (int g = 0; g < pl.nseg; ++g) {
        const Seg sg = pl.seg[g];
        for (int a = 0; a < sg.count; ++a) {
            double *o = sg.out ? sg.out + s + S * a : nullptr;
            const int64_t ostep = S * (int64_t)sg.count;
            if (sg.kind == SEG_SIMPLEX) {
                /* simplex_constrain: stick-breaking over n - 1 values */
                const int km1 = sg.n - 1;
                double stick = 1.0;
                for (int k = 0; k < km1; ++k) {
                    const double z = stan_inv_logit(theta[s + S * (i + k)] - hhmm_cr_log((double)(km1 - k)));
                    const double x = stick * z;
                    stick -= x;
                    if (o)
                        o[ostep * k] = x;
                }
                if (o)
                    o[ostep * km1] = stick;
                i += km1;
            } else if (sg.kind == SEG_ORDERED) {
                double y = theta[s + S * i];
                if (o)
                    o[0] = y;
                for (int k = 1; k < sg.n; ++k) {
                    y = y + hhmm_cr_exp(theta[s + S * (i + k)]);
                    if (o)
                        o[ostep * k] = y;
                }
                i += sg.n;
            } else {
                for (int k = 0; k < sg.n; ++k) {
                    const double u = theta[s + S * (i + k)];
                    double v = u;
                    if (sg.kind == SEG_LB)
                        v = hhmm_cr_exp(u) + sg.lb;
                    else if (sg.kind == SEG_LUB01)
                        v = stan_lub01(u);
                    if (o)
                        o[ostep * k] = v;
                }
                i += sg.n;
            }
        }
    }
}

/* The parameters block of each program as segments (include/hhmm_params.h). */
static bool make_plan(int model, int K, int L, int M, const hhmm_param_out *o, ParamPlan &pl)
{
    pl.nseg = 0;
    auto add = [&](int kind, int count, int n, double lb, double *out) {
        pl.seg[pl.nseg++] = Seg{kind, count, n, lb, out};
    };
    hhmm_param_out z = {};
    if (!o)
        o = &z;
    switch (model) {
    case HHMM_MODEL_HMM_GAUSS: /* hmm.stan:13-22 */
        add(SEG_SIMPLEX, 1, K, 0, o->p_1k);
        add(SEG_SIMPLEX, K, K, 0, o->A_ij);
        add(SEG_ORDERED, 1, K, 0, o->mu_k);
        add(SEG_LB, K, 1, 0.0001, o->sigma_k);
        return K >= 1;
    case HHMM_MODEL_HMM_MULTINOM: /* hmm-multinom.stan:14-22 */
    case HHMM_MODEL_HMM_MULTINOM_SEMISUP: /* hmm-multinom-semisup.stan:16-24 */
        add(SEG_SIMPLEX, 1, K, 0, o->p_1k);
        add(SEG_SIMPLEX, K, K, 0, o->A_ij);
        add(SEG_SIMPLEX, K, L, 0, o->phi_k);
        return K >= 1 && L >= 1;
    case HHMM_MODEL_IOHMM_REG: /* iohmm-reg.stan:16-24 */
        add(SEG_SIMPLEX, 1, K, 0, o->p_1k);
        add(SEG_IDENT, K, M, 0, o->w_km);
        add(SEG_IDENT, K, M, 0, o->b_km);
        add(SEG_LB, K, 1, 0.0001, o->s_k);
        return K >= 1 && M >= 1;
    case HHMM_MODEL_IOHMM_MIX: /* iohmm-mix.stan:17-26 */
    case HHMM_MODEL_IOHMM_HMIX: /* iohmm-hmix.stan:13-23 */
    case HHMM_MODEL_IOHMM_HMIX_LITE: /* iohmm-hmix-lite.stan:13-23 */
        add(SEG_SIMPLEX, 1, K, 0, o->p_1k);
        add(SEG_IDENT, K, M, 0, o->w_km);
        add(SEG_SIMPLEX, K, L, 0, o->lambda_kl);
        add(SEG_ORDERED, K, L, 0, o->mu_kl);
        add(SEG_LB, K, L, 0.0, o->s_kl);
        if (model == HHMM_MODEL_IOHMM_HMIX)
            add(SEG_ORDERED, 1, K, 0, o->hypermu_k);
        if (model == HHMM_MODEL_IOHMM_HMIX_LITE)
            add(SEG_IDENT, K, 1, 0, o->hypermu_k);
        return K >= 1 && M >= 1 && L >= 1;
    case HHMM_MODEL_TAYAL: /* hhmm-tayal2009.stan:15-22 */
    case HHMM_MODEL_TAYAL_LITE: /* hhmm-tayal2009-lite.stan:19-26 */
        add(SEG_LUB01, 1, 1, 0, o->p_11);
        add(SEG_SIMPLEX, 2, 2, 0, o->A_row);
        add(SEG_SIMPLEX, K, L, 0, o->phi_k);
        return K == 4 && L >= 1;
    default:
        return false;
    }
}

static int64_t plan_len(const ParamPlan &pl)
{
    int64_t n = 0;
    for (int g = 0; g < pl.nseg; ++g)
        n += (int64_t)pl.seg[g].count * (pl.seg[g].kind == SEG_SIMPLEX ? pl.seg[g].n - 1 : pl.seg[g].n);
    return n;
}

} // namespace hhmm

using namespace hhmm;

extern "C" {

int64_t hhmm_num_unconstrained(int model, int K, int L, int M)
{
    ParamPlan pl;
    if (K < 1 || K > 64 || L < 0 || L > 4096 || M < 0 || M > 4096 || !make_plan(model, K, L, M, nullptr, pl))
        return -1;
    return plan_len(pl);
}

static hhmm_status constrain_check(int model, int K, int L, int M, int64_t S, const double *theta,
                                   const hhmm_param_out *out, ParamPlan &pl)
{
    if (!theta || !out || S < 1) {
        set_error("constrain: NULL theta / out or S < 1");
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    if (hhmm_num_unconstrained(model, K, L, M) < 0 || !make_plan(model, K, L, M, out, pl)) {
        set_error("constrain: model %d with K=%d L=%d M=%d has no parameters block here", model, K, L, M);
        return HHMM_ERR_INVALID_ARGUMENT;
    }
    pl.S = S;
    pl.n_unc = plan_len(pl);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        (void)hipGetLastError();
        set_error("no HIP device visible: libhhmm has no CPU path (gfx950 required)");
        return HHMM_ERR_NO_DEVICE;
    }
    return HHMM_OK;
}

static hhmm_status constrain_launch(const ParamPlan &pl, const double *theta, hipStream_t st)
{
    hipLaunchKernelGGL(constrain_kernel, dim3((unsigned)((pl.S + 255) / 256)), dim3(256), 0, st, pl, theta);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("constrain_kernel launch: %s", hipGetErrorString(e));
        return HHMM_ERR_HIP;
    }
    return HHMM_OK;
}

hhmm_status hhmm_constrain_draws_device(int model, int K, int L, int M, int64_t S, const double *theta,
                                        hhmm_param_out *out, void *stream)
{
    ParamPlan pl;
    hhmm_status s = constrain_check(model, K, L, M, S, theta, out, pl);
    if (s != HHMM_OK)
        return s;
    return constrain_launch(pl, theta, (hipStream_t)stream);
}

hhmm_status hhmm_constrain_draws(int model, int K, int L, int M, int64_t S, const double *theta,
                                 hhmm_param_out *out, int device)
{
    ParamPlan pl;
    hhmm_status s = constrain_check(model, K, L, M, S, theta, out, pl);
    if (s != HHMM_OK)
        return s;
    if (device >= 0 && hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice(%d) failed", device);
        return HHMM_ERR_HIP;
    }
    std::vector<void *> owned;
    hipError_t e = hipSuccess;
    double *dtheta = nullptr;
    e = hipMalloc(&dtheta, sizeof(double) * (size_t)(S * (pl.n_unc > 0 ? pl.n_unc : 1)));
    if (e == hipSuccess) {
        owned.push_back(dtheta);
        e = hipMemcpy(dtheta, theta, sizeof(double) * (size_t)(S * pl.n_unc), hipMemcpyHostToDevice);
    }
    ParamPlan dpl = pl;
    for (int g = 0; g < dpl.nseg && e == hipSuccess; ++g) {
        if (!pl.seg[g].out)
            continue;
        void *p = nullptr;
        e = hipMalloc(&p, sizeof(double) * (size_t)(S * pl.seg[g].count * pl.seg[g].n));
        if (e == hipSuccess) {
            owned.push_back(p);
            dpl.seg[g].out = (double *)p;
        }
    }
    if (e == hipSuccess) {
        s = constrain_launch(dpl, dtheta, nullptr);
        for (int g = 0; g < dpl.nseg && s == HHMM_OK && e == hipSuccess; ++g)
            if (pl.seg[g].out)
                e = hipMemcpy(pl.seg[g].out, dpl.seg[g].out,
                              sizeof(double) * (size_t)(S * pl.seg[g].count * pl.seg[g].n), hipMemcpyDeviceToHost);
    }
    for (void *p : owned)
        (void)hipFree(p);
    if (e != hipSuccess) {
        set_error("constrain: %s", hipGetErrorString(e));
        return (e == hipErrorOutOfMemory) ? HHMM_ERR_OUT_OF_MEMORY : HHMM_ERR_HIP;
    }
    return s;
}

} // extern "C"
