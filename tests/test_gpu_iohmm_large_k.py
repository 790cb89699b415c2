"""GPU: the IOHMM programs at large K (8 < K <= 32; hhmm_lkio.h) against the
oracle -- iohmm-reg, iohmm-mix, iohmm-hmix and iohmm-hmix-lite with Stan's free
K (iohmm-reg/stan/iohmm-reg.stan:9).  One group of 16 or 32 lanes owns a pair,
lane j state j; the softmax over states is each lane's sequential max / sum
over the exchanged vector, so A_t, log A_t, the Viterbi paths, logp_zstar and
pair_status are bit-exact, the posteriors within tests/tolerances.py; the
fitted-output draws (lkfit_kernel, same layout) bit-exact given hat_rand."""
import numpy as np
import pytest

from hhmm_amd import synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

MODELS = ["iohmm-reg", "iohmm-mix", "iohmm-hmix", "iohmm-hmix-lite"]
NO = {"z_ffbs", "hatpi_tk", "hatz_t", "hatl_t", "hatx_t"}


def pars_of(model):
    return [p for p in synth.PARS[model] if p not in NO]


def run_both(engine, oracle, model, data, draws, pars, pairing="grid"):
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, pairing=pairing, lib=engine, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, pairing=pairing, return_status=True, nthreads=8)
    compare_all(got, ref, pars + ["pair_status"])
    assert got["status"] == ref["status"]


@pytest.mark.parametrize("K", [9, 12, 16, 17, 23, 24, 32])
@pytest.mark.parametrize("T", [1, 2, 37, 200])
@pytest.mark.parametrize("model", MODELS)
def test_iohmm_large_K(engine, oracle, model, K, T):
    data, draws = synth.GENERATORS[model](N=2, S=5, T=T, K=K, M=4)
    run_both(engine, oracle, model, data, draws, pars_of(model))


@pytest.mark.parametrize("K", [12, 23])
@pytest.mark.parametrize("model", MODELS)
def test_iohmm_large_K_ragged(engine, oracle, model, K):
    N = 5
    data, draws = synth.GENERATORS[model](N=N, S=3, T=300, K=K, M=4)
    data["T"] = np.array([300, 1, 65, 17, 211], dtype=np.int32)
    run_both(engine, oracle, model, data, draws, pars_of(model))


@pytest.mark.parametrize("pairing", ["zip", "block"])
def test_iohmm_large_K_pairings(engine, oracle, pairing):
    N = 6
    S = N if pairing == "zip" else 2 * N
    data, draws = synth.iohmm_reg(N=N, S=S, T=120, K=20, M=4)
    run_both(engine, oracle, "iohmm-reg", data, draws, pars_of("iohmm-reg"), pairing=pairing)


@pytest.mark.parametrize("pars", [["zstar_t", "logp_zstar"], ["loglik", "gamma_tk"], ["loglik", "zstar_t"]],
                         ids=["viterbi-only", "posteriors-only", "mixed"])
@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-hmix"])
def test_iohmm_large_K_profiles(engine, oracle, model, pars):
    """The correctly rounded sweep (any Viterbi output) and the libm sweep
    (posteriors only) on their own."""
    data, draws = synth.GENERATORS[model](N=3, S=4, T=150, K=23, M=4)
    run_both(engine, oracle, model, data, draws, pars)


@pytest.mark.parametrize("scale", [1.0, 40.0, 400.0])
def test_iohmm_large_K_softmax_regimes(engine, oracle, scale):
    """Mild to saturated transitions (one state takes A = 1 - tiny): the
    sequential softmax and the correctly rounded log A stay bit-exact.  At
    scale 400 A_t underflows to 0 on every state the linear filter's
    renormalised mass sits on (s_t = 0; tests/test_iohmm_underflow.py), and
    the pairs' filter outputs come from the log-space re-run
    (hhmm_iolog.hip), finite like the reference's."""
    data, draws = synth.iohmm_reg(N=2, S=6, T=120, K=16, M=4)
    draws["w_km"] = draws["w_km"] * scale
    pars = ["zstar_t", "logp_zstar", "logA_ij", "loglik", "alpha_tk", "unbeta_tk"]
    run_both(engine, oracle, "iohmm-reg", data, draws, pars)


@pytest.mark.parametrize("K", [9, 16, 23, 32])
@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-mix", "iohmm-hmix"])
def test_iohmm_large_K_ffbs(engine, oracle, model, K):
    """FFBS draws at large K (the contract's IO_DET arithmetic, its own sweep),
    bit-exact with the oracle, beside the posterior and Viterbi outputs of
    the same request; ragged T."""
    import hhmm_amd
    N, S, T = 3, 4, 150
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T, K=K, M=4)
    data["T"] = np.array([150, 1, 77], dtype=np.int32)
    u = synth.ffbs_uniforms(N * S, T)
    pars = ["loglik", "gamma_tk", "z_ffbs", "zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, uniforms=u, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, uniforms=u, return_status=True, nthreads=8)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("K", [12, 23, 32])
@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-mix", "iohmm-hmix"])
def test_iohmm_large_K_fitted_draws(engine, oracle, model, K):
    """SURVEY §8 F4 at large K (iohmm-reg.stan:131-148, iohmm-hmix.stan:145-158; K is data,
    iohmm-reg.stan:9): hatpi_tk / hatz_t / hatl_t / hatx_t bit-exact given hat_rand,
    ragged series, alone and together with the recursion outputs (one call, two kernels)."""
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=3, S=24, T=41, K=K, M=4)
    data["T"] = np.array([41, 17, 1], dtype=np.int32)
    P = 72
    hr = synth.hat_rand(P, 41, seed=K)
    hat = synth.HAT_PARS[model]
    Tn = np.repeat(data["T"], 24)
    for pars in (hat, pars_of(model) + hat):
        got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, hat_rand=hr, return_status=True)
        ref = oracle.gqs(model, data, draws, pars=pars, hat_rand=hr, return_status=True, nthreads=8)
        for name in hat:
            for p in range(P):
                g, r = got[name][p, :Tn[p]], ref[name][p, :Tn[p]]
                assert np.array_equal(g.view(np.int64) if g.dtype == np.float64 else g,
                                      r.view(np.int64) if r.dtype == np.float64 else r), (model, K, name, p)
        rest = [n for n in pars if n not in hat]
        # pair_status is the Viterbi's (the oracle always decodes: T = 1 pairs are Q3's
        # unset back-pointer); compared where the engine decodes too
        names = rest + (["pair_status"] if "zstar_t" in pars else [])
        if names:  # (compare_all compares every output when given none)
            compare_all(got, ref, names)
