"""GPU: the IOHMM filter where its linear-space form underflows (VERDICT r3,
"no log-space fallback").  Saturated softmax transitions (w scaled x400 /
x2000) put A_t = 0 in double on every state the renormalised linear filter
holds, so s_t = 0 there (tests/test_iohmm_underflow.py shows these inputs do
that); the reference's log-space recursion (iohmm-reg/stan/iohmm-reg.stan:59-102,
iohmm-mix/stan/iohmm-hmix.stan:64-121) stays finite.  The sweeps list such
pairs and hhmm_iolog.hip re-runs their filter outputs in log space, so loglik,
alpha, beta, gamma, ungamma, unalpha, unbeta and oblik_t match the oracle
within tests/tolerances.py; the Viterbi stays bit-exact.  Every IOHMM layout
that writes a filter output is covered: the lane sweep (K <= 8, with and
without the Viterbi), the state-parallel sweep (loglik / alpha / gamma, and with
FFBS), and the large-K group sweep."""
import numpy as np
import pytest

from hhmm_amd import synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

FULL = ["loglik", "alpha_tk", "unalpha_tk", "beta_tk", "unbeta_tk", "ungamma_tk", "gamma_tk"]
VIT = ["zstar_t", "logp_zstar"]


def pars_for(model, base):
    """The outputs of `base` the model declares (synth.PARS), plus oblik_t where it has one."""
    extra = ["oblik_t"] if "oblik_t" in synth.PARS[model] else []
    return [p for p in base if p in synth.PARS[model]] + extra


def run_both(engine, oracle, model, data, draws, pars, uniforms=None, flags=0):
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, return_status=True, uniforms=uniforms,
                       flags=flags)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True, nthreads=8, uniforms=uniforms)
    assert np.isfinite(ref["loglik"]).all()
    # pair_status is the Viterbi's (the oracle always decodes; the engine only when asked)
    compare_all(got, ref, pars + (["pair_status"] if "zstar_t" in pars else []))


@pytest.mark.parametrize("scale", [400.0, 2000.0])
@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-mix", "iohmm-hmix", "iohmm-hmix-lite"])
@pytest.mark.parametrize("profile", ["lanes-viterbi", "lanes", "states"])
def test_iohmm_k4_saturated_T10k(engine, oracle, model, scale, profile):
    """K = 4, T = 10^4: the lane sweep with the Viterbi (IO_CR), the lane sweep
    without it (every filter output), the state-parallel sweep (loglik /
    alpha / gamma)."""
    data, draws = synth.GENERATORS[model](N=2, S=6, T=10_000, K=4, M=4)
    draws["w_km"] = draws["w_km"] * scale
    if profile == "states":
        pars = pars_for(model, ["loglik", "alpha_tk", "gamma_tk"])
    else:
        pars = pars_for(model, FULL) + (VIT if profile == "lanes-viterbi" and model != "iohmm-hmix-lite" else [])
    run_both(engine, oracle, model, data, draws, pars)


@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-hmix"])
def test_iohmm_k4_saturated_with_ffbs(engine, oracle, model):
    """The state-parallel IO_DET sweep (loglik, gamma and FFBS draws): the
    filter outputs come from the log-space re-run, the draws stay the
    contract's bit for bit."""
    N, S, T = 2, 6, 4000
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T, K=4, M=4)
    draws["w_km"] = draws["w_km"] * 400.0
    run_both(engine, oracle, model, data, draws, pars_for(model, ["loglik", "gamma_tk"]) + ["z_ffbs"],
             uniforms=synth.ffbs_uniforms(N * S, T))


def test_iohmm_mixed_batch_only_some_pairs_rerun(engine, oracle):
    """Draws 1 and 4 saturated, the rest mild, ragged T: the list holds only
    some pairs of a wave, and the others keep the linear sweep's outputs."""
    data, draws = synth.iohmm_reg(N=3, S=6, T=3000, K=4, M=4)
    data["T"] = np.array([3000, 17, 2411], dtype=np.int32)
    w = np.array(draws["w_km"])
    w[[1, 4]] *= 800.0
    draws["w_km"] = w
    run_both(engine, oracle, "iohmm-reg", data, draws, FULL + VIT)


@pytest.mark.parametrize("K", [12, 16, 23])
@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-hmix"])
def test_iohmm_large_K_saturated(engine, oracle, model, K):
    """The large-K group sweep (hhmm_lkio.h) at T = 2000, w x400."""
    data, draws = synth.GENERATORS[model](N=2, S=3, T=2000, K=K, M=4)
    draws["w_km"] = draws["w_km"] * 400.0
    run_both(engine, oracle, model, data, draws, pars_for(model, FULL) + VIT)
