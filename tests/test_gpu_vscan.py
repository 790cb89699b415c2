"""GPU: the T-parallel exact Viterbi (gsoc17-hhmm_amd/csrc/hhmm_vscan.h) against the
oracle, bit for bit -- paths, logp_zstar and pair_status -- on the HMM family at
K = 2 and 4 (HHMM_FLAG_VIT_SCAN forces it below its automatic range; the C5
config tests in test_gpu_configs.py run it through the automatic dispatch).
Covers chunk edges (T = 1, 511..513, partial last chunks), ragged series, long
series crossing many binades of |delta|, the Tayal OOS pass and the invalid
back-pointer flag."""
import numpy as np
import pytest

from hhmm_amd import _abi, synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

VIT = ["zstar_t", "logp_zstar"]
SCAN = _abi.FLAG_VIT_SCAN


def run(engine, oracle, model, data, draws, pars=VIT, flags=SCAN):
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, return_status=True, flags=flags)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True, nthreads=8)
    compare_all(got, ref, pars + ["pair_status"])
    return got, ref


CASES = [("hhmm-tayal2009", {}), ("hmm-multinom", dict(K=4, L=9)), ("hmm-multinom", dict(K=2, L=5)),
         ("hmm", dict(K=4)), ("hmm", dict(K=2)), ("hmm-multinom-semisup", dict(K=4, L=9))]


@pytest.mark.parametrize("model,kw", CASES)
@pytest.mark.parametrize("T", [1, 37, 511, 512, 513, 5000])
def test_vscan_matches_oracle(engine, oracle, model, kw, T):
    data, draws = synth.GENERATORS[model](N=2, S=5, T=T, **kw)
    run(engine, oracle, model, data, draws)


@pytest.mark.parametrize("model,kw", CASES[:4])
def test_vscan_ragged(engine, oracle, model, kw):
    data, draws = synth.GENERATORS[model](N=4, S=3, T=3000, **kw)
    data["T"] = np.array([3000, 1, 1024, 1537], dtype=np.int32)
    run(engine, oracle, model, data, draws)


@pytest.mark.parametrize("model,kw", [("hhmm-tayal2009", {}), ("hmm", dict(K=4)), ("hmm-multinom", dict(K=2, L=5))])
def test_vscan_long_series(engine, oracle, model, kw):
    """T = 2e5: |delta| grows through ~10 binades; automatic dispatch (6 pairs)."""
    data, draws = synth.GENERATORS[model](N=2, S=3, T=200_000, **kw)
    run(engine, oracle, model, data, draws, flags=0)


def test_vscan_with_forward_backward(engine, oracle):
    """The hot request (loglik + gamma + path) with the scan forced on both passes
    (gamma's Tayal NaN rows are test_gpu_configs.compare_tayal_gamma's business)."""
    data, draws = synth.tayal(N=1, S=6, T=20_000)
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    import hhmm_amd
    got = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=pars, lib=engine, return_status=True,
                       flags=SCAN | _abi.FLAG_SCAN_FORCE)
    ref = oracle.gqs("hhmm-tayal2009", data, draws, pars=pars, return_status=True, nthreads=8)
    compare_all(got, ref, ["loglik"] + VIT + ["pair_status"])


def test_vscan_tayal_lite_oos(engine, oracle):
    data, draws = synth.tayal(N=2, S=3, T=700, T_oos=2600)
    data["T_oos"] = np.array([2600, 513], dtype=np.int32)
    run(engine, oracle, "hhmm-tayal2009-lite", data, draws, pars=["loglik", "alpha_tk_oos"] + VIT)


def test_vscan_invalid_backpointer(engine, oracle):
    """All delta_T = -inf: flagged, zstar zeroed, as the sequential decoders do."""
    data, draws = synth.hmm_multinom(N=1, S=4, T=1500, K=4, L=5)
    draws["phi_k"][:, :, 4] = 0.0
    draws["phi_k"] /= draws["phi_k"].sum(axis=2, keepdims=True)
    data["x"][0, 900] = 5
    got, ref = run(engine, oracle, "hmm-multinom", data, draws)
    assert (ref["pair_status"] == 1).all()


def test_vscan_agrees_with_sequential(engine):
    """Forced scan against the forced state-parallel decoder on the device, 64 pairs at T = 50k."""
    import hhmm_amd
    data, draws = synth.tayal(N=1, S=64, T=50_000)
    a = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=VIT, lib=engine, return_status=True, flags=SCAN)
    b = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=VIT, lib=engine, return_status=True,
                     flags=_abi.FLAG_VIT_STATES)
    assert np.array_equal(a["zstar_t"], b["zstar_t"])
    assert np.array_equal(a["logp_zstar"].view(np.int64), b["logp_zstar"].view(np.int64))
    assert np.array_equal(a["pair_status"], b["pair_status"])


def _tie_values(oracle, k, count, seed=5):
    """Probabilities whose correctly rounded log is an odd multiple of 2^(k-53): a
    rounding tie on the grid of binade k (the parity-dependent products of
    hhmm_vscan.h's vs_prod_tie_kernel)."""
    g = np.random.Generator(np.random.Philox(seed))
    found = []
    while len(found) < count:
        x = g.uniform(0.05, 0.9, 400_000)
        s = oracle.log_array(x, "cr") * 2.0 ** (53 - k)
        ok = (s == np.round(s)) & (np.abs(np.fmod(s, 2.0)) == 1.0)
        found.extend(x[ok][: count - len(found)])
    return np.array(found)


@pytest.mark.parametrize("model", ["hmm-multinom", "hhmm-tayal2009"])
def test_vscan_rounding_ties(engine, oracle, model):
    """Emission and transition log-probabilities that tie on the grid of the binades
    |delta| crosses (k = 11, 12, 13): those chunks take the even / odd entry-value
    products, still bit-exact."""
    T = 20_000
    if model == "hmm-multinom":
        data, draws = synth.hmm_multinom(N=1, S=4, T=T, K=4, L=9)
        phi = draws["phi_k"]
        for s, k in enumerate((11, 12, 13, 13)):
            v = _tie_values(oracle, k, 3, seed=5 + s)
            phi[s, 0, :3] = v
            draws["A_ij"][s, 1, 2] = v[0]
    else:
        data, draws = synth.tayal(N=1, S=4, T=T)
        phi = draws["phi_k"]
        for s, k in enumerate((11, 12, 13, 13)):
            v = _tie_values(oracle, k, 4, seed=9 + s)
            phi[s, :, 4] = v
    run(engine, oracle, model, data, draws)
