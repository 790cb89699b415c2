"""GPU: the state-parallel IOHMM sweep (hhmm_iohmm.h: iohmm_sp_sweep, one lane per
(pair, state)) -- loglik, alpha / gamma and FFBS draws -- bit-identical to the
lane-per-pair sweep and against the oracle (draws exact, floats within
tests/tolerances.py)."""
import numpy as np
import pytest

from hhmm_amd import _abi, synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

PARS = ["loglik", "gamma_tk", "alpha_tk", "z_ffbs"]
CASES = [("iohmm-reg", dict(K=2, M=3)), ("iohmm-reg", dict(K=3, M=4)), ("iohmm-reg", dict(K=4, M=7)),
         ("iohmm-mix", dict(K=4, L=3, M=4)), ("iohmm-mix", dict(K=3, L=6, M=8)), ("iohmm-hmix", dict(K=4, L=3, M=4)),
         ("iohmm-hmix", dict(K=2, L=2, M=5))]


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f":
        return np.array_equal(a.view(np.int64), b.view(np.int64))
    return np.array_equal(a, b)


@pytest.mark.parametrize("model,kw", CASES)
@pytest.mark.parametrize("T", [1, 2, 57])
def test_states_layout_matches_lanes_and_oracle(engine, oracle, model, kw, T):
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=3, S=5, T=T, **kw)
    uu = synth.ffbs_uniforms(15, T, seed=4)
    got = {f: hhmm_amd.gqs(model, data, draws, pars=PARS, lib=engine, uniforms=uu, flags=f, return_status=True)
           for f in (_abi.FLAG_VIT_STATES, _abi.FLAG_VIT_LANES)}
    s, ln = got[_abi.FLAG_VIT_STATES], got[_abi.FLAG_VIT_LANES]
    for k in PARS:
        assert _same(s[k], ln[k]), k
    ref = oracle.gqs(model, data, draws, pars=PARS, uniforms=uu, return_status=True)
    compare_all(s, ref, PARS)


@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-hmix"])
def test_states_layout_ragged(engine, oracle, model):
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=3, S=4, T=40)
    data["T"] = np.array([40, 1, 23], dtype=np.int32)
    uu = synth.ffbs_uniforms(12, 40, seed=6)
    got = hhmm_amd.gqs(model, data, draws, pars=PARS, lib=engine, uniforms=uu, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=PARS, uniforms=uu, return_status=True)
    compare_all(got, ref, PARS)
