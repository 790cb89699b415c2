"""GPU: the HMM family at large K (hhmm_large.h) against the
oracle -- hmm.stan and hmm-multinom.stan at 8 < K <= 32, where one group of
32 lanes owns a pair and the K x K transitions are spread over the group.
Posteriors and log-likelihoods within tests/tolerances.py, Viterbi paths,
logp_zstar and pair_status bit-exact."""
import numpy as np
import pytest

from hhmm_amd import api, synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

PARS = ["loglik", "alpha_tk", "beta_tk", "ungamma_tk", "gamma_tk", "zstar_t", "logp_zstar"]


def run_both(engine, oracle, model, data, draws, pars=PARS, pairing="grid"):
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, pairing=pairing, lib=engine, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, pairing=pairing, return_status=True, nthreads=8)
    compare_all(got, ref, pars + ["pair_status"])
    assert got["status"] == ref["status"]


@pytest.mark.parametrize("K", [9, 12, 16, 17, 23, 24, 25, 32])
@pytest.mark.parametrize("T", [1, 2, 37, 300])
def test_multinom_large_K(engine, oracle, K, T):
    data, draws = synth.hmm_multinom(N=3, S=21, T=T, K=K, L=9)
    run_both(engine, oracle, "hmm-multinom", data, draws)


@pytest.mark.parametrize("K", [12, 23, 25])
@pytest.mark.parametrize("T", [1, 2, 130])
def test_gauss_large_K(engine, oracle, K, T):
    data, draws = synth.hmm_gauss(N=2, S=17, T=T, K=K)
    run_both(engine, oracle, "hmm", data, draws)


@pytest.mark.parametrize("K,L", [(12, 31), (23, 4)])
def test_multinom_large_K_T1000_ragged(engine, oracle, K, L):
    data, draws = synth.hmm_multinom(N=4, S=9, T=1000, K=K, L=L)
    data["T"] = np.array([1000, 1, 333, 999], dtype=np.int32)
    run_both(engine, oracle, "hmm-multinom", data, draws)


@pytest.mark.parametrize("pairing", ["zip", "block"])
def test_large_K_pairings(engine, oracle, pairing):
    N = 40
    S = N if pairing == "zip" else 3 * N
    data, draws = synth.hmm_multinom(N=N, S=S, T=64, K=16, L=9)
    run_both(engine, oracle, "hmm-multinom", data, draws, pairing=pairing)


def test_large_K_invalid_backpointer(engine, oracle):
    """A symbol impossible under every state: all delta_T = -inf, Stan would
    throw while backtracking; flagged, path zeroed -- as at small K."""
    data, draws = synth.hmm_multinom(N=1, S=5, T=20, K=12, L=9)
    draws["phi_k"][:, :, 8] = 0.0
    draws["phi_k"] /= draws["phi_k"].sum(axis=2, keepdims=True)
    data["x"][0, 7] = 9
    run_both(engine, oracle, "hmm-multinom", data, draws)


def test_large_K_unsupported_outputs(engine):
    import hhmm_amd
    data, draws = synth.hmm_multinom(N=1, S=2, T=10, K=12, L=9)
    with pytest.raises(api.HHMMError):
        hhmm_amd.gqs("hmm-multinom", data, draws, pars=["unalpha_tk"], lib=engine)
