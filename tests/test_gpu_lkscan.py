"""GPU: the parallel scan over T at large K (hhmm_lkscan.h; SURVEY.md §8 A16
at 8 < K <= 32, the verdict's N2) against the oracle -- hmm-multinom with few
pairs and long series: MFMA chunk products (v_mfma_f64_4x4x4_f64 blocks), the
scan over chunks, the chunks' forward-backward sweeps.  Posteriors and the
log-likelihood within tests/tolerances.py (the products reassociate the
sums); the Viterbi (sequential, beside it) bit-exact."""
import numpy as np
import pytest

from hhmm_amd import _abi, synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

FB = ["loglik", "gamma_tk"]


def scan_flags(log2=None):
    return _abi.FLAG_SCAN_FORCE | (_abi.flag_scan_chunk_log2(log2) if log2 else 0)


def run_both(engine, oracle, data, draws, pars, flags=0, pairing="grid"):
    import hhmm_amd
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, pairing=pairing, lib=engine, return_status=True,
                       flags=flags)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, pairing=pairing, return_status=True, nthreads=16)
    # pair_status is the decoder's (the oracle flags T = 1 pairs, Q3); compared when it runs
    extra = ["pair_status"] if "zstar_t" in pars else []
    compare_all(got, ref, pars + extra)
    return got, ref


@pytest.mark.parametrize("K", [9, 12, 16, 17, 23, 24, 32])
@pytest.mark.parametrize("T,log2", [(1, 5), (31, 5), (32, 5), (33, 5), (700, 6), (4000, 8)])
def test_forced_scan_matches_oracle(engine, oracle, K, T, log2):
    """Chunks of 32 / 64 / 256 steps, chunk boundaries inside and at the
    series' end, every state-capacity instantiation (16, 24, 32)."""
    data, draws = synth.hmm_multinom(N=2, S=3, T=T, K=K, L=9)
    run_both(engine, oracle, data, draws, ["loglik", "alpha_tk", "beta_tk", "ungamma_tk", "gamma_tk"],
             flags=scan_flags(log2))


@pytest.mark.parametrize("K", [12, 23])
def test_forced_scan_ragged_with_viterbi(engine, oracle, K):
    data, draws = synth.hmm_multinom(N=4, S=5, T=3000, K=K, L=9)
    data["T"] = np.array([3000, 1, 1999, 64], dtype=np.int32)
    run_both(engine, oracle, data, draws, FB + ["zstar_t", "logp_zstar"], flags=scan_flags(7))


@pytest.mark.parametrize("pairing", ["zip", "block"])
def test_forced_scan_pairings(engine, oracle, pairing):
    N = 6
    S = N if pairing == "zip" else 2 * N
    data, draws = synth.hmm_multinom(N=N, S=S, T=900, K=16, L=9)
    run_both(engine, oracle, data, draws, FB, flags=scan_flags(6), pairing=pairing)


@pytest.mark.parametrize("K", [16, 23])
def test_auto_scan_T1e5(engine, oracle, K):
    """T = 10^5 on 3 pairs: the automatic dispatch takes the scan (P < 4096,
    T >= 8192); the decoder runs sequentially beside it."""
    data, draws = synth.hmm_multinom(N=1, S=3, T=100_000, K=K, L=9)
    run_both(engine, oracle, data, draws, FB + ["zstar_t", "logp_zstar"])


@pytest.mark.parametrize("tiny", [1e-90, 1e-200])
def test_scan_near_impossible_runs(engine, oracle, tiny):
    """A run of a symbol every state emits with probability `tiny`: the chunk
    products renormalise every column every step, the row exponents carry
    the scale exactly across chunks."""
    K = 23
    data, draws = synth.hmm_multinom(N=1, S=3, T=2000, K=K, L=9)
    phi = np.array(draws["phi_k"], dtype=np.float64)
    phi[:, :, 8] = tiny
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    x = np.array(data["x"])
    x[:, 600:700] = 9
    data["x"] = x
    got, _ = run_both(engine, oracle, data, draws, FB, flags=scan_flags(6))
    assert np.isfinite(got["loglik"]).all()


def test_scan_transient_states(engine, oracle):
    """Rows of the chunk products that die out (a state that cannot produce
    the chunk's symbols: zero emission probability) carry no exponent; the
    scan ignores them."""
    K = 12
    data, draws = synth.hmm_multinom(N=1, S=2, T=1500, K=K, L=9)
    phi = np.array(draws["phi_k"], dtype=np.float64)
    phi[:, 0, 3] = 0.0  # state 1 never emits symbol 4
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    run_both(engine, oracle, data, draws, FB + ["alpha_tk", "beta_tk"], flags=scan_flags(5))


# ---- hmm.stan (Gaussian emissions) on the large-K scan (Missing 4) ----------------
def run_gauss(engine, oracle, data, draws, pars, flags=0):
    import hhmm_amd
    got = hhmm_amd.gqs("hmm", data, draws, pars=pars, lib=engine, return_status=True, flags=flags)
    ref = oracle.gqs("hmm", data, draws, pars=pars, return_status=True, nthreads=16)
    extra = ["pair_status"] if "zstar_t" in pars else []
    compare_all(got, ref, pars + extra)


@pytest.mark.parametrize("K", [9, 16, 23, 32])
@pytest.mark.parametrize("T,log2", [(1, 5), (33, 5), (700, 6), (4000, 8)])
def test_forced_scan_gauss(engine, oracle, K, T, log2):
    """hmm.stan at K > 8 (K is data, hmm/stan/hmm.stan:8): e_t(j) = exp(lpdf_j - m_t)
    in the chunk products, each chunk's sum of the shifts m_t its log scale, the
    summed t = 1 emission (Q2) in phase 2's initial log scale."""
    data, draws = synth.hmm_gauss(N=2, S=3, T=T, K=K)
    run_gauss(engine, oracle, data, draws, ["loglik", "alpha_tk", "beta_tk", "ungamma_tk", "gamma_tk"],
              flags=scan_flags(log2))


@pytest.mark.parametrize("K", [9, 23])
@pytest.mark.parametrize("log2", [5, 6])
def test_forced_scan_gauss_ragged(engine, oracle, K, log2):
    """ragged series on the Gaussian large-K scan -- partial last
    chunks, T = 1, lengths that are not multiples of the chunk, and columns past
    a pair's own chunk count (their log scale sc_bl never accumulates)."""
    Ts = [1, 700, 33, 64, 65, 451]
    data, draws = synth.hmm_gauss(N=len(Ts), S=3, T=max(Ts), K=K)
    data["T"] = np.array(Ts, dtype=np.int32)
    run_gauss(engine, oracle, data, draws, ["loglik", "alpha_tk", "beta_tk", "ungamma_tk", "gamma_tk"],
              flags=scan_flags(log2))


def test_auto_scan_gauss_T1e5(engine, oracle):
    """Few pairs, long T: the automatic dispatch takes the scan for hmm.stan too."""
    data, draws = synth.hmm_gauss(N=1, S=3, T=100_000, K=12)
    data["T"] = np.array([100_000], dtype=np.int32)
    run_gauss(engine, oracle, data, draws, FB + ["zstar_t", "logp_zstar"])
