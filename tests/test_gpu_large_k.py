"""GPU: the HMM family at large K (hhmm_large.h) against the
oracle -- hmm.stan and hmm-multinom.stan at 8 < K <= 32, where one group of
32 lanes owns a pair and the K x K transitions are spread over the group.
Posteriors and log-likelihoods within tests/tolerances.py, Viterbi paths,
logp_zstar and pair_status bit-exact."""
import numpy as np
import pytest

from hhmm_amd import _abi, api, synth
from tolerances import compare_all

pytestmark = pytest.mark.gpu

PARS = ["loglik", "alpha_tk", "beta_tk", "ungamma_tk", "gamma_tk", "zstar_t", "logp_zstar"]


def run_both(engine, oracle, model, data, draws, pars=PARS, pairing="grid", flags=0):
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, pairing=pairing, lib=engine, return_status=True, flags=flags)
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


def twin_states(draws, a, b, rel):
    """States a and b made twins: the same incoming transitions and emissions,
    so their deltas are equal at every step, and b's outgoing row is a's times
    (1 + rel): rel = 0 gives exact ties in the max-plus step, a tiny rel
    candidates an ulp or two apart (lk_viterbi_kernel's fast step marks both,
    and the block is replayed in the reference's order)."""
    A = np.array(draws["A_ij"], dtype=np.float64)
    A[:, :, a] += 4.0  # make the twins likely winners
    A[:, :, b] = A[:, :, a]
    A /= A.sum(axis=2, keepdims=True)
    A[:, b, :] = A[:, a, :] * (1.0 + rel)
    draws["A_ij"] = A
    phi = np.array(draws["phi_k"], dtype=np.float64)
    phi[:, b, :] = phi[:, a, :]
    draws["phi_k"] = phi


@pytest.mark.parametrize("K", [12, 23, 32])
@pytest.mark.parametrize("rel", [0.0, 2.0 ** -52, -(2.0 ** -50), 2.0 ** -44, 2.0 ** -40])
def test_large_K_viterbi_ties(engine, oracle, K, rel):
    """Exact and near ties between two states' candidates: the Viterbi keeps
    the reference's first-i-on-ties order bit for bit."""
    data, draws = synth.hmm_multinom(N=3, S=6, T=300, K=K, L=9)
    twin_states(draws, 2, K - 3, rel)
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["zstar_t", "logp_zstar"])


def test_large_K_viterbi_ties_gauss(engine, oracle):
    data, draws = synth.hmm_gauss(N=2, S=5, T=200, K=17)
    twin_states_g = dict(draws)
    A = np.array(draws["A_ij"], dtype=np.float64)
    A[:, :, 4] += 4.0
    A[:, :, 9] = A[:, :, 4]
    A /= A.sum(axis=2, keepdims=True)
    A[:, 9, :] = A[:, 4, :]
    twin_states_g["A_ij"] = A
    for k in ("mu_k", "sigma_k"):
        v = np.array(draws[k], dtype=np.float64)
        v[:, 9] = v[:, 4]
        twin_states_g[k] = v
    run_both(engine, oracle, "hmm", data, twin_states_g, pars=["zstar_t", "logp_zstar"])


@pytest.mark.parametrize("K", [12, 23, 32])
def test_gamma_only_large_K_ragged(engine, oracle, K):
    """The bench's N1 output set (loglik, gamma, zstar, logp_zstar) runs the
    one-group-sum gamma (alpha .* beta / sum, lk_fb_kernel's gamma_only
    branch); ragged T inside the wave's two groups."""
    data, draws = synth.hmm_multinom(N=5, S=7, T=400, K=K, L=9)
    data["T"] = np.array([400, 1, 257, 399, 64], dtype=np.int32)
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["loglik", "gamma_tk", "zstar_t", "logp_zstar"])


def test_gamma_only_large_K_disjoint_filters(engine, oracle):
    """alpha and beta nearly disjoint (states that the forward pass makes
    improbable are the ones the backward pass favours) so the product's sum
    drops below kGammaDirect = 2^-240 (hhmm_internal.h) and the gamma-only branch takes the reference's
    normalised-vector formula."""
    K = 12
    data, draws = synth.hmm_multinom(N=1, S=4, T=600, K=K, L=9)
    A = np.full((4, K, K), 1e-300)
    for i in range(K):
        A[:, i, i] = 1.0
    A /= A.sum(axis=2, keepdims=True)
    draws["A_ij"] = A
    phi = np.full((4, K, 9), 1e-3)
    phi[:, : K // 2, 0] = 1.0
    phi[:, K // 2:, 1] = 1.0
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    x = np.ones((1, 600), dtype=np.int32)
    x[0, 300:] = 2
    data["x"] = x
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["loglik", "gamma_tk", "zstar_t", "logp_zstar"])


def test_large_K_unsupported_outputs(engine):
    """Past the state capacity (K > 32) every program is unsupported, with a
    message (the IOHMM programs at 8 < K <= 32: tests/test_gpu_iohmm_large_k.py)."""
    import hhmm_amd
    data, draws = synth.iohmm_reg(N=1, S=2, T=10, K=33, M=4)
    with pytest.raises(api.HHMMError, match="K <= 32"):
        hhmm_amd.gqs("iohmm-reg", data, draws, pars=["loglik"], lib=engine)


LOGPARS = ["loglik", "unalpha_tk", "alpha_tk", "unbeta_tk", "beta_tk", "ungamma_tk", "gamma_tk"]


@pytest.mark.parametrize("model", ["hmm-multinom", "hmm"])
@pytest.mark.parametrize("K", [9, 16, 23, 32])
@pytest.mark.parametrize("T", [1, 2, 37, 300])
def test_log_profile_large_K(engine, oracle, model, K, T):
    """unalpha_tk / unbeta_tk at large K (lk_log_kernel): the reference's
    log-space recursion with every posterior of the request."""
    gen = synth.hmm_multinom if model == "hmm-multinom" else synth.hmm_gauss
    kw = dict(L=9) if model == "hmm-multinom" else {}
    data, draws = gen(N=2, S=5, T=T, K=K, **kw)
    run_both(engine, oracle, model, data, draws, pars=LOGPARS + ["zstar_t", "logp_zstar"])


def test_log_profile_large_K_far_states(engine, oracle):
    """A state thousands of nats below the others: its linear-space filter
    underflows, the log-space unalpha / unbeta stay finite as in Stan."""
    K = 12
    data, draws = synth.hmm_multinom(N=1, S=3, T=800, K=K, L=9)
    phi = np.array(draws["phi_k"], dtype=np.float64)
    phi[:, 0, :] = 1e-6
    phi[:, 0, 0] = 1.0
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    data["x"] = np.where(np.asarray(data["x"]) == 1, 2, np.asarray(data["x"]))
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=LOGPARS)


def test_log_profile_forward_only_large_K(engine, oracle):
    data, draws = synth.hmm_multinom(N=2, S=4, T=100, K=20, L=9)
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["loglik", "unalpha_tk", "alpha_tk"])


@pytest.mark.parametrize("model", ["hmm-multinom", "hmm"])
@pytest.mark.parametrize("K", [9, 16, 23, 32])
@pytest.mark.parametrize("T", [1, 2, 37, 300])
def test_ffbs_large_K(engine, oracle, model, K, T):
    """FFBS at large K (lk_ffbs_kernel): the contract's filter (state-order fma
    sums, per-step power-of-two renormalisation) and draws, bit-exact against
    the oracle's ffbs_contract given the same uniforms."""
    import hhmm_amd
    gen = synth.hmm_multinom if model == "hmm-multinom" else synth.hmm_gauss
    kw = dict(L=9) if model == "hmm-multinom" else {}
    data, draws = gen(N=2, S=7, T=T, K=K, **kw)
    P = 14
    u = synth.ffbs_uniforms(P, T)
    pars = ["loglik", "gamma_tk", "z_ffbs"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, uniforms=u, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, uniforms=u, return_status=True, nthreads=8)
    compare_all(got, ref, pars)


def test_ffbs_large_K_ragged_with_viterbi(engine, oracle):
    import hhmm_amd
    data, draws = synth.hmm_multinom(N=3, S=5, T=500, K=23, L=9)
    data["T"] = np.array([500, 3, 257], dtype=np.int32)
    u = synth.ffbs_uniforms(15, 500)
    pars = ["loglik", "gamma_tk", "z_ffbs", "zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, uniforms=u, return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, uniforms=u, return_status=True, nthreads=8)
    compare_all(got, ref, pars + ["pair_status"])


# ---- GRID batches with >= 16 series per draw: the forward-backward on the matrix cores (lkm_fb_kernel,
# opt-in HHMM_FLAG_LKM_MFMA)
MF = _abi.FLAG_LKM_MFMA

@pytest.mark.parametrize("K", [9, 12, 16, 17, 23, 24, 32])
@pytest.mark.parametrize("T", [1, 2, 37, 300])
def test_mfma_grid_fb(engine, oracle, K, T):
    data, draws = synth.hmm_multinom(N=20, S=3, T=T, K=K, L=9)
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
             flags=MF)


@pytest.mark.parametrize("K", [12, 23])
def test_mfma_grid_fb_ragged_matches_state_parallel(engine, oracle, K):
    """Ragged series inside a tile; the matrix-core path against the oracle
    and against the state-parallel kernels (the default) on the same
    request (both within tolerance of each other: the sums reassociate)."""
    import hhmm_amd
    from tolerances import compare
    N = 37
    data, draws = synth.hmm_multinom(N=N, S=4, T=700, K=K, L=9)
    data["T"] = np.random.default_rng(K).integers(1, 701, N).astype(np.int32)
    pars = ["loglik", "gamma_tk"]
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=pars, flags=MF)
    a = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=MF)
    b = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine)
    for k in pars:
        compare(k, a[k], b[k])


@pytest.mark.parametrize("tiny", [1e-90, 1e-200])
def test_mfma_grid_fb_near_impossible_runs(engine, oracle, tiny):
    K = 23
    data, draws = synth.hmm_multinom(N=16, S=3, T=400, K=K, L=9)
    phi = np.array(draws["phi_k"], dtype=np.float64)
    phi[1, :, 8] = tiny
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    x = np.array(data["x"])
    x[:, 100:160] = 9
    data["x"] = x
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["loglik", "gamma_tk"], flags=MF)


def test_mfma_grid_fb_disjoint_filters(engine, oracle):
    """The gamma sum below kGammaDirect = 2^-240 (hhmm_internal.h): the
    reference's normalised-vector formula."""
    K = 12
    data, draws = synth.hmm_multinom(N=16, S=2, T=600, K=K, L=9)
    A = np.full((2, K, K), 1e-300)
    for i in range(K):
        A[:, i, i] = 1.0
    A /= A.sum(axis=2, keepdims=True)
    draws["A_ij"] = A
    phi = np.full((2, K, 9), 1e-3)
    phi[:, : K // 2, 0] = 1.0
    phi[:, K // 2:, 1] = 1.0
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    x = np.ones((16, 600), dtype=np.int32)
    x[:, 300:] = 2
    data["x"] = x
    run_both(engine, oracle, "hmm-multinom", data, draws, pars=["loglik", "gamma_tk"], flags=MF)
