"""CPU: the C oracle against an independent transcription and analytic answers.

The reference has no tests, fixtures or runnable toolchain here (SURVEY.md §4,
§8c), so parity of the oracle with Stan is pinned by (i) an independent
pure-Python transcription of each .stan file (tests/oracle_numpy.py) that
must agree BIT-FOR-BIT with the oracle's libm build, (ii) analytic
known-answer tests, and (iii) committed fixtures (test_golden.py).
"""
import math

import numpy as np
import pytest

import oracle_numpy as onp
from hhmm_amd import synth

ALL_MODELS = list(synth.GENERATORS)


def _compare_exact(model, ref, rows, pars):
    for p, r in enumerate(rows):
        T = r["T"]
        assert int(ref["pair_status"][p]) == r["pair_status"], (model, p)
        for k in pars:
            a = np.asarray(ref[k][p])
            b = np.asarray(r[k])
            if a.ndim:
                a = a[: b.shape[0]]
            same = (a == b) | (np.isnan(a) & np.isnan(b))
            assert np.all(same), f"{model} pair {p} {k}: oracle and transcription differ (T={T})"


@pytest.mark.parametrize("model", ALL_MODELS)
@pytest.mark.parametrize("T", [1, 2, 23])
def test_oracle_matches_transcription(oracle, model, T):
    data, draws = synth.GENERATORS[model](N=2, S=2, T=T)
    pars = synth.PARS[model]
    ref = oracle.gqs(model, data, draws, pars=pars, variant="libm", return_status=True)
    rows = onp.run(model, data, draws)
    _compare_exact(model, ref, rows, pars)


@pytest.mark.parametrize("model", ["hmm", "hmm-multinom", "hhmm-tayal2009", "iohmm-reg", "iohmm-hmix"])
def test_oracle_ragged_matches_transcription(oracle, model):
    data, draws = synth.GENERATORS[model](N=3, S=2, T=19)
    data["T"] = np.array([19, 4, 11], dtype=np.int32)
    pars = synth.PARS[model]
    ref = oracle.gqs(model, data, draws, pars=pars, variant="libm", return_status=True)
    rows = onp.run(model, data, draws)
    _compare_exact(model, ref, rows, pars)


@pytest.mark.parametrize("model", ALL_MODELS)
def test_cr_and_libm_builds_agree(oracle, model):
    """The correctly rounded log moves results by at most an ulp-scale amount;
    Viterbi paths agree on random (tie-free) draws."""
    data, draws = synth.GENERATORS[model](N=3, S=4, T=60)
    pars = synth.PARS[model]
    a = oracle.gqs(model, data, draws, pars=pars, variant="cr", return_status=True)
    b = oracle.gqs(model, data, draws, pars=pars, variant="libm", return_status=True)
    for k in pars:
        if k == "zstar_t":
            assert np.array_equal(a[k], b[k])
        else:
            x, y = a[k], b[k]
            m = np.isfinite(y)
            assert np.array_equal(np.isnan(x), np.isnan(y))
            assert np.all(np.abs(x[m] - y[m]) <= 1e-12 * np.maximum(np.abs(y[m]), 1.0)), k


# ---------------- analytic known-answer tests ----------------

def test_kat_single_state(oracle):
    """K = 1: alpha = beta = gamma = 1, loglik = sum_t log phi(1, x_t),
    Viterbi path all ones, logp_zstar = sum_{t>=1} log phi (log A = 0, no log p)."""
    T = 30
    g = np.random.Generator(np.random.Philox(1))
    x = g.integers(1, 4, size=T)
    phi = np.array([0.2, 0.3, 0.5])
    data = {"K": 1, "L": 3, "x": x.reshape(1, T)}
    draws = {"p_1k": np.ones((1, 1)), "A_ij": np.ones((1, 1, 1)), "phi_k": phi.reshape(1, 1, 3)}
    out = oracle.gqs("hmm-multinom", data, draws, pars=synth.PARS["hmm-multinom"])
    ll = sum(math.log(phi[v - 1]) for v in x)
    assert abs(out["loglik"][0] - ll) <= 1e-12 * abs(ll)
    assert np.all(out["alpha_tk"] == 1.0) and np.all(out["gamma_tk"] == 1.0)
    assert np.all(out["zstar_t"] == 1)
    assert abs(out["logp_zstar"][0] - ll) <= 1e-12 * abs(ll)


def test_kat_uniform_chain(oracle):
    """Uniform p, A and emissions: every state equally likely, loglik = T log(1/L)."""
    K, L, T = 4, 5, 40
    x = (np.arange(T) % L) + 1
    data = {"K": K, "L": L, "x": x.reshape(1, T)}
    draws = {"p_1k": np.full((1, K), 1 / K), "A_ij": np.full((1, K, K), 1 / K), "phi_k": np.full((1, K, L), 1 / L)}
    out = oracle.gqs("hmm-multinom", data, draws, pars=synth.PARS["hmm-multinom"])
    assert abs(out["loglik"][0] - T * math.log(1 / L)) < 1e-11
    assert np.allclose(out["gamma_tk"], 1 / K, rtol=1e-13)
    # all paths tie: strict '>' keeps the FIRST i per step, the LAST j at T (Q4),
    # and the buggy init leaves only state K alive at t = 1 (Q3).
    z = out["zstar_t"][0]
    assert z[0] == K and z[-1] == K and np.all(z[1:-1] == 1)


def test_kat_viterbi_init_quirk_and_t1(oracle):
    """Q3: zstar_t[1] = K for the buggy-init models.  At T = 1 the delta row is
    (NaN, ..., NaN, e_K): max() follows Eigen's SSE2 maxCoeff, which returns
    e_K for K = 2, 4 (valid path) and NaN for K = 3 (Stan would throw)."""
    for K, expect_valid in ((4, True), (3, False), (2, True), (1, True)):
        data, draws = synth.hmm_multinom(N=1, S=2, T=1, K=K, L=5)
        out = oracle.gqs("hmm-multinom", data, draws, pars=["zstar_t", "logp_zstar"], return_status=True)
        if expect_valid:
            assert np.all(out["zstar_t"][:, 0] == K) and np.all(out["pair_status"] == 0)
        else:
            assert np.all(out["pair_status"] == 1) and np.all(np.isnan(out["logp_zstar"]))
    data, draws = synth.hmm_multinom(N=1, S=3, T=50, K=4, L=9)
    out = oracle.gqs("hmm-multinom", data, draws, pars=["zstar_t"])
    assert np.all(out["zstar_t"][:, 0] == 4)


def test_kat_unbeta_offset(oracle):
    """Q1: unbeta_tk[T] = 1, and every unbeta carries the +1 offset."""
    data, draws = synth.hmm_multinom(N=1, S=2, T=10, K=3, L=5)
    out = oracle.gqs("hmm-multinom", data, draws, pars=["unbeta_tk", "beta_tk"])
    assert np.all(out["unbeta_tk"][:, -1, :] == 1.0)
    assert np.allclose(out["beta_tk"][:, -1, :], 1 / 3, rtol=1e-15)


def test_kat_gaussian_t1_summed_emission(oracle):
    """Q2: hmm.stan adds the SUM over states of normal_lpdf(x[1]) at t = 1, so
    alpha_tk[1] = p_1k exactly in value and loglik carries that constant."""
    data, draws = synth.hmm_gauss(N=1, S=3, T=15, K=3)
    out = oracle.gqs("hmm", data, draws, pars=["alpha_tk", "unalpha_tk"])
    assert np.allclose(out["alpha_tk"][:, 0, :], draws["p_1k"], rtol=1e-14)
    x1 = data["x"][0, 0]
    for s in range(3):
        tot = sum(-math.log(math.sqrt(2 * math.pi)) - math.log(sg) - 0.5 * ((x1 - m) / sg) ** 2
                  for m, sg in zip(draws["mu_k"][s], draws["sigma_k"][s]))
        assert np.allclose(out["unalpha_tk"][s, 0, :], np.log(draws["p_1k"][s]) + tot, rtol=1e-13)


def test_kat_tayal_masks(oracle):
    """Q6 (hhmm-tayal2009.stan:49-54, :60-64): unalpha_1(j) = log phi(j, x_1)
    plus log p_1k[j] only for (sign 1, j = 3) or (sign 2, j = 1); at t >= 2 the
    transition term is added only for the sign-consistent states, so the
    other states accumulate without a transition penalty (the reference's
    semantics, reproduced as written)."""
    data, draws = synth.tayal(N=1, S=2, T=40)
    out = oracle.gqs("hhmm-tayal2009", data, draws, pars=["unalpha_tk", "gamma_tk"], return_status=True)
    assert np.all(out["pair_status"] == 0)
    x1, s1 = data["x"][0, 0], data["sign"][0, 0]
    for s in range(2):
        p11 = draws["p_11"][s]
        p = [p11, 0.0, 1 - p11, 0.0]
        for j in range(4):
            e = math.log(draws["phi_k"][s, j, x1 - 1])
            if (s1 == 1 and j == 2) or (s1 == 2 and j == 0):
                e += math.log(p[j]) if p[j] > 0 else -math.inf
            assert out["unalpha_tk"][s, 0, j] == pytest.approx(e, rel=1e-14)
    # t = 2, a sign-inconsistent state j: LSE_i(unalpha_1(i)) + log phi(j, x_2)
    s2, x2 = data["sign"][0, 1], data["x"][0, 1]
    j = 0 if s2 == 1 else 1
    un1 = out["unalpha_tk"][0, 0]
    lse = np.logaddexp.reduce(un1[np.isfinite(un1)])
    assert out["unalpha_tk"][0, 1, j] == pytest.approx(lse + math.log(draws["phi_k"][0, j, x2 - 1]), rel=1e-13)
    assert np.allclose(out["gamma_tk"].sum(axis=2), 1.0, rtol=1e-13)


def test_kat_iohmm_backward_is_state_independent(oracle):
    """Q5: the IOHMM backward accumulator does not depend on j, so beta_tk is
    uniform at every t (iohmm-reg.stan:90-97)."""
    data, draws = synth.iohmm_reg(N=1, S=2, T=25, K=3)
    out = oracle.gqs("iohmm-reg", data, draws, pars=["beta_tk", "unbeta_tk"])
    assert np.allclose(out["beta_tk"], 1 / 3, rtol=1e-14)
    assert np.all(out["unbeta_tk"] == out["unbeta_tk"][:, :, :1])


@pytest.mark.parametrize("model", ["hmm", "hmm-multinom"])
@pytest.mark.parametrize("K", [12, 23])
def test_oracle_large_K_matches_transcription(oracle, model, K):
    """The oracle at the large K of SURVEY §8 N1 (free `int<lower=1> K`,
    hmm-multinom.stan:9; 23 flattened states, log.md:657)."""
    data, draws = synth.GENERATORS[model](N=2, S=2, T=17, K=K)
    pars = synth.PARS[model]
    ref = oracle.gqs(model, data, draws, pars=pars, variant="libm", return_status=True)
    rows = onp.run(model, data, draws)
    _compare_exact(model, ref, rows, pars)
