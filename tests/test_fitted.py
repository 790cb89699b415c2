"""IOHMM fitted-output draws: hatpi_tk, hatz_t, hatl_t, hatx_t.

Reference: iohmm-reg/stan/iohmm-reg.stan:131-148, iohmm-mix/stan/iohmm-mix.stan:140-160,
iohmm-mix/stan/iohmm-hmix.stan:146-157.  Stan draws these with its own RNG
(categorical_rng / normal_rng), so parity with the reference is unpinned for the
draws themselves; the contract (include/hhmm.h, HHMM_OUT_HATZ..) fixes the
randomness as caller-supplied uniforms / normal deviates and keeps Stan's
arithmetic: Eigen dot order, Stan Math softmax, categorical_rng's inverse CDF
over cumulative_sum(theta), boost normal_distribution's `z * sigma + mu`.

CPU: the C oracle (libm build) against an independent Python transcription of
the three GQ blocks, plus known answers.  GPU: libhhmm against the oracle's CR
build, bit for bit (hatpi_tk included: the softmax uses the shared correctly
rounded exp on both sides).
"""
import numpy as np
import pytest

import oracle_numpy as onp
from hhmm_amd import synth

HAT_MODELS = ["iohmm-reg", "iohmm-mix", "iohmm-hmix"]


def _categorical(theta, u):
    """categorical_rng: cumulative_sum(theta); b = 0; while (u > cum[b]) b++ (1-based)."""
    b, cum = 0, theta[0]
    while b < len(theta) - 1 and u > cum:
        b += 1
        cum = cum + theta[b]
    return b + 1


def transcribe(model, data, draws, hat_rand):
    """Pure-Python restatement of the GQ blocks, grid pairing p = s + S*n."""
    x = np.asarray(data["x_t"])
    N, T = x.shape
    K, M = int(data["K"]), int(data["M"])
    u = np.asarray(data["u_tm"])
    S = draws["w_km"].shape[0]
    out = {"hatpi_tk": np.zeros((N * S, T, K)), "hatz_t": np.zeros((N * S, T), np.int32),
           "hatl_t": np.zeros((N * S, T), np.int32), "hatx_t": np.zeros((N * S, T))}
    for n in range(N):
        for s in range(S):
            p = s + S * n
            for t in range(T):
                ut = [float(v) for v in u[n, t, :M]]
                reg = [onp.eigen_dot(ut, [float(v) for v in draws["w_km"][s, j, :M]]) for j in range(K)]
                th = onp.softmax(reg)
                out["hatpi_tk"][p, t] = th
                z = _categorical(th, hat_rand[p, t, 0])
                out["hatz_t"][p, t] = z
                if model == "iohmm-reg":
                    mu = onp.eigen_dot(ut, [float(v) for v in draws["b_km"][s, z - 1, :M]])
                    out["hatx_t"][p, t] = hat_rand[p, t, 2] * float(draws["s_k"][s, z - 1]) + mu
                else:
                    lam = [float(v) for v in draws["lambda_kl"][s, z - 1]]
                    lz = _categorical(lam, hat_rand[p, t, 1])
                    out["hatl_t"][p, t] = lz
                    out["hatx_t"][p, t] = (hat_rand[p, t, 2] * float(draws["s_kl"][s, z - 1, lz - 1])
                                           + float(draws["mu_kl"][s, z - 1, lz - 1]))
    return out


@pytest.mark.parametrize("model", HAT_MODELS)
@pytest.mark.parametrize("T", [1, 2, 23])
def test_oracle_matches_transcription(oracle, model, T):
    data, draws = synth.GENERATORS[model](N=2, S=3, T=T)
    hr = synth.hat_rand(6, T, seed=5)
    pars = synth.HAT_PARS[model]
    got = oracle.gqs(model, data, draws, pars=pars, variant="libm", hat_rand=hr)
    want = transcribe(model, data, draws, hr)
    for name in pars:
        assert np.array_equal(got[name], want[name]), (model, name)


def test_oracle_known_answers(oracle):
    """u -> 0 picks state 1, u -> 1 the last state; z = 0 gives hatx = the mean."""
    model = "iohmm-mix"
    data, draws = synth.GENERATORS[model](N=1, S=2, T=9)
    hr = synth.hat_rand(2, 9, seed=6)
    hr[:, :, 0] = 1e-300
    hr[:, :, 1] = 1.0 - 2 ** -53
    hr[:, :, 2] = 0.0
    got = oracle.gqs(model, data, draws, pars=["hatz_t", "hatl_t", "hatx_t"], hat_rand=hr)
    L = int(data["L"])
    assert (got["hatz_t"] == 1).all()
    assert (got["hatl_t"] == L).all()
    for s in range(2):
        assert np.array_equal(got["hatx_t"][s], np.full(9, draws["mu_kl"][s, 0, L - 1]))


def test_oracle_hatz_follows_hatpi(oracle):
    """Over many uniforms the hatz frequencies match the average hatpi (z-score)."""
    model = "iohmm-reg"
    data, draws = synth.GENERATORS[model](N=1, S=1, T=4000)
    data["u_tm"][:] = data["u_tm"][:, :1, :]  # one input vector: hatpi is constant over t
    hr = synth.hat_rand(1, 4000, seed=7)
    got = oracle.gqs(model, data, draws, pars=["hatpi_tk", "hatz_t"], hat_rand=hr)
    pi = got["hatpi_tk"][0, 0]
    K = pi.size
    freq = np.bincount(got["hatz_t"][0] - 1, minlength=K) / 4000
    se = np.sqrt(pi * (1 - pi) / 4000) + 1e-12
    assert (np.abs(freq - pi) / se < 5).all(), (freq, pi)


def test_hat_requires_rand():
    from hhmm_amd.api import PreparedRequest
    data, draws = synth.GENERATORS["iohmm-reg"](N=1, S=2, T=5)
    with pytest.raises(ValueError):
        PreparedRequest("iohmm-reg", data, draws, ["hatz_t"])


@pytest.mark.gpu
@pytest.mark.parametrize("model", HAT_MODELS)
@pytest.mark.parametrize("K", [2, 4, 7])
def test_gpu_hat_bit_exact(engine, oracle, model, K):
    import hhmm_amd
    kw = {"K": K} if model != "iohmm-reg" else {"K": K}
    data, draws = synth.GENERATORS[model](N=3, S=70, T=37, **kw)
    data["T"] = np.array([37, 12, 1], dtype=np.int32)
    P = 210
    hr = synth.hat_rand(P, 37, seed=K)
    pars = synth.HAT_PARS[model]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, hat_rand=hr)
    ref = oracle.gqs(model, data, draws, pars=pars, hat_rand=hr)
    Tn = np.repeat(data["T"], 70)
    for name in pars:
        for p in range(P):
            g, r = got[name][p, :Tn[p]], ref[name][p, :Tn[p]]
            assert np.array_equal(g.view(np.int64) if g.dtype == np.float64 else g,
                                  r.view(np.int64) if r.dtype == np.float64 else r), (model, name, p)


@pytest.mark.gpu
def test_gpu_hat_with_hot_outputs(engine, oracle):
    """Fitted draws requested together with the recursion outputs (two kernels, one call)."""
    import hhmm_amd
    from tolerances import compare_all
    model = "iohmm-mix"
    data, draws = synth.GENERATORS[model](N=2, S=64, T=50)
    hr = synth.hat_rand(128, 50, seed=3)
    pars = ["loglik", "gamma_tk", "zstar_t"] + synth.HAT_PARS[model]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, hat_rand=hr)
    ref = oracle.gqs(model, data, draws, pars=pars, hat_rand=hr)
    compare_all(got, ref, ["loglik", "gamma_tk", "zstar_t"])
    for name in synth.HAT_PARS[model]:
        assert np.array_equal(got[name], ref[name]), name
