"""Seeded synthetic inputs for every model on the path.

The reference simulates its calibration data with R's RNG (hmm/R/hmm-sim.R:17-42,
iohmm-reg/R/iohmm-sim.R:26-131) from the true parameters in its driver
scripts.  We cannot reproduce R's Mersenne-Twister stream, so this module
re-implements the same generative models with numpy's counter-based Philox
(seed 9000 by default, the reference's n.seed, hmm/main.R:18) and draws
"posterior draws" jittered around the true parameters:
simplex rows ~ Dirichlet(200 * row + 1), means + N(0, 0.05 * scale),
standard deviations * exp(N(0, 0.05)).

Every generator returns (data, draws) dicts in the shapes hhmm_amd.gqs takes:
series arrays (N, T), draw arrays (S, ...) -- extract()'s layout.
"""
import numpy as np

SEED = 9000


def rng(seed=SEED, stream=0):
    return np.random.Generator(np.random.Philox(key=int(seed) + (int(stream) << 40)))


def _dirichlet_rows(g, rows, S, conc=200.0):
    """S draws of each simplex row: Dirichlet(conc * row + 1)."""
    rows = np.atleast_2d(np.asarray(rows, dtype=np.float64))
    out = np.empty((S,) + rows.shape)
    for r in range(rows.shape[0]):
        out[:, r, :] = g.dirichlet(conc * rows[r] + 1.0, size=S)
    return out


def _markov_chain(g, N, T, A, p1):
    """z[n, t] in 0..K-1 for N independent chains (inverse-CDF sampling)."""
    A = np.asarray(A, dtype=np.float64)
    cA = np.cumsum(A, axis=1)
    cp = np.cumsum(np.asarray(p1, dtype=np.float64))
    z = np.empty((N, T), dtype=np.int64)
    u = g.random((N, T))
    z[:, 0] = np.minimum(np.searchsorted(cp, u[:, 0] * cp[-1], side="right"), len(cp) - 1)
    for t in range(1, T):
        rows = cA[z[:, t - 1]]
        z[:, t] = np.minimum((u[:, t, None] * rows[:, -1:] >= rows).sum(axis=1), A.shape[0] - 1)
    return z


def _categorical(g, probs_rows, z):
    """x[n, t] ~ Cat(probs_rows[z[n, t]]) (1-based)."""
    c = np.cumsum(probs_rows, axis=1)
    u = g.random(z.shape)
    rows = c[z]
    return np.minimum((u[..., None] * rows[..., -1:] >= rows).sum(axis=-1), probs_rows.shape[1] - 1) + 1


def default_A(K):
    """Diagonal-heavy K x K transition matrix (hmm/main.R:9 generalised)."""
    if K == 2:
        return np.array([[0.80, 0.20], [0.35, 0.65]])
    A = np.full((K, K), 0.2 / max(K - 1, 1))
    np.fill_diagonal(A, 0.8)
    if K == 1:
        A[:] = 1.0
    return A


# hmm/main-multinom-semisup.R:12-17 (K = 4)
A_SEMISUP = np.array([[0.00, 0.50, 0.50, 0.00],
                      [1.00, 0.00, 0.00, 0.00],
                      [0.50, 0.00, 0.00, 0.50],
                      [0.00, 0.00, 1.00, 0.00]])
P1_SEMISUP = np.array([0.50, 0.00, 0.50, 0.00])
G_OF_STATE = np.array([1, 2, 2, 1])  # semisup.R:9, 1 = D, 2 = U

# tayal2009/main-sim.R:10-15
A_TAYAL = np.array([[0.00, 0.80, 0.20, 0.00],
                    [1.00, 0.00, 0.00, 0.00],
                    [0.35, 0.00, 0.00, 0.65],
                    [0.00, 0.00, 1.00, 0.00]])
P1_TAYAL = np.array([0.50, 0.00, 0.50, 0.00])


def smoothed_identity(K, L, weight=9.0):
    """Emission rows normalize(1 + weight * e_k) (state k favours symbol k)."""
    B = np.ones((K, L))
    for k in range(K):
        B[k, k % L] += weight
    return B / B.sum(axis=1, keepdims=True)


def hmm_gauss(N=1, S=8, T=64, K=3, seed=SEED):
    """hmm/stan/hmm.stan: mu = 10, 20, ..., sigma = 3 (hmm/main.R:7-11, App. C)."""
    g = rng(seed, 1)
    A = default_A(K)
    p1 = np.full(K, 1.0 / K)
    mu = 10.0 * np.arange(1, K + 1)
    z = _markov_chain(g, N, T, A, p1)
    x = g.normal(mu[z], 3.0)
    draws = {
        "p_1k": _dirichlet_rows(g, p1, S)[:, 0, :],
        "A_ij": _dirichlet_rows(g, A, S),
        "mu_k": np.sort(mu[None, :] + g.normal(0, 0.05 * 10, (S, K)), axis=1),
        "sigma_k": 3.0 * np.exp(g.normal(0, 0.05, (S, K))),
    }
    return {"K": K, "x": x}, draws


def hmm_multinom(N=1, S=8, T=64, K=4, L=9, seed=SEED, A=None, p1=None, B=None):
    """hmm/stan/hmm-multinom.stan; A, p1 of hmm/main-multinom-semisup.R for K = 4."""
    g = rng(seed, 2)
    if A is None:
        A = A_SEMISUP if K == 4 else default_A(K)
    if p1 is None:
        p1 = P1_SEMISUP if K == 4 else np.full(K, 1.0 / K)
    if B is None:
        B = smoothed_identity(K, L)
    z = _markov_chain(g, N, T, A, p1)
    x = _categorical(g, B, z)
    draws = {
        "p_1k": _dirichlet_rows(g, p1, S)[:, 0, :],
        "A_ij": _dirichlet_rows(g, A, S),
        "phi_k": _dirichlet_rows(g, B, S),
    }
    return {"K": K, "L": L, "x": x}, draws


def hmm_multinom_semisup(N=1, S=8, T=64, K=4, L=9, seed=SEED):
    """hmm/stan/hmm-multinom-semisup.stan: g[t] = group of the true state."""
    data, draws = hmm_multinom(N, S, T, K, L, seed)
    g = rng(seed, 3)
    # groups follow the state pattern of semisup.R:9; extra states alternate
    gmap = np.array([G_OF_STATE[k % 4] for k in range(K)])
    # the true states are not returned by hmm_multinom; regenerate groups from x
    z_guess = (np.asarray(data["x"]) - 1) % K
    data["g"] = gmap[z_guess]
    flip = g.random(data["g"].shape) < 0.05
    data["g"] = np.where(flip, 3 - data["g"], data["g"])
    data["G"] = 2
    return data, draws


def tayal(N=1, S=8, T=64, L=9, seed=SEED, T_oos=None):
    """tayal2009/stan/hhmm-tayal2009[-lite].stan, A / p1 of tayal2009/main-sim.R:10-15.
    U states {2,3} emit with sign = 1 (up), D states {1,4} with sign = 2."""
    K = 4
    g = rng(seed, 4)
    B = smoothed_identity(K, L, weight=4.0)

    def sim(TT):
        z = _markov_chain(g, N, TT, A_TAYAL, P1_TAYAL)
        x = _categorical(g, B, z)
        sign = np.where((z == 1) | (z == 2), 1, 2)
        return x, sign

    x, sign = sim(T)
    data = {"K": K, "L": L, "x": x, "sign": sign}
    if T_oos:
        xo, so = sim(T_oos)
        data.update({"x_oos": xo, "sign_oos": so})
    A_row = np.empty((S, 2, 2))
    A_row[:, 0, :] = g.dirichlet(200 * np.array([0.8, 0.2]) + 1, size=S)
    A_row[:, 1, :] = g.dirichlet(200 * np.array([0.35, 0.65]) + 1, size=S)
    draws = {
        "p_11": g.beta(100.0, 100.0, size=S),
        "A_row": A_row,
        "phi_k": _dirichlet_rows(g, B, S),
    }
    return data, draws


# iohmm-reg/main.R:14-22 (K = 3); C3 extends to K = 4 with a fourth row.
W_REG = np.array([[1.2, 0.5, 0.3, 0.1], [0.5, 1.2, 0.3, 0.1], [0.5, 0.1, 1.2, 0.1], [0.1, 0.1, 0.1, 1.2]])
B_REG = np.array([[5.0, 6.0, 7.0, 0.5], [1.0, 5.0, 0.1, -0.5], [0.1, -1.0, -5.0, 0.2], [-3.0, 2.0, 1.0, 4.0]])
S_REG = np.array([0.2, 1.0, 2.5, 1.5])
P1_REG = np.array([0.4, 0.2, 0.4, 0.0])


def _softmax_rows(v):
    m = v.max(axis=-1, keepdims=True)
    e = np.exp(v - m)
    return e / e.sum(axis=-1, keepdims=True)


def _iohmm_states(g, u, w, p1):
    N, T, M = u.shape
    z = np.empty((N, T), dtype=np.int64)
    cp = np.cumsum(p1)
    z[:, 0] = np.minimum(np.searchsorted(cp, g.random(N) * cp[-1], side="right"), len(p1) - 1)
    P = _softmax_rows(np.einsum("ntm,km->ntk", u, w))
    c = np.cumsum(P, axis=-1)
    uu = g.random((N, T))
    z[:, 1:] = np.minimum((uu[:, 1:, None] >= c[:, 1:, :]).sum(-1), len(p1) - 1)
    return z


def _pad(a, shape, fill):
    """The reference's K = 3..4 / M = 4 / L = 3 values, extended deterministically to larger shapes."""
    out = np.empty(shape)
    out[...] = fill(np.indices(shape))
    sl = tuple(slice(0, min(n, m)) for n, m in zip(shape, a.shape))
    out[sl] = a[sl]
    return out


def iohmm_reg(N=1, S=8, T=64, K=3, M=4, seed=SEED):
    g = rng(seed, 5)
    w = _pad(W_REG, (K, M), lambda ix: np.where(ix[0] == ix[1] % K, 1.2, 0.1))
    b = _pad(B_REG, (K, M), lambda ix: 2.0 * np.cos(1.0 + ix[0] * 1.7 + ix[1] * 0.9))
    s = _pad(S_REG, (K,), lambda ix: 0.5 + 0.3 * ix[0])
    p1 = _pad(P1_REG, (K,), lambda ix: 0.1 + 0 * ix[0])
    p1 = np.where(p1 > 0, p1, 0.1)
    p1 /= p1.sum()
    u = g.normal(0, 1, (N, T, M))
    z = _iohmm_states(g, u, w, p1)
    mean = np.einsum("ntm,ntm->nt", u, b[z])
    x = g.normal(mean, s[z])
    draws = {
        "p_1k": _dirichlet_rows(g, p1, S)[:, 0, :],
        "w_km": w[None] + g.normal(0, 0.05, (S, K, M)),
        "b_km": b[None] + g.normal(0, 0.05, (S, K, M)),
        "s_k": s[None] * np.exp(g.normal(0, 0.05, (S, K))),
    }
    return {"K": K, "M": M, "x_t": x, "u_tm": u}, draws


def _mix_true(K, L):
    # iohmm-mix/main.R:16-28; the 12 w values fill a 4 x 4 matrix by R recycling
    wv = [1.2, 0.5, 0.3, 0.1, 0.5, 1.2, 0.3, 0.1, 0.5, 0.1, 1.2, 0.1]
    w = np.array([wv[i % 12] for i in range(16)]).reshape(4, 4)
    lam = np.array([[2, 0.1, 0.5], [1.2, 0.3, 1.6], [0.1, 0.5, 0.5], [0.1, 1.2, 0.1]])
    mu = np.arange(1, 13, dtype=np.float64).reshape(4, 3)
    s = np.tile([0.1, 0.3, 0.5], (4, 1))
    p1 = np.array([0.25, 0.10, 0.45, 0.15])
    lam = _pad(lam, (K, L), lambda ix: 0.3 + 0.2 * ((ix[0] + ix[1]) % 3))
    lam = lam / lam.sum(axis=1, keepdims=True)
    mu = _pad(mu, (K, L), lambda ix: 1.0 + 3 * ix[0] + ix[1])
    s = _pad(s, (K, L), lambda ix: 0.1 + 0.2 * (ix[1] % 3))
    p1 = _pad(p1, (K,), lambda ix: 0.1 + 0 * ix[0])
    return w[:K], lam, mu, s, p1 / p1.sum()


def iohmm_mix(N=1, S=8, T=64, K=4, L=3, M=4, seed=SEED):
    """iohmm-mix / iohmm-hmix / iohmm-hmix-lite inputs (same data and parameters)."""
    g = rng(seed, 6)
    w, lam, mu, s, p1 = _mix_true(K, L)
    w = _pad(w, (K, M), lambda ix: np.where(ix[0] == ix[1] % K, 1.2, 0.1))
    u = g.normal(0, 1, (N, T, M))
    z = _iohmm_states(g, u, w, p1)
    comp = _categorical(g, lam, z) - 1
    x = g.normal(mu[z, comp], s[z, comp])
    draws = {
        "p_1k": _dirichlet_rows(g, p1, S)[:, 0, :],
        "w_km": w[None] + g.normal(0, 0.05, (S, K, M)),
        "lambda_kl": _dirichlet_rows(g, lam, S),
        "mu_kl": np.sort(mu[None] + g.normal(0, 0.05, (S, K, L)), axis=2),
        "s_kl": s[None] * np.exp(g.normal(0, 0.05, (S, K, L))),
    }
    data = {"K": K, "M": M, "L": L, "x_t": x, "u_tm": u,
            "hyperparams": np.array([0, 5, 10, 0, 5, 1, 1, 0, 10], dtype=np.float64)}
    return data, draws


def ffbs_uniforms(P, T, seed=SEED):
    """Caller-supplied FFBS uniforms in (0, 1), shape (P, T) (Philox stream 7)."""
    u = rng(seed, 7).random((P, T))
    return np.where(u > 0.0, u, 0.5)


def hat_rand(P, T, seed=SEED):
    """Caller randomness of the IOHMM fitted-output draws, shape (P, T, 3):
    [..., 0] uniform for hatz_t, [..., 1] uniform for hatl_t (both in (0, 1)),
    [..., 2] standard normal deviate for hatx_t (Philox stream 8)."""
    g = rng(seed, 8)
    r = np.empty((P, T, 3))
    u = g.random((P, T, 2))
    r[..., :2] = np.where(u > 0.0, u, 0.5)
    r[..., 2] = g.standard_normal((P, T))
    return r


GENERATORS = {
    "hmm": hmm_gauss,
    "hmm-multinom": hmm_multinom,
    "hmm-multinom-semisup": hmm_multinom_semisup,
    "hhmm-tayal2009": tayal,
    "hhmm-tayal2009-lite": lambda **kw: tayal(T_oos=kw.pop("T_oos", 48), **kw),
    "iohmm-reg": iohmm_reg,
    "iohmm-mix": iohmm_mix,
    "iohmm-hmix": iohmm_mix,
    "iohmm-hmix-lite": iohmm_mix,
}


# Every TP / GQ output each Stan program declares.
PARS = {
    "hmm": ["loglik", "unalpha_tk", "alpha_tk", "unbeta_tk", "beta_tk", "ungamma_tk", "gamma_tk", "zstar_t",
            "logp_zstar"],
    "iohmm-reg": ["loglik", "unalpha_tk", "alpha_tk", "unbeta_tk", "beta_tk", "ungamma_tk", "gamma_tk",
                  "zstar_t", "logp_zstar", "oblik_tk", "logA_ij"],
    "iohmm-hmix": ["loglik", "unalpha_tk", "alpha_tk", "beta_tk", "gamma_tk", "oblik_tk", "oblik_t", "logA_ij",
                   "zstar_t", "logp_zstar"],
    "iohmm-hmix-lite": ["loglik", "unalpha_tk", "oblik_tk", "oblik_t", "logA_ij"],
    "hhmm-tayal2009-lite": ["loglik", "unalpha_tk", "alpha_tk", "unalpha_tk_oos", "alpha_tk_oos", "zstar_t",
                            "logp_zstar"],
}
PARS["hmm-multinom"] = PARS["hmm"]
PARS["hmm-multinom-semisup"] = PARS["hmm"]
PARS["hhmm-tayal2009"] = PARS["hmm"]
PARS["iohmm-mix"] = PARS["iohmm-reg"]

# Fitted-output GQ draws each IOHMM program declares.
HAT_PARS = {
    "iohmm-reg": ["hatpi_tk", "hatz_t", "hatx_t"],
    "iohmm-mix": ["hatpi_tk", "hatz_t", "hatl_t", "hatx_t"],
    "iohmm-hmix": ["hatz_t", "hatl_t", "hatx_t"],
}
