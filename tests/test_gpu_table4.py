"""GPU parity at the reference-pinned Tayal parameter point.

tests/test_rdata.py pins the oracle's hhmm-tayal2009-lite forward to Table 4 of the
reference's rendered report (tayal2009/main.pdf; main.Rmd:596-602, 704-723) at the
posterior means printed in its Table 8 (main.Rmd:869-907).  The real ticks (CC-BY-NC,
tayal2009/data) cannot travel to the GPU box, so this test drives the engine at the
same parameter point over synthetic leg sequences with the report's symbol mix: the
18 feature counts of Table 4 (its column sums), drawn i.i.d. and as runs, in-sample
T = 8386 and out-of-sample T = 1380 (the G.TO windows).  The engine's alpha_tk,
alpha_tk_oos, unalpha_tk(_oos), loglik, OOS zstar_t and logp_zstar must match the
oracle (tests/tolerances.py), and so must the Table-4-style tabulation of
which.max(alpha_tk).  The full model (hhmm-tayal2009: backward, gamma, in-sample
Viterbi) runs at the same point too.
"""
import numpy as np
import pytest

from hhmm_amd import synth
from test_rdata import TABLE4, table8_draw, tabulate
from tolerances import compare, compare_all

pytestmark = pytest.mark.gpu

T_INS, T_OOS = 8386, 1380


def _legs(g, n, runs):
    """Feature codes 1..18 with Table 4's marginal mix (U1..U9 = 1..9, D1..D9 = 10..18)."""
    p = TABLE4.sum(axis=0) / TABLE4.sum()
    if not runs:
        return g.choice(18, size=n, p=p) + 1
    out = np.empty(n, dtype=np.int64)  # runs of geometric length: regimes as in the real series
    t = 0
    while t < n:
        k = min(n - t, int(g.geometric(0.3)))
        out[t:t + k] = g.choice(18, p=p) + 1
        t += k
    return out


def _data(N, runs, seed=4):
    g = synth.rng(synth.SEED, seed)
    fi = np.stack([_legs(g, T_INS, runs) for _ in range(N)])
    fo = np.stack([_legs(g, T_OOS, runs) for _ in range(N)])
    split = lambda f: (np.where(f <= 9, f, f - 9), np.where(f <= 9, 1, 2))  # noqa: E731 (main.Rmd:442-446)
    x, s = split(fi)
    xo, so = split(fo)
    return fi, {"K": 4, "L": 9, "x": x, "sign": s, "x_oos": xo, "sign_oos": so}


def _draws(S, seed=5):
    """Table 8's point first, then S-1 draws jittered around it (SURVEY §8d's Dirichlet rule)."""
    d = table8_draw()
    if S == 1:
        return d
    g = synth.rng(synth.SEED, seed)
    p11 = np.concatenate([d["p_11"], g.beta(200 * 0.51 + 1, 200 * 0.49 + 1, size=S - 1)])
    A_row = np.concatenate([d["A_row"], np.stack([g.dirichlet(200 * np.array(r) + 1, size=S - 1)
                                                  for r in d["A_row"][0]], axis=1)])
    phi = np.concatenate([d["phi_k"], np.stack([g.dirichlet(200 * r + 1, size=S - 1)
                                                for r in d["phi_k"][0]], axis=1)])
    return {"p_11": p11, "A_row": A_row, "phi_k": phi}


LITE = ["loglik", "unalpha_tk", "alpha_tk", "unalpha_tk_oos", "alpha_tk_oos", "zstar_t", "logp_zstar"]


@pytest.mark.parametrize("runs", [False, True], ids=["iid", "runs"])
def test_table8_point_lite(engine, oracle, runs):
    """One series under one draw: the report's own request shape."""
    import hhmm_amd
    feat, data = _data(1, runs)
    draw = _draws(1)
    got = hhmm_amd.gqs("hhmm-tayal2009-lite", data, draw, pars=LITE, lib=engine, return_status=True)
    ref = oracle.gqs("hhmm-tayal2009-lite", data, draw, pars=LITE, return_status=True)
    compare_all(got, ref, LITE + ["pair_status"])
    tg = tabulate(feat[0], np.argmax(got["alpha_tk"][0], axis=1) + 1)
    tr = tabulate(feat[0], np.argmax(ref["alpha_tk"][0], axis=1) + 1)
    assert np.array_equal(tg, tr) and tg.sum() == T_INS


@pytest.mark.parametrize("S", [64, 1024])
def test_table8_neighbourhood_lite_batch(engine, oracle, S):
    """4 series x S draws around the Table 8 point (grid pairing): the batched lane path."""
    import hhmm_amd
    _, data = _data(4, True, seed=6)
    draws = _draws(S)
    got = hhmm_amd.gqs("hhmm-tayal2009-lite", data, draws, pars=LITE, lib=engine, return_status=True)
    idx = np.unique(np.r_[0:8, S - 8:S, S:S + 4, 3 * S + S // 2, 4 * S - 1])  # pairs p = s + S n
    sub_n = idx // S
    sub_s = idx % S
    for n in np.unique(sub_n):
        ss = sub_s[sub_n == n]
        dn = {k: v[n:n + 1] for k, v in data.items() if k not in ("K", "L")}
        dn.update(K=4, L=9)
        dd = {k: v[ss] for k, v in draws.items()}
        ref = oracle.gqs("hhmm-tayal2009-lite", dn, dd, pars=LITE, return_status=True)
        for name in LITE + ["pair_status"]:
            compare(name, np.asarray(got[name])[ss + S * n], ref[name])


# LIN: the probability-space outputs (the scaled linear filters, the T-scan); with unalpha_tk /
# unbeta_tk requested the engine runs the log-space recursions instead (FULL).
LIN = ["loglik", "alpha_tk", "beta_tk", "gamma_tk", "zstar_t", "logp_zstar"]
FULL = LIN + ["unalpha_tk", "unbeta_tk"]


@pytest.mark.parametrize("pars", [LIN, FULL], ids=["linear", "log-space"])
def test_table8_point_full_model(engine, oracle, pars):
    """hhmm-tayal2009.stan at the same point: backward (Q6 previous-state mask), gamma, Viterbi."""
    import hhmm_amd
    _, data = _data(2, True, seed=7)
    data = {k: v for k, v in data.items() if not k.endswith("_oos")}
    draws = _draws(16)
    got = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=pars, lib=engine, return_status=True)
    ref = oracle.gqs("hhmm-tayal2009", data, draws, pars=FULL, return_status=True)
    compare_all(got, ref, [n for n in pars if n != "gamma_tk"] + ["pair_status"])
    from test_gpu_configs import compare_tayal_gamma
    compare_tayal_gamma(got, ref, max_forgiven=0)


# ---- degenerate draws on the sign-class paths ------------------------------------
# The Tayal kernels skip the flattened HHMM's structural transition zeros when a wave's lanes
# share a step's sign (hhmm_hmm.h tayal_nz / tayal_dispatch).  0 x f adds nothing to a sum of
# finite terms, but the reference computes in log space, where a NaN on a skipped path still
# reaches every accumulator (NaN + -inf = NaN, hhmm-tayal2009.stan:60-71).  The skip is taken
# only where the wave's p_11, A_row and phi_k are all probabilities; these draws are not, and
# must give the oracle's values and NaN placement exactly.
# (An infinite phi entry is left out: there log space gives inf + log 0 = NaN for every
# transition with a zero probability while linear space gives 0 x inf only where the whole
# sum is zero -- the two arithmetics part there with or without the skip.)
DEGENERATE = ["p11_nan", "phi_nan", "arow_above_one", "arow_zero"]


def _degenerate(kind, S=64):
    d = _draws(S)
    d = {k: v.copy() for k, v in d.items()}
    s = 5
    if kind == "p11_nan":
        d["p_11"][s] = np.nan
    elif kind == "phi_nan":
        d["phi_k"][s, 1, 4] = np.nan
    elif kind == "arow_above_one":
        d["A_row"][s, 1, 0] = 1.5
    elif kind == "arow_zero":  # a valid draw with an extra zero: the skip stays on
        d["A_row"][s, 0] = (0.0, 1.0)
    return d


@pytest.mark.parametrize("kind", DEGENERATE)
@pytest.mark.parametrize("T,flags", [(300, 0), (40_000, 0), (40_000, 2)], ids=["lanes", "scan", "scan-off"])
def test_degenerate_draw_sign_class_paths(engine, oracle, kind, T, flags):
    """One series under 64 draws (C5's wave shape: every lane shares each step's sign)."""
    import hhmm_amd
    g = synth.rng(synth.SEED, 9)
    f = _legs(g, T, True)
    data = {"K": 4, "L": 9, "x": np.where(f <= 9, f, f - 9)[None], "sign": np.where(f <= 9, 1, 2)[None]}
    draws = _degenerate(kind)
    got = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=LIN, lib=engine, return_status=True, flags=flags)
    ref = oracle.gqs("hhmm-tayal2009", data, draws, pars=FULL, return_status=True, nthreads=8)
    names = ["loglik", "alpha_tk", "beta_tk", "zstar_t", "logp_zstar", "pair_status"]
    compare_all(got, ref, names)
    from test_gpu_configs import compare_tayal_gamma
    compare_tayal_gamma(got, ref, max_forgiven=0)


def test_c5_scale_gamma_at_table8_point(engine, oracle):
    """C5's shape (one series of 10^6 legs under many draws; the T-scan and the V-scan) at
    the reference's own parameter point, over the report's symbol mix in runs.  On C5's
    synthetic data gamma is ~99.7 % NaN rows (Q6: the forward and backward masks drive
    alpha and beta apart until their overlap underflows); at Table 8's
    point and Table 4's mix the overlap stays finite, so gamma itself is compared at every
    one of the 10^6 steps of 8 pairs -- with loglik, alpha, beta and the Viterbi."""
    import hhmm_amd
    T = 1_000_000
    g = synth.rng(synth.SEED, 10)
    f = _legs(g, T, True)
    data = {"K": 4, "L": 9, "x": np.where(f <= 9, f, f - 9)[None], "sign": np.where(f <= 9, 1, 2)[None]}
    draws = _draws(8, seed=11)
    got = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=LIN, lib=engine, return_status=True)
    ref = oracle.gqs("hhmm-tayal2009", data, draws, pars=FULL, return_status=True, nthreads=8)
    nan_rows = int(np.isnan(ref["gamma_tk"]).any(axis=-1).sum())
    print(f"oracle gamma NaN rows: {nan_rows} of {8 * T}")
    assert nan_rows < 0.01 * 8 * T
    compare_all(got, ref, [n for n in LIN if n != "gamma_tk"] + ["pair_status"])
    from test_gpu_configs import compare_tayal_gamma
    compare_tayal_gamma(got, ref, max_forgiven=64)
