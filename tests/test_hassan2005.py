"""IOHMM-reg pinned to the reference's second rendered output: hassan2005.

hassan2005/main.Rmd:250-476 simulates one iohmm-reg series with set.seed(9000)
and fits iohmm-reg.stan (the C3 model with the
previous-state-indexed transition of SURVEY App. A Q5).  main.html prints:

* the true state counts after relabelling, 102 / 108 / 90 (main.html:749-753);
* the posterior summary (main.html:440-725);
* the "Hard classification" table of which.max(round(median alpha_tk))
  against the relabelled truth: 89 4 1 / 10 100 1 / 3 4 88 (main.html:1131-1161).

R is not in the image, so the inputs come from a Python restatement of R 3.3's
stream (tests/r_rng.py, itself checked against values R prints for known
seeds in tests/test_r_rng.py).  The checks, in order:

1. the regenerated hidden path has exactly the printed state counts (90/108/102
   for original labels 1/2/3) -- this pins the RNG restatement and the
   simulation (u, z; x is drawn from the same stream after z);
2. the oracle's iohmm-reg alpha_tk at the printed posterior means (and, as a
   second point, the printed medians) reproduces the printed relabelling table
   exactly and the printed hard-classification table up to ONE step: the
   reference classifies with the per-step median of alpha over 200 draws, we
   with alpha at one parameter point, and the single step that moves (t=226,
   alpha = 0.504 / 0.496 at the means) is a near-tie.  The residual is
   asserted to be at most one step, and to sit on a step whose winning margin
   is under 0.05, where the median step's margin is above 0.9;
3. discrimination: the techreview form that indexes the transition by the
   CURRENT state (techreview/Rmd/iohmm.Rmd:20-23), and alpha at the
   TRUE parameters, both score measurably worse (L1 distance >= 6);
4. (GPU) the HIP path at the same point agrees with the oracle on every
   output of the program (1e-9 relative, paths bit-exact).
"""
import numpy as np
import pytest

import hassan2005 as h
from tolerances import compare

ALL = ["loglik", "unalpha_tk", "alpha_tk", "unbeta_tk", "beta_tk", "ungamma_tk", "gamma_tk", "zstar_t",
       "logp_zstar", "oblik_tk", "logA_ij"]


@pytest.fixture(scope="module")
def sim():
    return h.simulate()


def _alpha(oracle, sim, point):
    u, z, x = sim
    out = oracle.gqs("iohmm-reg", h.stan_data(u, x), h.draws(point), pars=["alpha_tk", "oblik_tk", "logA_ij"])
    return out


def test_state_counts(sim):
    _, z, _ = sim
    assert [int((z == k).sum()) for k in (1, 2, 3)] == [90, 108, 102]
    assert z.shape == (h.T,) and set(np.unique(z)) == {1, 2, 3}


@pytest.mark.parametrize("point", ["mean", "median"])
def test_hard_classification(oracle, sim, point):
    _, z, _ = sim
    params = h.POSTERIOR_MEAN if point == "mean" else h.POSTERIOR_MEDIAN
    al = _alpha(oracle, sim, params)["alpha_tk"][0]
    zr = h.relabel(al, z)
    assert np.array_equal(h.table(zr, z), h.RELABEL_TABLE)
    got = h.hard_table(al, zr)
    print(point, got.tolist())
    assert got.sum() == h.T and np.array_equal(got.sum(axis=0), h.HARD_TABLE.sum(axis=0))
    assert np.abs(got - h.HARD_TABLE).sum() <= 2  # at most one step moved between two cells
    est = np.array([h.which_max(np.round(a)) for a in al])
    # the moved step is a near-tie: its top two alpha components are within 0.05
    # (0.008 at the means, 0.035 at the medians; the median step margin is > 0.9)
    if np.abs(got - h.HARD_TABLE).sum() == 2:
        d = got - h.HARD_TABLE
        (ri, ci), = np.argwhere(d > 0)
        cand = np.flatnonzero((est == ri + 1) & (zr == ci + 1))
        top2 = np.sort(al[cand], axis=1)[:, -2:]
        assert (top2[:, 1] - top2[:, 0]).min() < 0.05
    margins = np.diff(np.sort(al, axis=1)[:, -2:], axis=1)
    assert np.median(margins) > 0.9


def test_discrimination(oracle, sim):
    """Indexing A_ij[t] by the current state, or using the true parameters,
    moves the table away from the printed one by far more than one step."""
    from scipy.special import logsumexp
    _, z, _ = sim
    out = _alpha(oracle, sim, h.POSTERIOR_MEAN)
    ob, A = out["oblik_tk"][0], out["logA_ij"][0]
    un = np.empty((h.T, h.K))
    un[0] = np.log(h.POSTERIOR_MEAN["p_1k"]) + ob[0]
    for t in range(1, h.T):  # techreview form: log A_ij[t][j] for the current state j
        un[t] = logsumexp(un[t - 1]) + np.log(A[t]) + ob[t]
    al2 = np.exp(un - logsumexp(un, axis=1, keepdims=True))
    d_cur = np.abs(h.hard_table(al2, h.relabel(al2, z)) - h.HARD_TABLE).sum()
    true = dict(p_1k=h.P1_TRUE, w_km=h.W_TRUE, b_km=h.B_TRUE, s_k=h.S_TRUE)
    al3 = _alpha(oracle, sim, true)["alpha_tk"][0]
    d_true = np.abs(h.hard_table(al3, h.relabel(al3, z)) - h.HARD_TABLE).sum()
    print("L1 distance: current-state form", d_cur, "true parameters", d_true)
    assert d_cur >= 6 and d_true >= 6


def test_oracle_variants_agree(oracle, sim):
    """The correctly rounded and the libm oracle builds agree on this point."""
    u, _, x = sim
    a = oracle.gqs("iohmm-reg", h.stan_data(u, x), h.draws(h.POSTERIOR_MEAN), pars=ALL)
    b = oracle.gqs("iohmm-reg", h.stan_data(u, x), h.draws(h.POSTERIOR_MEAN), pars=ALL, variant="libm")
    for k in ALL:
        if k != "zstar_t":
            compare(k, b[k], a[k])


@pytest.mark.gpu
@pytest.mark.parametrize("point", ["mean", "median", "true"])
def test_gpu_parity_at_hassan2005(engine, oracle, sim, point):
    import hhmm_amd
    u, z, x = sim
    params = {"mean": h.POSTERIOR_MEAN, "median": h.POSTERIOR_MEDIAN,
              "true": dict(p_1k=h.P1_TRUE, w_km=h.W_TRUE, b_km=h.B_TRUE, s_k=h.S_TRUE)}[point]
    data, dr = h.stan_data(u, x), h.draws(params)
    got = hhmm_amd.gqs("iohmm-reg", data, dr, pars=ALL, lib=engine, return_status=True)
    ref = oracle.gqs("iohmm-reg", data, dr, pars=ALL, return_status=True)
    assert np.array_equal(got["pair_status"], ref["pair_status"])
    for k in ALL:
        compare(k, got[k], ref[k])
    if point != "true":
        al = got["alpha_tk"][0]
        zr = h.relabel(al, z)
        assert np.array_equal(h.table(zr, z), h.RELABEL_TABLE)
        assert np.abs(h.hard_table(al, zr) - h.HARD_TABLE).sum() <= 2
