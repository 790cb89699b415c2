"""Parity tolerances (north_star: 1e-9 relative in fp64; paths bit-exact).

* probability-space outputs (alpha, beta, gamma, ungamma): |a - b| <= 1e-9 |b| + 1e-250.
  The reference normalises in probability space, so components below ~1e-308
  flush to 0; the floor keeps such underflow from counting.
* log-space outputs (loglik, unalpha, unbeta, logp_zstar, oblik): |a - b| <= 1e-9 max(|b|, 1),
  i.e. 1e-9 relative to the log value (north_star's bound for the
  log-likelihood), with an absolute floor of 1e-9 near 0 where a relative
  error is meaningless.  This is NOT 1e-9 relative in probability for the
  per-step log outputs of a long series: at T = 10^6 |unalpha_tk| reaches
  ~2e6, so the bound is 2e-3 in log space there.  The per-step
  posteriors are held to 1e-9 relative in probability by the alpha / beta /
  gamma comparisons (PROB above), which every long-series test makes; the
  log-space bound is reported (max_log_abs_err) where those tests print it.
* NaN / +-inf must sit in the same places on both sides.
* integer outputs (zstar_t, z_ffbs, pair_status): exact.
"""
import numpy as np

PROB = {"alpha_tk", "beta_tk", "gamma_tk", "ungamma_tk", "alpha_tk_oos"}
LOG = {"loglik", "unalpha_tk", "unbeta_tk", "logp_zstar", "oblik_tk", "oblik_t", "unalpha_tk_oos", "logA_ij"}
INT = {"zstar_t", "z_ffbs", "pair_status"}
RTOL = 1e-9


def compare(name, got, ref):
    got = np.asarray(got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    if name in INT:
        bad = np.flatnonzero((got != ref).ravel(order="F"))
        assert bad.size == 0, f"{name}: {bad.size} mismatches, first at flat index {bad[:5]}"
        return
    gn, rn = np.isnan(got), np.isnan(ref)
    assert np.array_equal(gn, rn), f"{name}: NaN placement differs ({gn.sum()} vs {rn.sum()})"
    gi, ri = np.isinf(got), np.isinf(ref)
    assert np.array_equal(gi, ri) and np.array_equal(got[gi], ref[ri]), f"{name}: inf placement differs"
    m = ~(gn | gi)
    g, r = got[m], ref[m]
    if name in PROB:
        tol = RTOL * np.abs(r) + 1e-250
    elif name in LOG:
        tol = RTOL * np.maximum(np.abs(r), 1.0)
    else:
        raise KeyError(name)
    err = np.abs(g - r)
    worst = int(np.argmax(err - tol)) if err.size else 0
    assert np.all(err <= tol), (f"{name}: max err {err.max():.3e} exceeds tolerance "
                                f"(got {g[worst]!r}, ref {r[worst]!r})")


def compare_all(got, ref, names=None):
    for k in names or ref:
        if k in ("status",):
            continue
        compare(k, got[k], ref[k])
