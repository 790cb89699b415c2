"""CPU: the chaining of segment summaries (hhmm_amd.segment.boundaries) against
a direct forward / backward product on random K x K factors -- the host
arithmetic of SURVEY.md §8e's exchange step, without a GPU."""
import numpy as np

from hhmm_amd import segment


def _summary(F, Q, fex, lsc, qex):
    K = F.shape[1]
    P = F.shape[0]
    s = np.zeros((2 * K * K + 3, P))
    s[:K * K] = F.reshape(P, K * K).T
    s[K * K:2 * K * K] = Q.reshape(P, K * K).T
    s[2 * K * K] = fex
    s[2 * K * K + 1] = lsc
    s[2 * K * K + 2] = qex
    return s


def test_boundaries_match_direct_products():
    rng = np.random.default_rng(7)
    P, K, R = 5, 4, 4
    f0 = rng.random((P, K))
    Fs = [np.repeat(f0[:, None, :], K, axis=1)] + [rng.random((P, K, K)) for _ in range(R - 1)]
    Qs = [rng.random((P, K, K)) for _ in range(R)]
    fex = [rng.integers(-40, 40, P).astype(float) for _ in range(R)]
    lsc = [rng.normal(size=P) for _ in range(R)]
    qex = [rng.integers(-40, 40, P).astype(float) for _ in range(R)]
    sums = [_summary(Fs[r], Qs[r], fex[r], lsc[r], qex[r]) for r in range(R)]
    enter, leave, loglik = segment.boundaries(sums, K)
    assert enter[0] is None and leave[R - 1] is None
    for p in range(P):
        # forward: f leaving window r = f0-row of window 0, then times each later window, with scales
        f = Fs[0][p, 0].copy()
        logsc = lsc[0][p] + np.log(2.0) * fex[0][p]
        for r in range(1, R):
            e = enter[r][:, p]
            np.testing.assert_allclose(e[:K] * np.exp(e[K] - logsc), f, rtol=1e-12)
            f = f @ Fs[r][p]
            logsc += lsc[r][p] + np.log(2.0) * fex[r][p]
        np.testing.assert_allclose(loglik[p], np.log(f.sum()) + logsc, rtol=1e-12)
        b = np.ones(K)
        bl = 0.0
        for r in range(R - 1, 0, -1):
            b = Qs[r][p] @ b
            bl += lsc[r][p] + np.log(2.0) * qex[r][p]
            v = leave[r - 1][:, p]
            np.testing.assert_allclose(v[:K] * np.exp(v[K] - bl), b, rtol=1e-12)


def test_windows_cover_the_series():
    for T in (1, 7, 1000, 1_000_001):
        for R in (1, 2, 3, 8):
            w = segment.windows(T, R)
            assert w[0][0] == 0 and w[-1][1] == T
            assert all(w[i][1] == w[i + 1][0] for i in range(R - 1))
