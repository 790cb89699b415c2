"""Nearest-neighbour forecast over oblik_t.

Reference: neighbouring_forecast(x, oblik_t, h, threshold), hassan2005/R/forecast.R:1-31,
fed by iohmm-hmix(-lite)'s oblik_t (hassan2005/main.R:94,138).  R is absent, so parity
with R is unpinned; the C oracle (oracle/forecast_oracle.c) is pinned by the
transcription below (80-bit long-double sums like R's sum(), math.exp like R's exp).
The GPU sums in double in the same order and uses the correctly rounded exp:
forecasts agree within 1e-12 relative; the neighbour selection is exact.
"""
import math

import numpy as np
import pytest

from hhmm_amd import forecast as Fc
from hhmm_amd import synth


def transcribe(x, oblik_t, h=1, threshold=0.05):
    """forecast.R line by line for one series x[T] and oblik_t[S, T]."""
    S, T = oblik_t.shape
    out = []
    for n in range(S):
        target = float(oblik_t[n, T - 1])                      # :20
        cand = [float(v) for v in oblik_t[n, :T - h]]          # :21
        dist = [abs(target - c) for c in cand]
        ind = [i for i, d in enumerate(dist) if d < abs(target) * threshold]   # :10
        if not ind:                                            # :12-13
            if any(math.isnan(d) for d in dist):
                out.append(float("nan"))
                continue
            m = min(dist)
            ind = [i for i, d in enumerate(dist) if d == m]
        num, den = np.longdouble(0), np.longdouble(0)
        for i in ind:                                          # :24-27
            w = math.exp(abs(target - float(oblik_t[n, i])))
            num += np.longdouble((float(x[i + h]) - float(x[i])) * w)
            den += np.longdouble(w)
        out.append(float(x[T - 1]) + float(num) / float(den))
    return np.array(out)


def _cases():
    g = np.random.Generator(np.random.Philox(key=21))
    T, S = 120, 40
    x = np.cumsum(g.normal(0, 1, T)) + 50
    ob = g.normal(-3.0, 1.0, (S, T))
    yield "random", x, ob, 1, 0.05
    yield "h3_wide", x, ob, 3, 0.3
    ob2 = ob.copy()
    ob2[:, -1] = 1e-9                  # tiny |target|: no candidate inside the threshold -> minimisers
    ob2[:5, 10] = ob2[:5, 20] = 0.25   # exact ties of the minimum
    yield "min_ties", x, ob2, 1, 0.05
    ob3 = ob.copy()
    ob3[:3, 7] = np.nan                # NaN distance: min() is NA when nothing is within the threshold
    ob3[:3, -1] = 1e-12
    yield "nan", x, ob3, 1, 0.05
    yield "short", x[:2], ob[:, :2], 1, 0.05


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_oracle_matches_transcription(oracle, case):
    _, x, ob, h, thr = case
    got = oracle.neighbouring_forecast(x, ob, h, thr)
    want = transcribe(x, ob, h, thr)
    assert np.array_equal(got, want, equal_nan=True)


def test_oracle_batched_series(oracle):
    g = np.random.Generator(np.random.Philox(key=22))
    N, S, T = 3, 7, 50
    x = g.normal(0, 1, (N, T))
    ob = g.normal(-2, 1, (N * S, T))
    got = oracle.neighbouring_forecast(x, ob)
    for n in range(N):
        rows = ob[[s + S * n for s in range(S)]]
        assert np.array_equal(got[[s + S * n for s in range(S)]], transcribe(x[n], rows), equal_nan=True)


def test_bad_shapes():
    with pytest.raises(ValueError):
        Fc.make_request(np.zeros(10), np.zeros((4, 9)))


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_gpu_matches_oracle(engine, oracle, case):
    _, x, ob, h, thr = case
    got = Fc.neighbouring_forecast(x, ob, h, thr, lib=engine)
    ref = oracle.neighbouring_forecast(x, ob, h, thr)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    ok = ~np.isnan(ref)
    assert np.allclose(got[ok], ref[ok], rtol=1e-12, atol=0)


@pytest.mark.gpu
def test_gpu_end_to_end_hmix_lite(engine, oracle):
    """iohmm-hmix-lite oblik_t on the GPU -> forecast on the GPU, against the oracle chain
    (hassan2005/main.R:94,138)."""
    import hhmm_amd
    model = "iohmm-hmix-lite"
    data, draws = synth.GENERATORS[model](N=2, S=96, T=200)
    got_ob = hhmm_amd.gqs(model, data, draws, pars=["oblik_t"], lib=engine)["oblik_t"]
    ref_ob = oracle.gqs(model, data, draws, pars=["oblik_t"])["oblik_t"]
    x = np.asarray(data["x_t"])
    got = Fc.neighbouring_forecast(x, got_ob, lib=engine)
    ref = oracle.neighbouring_forecast(x, ref_ob)
    assert np.allclose(got, ref, rtol=1e-9, atol=0)
