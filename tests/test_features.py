"""Tick -> zig-zag -> leg feature extractor.

Reference: extract_features(tdata, alpha), tayal2009/R/feature-extraction.R:8-133,
with the constants of tayal2009/R/constants.R:2-14 and the Tayal data coding of
tayal2009/main.R:85-89.  R and the xts / highfrequency packages are absent here
and on the GPU box, and the reference stores no extracted features, so parity
with R is unpinned; the C oracle (oracle/features_oracle.c) is pinned by the
independent transcription below (written from the R source, step by step) and
by hand-built known answers.  The GPU path must equal the oracle exactly on
every column (integer-valued sizes, as trade volumes are, keep R's long-double
sum exact in double).
"""
import numpy as np
import pytest

from hhmm_amd import features as F

LEGS = [(1, 1, 1, 1), (1, -1, 1, 2), (1, 1, 0, 3), (1, 0, 1, 4), (1, 0, 0, 5), (1, 0, -1, 6), (1, -1, 0, 7),
        (1, 1, -1, 8), (1, -1, -1, 9), (-1, 1, -1, 10), (-1, -1, -1, 11), (-1, 1, 0, 12), (-1, 0, -1, 13),
        (-1, 0, 0, 14), (-1, 0, 1, 15), (-1, -1, 0, 16), (-1, 1, 1, 17), (-1, -1, 1, 18)]


def _difftime_secs(t1, t0):
    z = t1 - t0
    az = abs(z)
    if not np.isfinite(az) or az < 60:
        return z
    unit = 60.0 if az < 3600 else (3600.0 if az < 86400 else 86400.0)
    return (z / unit) * unit


def transcribe(price, size, time, alpha=0.25):
    """Step-by-step restatement of feature-extraction.R with R's NA rules (None = NA)."""
    price = [float(v) for v in price]
    n = len(price)
    direction = [0] + [1 if price[t] > price[t - 1] else (-1 if price[t] < price[t - 1] else 0)
                       for t in range(1, n)]                                      # :20-24
    ldirection = [None] + direction[:-1]                                          # :26
    chg = [d != 0 and (l is None or d != l) if d != 0 else False
           for d, l in zip(direction, ldirection)]                                # :27
    where = [t + 1 for t in range(n) if chg[t]]                                   # which(direction.chg)
    zp = [price[i - 2] for i in where]                                            # :30
    start = [1] + where[:-1]                                                      # :33
    end = [s - 1 for s in start[1:]] + [n]                                        # :35-36
    m = len(zp)
    sav = [float(sum(int(v) for v in size[s - 1:e])) / (_difftime_secs(time[e - 1], time[s - 1]) + 1)
           for s, e in zip(start, end)]                                           # :41-47
    f0 = [None] + [1 if zp[r - 1] < zp[r] else -1 for r in range(1, m)]           # :50
    f0[0] = -1 if f0[1] == 1 else 1                                               # :51
    f1 = []
    for r in range(m):                                                            # :55-70
        if r + 1 <= 4:
            f1.append(0)
            continue
        e = zp[r - 4:r + 1]
        if e[0] < e[2] < e[4] and e[1] < e[3]:
            f1.append(1)
        elif e[0] > e[2] > e[4] and e[1] > e[3]:
            f1.append(-1)
        else:
            f1.append(0)

    def lag(v, k):
        return [None] * k + v[:len(v) - k]

    def ratio(a, b):
        return [None if (x is None or y is None) else (np.float64(x) / np.float64(y)) for x, y in zip(a, b)]

    def disc(v):                                                                   # :77-79
        out = []
        for x in v:
            if x is None or np.isnan(x):
                out.append(None)
            else:
                out.append(1 if x - 1 > alpha else (-1 if 1 - x > alpha else 0))
        return out

    s1 = disc(ratio(sav, lag(sav, 1)))
    s2 = disc(ratio(sav, lag(sav, 2)))
    s3 = disc(ratio(lag(sav, 1), lag(sav, 2)))

    def r_and(*xs):  # R's three-valued &
        if any(x is False for x in xs):
            return False
        if any(x is None for x in xs):
            return None
        return True

    def cmp(x, f):
        return None if x is None else f(x)

    f2 = [0] * m                                                                  # :85
    for r in range(m):
        if r_and(cmp(s1[r], lambda v: v == 1), cmp(s2[r], lambda v: v > -1), cmp(s3[r], lambda v: v < 1)) is True:
            f2[r] = 1                                                             # :86
    for r in range(m):
        if r_and(cmp(s1[r], lambda v: v == -1), cmp(s2[r], lambda v: v < 1), cmp(s3[r], lambda v: v > -1)) is True:
            f2[r] = -1                                                            # :87
    f2[0:2] = [0, 0]                                                              # :89
    feature = []
    for a, b, c in zip(f0, f1, f2):                                               # :113-125
        for row in LEGS:
            if row[:3] == (a, b, c):
                feature.append(row[3])
                break
        else:
            raise ValueError("Not a valid leg")
    trend = [-1 if c in (6, 7, 8, 9, 15, 16, 17, 18) else (0 if c in (5, 14) else 1) for c in feature]
    return {"price": np.array(zp), "start": np.array(start), "end": np.array(end), "size_av": np.array(sav),
            "f0": np.array(f0), "f1": np.array(f1), "f2": np.array(f2), "feature": np.array(feature),
            "trend": np.array(trend),
            "sign": np.array([1 if c < 10 else 2 for c in feature]),              # tayal2009/main.R:87
            "x": np.array([c if c < 10 else c - 9 for c in feature])}             # :88


def _same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype.kind == "f" or b.dtype.kind == "f":
        a64, b64 = np.asarray(a, np.float64), np.asarray(b, np.float64)
        return a64.shape == b64.shape and (np.array_equal(a64.view(np.int64), b64.view(np.int64))
                                           or np.array_equal(a64, b64))
    return np.array_equal(a, b)


def _assert_same(got, want):
    for k in F.COLUMNS:
        assert _same(got[k], want[k]), (k, got[k][:12], want[k][:12])


def _edge_series():
    g = np.random.Generator(np.random.Philox(key=3))
    cases = []
    p, s, t = F.synth_ticks(2500, seed=1)
    cases.append(("synth", p, s, t))
    # alternating prices: a leg boundary at every tick
    n = 64
    cases.append(("alternating", 10 + 0.01 * (np.arange(n) % 2), np.full(n, 100.0), np.arange(n, dtype=float)))
    # equal closing prices (f0 ties), zero sizes (0/0 ratios -> NA), long pauses (mins/hours/days units)
    p = np.array([10, 11, 10, 11, 10, 12, 12, 12, 11, 13, 11, 13, 10, 14, 9, 15, 9, 9, 16], dtype=float)
    s = np.array([0, 0, 0, 0, 0, 100, 0, 0, 200, 300, 0, 0, 100, 100, 100, 500, 0, 0, 100], dtype=float)
    t = np.cumsum(np.array([0, 1, 61, 2, 3700, 5, 90000, 1.5, 2, 0.25, 7, 59.999, 60.001, 3599.5, 3600.5, 86399,
                            86401, 3, 4], dtype=float)) + 1e9
    cases.append(("ties_zero_pauses", p, s, t))
    # flat runs between moves
    steps = g.choice([-1, 0, 0, 0, 0, 1], size=3000)
    cases.append(("flat_runs", 50 + 0.05 * np.cumsum(steps), 100.0 * g.integers(0, 5, 3000),
                  1e9 + np.cumsum(g.exponential(2.0, 3000))))
    return cases


@pytest.mark.parametrize("case", _edge_series(), ids=lambda c: c[0])
def test_oracle_matches_transcription(oracle, case):
    _, p, s, t = case
    got = oracle.extract_features(p, s, t, alpha=0.25)
    _assert_same(got, transcribe(p, s, t, 0.25))


@pytest.mark.parametrize("alpha", [0.0, 0.1, 0.5])
def test_oracle_alpha(oracle, alpha):
    p, s, t = F.synth_ticks(1500, seed=2)
    _assert_same(oracle.extract_features(p, s, t, alpha=alpha), transcribe(p, s, t, alpha))


def test_known_answer(oracle):
    """Hand-worked: prices 10 11 12 11 10 11 -> directions 0 + + - - +, so legs
    start at ticks 2 (first move off `lt`), 4 and 6."""
    p = np.array([10, 11, 12, 11, 10, 11], dtype=float)
    s = np.array([100, 200, 300, 400, 500, 600], dtype=float)
    t = np.array([0, 1, 2, 3, 4, 5], dtype=float)
    got = oracle.extract_features(p, s, t)
    assert list(got["start"]) == [1, 2, 4] and list(got["end"]) == [1, 3, 6]
    assert list(got["price"]) == [10.0, 12.0, 10.0]     # ticks 1, 3 and 5 (the last leg's end is n)
    assert list(got["size_av"]) == [100.0, 250.0, 500.0]  # 100/(0+1), 500/(1+1), 1500/(2+1)
    assert list(got["f0"]) == [-1, 1, -1]
    assert list(got["f1"]) == [0, 0, 0]
    assert list(got["f2"]) == [0, 0, 0]                 # s1 = s2 = s3 = 1: neither rule fires
    assert list(got["feature"]) == [14, 5, 14] and list(got["trend"]) == [0, 0, 0]
    assert list(got["sign"]) == [2, 1, 2] and list(got["x"]) == [5, 5, 5]


def test_oracle_too_few_legs(oracle):
    p = np.array([10, 11, 12, 13], dtype=float)
    with pytest.raises(RuntimeError):
        oracle.extract_features(p, np.ones(4), np.arange(4.0))


@pytest.mark.gpu
@pytest.mark.parametrize("case", _edge_series(), ids=lambda c: c[0])
def test_gpu_matches_oracle_edge(engine, oracle, case):
    _, p, s, t = case
    _assert_same(F.extract_features(p, s, t, lib=engine), oracle.extract_features(p, s, t))


@pytest.mark.gpu
@pytest.mark.parametrize("n", [3, 4095, 4096, 4097, 8193, 300_001, 2_000_000])
def test_gpu_matches_oracle_sizes(engine, oracle, n):
    p, s, t = F.synth_ticks(n, seed=n)
    if n == 3:
        p = np.array([10.0, 11.0, 10.0])
    _assert_same(F.extract_features(p, s, t, lib=engine), oracle.extract_features(p, s, t))


@pytest.mark.gpu
def test_gpu_too_few_legs(engine):
    from hhmm_amd.api import HHMMError
    with pytest.raises(HHMMError):
        F.extract_features(np.array([1.0, 2.0, 3.0, 4.0]), np.ones(4), np.arange(4.0), lib=engine)


@pytest.mark.gpu
def test_gpu_legs_feed_tayal(engine, oracle):
    """End to end: ticks -> legs -> hhmm-tayal2009-lite data block on the GPU (tayal2009/main.R:84-90)."""
    import hhmm_amd
    from hhmm_amd import synth
    p, s, t = F.synth_ticks(20_000, seed=5)
    legs = F.extract_features(p, s, t, lib=engine)
    T = legs["x"].size
    data, draws = synth.GENERATORS["hhmm-tayal2009"](N=1, S=4, T=T)
    data["x"] = legs["x"].reshape(1, T)
    data["sign"] = legs["sign"].reshape(1, T)
    pars = ["loglik", "zstar_t"]
    got = hhmm_amd.gqs("hhmm-tayal2009", data, draws, pars=pars, lib=engine)
    ref = oracle.gqs("hhmm-tayal2009", data, draws, pars=pars)
    assert np.array_equal(got["zstar_t"], ref["zstar_t"])
    assert np.allclose(got["loglik"], ref["loglik"], rtol=1e-9, atol=0)


def test_no_gpu_fails_loudly(engine):
    """Without a gfx950 device the product path errors; it never falls back to the oracle."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from hhmm_amd import _abi
    from hhmm_amd.api import HHMMError
    p, s, t = F.synth_ticks(1000, seed=4)
    with pytest.raises(HHMMError) as e:
        F.extract_features(p, s, t, lib=engine)
    assert e.value.status == _abi.ERR_NO_DEVICE
