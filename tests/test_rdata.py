"""RDX2 reader for the reference's tick files (SURVEY.md §8 F1 input side;
tayal2009/main.R:47-58 loads tayal2009/data/<SYM>/*.RData with `load()`).

CPU only.  A hand-serialised xts (the same layout the reference's files carry:
REALSXP matrix + dim / dimnames / index / class attributes, XDR, gzip) checks
the decoder everywhere; when /root/reference is present the real G.TO files
are decoded and pushed through the feature oracle, which must agree with the
R-semantics transcription (tests/test_features.py) on real ticks.  The data
(CC-BY-NC, tayal2009/data/LICENSE.md) is read in place, never copied.
"""
import gzip
import pathlib
import struct

import numpy as np
import pytest

from hhmm_amd import rdata

DATA = pathlib.Path("/root/reference/tayal2009/data")


def _i(v):
    return struct.pack(">i", v)


def _flags(t, attr=False, tag=False, obj=False):
    return _i(t | (1 << 9 if attr else 0) | (1 << 10 if tag else 0) | (1 << 8 if obj else 0))


def _charsxp(s):
    b = s.encode()
    return _i(0x00040009) + _i(len(b)) + b


def _sym(name):
    return _i(rdata.SYMSXP) + _charsxp(name)


def _strsxp(vals):
    return _i(rdata.STRSXP) + _i(len(vals)) + b"".join(_charsxp(v) for v in vals)


def _real(vals, attrs=b""):
    v = np.asarray(vals, dtype=">f8")
    return _flags(rdata.REALSXP, attr=bool(attrs)) + _i(v.size) + v.tobytes() + attrs


def _pairlist(items):
    out = b""
    for tag, val in items:
        out += _flags(rdata.LISTSXP, tag=True) + _sym(tag) + val
    return out + _i(rdata.NILVALUE)


def _xts_file(name, price, size, index):
    n = len(price)
    dim = _flags(rdata.INTSXP) + _i(2) + _i(n) + _i(2)
    dimnames = _flags(rdata.VECSXP) + _i(2) + _i(rdata.NILVALUE) + _strsxp(["PRICE", "SIZE"])
    attrs = _pairlist([("dim", dim), ("dimnames", dimnames), ("index", _real(index)),
                       ("class", _strsxp(["xts", "zoo"]))])
    body = _real(np.concatenate([price, size]), attrs)
    raw = b"RDX2\nX\n" + _i(2) + _i(0x030303) + _i(0x020300) + _pairlist([(name, body)])
    return gzip.compress(raw)


def test_reader_roundtrip(tmp_path):
    price = np.array([10.0, np.nan, 10.01, 10.0, 9.99])
    size = np.array([100.0, 200.0, 300.0, np.nan, 500.0])
    index = 1.17802622e9 + np.arange(5.0)
    f = tmp_path / "2007.05.01.X.TO.RData"
    f.write_bytes(_xts_file("X.TO", price, size, index))
    objs = rdata.read_rdata(f)
    assert list(objs) == ["X.TO"]
    idx, cols = rdata.xts_columns(objs["X.TO"])
    assert list(cols) == ["PRICE", "SIZE"] and np.array_equal(idx, index)
    p, s, t = rdata.load_ticks(f)  # na.omit drops rows 2 and 4
    assert np.array_equal(p, [10.0, 10.01, 9.99]) and np.array_equal(s, [100.0, 300.0, 500.0])
    assert np.array_equal(t, index[[0, 2, 4]])


def test_reader_refuses_code(tmp_path):
    raw = b"RDX2\nX\n" + _i(2) + _i(0) + _i(0) + _flags(rdata.LISTSXP, tag=True) + _sym("f") + _i(3)
    f = tmp_path / "closure.RData"
    f.write_bytes(raw)
    with pytest.raises(ValueError):
        rdata.read_rdata(f)


@pytest.mark.skipif(not DATA.exists(), reason="reference tick data not present (GPU box)")
def test_real_ticks_through_feature_oracle(oracle):
    import test_features
    files = sorted((DATA / "G.TO").glob("*.RData"))[:3]
    price, size, time = rdata.load_ticks(files)
    assert price.size > 10_000
    assert (size == np.round(size)).all()  # integer volumes: R's long-double sum is exact in double
    got = oracle.extract_features(price, size, time, alpha=0.25)
    test_features._assert_same(got, test_features.transcribe(price, size, time, 0.25))


# tayal2009/main.Rmd:65-74 -- the data set and windows its rendered report (main.pdf) uses
RMD_DAYS = ("2007.05.04", "2007.05.07", "2007.05.08", "2007.05.09", "2007.05.10", "2007.05.11")
RMD_INS = "2007-05-04 09:30:00/2007-05-10 16:30:00"
RMD_OOS = "2007-05-11 09:30:00/2007-05-11 16:30:00"


@pytest.mark.skipif(not DATA.exists(), reason="reference tick data not present (GPU box)")
def test_in_sample_zigzag_count_matches_report(oracle):
    """Reference-held pin for F1: main.Rmd:410 prints nrow(zig.ins), and the
    rendered tayal2009/main.pdf reads "In-sample dataset reduced to 8386
    zig-zags".  The chain is the report's own: load() + rbind + na.omit of the
    six files (:386-395), extract_features(tdata, 0.25) (:405), zig[ins] with
    the index in America/Toronto (:406, main.R:52)."""
    from hhmm_amd import features as F
    files = [DATA / "G.TO" / f"{d}.G.TO.RData" for d in RMD_DAYS]
    price, size, time = rdata.load_ticks(files)
    legs = oracle.extract_features(price, size, time, alpha=0.25)
    when = time[F.index_ticks(legs, price)]
    assert int(F.xts_window(when, RMD_INS).sum()) == 8386
    assert int(F.xts_window(when, RMD_OOS).sum()) > 0


# Column sums of Table 4 ("tab:tseg-filtered-ins") of the rendered tayal2009/main.pdf:
# main.Rmd:704-723 prints table(x.ins, state.filtered.ins) with the rows labelled by
# expand.grid(1:9, c("U", "D")), i.e. feature codes 1..9 = U1..U9 and 10..18 = D1..D9.
# Summed over the four states they are the in-sample count of each leg feature.
TABLE4_U = (58, 15, 158, 810, 2155, 828, 33, 49, 17)
TABLE4_D = (15, 72, 34, 831, 2209, 846, 181, 16, 59)


@pytest.mark.skipif(not DATA.exists(), reason="reference tick data not present (GPU box)")
def test_in_sample_feature_histogram_matches_report_table4(oracle):
    """Second reference-held pin for F1, symbol by symbol: the per-feature counts
    of the same 8386 in-sample zig-zags pin the leg coding of
    feature-extraction.R:92-110, and the (x, sign) split of tayal2009/main.R:85-89
    (sign = 1 for codes 1..9 = U, x = code; sign = 2 for 10..18 = D, x = code - 9)."""
    from hhmm_amd import features as F
    files = [DATA / "G.TO" / f"{d}.G.TO.RData" for d in RMD_DAYS]
    price, size, time = rdata.load_ticks(files)
    legs = oracle.extract_features(price, size, time, alpha=0.25)
    ins = F.xts_window(time[F.index_ticks(legs, price)], RMD_INS)
    counts = np.bincount(legs["feature"][ins], minlength=19)
    assert counts[0] == 0 and counts.size == 19
    assert tuple(counts[1:10]) == TABLE4_U
    assert tuple(counts[10:19]) == TABLE4_D
    assert sum(TABLE4_U) + sum(TABLE4_D) == 8386
    x, sign = legs["x"][ins], legs["sign"][ins]
    assert tuple(np.bincount(x[sign == 1], minlength=10)[1:]) == TABLE4_U
    assert tuple(np.bincount(x[sign == 2], minlength=10)[1:]) == TABLE4_D


# ---- Reference-held pin of the Tayal forward (A2/A6/A7/A12 with the Q6 mask) -------------------
#
# Table 4 of main.pdf (main.Rmd:704-723) is table(x.ins, state.filtered.ins), where
# state.filtered.ins is the per-t which.max of the median over draws of hhmm-tayal2009-lite's
# alpha_tk (main.Rmd:436, 596-602).  Rows = bottom states 1..4, columns = U1..U9, D1..D9.
TABLE4 = np.array([
    [0, 15, 0, 810, 0, 828, 33, 0, 17, 0, 0, 0, 0, 0, 0, 0, 0, 0],
    [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 72, 0, 0, 2208, 0, 181, 0, 59],
    [0, 0, 0, 0, 0, 0, 0, 27, 0, 15, 0, 34, 831, 0, 846, 0, 16, 0],
    [58, 0, 158, 0, 2155, 0, 0, 22, 0, 0, 0, 0, 0, 1, 0, 0, 0, 0]])

# Table 8 of main.pdf (main.Rmd:869-907): posterior means of the same fit, printed to 2 decimals.
# p_1k = (.51, 0, .49, 0); A_ij: a12 .46, a13 .54, a21 1, a31 .09, a34 .91, a43 1.
TABLE8_P11 = 0.51
TABLE8_A_ROW = ((0.46, 0.54), (0.09, 0.91))
TABLE8_PHI = np.array([
    [.01, .02, .01, .34, .22, .35, .03, .01, .02],
    [.00, .02, .00, .05, .80, .02, .08, .00, .02],
    [.01, .00, .03, .36, .20, .39, .00, .02, .00],
    [.02, .00, .06, .02, .88, .01, .00, .01, .00]])
# A printed 0.00 is a simplex entry below 0.005, never exactly 0 (simplex[L] phi_k, lite.stan:25);
# it is floored at the midpoint of [0, 0.005) and each row renormalised.
PHI_FLOOR = 0.0025


def table8_draw():
    phi = np.where(TABLE8_PHI == 0.0, PHI_FLOOR, TABLE8_PHI)
    phi = phi / phi.sum(axis=1, keepdims=True)
    return {"p_11": np.array([TABLE8_P11]), "A_row": np.array([TABLE8_A_ROW]), "phi_k": phi[None]}


def table8_flat(draw):
    """hhmm-tayal2009-lite.stan:34-48: the transformed-parameters expansion."""
    p11, (r1, r2) = draw["p_11"][0], draw["A_row"][0]
    p_1k = np.array([[p11, 0.0, 1.0 - p11, 0.0]])
    A = np.zeros((1, 4, 4))
    A[0, 0, 1], A[0, 0, 2], A[0, 1, 0], A[0, 2, 0], A[0, 2, 3], A[0, 3, 2] = r1[0], r1[1], 1, r2[0], r2[1], 1
    return p_1k, A


def tabulate(feature, state):
    """table(x.ins, state) laid out like Table 4: [state, feature]."""
    t = np.zeros((4, 18), dtype=np.int64)
    np.add.at(t, (state - 1, feature - 1), 1)
    return t


def table_agreement(got):
    """Observations whose (feature, state) cell is shared with Table 4: sum of cell-wise minima."""
    return int(np.minimum(got, TABLE4).sum())


def _gto_legs(oracle):
    from hhmm_amd import features as F
    files = [DATA / "G.TO" / f"{d}.G.TO.RData" for d in RMD_DAYS]
    price, size, time = rdata.load_ticks(files)
    legs = oracle.extract_features(price, size, time, alpha=0.25)
    when = time[F.index_ticks(legs, price)]
    return legs, F.xts_window(when, RMD_INS), F.xts_window(when, RMD_OOS)


@pytest.mark.skipif(not DATA.exists(), reason="reference tick data not present (GPU box)")
def test_tayal_forward_reproduces_report_table4(oracle):
    """Pins the oracle's Tayal forward to the reference's own output.  The report's chain on
    CPU: six G.TO files -> extract_features -> in-sample / OOS windows (main.Rmd:405-446) ->
    hhmm-tayal2009-lite at Table 8's posterior means -> which.max(alpha_tk) per t, tabulated
    against the 18 features.  A point estimate stands in for the median over 250 draws, so a
    few observations near a decision boundary may move (U6, U8); every other cell must agree,
    including the Q6-mask cells where up legs go to the bear state 1 (U2/U4/U6/U7/U9) and the
    single D5 observation in state 4."""
    legs, ins, oos = _gto_legs(oracle)
    feat, x, sign = legs["feature"][ins], legs["x"][ins], legs["sign"][ins]
    assert feat.size == 8386 and np.array_equal(feat, np.where(sign == 1, x, x + 9))
    data = {"K": 4, "L": 9, "x": x, "sign": sign, "x_oos": legs["x"][oos], "sign_oos": legs["sign"][oos]}
    draw = table8_draw()
    out = oracle.gqs("hhmm-tayal2009-lite", data, draw, pars=["alpha_tk", "alpha_tk_oos", "zstar_t"])
    got = tabulate(feat, np.argmax(out["alpha_tk"][0], axis=1) + 1)
    assert got.sum() == 8386
    agree = table_agreement(got)
    assert agree >= 8350, (agree, got)
    # the 16 features other than U6 and U8 land exactly where the report put them
    exact = [c for c in range(18) if c not in (5, 7)]
    assert np.array_equal(got[:, exact], TABLE4[:, exact]), got
    assert got[1, 13] == 2208 and got[3, 13] == 1  # D5: 2208 in state 2, one in state 4
    assert got[0, 5] + got[2, 5] == 828 and got[0, 5] >= 800  # U6 mostly in state 1, as the report
    assert got[2, 7] + got[3, 7] == 49  # U8 split between states 3 and 4, as the report
    print(f"Table 4 agreement {agree} / 8386; U6 {got[:, 5]}, U8 {got[:, 7]}")

    # The check discriminates: without the sign mask (the transition applied for every j and the
    # initial distribution for every j, i.e. the plain multinomial HMM of hmm-multinom.stan at the
    # same expanded parameters) the table falls apart.
    p_1k, A = table8_flat(draw)
    plain = oracle.gqs("hmm-multinom", {"K": 4, "L": 9, "x": x},
                       {"p_1k": p_1k, "A_ij": A, "phi_k": draw["phi_k"]}, pars=["alpha_tk"])
    nomask = table_agreement(tabulate(feat, np.argmax(plain["alpha_tk"][0], axis=1) + 1))
    print(f"no-mask agreement {nomask} / 8386")
    assert nomask < 5000, nomask


@pytest.mark.skipif(not DATA.exists(), reason="reference tick data not present (GPU box)")
def test_table4_point_oracle_vs_numpy_transcription(oracle):
    """The same real-data request through the independent pure-Python transcription
    (tests/oracle_numpy.py): every in-sample and OOS output of the lite model agrees with the
    C oracle, so the Table 4 pin above covers both restatements."""
    import oracle_numpy as onp
    from tolerances import compare
    legs, ins, oos = _gto_legs(oracle)
    x, sign, xo, so = legs["x"][ins], legs["sign"][ins], legs["x"][oos], legs["sign"][oos]
    data = {"K": 4, "L": 9, "x": x, "sign": sign, "x_oos": xo, "sign_oos": so}
    draw = table8_draw()
    pars = ["loglik", "unalpha_tk", "alpha_tk", "unalpha_tk_oos", "alpha_tk_oos", "zstar_t", "logp_zstar"]
    got = oracle.gqs("hhmm-tayal2009-lite", data, draw, pars=pars)
    ref = onp.tayal_lite(x.size, x, sign, xo.size, xo, so, draw["p_11"][0], draw["A_row"][0], draw["phi_k"][0])
    for name in pars:
        compare(name, np.asarray(got[name])[0], np.asarray(ref[name]))
