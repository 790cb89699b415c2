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
