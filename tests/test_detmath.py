"""CPU: the FFBS contract's deterministic exp / log (gsoc17-hhmm_amd/csrc/hhmm_detmath.h).

The oracle's C functions (the ones the device compiles from the same header)
against the independent Python restatement in tests/ffbs_contract.py, bit for
bit, and their accuracy against the correctly rounded functions (a few ulp:
the float outputs computed from them carry a 1e-9 tolerance).
"""
import math

import numpy as np

import ffbs_contract as fc


def _args_exp():
    g = np.random.Generator(np.random.Philox(21))
    return np.concatenate([(g.random(3000) - 0.5) * 1500.0, (g.random(3000) - 0.5) * 40.0,
                           -g.random(2000) * 30.0, (g.random(500) - 0.5) * 1e-9,
                           np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 709.78, 709.79, 710.0, 711.0,
                                     -708.39, -708.4, -745.13, -745.14, -746.0, -747.0, 5e-324, -5e-324,
                                     -744.4400719213812, -1022 * math.log(2), 1022 * math.log(2)])])


def _args_log():
    g = np.random.Generator(np.random.Philox(22))
    bits = g.integers(1, 0x7FF0000000000000, size=3000, dtype=np.int64).view(np.float64)
    return np.concatenate([bits, 1.0 + (g.random(2000) - 0.5) * 2.0 ** -6, g.random(2000),
                           np.array([1.0, 2.0, 0.5, 0.0, -0.0, -1.0, np.inf, -np.inf, np.nan, 5e-324,
                                     2.2250738585072014e-308, 1.7976931348623157e308, 1 - 2 ** -53, 1 + 2 ** -52,
                                     math.sqrt(2), np.nextafter(math.sqrt(2), 2), np.nextafter(math.sqrt(2), 0)])])


def _same(a, b):
    return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))


def test_det_exp_oracle_matches_python_restatement(oracle):
    x = _args_exp()
    got = oracle.det_array("exp", x)
    want = np.array([fc.det_exp(float(v)) for v in x])
    same = _same(got, want)
    assert same.all(), x[~same][:5]


def test_det_exp_subnormal_and_overflow_edges(oracle):
    """The result's scaling by 2^k (ldexp in hhmm_detmath.h) against the
    restatement's two exact power-of-two factors, densely where it matters:
    the subnormal results (x in [-746, -708]) and the overflow edge."""
    g = np.random.Generator(np.random.Philox(23))
    x = np.concatenate([-708.0 - g.random(20000) * 38.0, 700.0 + g.random(4000) * 11.0])
    got = oracle.det_array("exp", x)
    want = np.array([fc.det_exp(float(v)) for v in x])
    same = _same(got, want)
    assert same.all(), x[~same][:5]


def test_det_log_oracle_matches_python_restatement(oracle):
    x = _args_log()
    got = oracle.det_array("log", x)
    want = np.array([fc.det_log(float(v)) for v in x])
    same = _same(got, want)
    assert same.all(), x[~same][:5]


def test_det_accuracy_against_correctly_rounded(oracle):
    for which, x, ref in (("exp", _args_exp(), oracle.exp_array), ("log", _args_log(), oracle.log_array)):
        got = oracle.det_array(which, x)
        cr = ref(x, "cr")
        fin = np.isfinite(cr) & (cr != 0)
        # specials identical
        assert _same(got[~fin & ~np.isnan(cr)], cr[~fin & ~np.isnan(cr)]).all(), which
        assert np.isnan(got[np.isnan(cr)]).all(), which
        normal = fin & (np.abs(cr) > 1e-300)
        ulp = np.abs(got[normal] - cr[normal]) / np.spacing(np.abs(cr[normal]))
        assert ulp.max() <= 4, (which, ulp.max())
