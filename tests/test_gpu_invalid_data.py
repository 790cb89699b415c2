"""The device entry enforces the data block's bounds pair by pair.

Stan rejects a data block whose int arrays leave their declared bounds:
int<lower=1,upper=L> x[T] (hmm/stan/hmm-multinom.stan:11), int<lower=1,upper=2>
sign[T] (tayal2009/stan/hhmm-tayal2009.stan:11-12; -lite.stan:11-16 for the
out-of-sample arrays), int<lower=1,upper=G> g[T] (hmm-multinom-semisup.stan:7-14).
hhmm_run checks them on the host and rejects the request (tests/test_abi.py).
hhmm_run_device cannot read its device arrays on the host: it flags each pair
whose series breaks a bound with HHMM_PAIR_INVALID_DATA and computes every other
pair as usual.  Each case corrupts one value of one series (and one ragged length)
and checks (a) exactly that series' pairs are flagged, (b) every other pair matches
the oracle on the clean data (tests/tolerances.py)."""
import numpy as np
import pytest

from hhmm_amd import _abi, synth
from tolerances import compare

pytestmark = pytest.mark.gpu

INVALID_DATA = _abi.PAIR_INVALID_DATA


def _run(engine, oracle, model, data, bad_data, draws, pars, bad_series, pairing="grid", flags=0):
    from devrun import DeviceRequest
    r = DeviceRequest(engine, model, bad_data, draws, pars, pairing=pairing, flags=flags)
    r.run()
    status = r.status.cpu().numpy()
    N = np.asarray(data["x"]).shape[0]
    S = np.asarray(next(iter(draws.values()))).shape[0]
    pairs = np.arange(r.P)
    series = pairs // S if pairing == "grid" else pairs
    flagged = np.isin(series, bad_series)
    assert (status[flagged] == INVALID_DATA).all(), status[flagged]
    assert (status[~flagged] == 0).all(), np.flatnonzero(status[~flagged])
    ok = pairs[~flagged]
    ref = oracle.gqs(model, data, draws, pars=pars, pairing=pairing, return_status=True, nthreads=8)
    for name in pars:
        compare(name, r.host_pairs(name, ok), np.asarray(ref[name])[ok])
    assert N == len(np.unique(series)) or pairing != "grid"
    return status


def _corrupt(data, key, n, t, v):
    bad = dict(data)
    a = np.array(data[key], copy=True)
    a[n, t] = v
    bad[key] = a
    return bad


C2_PARS = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]


@pytest.mark.parametrize("flags", [0, _abi.FLAG_VFB_OFF], ids=["phased-sweep", "two-kernels"])
def test_multinom_symbol_out_of_range(engine, oracle, flags):
    """C2's profile: the phased sweep checks x while it packs the symbols; with it off,
    the separate check pass does."""
    data, draws = synth.hmm_multinom(N=512, S=512, T=200, K=4, L=9)
    bad = _corrupt(data, "x", 37, 101, 10)       # L + 1
    bad = _corrupt(bad, "x", 200, 0, 0)          # below 1
    bad = _corrupt(bad, "x", 311, 199, -7)
    _run(engine, oracle, "hmm-multinom", data, bad, draws, C2_PARS, [37, 200, 311], pairing="zip", flags=flags)


def test_multinom_grid_ragged_length(engine, oracle):
    """GRID pairing: every draw of the broken series is flagged; a T[n] past T_max too.
    A step past a series' own length is padding and is not checked."""
    data, draws = synth.hmm_multinom(N=6, S=64, T=300, K=4, L=9)
    T = np.array([300, 250, 300, 120, 300, 300], dtype=np.int32)
    data = dict(data, T=T)
    bad = dict(data, T=T.copy())
    bad["T"][4] = 301
    bad = _corrupt(bad, "x", 1, 20, 99)
    bad = _corrupt(bad, "x", 3, 200, 0)          # t >= T[3]: padding, not a violation
    _run(engine, oracle, "hmm-multinom", data, bad, draws, ["loglik", "gamma_tk", "zstar_t"], [1, 4])


def test_semisup_group_out_of_range(engine, oracle):
    data, draws = synth.hmm_multinom_semisup(N=8, S=32, T=150)
    bad = _corrupt(data, "g", 5, 77, 3)          # G + 1
    _run(engine, oracle, "hmm-multinom-semisup", data, bad, draws, ["loglik", "gamma_tk", "zstar_t"], [5])


def test_tayal_sign_out_of_range(engine, oracle):
    data, draws = synth.tayal(N=4, S=32, T=400)
    bad = _corrupt(data, "sign", 2, 399, 0)
    bad = _corrupt(bad, "x", 0, 3, 12)
    _run(engine, oracle, "hhmm-tayal2009", data, bad, draws, ["loglik", "gamma_tk", "zstar_t"], [0, 2])


def test_tayal_lite_out_of_sample(engine, oracle):
    data, draws = synth.tayal(N=4, S=16, T=300, T_oos=120)
    bad = _corrupt(data, "sign_oos", 1, 50, 3)
    bad = _corrupt(bad, "x_oos", 3, 0, 10)
    _run(engine, oracle, "hhmm-tayal2009-lite", data, bad, draws,
         ["loglik", "alpha_tk", "alpha_tk_oos", "zstar_t"], [1, 3])


def test_tayal_long_series_scan(engine, oracle):
    """One series under many draws, long T: the T-scan and the V-scan (C5's dispatch)."""
    data, draws = synth.tayal(N=2, S=8, T=40_000)
    bad = _corrupt(data, "x", 1, 39_999, 0)
    # alpha / beta, not gamma: past t ~ 2000 the Q6 masks underflow gamma's overlap to
    # NaN at the subnormal edge (tests/test_gpu_configs.py compare_tayal_gamma)
    _run(engine, oracle, "hhmm-tayal2009", data, bad, draws, ["loglik", "alpha_tk", "beta_tk", "zstar_t"], [1])


def test_large_k_symbol_out_of_range(engine, oracle):
    data, draws = synth.hmm_multinom(N=6, S=16, T=200, K=12, L=9)
    bad = _corrupt(data, "x", 2, 150, 10)
    _run(engine, oracle, "hmm-multinom", data, bad, draws, ["loglik", "gamma_tk", "zstar_t"], [2])


_LANES = _abi.FLAG_SCAN_OFF | _abi.FLAG_VIT_SCAN_OFF | _abi.FLAG_VIT_LANES
SCHEDULES = [
    # (id, outputs, flags): which kernels read x, hence which check runs
    ("fb", ["loglik", "gamma_tk"], _LANES),                         # fb_kernel, inline
    ("forward", ["loglik"], _LANES),                                # fb_kernel forward only, inline
    ("alpha-beta", ["alpha_tk", "beta_tk"], _LANES),                # fb_kernel FB_FULL, inline
    ("log-space", ["unalpha_tk"], _LANES),                          # fb_log_kernel: check pass
    ("viterbi", ["zstar_t", "logp_zstar"], _LANES),                 # viterbi_kernel, inline
    ("viterbi-states", ["zstar_t"], _abi.FLAG_VIT_STATES),          # viterbi_sp_kernel: check pass
    ("two", C2_PARS, _LANES | _abi.FLAG_VFB_OFF),                   # both inline, two streams
    ("split", C2_PARS, _LANES | _abi.FLAG_FB_SPLIT),                # forward launch inline
    ("fused", C2_PARS, _LANES | _abi.FLAG_FUSED),                   # fbv_kernel: check pass
    ("scan", ["loglik", "gamma_tk"], _abi.FLAG_SCAN_FORCE),         # T-scan: check pass
]


@pytest.mark.parametrize("outs,flags", [s[1:] for s in SCHEDULES], ids=[s[0] for s in SCHEDULES])
def test_multinom_schedules_ragged(engine, oracle, outs, flags):
    """Every schedule of the hmm-multinom request flags the same series: the sweeps
    that read x over whole series check it inline (fb_sweep, viterbi_block, the phased
    sweep), the others leave it to data_check_kernel.  Ragged lengths put violations
    in a wave's full chunks, in its partial chunks, and in the padding past a
    series' own length (not a violation)."""
    N, T = 300, 203
    data, draws = synth.hmm_multinom(N=N, S=N, T=T, K=4, L=9, seed=11)
    rng = np.random.default_rng(5)
    Tn = rng.integers(150, T + 1, size=N).astype(np.int32)
    Tn[17] = 161
    Tn[29] = 170
    data = dict(data, T=Tn)
    bad = dict(data, T=Tn.copy())
    bad["T"][60] = T + 1                          # length past T_max
    bad = _corrupt(bad, "x", 5, 3, 10)            # a full chunk (every lane's steps valid)
    bad = _corrupt(bad, "x", 17, 160, 0)          # the series' last step (a partial chunk)
    bad = _corrupt(bad, "x", 29, 170, 0)          # t = T[29]: padding, not a violation
    bad = _corrupt(bad, "x", 41, 100, -3)
    bad = _corrupt(bad, "x", 299, 149, 12)        # the last pair (the final wave's padded lanes)
    _run(engine, oracle, "hmm-multinom", data, bad, draws, outs, [5, 17, 41, 60, 299], pairing="zip", flags=flags)


def test_multinom_check_past_grid_y_limit(engine, oracle):
    """T_max above 65535 strips of 64 steps (4,194,240) -- the check
    kernel caps grid.y and loops over strips, so the launch still succeeds and a bad
    symbol past the cap is found (the long series runs the parallel scan over T)."""
    T = 4_300_000
    data, draws = synth.hmm_multinom(N=2, S=1, T=64, K=4, L=9)
    data = dict(data, x=np.random.default_rng(11).integers(1, 10, size=(2, T)).astype(np.int32))
    bad = _corrupt(data, "x", 1, 4_250_000, 10)   # in the strips past the cap
    from devrun import DeviceRequest
    got = DeviceRequest(engine, "hmm-multinom", bad, draws, ["loglik"])
    got.run()
    clean = DeviceRequest(engine, "hmm-multinom", data, draws, ["loglik"])
    clean.run()
    assert list(got.status.cpu().numpy()) == [0, INVALID_DATA]
    assert list(clean.status.cpu().numpy()) == [0, 0]
    # the clean series' pair is computed as usual (the oracle's 77 s at this T is
    # spared: the same device path on the clean data is the reference here)
    assert got.host_pairs("loglik", [0])[0] == clean.host_pairs("loglik", [0])[0]
    assert np.isfinite(clean.host_pairs("loglik", [0, 1])).all()
