"""GPU parity: libhhmm.so (gfx950) against the CPU oracle on identical inputs.

Posteriors / log-likelihoods within the tolerances of tests/tolerances.py;
Viterbi paths, logp_zstar and pair_status bit-exact (the oracle and the
device share the correctly rounded log and the reference's operation order).
"""
import numpy as np
import pytest

from hhmm_amd import _abi, synth
from tolerances import compare, compare_all

pytestmark = pytest.mark.gpu

DEVICE_MODELS = ["hmm", "hmm-multinom", "hmm-multinom-semisup", "hhmm-tayal2009", "hhmm-tayal2009-lite",
                 "iohmm-reg", "iohmm-mix", "iohmm-hmix", "iohmm-hmix-lite"]

# the hot-path outputs of each program (what a batch caller asks for)
HOT_PARS = {m: ["loglik", "gamma_tk", "zstar_t", "logp_zstar"] for m in DEVICE_MODELS}
HOT_PARS["hhmm-tayal2009-lite"] = ["loglik", "alpha_tk", "alpha_tk_oos", "zstar_t", "logp_zstar"]
HOT_PARS["iohmm-hmix"] = ["loglik", "gamma_tk", "oblik_t", "zstar_t", "logp_zstar"]
HOT_PARS["iohmm-hmix-lite"] = ["loglik", "unalpha_tk", "oblik_t"]


def run_both(engine, oracle, model, data, draws, pars, pairing="grid"):
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, pairing=pairing, lib=engine, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, pairing=pairing, return_status=True)
    return got, ref


def test_cr_log_device_matches_oracle(engine, oracle):
    import ctypes as C
    g = np.random.Generator(np.random.Philox(7))
    bits = g.integers(1, 0x7FF0000000000000, size=200_000, dtype=np.int64).view(np.float64)
    near1 = 1.0 + (g.random(100_000) - 0.5) * 2.0 ** -6
    small = g.random(100_000)
    special = np.array([1.0, 2.0, 0.5, 0.0, -1.0, np.inf, np.nan, 5e-324, 2.2250738585072014e-308,
                        1.7976931348623157e308, 1 - 2 ** -53, 1 + 2 ** -52])
    x = np.concatenate([bits, near1, small, special])
    y = np.empty_like(x)
    st = engine.hhmm_selftest_cr_log(x.ctypes.data_as(C.POINTER(C.c_double)),
                                     y.ctypes.data_as(C.POINTER(C.c_double)), x.size)
    assert st == 0, engine.hhmm_last_error()
    ref = oracle.log_array(x, "cr")
    same = (y.view(np.int64) == ref.view(np.int64)) | (np.isnan(y) & np.isnan(ref))
    assert same.all(), f"{(~same).sum()} device logs differ from the oracle's"


def test_cr_exp_device_matches_oracle(engine, oracle):
    """Device exp (quick phase + accurate fallback) bit-identical to the
    oracle's, across the normal, subnormal-result and overflow ranges."""
    import ctypes as C
    g = np.random.Generator(np.random.Philox(8))
    wide = (g.random(200_000) - 0.5) * 1500.0
    small = (g.random(100_000) - 0.5) * 40.0
    neg = -g.random(100_000) * 30.0
    tiny = (g.random(50_000) - 0.5) * 1e-9
    special = np.array([0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, 709.78, 709.79, -708.39, -708.4,
                        -745.13, -745.14, -707.0, 693.0, 5e-324, -5e-324])
    x = np.concatenate([wide, small, neg, tiny, special])
    y = np.empty_like(x)
    st = engine.hhmm_selftest_cr_exp(x.ctypes.data_as(C.POINTER(C.c_double)),
                                     y.ctypes.data_as(C.POINTER(C.c_double)), x.size)
    assert st == 0, engine.hhmm_last_error()
    ref = oracle.exp_array(x, "cr")
    same = (y.view(np.int64) == ref.view(np.int64)) | (np.isnan(y) & np.isnan(ref))
    assert same.all(), f"{(~same).sum()} device exps differ from the oracle's"


@pytest.mark.parametrize("which", ["log", "exp"])
def test_det_math_device_matches_oracle(engine, oracle, which):
    """The FFBS contract's deterministic exp / log (hhmm_detmath.h): the device
    compilation bit-identical to the oracle's."""
    import ctypes as C
    from test_detmath import _args_exp, _args_log
    g = np.random.Generator(np.random.Philox(9))
    if which == "exp":
        x = np.concatenate([_args_exp(), (g.random(300_000) - 0.5) * 1500.0, (g.random(100_000) - 0.5) * 40.0])
        fn = engine.hhmm_selftest_det_exp
    else:
        x = np.concatenate([_args_log(), g.integers(1, 0x7FF0000000000000, size=300_000,
                                                    dtype=np.int64).view(np.float64), g.random(100_000)])
        fn = engine.hhmm_selftest_det_log
    y = np.empty_like(x)
    st = fn(x.ctypes.data_as(C.POINTER(C.c_double)), y.ctypes.data_as(C.POINTER(C.c_double)), x.size)
    assert st == 0, engine.hhmm_last_error()
    ref = oracle.det_array(which, x)
    same = (y.view(np.int64) == ref.view(np.int64)) | (np.isnan(y) & np.isnan(ref))
    assert same.all(), f"{(~same).sum()} device det_{which} differ from the oracle's"


CASES = [
    ("hmm", dict(K=1)), ("hmm", dict(K=2)), ("hmm", dict(K=3)), ("hmm", dict(K=4)), ("hmm", dict(K=6)),
    ("hmm-multinom", dict(K=1, L=3)), ("hmm-multinom", dict(K=2, L=5)), ("hmm-multinom", dict(K=3, L=5)),
    ("hmm-multinom", dict(K=4, L=9)), ("hmm-multinom", dict(K=5, L=7)), ("hmm-multinom", dict(K=8, L=9)),
    ("hmm-multinom-semisup", dict(K=4, L=9)), ("hhmm-tayal2009", dict()), ("hhmm-tayal2009-lite", dict()),
    ("iohmm-reg", dict(K=1, M=1)), ("iohmm-reg", dict(K=2, M=3)), ("iohmm-reg", dict(K=3, M=4)),
    ("iohmm-reg", dict(K=4, M=4)), ("iohmm-reg", dict(K=6, M=7)),
    ("iohmm-mix", dict(K=4, L=3, M=4)), ("iohmm-mix", dict(K=3, L=1, M=2)), ("iohmm-mix", dict(K=5, L=6, M=8)),
    ("iohmm-hmix", dict(K=4, L=3, M=4)), ("iohmm-hmix", dict(K=2, L=2, M=5)),
    ("iohmm-hmix-lite", dict(K=4, L=3, M=4)),
]


@pytest.mark.parametrize("model,kw", CASES, ids=[f"{m}-{'-'.join(f'{k}{v}' for k, v in kw.items())}"
                                                 for m, kw in CASES])
@pytest.mark.parametrize("T", [1, 2, 37, 130])
def test_parity_grid(engine, oracle, model, kw, T):
    data, draws = synth.GENERATORS[model](N=3, S=70, T=T, **kw)
    got, ref = run_both(engine, oracle, model, data, draws, synth.PARS[model])
    compare_all(got, ref, synth.PARS[model] + ["pair_status"])
    assert got["status"] == ref["status"]


@pytest.mark.parametrize("model", DEVICE_MODELS)
def test_parity_zip_many_pairs(engine, oracle, model):
    N = 1000
    data, draws = synth.GENERATORS[model](N=N, S=N, T=64)
    pars = HOT_PARS[model]
    got, ref = run_both(engine, oracle, model, data, draws, pars, pairing="zip")
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("model", DEVICE_MODELS)
def test_parity_ragged(engine, oracle, model):
    N, S, T = 5, 64, 90
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T)
    data["T"] = np.array([90, 1, 17, 64, 33], dtype=np.int32)
    if "x_oos" in data:
        data["T_oos"] = np.array([3, 48, 1, 20, 47], dtype=np.int32)
    pars = synth.PARS[model]
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True)
    # entries past a series' length are not written by either side (NaN-prefilled)
    compare_all(got, ref, pars + ["pair_status"])


def test_invalid_backpointer_flagged(engine, oracle):
    """All delta_T = -inf (an impossible observation under every state):
    Stan would throw while backtracking; the pair is flagged, zstar zeroed."""
    data, draws = synth.hmm_multinom(N=1, S=4, T=12, K=3, L=4)
    draws["phi_k"][:, :, 3] = 0.0
    draws["phi_k"] /= draws["phi_k"].sum(axis=2, keepdims=True)
    data["x"][0, 7] = 4
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    got, ref = run_both(engine, oracle, "hmm-multinom", data, draws, pars)
    assert (ref["pair_status"] == 1).all() and ref["status"] == 1
    compare_all(got, ref, pars + ["pair_status"])
    assert got["status"] == 1


def test_deterministic_emissions_recover_path(engine):
    """KAT (hmm/main-multinom-semisup.R:31-35: B = identity rows): with
    noise-free emissions the Viterbi path is the observed symbol sequence,
    except zstar[1] = K from the Q3 initialisation quirk."""
    import hhmm_amd
    K, L, T = 4, 4, 50
    g = np.random.Generator(np.random.Philox(3))
    z = g.integers(1, K + 1, size=T)
    z[0] = K  # otherwise delta_1 = (NaN, .., log 0): every path is -inf and Stan throws
    data = {"K": K, "L": L, "x": z.reshape(1, T)}
    draws = {"p_1k": np.full((1, K), 0.25), "A_ij": np.full((1, K, K), 0.25),
             "phi_k": np.eye(K).reshape(1, K, L)}
    out = hhmm_amd.gqs("hmm-multinom", data, draws, pars=["zstar_t"], lib=engine)
    path = out["zstar_t"][0]
    assert path[0] == K
    assert np.array_equal(path[1:], z[1:])


FFBS_MODELS = ["hmm", "hmm-multinom", "hmm-multinom-semisup", "hhmm-tayal2009", "iohmm-reg", "iohmm-mix",
               "iohmm-hmix"]


@pytest.mark.parametrize("model", FFBS_MODELS)
@pytest.mark.parametrize("T", [1, 2, 37, 130])
def test_ffbs_parity(engine, oracle, model, T):
    """FFBS draws bit-exact with the oracle's contract given the same uniforms,
    requested alone and together with every other output."""
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=3, S=70, T=T)
    uu = synth.ffbs_uniforms(210, T, seed=T)
    for pars in (["z_ffbs"], synth.PARS[model] + ["z_ffbs"]):
        got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, uniforms=uu, return_status=True)
        ref = oracle.gqs(model, data, draws, pars=pars, uniforms=uu, return_status=True)
        compare_all(got, ref, pars)


@pytest.mark.parametrize("model", ["hmm-multinom", "hhmm-tayal2009", "iohmm-hmix"])
def test_ffbs_parity_ragged(engine, oracle, model):
    import hhmm_amd
    N, S, T = 5, 64, 90
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T)
    data["T"] = np.array([90, 1, 17, 64, 33], dtype=np.int32)
    uu = synth.ffbs_uniforms(N * S, T, seed=4)
    pars = ["z_ffbs", "gamma_tk", "loglik"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, uniforms=uu)
    ref = oracle.gqs(model, data, draws, pars=pars, uniforms=uu)
    compare_all(got, ref, pars)


@pytest.mark.parametrize("model", DEVICE_MODELS)
def test_parity_long_full_profile(engine, oracle, model):
    """Every declared output at T = 1000: log-scale outputs (unalpha / unbeta)
    of states far below the others stay finite, as in Stan's log space."""
    data, draws = synth.GENERATORS[model](N=2, S=40, T=1000)
    got, ref = run_both(engine, oracle, model, data, draws, synth.PARS[model])
    compare_all(got, ref, synth.PARS[model] + ["pair_status"])


VIT_CASES = [("hmm", dict(K=2)), ("hmm", dict(K=3)), ("hmm", dict(K=4)), ("hmm-multinom", dict(K=2, L=5)),
             ("hmm-multinom", dict(K=3, L=5)), ("hmm-multinom", dict(K=4, L=9)),
             ("hmm-multinom-semisup", dict(K=4, L=9)), ("hhmm-tayal2009", dict()),
             ("hhmm-tayal2009-lite", dict())]


@pytest.mark.parametrize("layout", ["lanes", "states"])
@pytest.mark.parametrize("model,kw", VIT_CASES, ids=[f"{m}-{'-'.join(f'{k}{v}' for k, v in kw.items())}"
                                                     for m, kw in VIT_CASES])
@pytest.mark.parametrize("T", [1, 2, 37, 1000])
def test_viterbi_layouts_match_oracle(engine, oracle, model, kw, T, layout):
    """Both Viterbi decoders -- one lane per pair and one lane per (pair,
    state) -- are bit-exact with the oracle (paths, logp_zstar, status)."""
    import hhmm_amd
    flags = _abi.FLAG_VIT_LANES if layout == "lanes" else _abi.FLAG_VIT_STATES
    data, draws = synth.GENERATORS[model](N=3, S=30, T=T, **kw)
    pars = ["zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=flags, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("layout", ["lanes", "states"])
@pytest.mark.parametrize("model", ["hmm", "hmm-multinom", "hhmm-tayal2009"])
def test_viterbi_layouts_ragged(engine, oracle, model, layout):
    import hhmm_amd
    flags = _abi.FLAG_VIT_LANES if layout == "lanes" else _abi.FLAG_VIT_STATES
    N, S, T = 5, 13, 90
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T)
    data["T"] = np.array([90, 1, 17, 64, 33], dtype=np.int32)
    pars = ["zstar_t", "logp_zstar", "loglik"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=flags, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("sched", ["split", "vfb"])
@pytest.mark.parametrize("T", [1, 2, 9, 37, 130])
def test_split_schedule(engine, oracle, T, sched):
    """HHMM_FLAG_FB_SPLIT (hmm-multinom K = 4, gamma + path in one request):
    the forward launch packs the symbols, the Viterbi decodes them beside the
    backward launch -- bit-exact paths, gamma / loglik within tolerance, at
    series lengths around the 8-step chunk and 16-step block sizes.  `vfb`:
    the phased sweep (HHMM_FLAG_VFB), whose Viterbi packs the symbols its
    forward-backward reads."""
    import hhmm_amd
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    data, draws = synth.hmm_multinom(N=70, S=70, T=T, K=4, L=9)
    flags = _abi.FLAG_VIT_LANES | (_abi.FLAG_FB_SPLIT if sched == "split" else _abi.FLAG_VFB)
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=flags, pairing="zip",
                       return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("scale", [1.0, 8.0, 40.0, 400.0])
@pytest.mark.parametrize("model", ["iohmm-reg", "iohmm-hmix"])
def test_viterbi_log_softmax_regimes(engine, oracle, model, scale):
    """The Viterbi's log A_t(i) -- the correctly rounded log of each softmax
    output (and, in a -DHHMM_IO_ONELOG=1 build, derived from the softmax's own
    exps and one log of the sum: softmax_cr_log) -- bit-exact with the oracle
    from mild transitions (scale 1) to saturated ones where one state takes
    A = 1 - tiny (sum == 1, A within 2^-18 of 1) and the others underflow
    toward the exp's accurate phase."""
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=3, S=50, T=120, K=4, M=4)
    draws["w_km"] = draws["w_km"] * scale
    pars = ["zstar_t", "logp_zstar", "loglik"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


def _near_impossible_runs(tiny, K=4, N=192, which=(70,)):
    """hmm-multinom, zip pairing: the pairs in `which` emit symbol 9 with
    probability `tiny` under every state (others keep their Dirichlet draw),
    and every series holds a run of 40 nines -- so the waves of those pairs
    shrink the filter by ~tiny per step while the other waves do not."""
    data, draws = synth.hmm_multinom(N=N, S=N, T=200, K=K, L=9)
    phi = np.array(draws["phi_k"], dtype=np.float64)
    for p in which:
        phi[p, :, 8] = tiny
    phi /= phi.sum(axis=2, keepdims=True)
    draws["phi_k"] = phi
    x = np.array(data["x"])
    x[:, 60:100] = 9
    data["x"] = x
    return data, draws


@pytest.mark.parametrize("tiny", [1e-30, 1e-70, 1e-90, 1e-200])
@pytest.mark.parametrize("flags", [_abi.FLAG_VIT_LANES, _abi.FLAG_VIT_LANES | _abi.FLAG_FUSED,
                                   _abi.FLAG_VIT_LANES | _abi.FLAG_FB_SPLIT, _abi.FLAG_VIT_LANES | _abi.FLAG_VFB],
                         ids=["default", "fused", "split", "vfb"])
def test_gamma_profile_near_impossible_runs(engine, oracle, tiny, flags):
    """The gamma profile renormalises every 4 steps (FB_BIG, kBigRenorm) only
    in waves whose pairs bound the 4-step shrink (renorm_sparse_safe: the
    smallest emission times the smallest row / column max of A >= 2^-39);
    a wave holding a pair with a symbol of probability 1e-90 or 1e-200 under
    every state renormalises every step, which keeps the filter normal down to
    ~1e-300 per step like the reference's log space.  Every schedule of the
    C2 request (the bench's lane decoder, the fused sweep, the split
    launches), against the oracle, with the safe and the dense waves in one
    batch."""
    import hhmm_amd
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    data, draws = _near_impossible_runs(tiny)
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, pairing="zip", flags=flags,
                       return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", return_status=True)
    compare_all(got, ref, pars + ["pair_status"])
    assert np.isfinite(got["loglik"]).all()


@pytest.mark.parametrize("tiny", [1e-70, 1e-90, 1e-200])
@pytest.mark.parametrize("K", [12, 23])
@pytest.mark.parametrize("pars", [["loglik", "gamma_tk", "zstar_t", "logp_zstar"],
                                  ["loglik", "alpha_tk", "beta_tk", "gamma_tk"]], ids=["gamma-only", "full"])
def test_large_K_near_impossible_runs(engine, oracle, tiny, K, pars):
    """The large-K filters' every-kLRenorm-steps cadence under the same
    bound (hhmm_large.h, kLRenormSafeBound): pairs 5 and 70 carry the tiny
    symbol, so their waves renormalise every step and the rest keep the
    cadence; the gamma-only request runs the one-group-sum gamma."""
    import hhmm_amd
    data, draws = _near_impossible_runs(tiny, K=K, N=96, which=(5, 70))
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, pairing="zip", return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", return_status=True, nthreads=8)
    compare_all(got, ref, pars + ["pair_status"])
    assert np.isfinite(got["loglik"]).all()


def test_unsupported_shape_leaves_no_kernel_running(engine, oracle):
    """hmm-multinom K = 4 with L = 100: the forward-backward's emission table
    (L * 4 doubles per lane) does not fit in LDS while the state-parallel
    decoder's would.  The request fails before either kernel is enqueued (no
    decoder left writing into buffers the call hands back), and the next
    request on the same device is still bit-exact with the oracle."""
    import hhmm_amd
    from hhmm_amd.api import HHMMError
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    data, draws = synth.hmm_multinom(N=3, S=40, T=200, K=4, L=100)
    with pytest.raises(HHMMError, match="does not fit"):
        hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine)
    data, draws = synth.hmm_multinom(N=3, S=40, T=200, K=4, L=9)
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("sched", ["split", "vfb"])
def test_split_schedule_ragged(engine, oracle, sched):
    """Ragged lengths inside one wave: a lane's packed rows past its own end
    are padding the decoder never consumes."""
    import hhmm_amd
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    N = 130
    data, draws = synth.hmm_multinom(N=N, S=N, T=300, K=4, L=9)
    data["T"] = np.random.default_rng(5).integers(1, 301, N).astype(np.int32)
    flags = _abi.FLAG_VIT_LANES | (_abi.FLAG_FB_SPLIT if sched == "split" else _abi.FLAG_VFB)
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=flags, pairing="zip",
                       return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("model", ["hmm-multinom", "hhmm-tayal2009"])
def test_viterbi_states_backtrack_groups(engine, oracle, model):
    """The state-parallel decoder's backtrack reads its back-pointer words in
    groups of 8 chunks x 16 steps: series lengths on both sides of one and two
    group boundaries (ragged within the wave) stay bit-exact with the oracle."""
    import hhmm_amd
    N, S, T = 6, 7, 257
    data, draws = synth.GENERATORS[model](N=N, S=S, T=T)
    data["T"] = np.array([127, 128, 129, 255, 256, 257], dtype=np.int32)
    pars = ["zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=_abi.FLAG_VIT_STATES, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, return_status=True)
    compare_all(got, ref, pars + ["pair_status"])


def test_vfb_invalid_backpointer(engine, oracle):
    """The phased sweep (HHMM_FLAG_VFB) on the all -inf delta_T pair: flagged,
    the path zeroed, gamma / loglik as the oracle; with a near-impossible
    symbol in another pair of the wave, so the wave takes the per-step
    renormalisation kernel (zstar_T parked in zstar[T-1])."""
    import hhmm_amd
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    data, draws = synth.hmm_multinom(N=3, S=3, T=40, K=4, L=9)
    draws["phi_k"][0, :, 8] = 0.0
    draws["phi_k"][2, :, 7] = 1e-200
    draws["phi_k"] /= draws["phi_k"].sum(axis=2, keepdims=True)
    data["x"][0, 7] = 9
    data["x"][2, 10:20] = 8
    for flags in (_abi.FLAG_VIT_LANES | _abi.FLAG_VFB,):
        got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=flags, pairing="zip",
                           return_status=True)
        ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", return_status=True)
        assert ref["pair_status"][0] == 1
        compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("layout", ["lanes", "states"])
def test_viterbi_layouts_invalid_backpointer(engine, oracle, layout):
    import hhmm_amd
    flags = _abi.FLAG_VIT_LANES if layout == "lanes" else _abi.FLAG_VIT_STATES
    data, draws = synth.hmm_multinom(N=1, S=4, T=12, K=3, L=4)
    draws["phi_k"][:, :, 3] = 0.0
    draws["phi_k"] /= draws["phi_k"].sum(axis=2, keepdims=True)
    data["x"][0, 7] = 4
    pars = ["zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, lib=engine, flags=flags, return_status=True)
    ref = oracle.gqs("hmm-multinom", data, draws, pars=pars, return_status=True)
    assert (ref["pair_status"] == 1).all()
    compare_all(got, ref, pars + ["pair_status"])


@pytest.mark.parametrize("model", ["hmm", "hhmm-tayal2009"])
def test_viterbi_layouts_agree_long(engine, model):
    """C5-like shape (few pairs, long T): the two decoders return identical
    paths and logp_zstar."""
    import hhmm_amd
    data, draws = synth.GENERATORS[model](N=2, S=150, T=50_000)
    pars = ["zstar_t", "logp_zstar"]
    a = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=_abi.FLAG_VIT_LANES)
    b = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, flags=_abi.FLAG_VIT_STATES)
    assert np.array_equal(a["zstar_t"], b["zstar_t"])
    assert np.array_equal(a["logp_zstar"].view(np.int64), b["logp_zstar"].view(np.int64))


@pytest.mark.parametrize("model", DEVICE_MODELS)
def test_parity_block_pairing(engine, oracle, model):
    """HHMM_PAIR_BLOCK: every series under its own block of draws (one fit per
    series, the walk-forward layout), ragged T."""
    N, B, T = 3, 20, 57
    data, draws = synth.GENERATORS[model](N=N, S=N * B, T=T)
    data["T"] = np.array([57, 1, 30], dtype=np.int32)
    if "x_oos" in data:
        data["T_oos"] = np.array([2, 48, 19], dtype=np.int32)
    pars = synth.PARS[model]
    import hhmm_amd
    got = hhmm_amd.gqs(model, data, draws, pars=pars, pairing="block", lib=engine, return_status=True)
    ref = oracle.gqs(model, data, draws, pars=pars, pairing="block", return_status=True)
    compare_all(got, ref, pars + ["pair_status"])
