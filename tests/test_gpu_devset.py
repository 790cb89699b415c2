"""GPU: hhmm_run over the device set (HHMM_DEVICE_SET; SURVEY.md §8b device set
{GPU 0..7}, §8e contiguous series ranges, one host thread per GPU).

The box has one GPU, so the set repeats it (hhmm_init_devices({0, 0, 0})):
three shards run in three host threads, each uploading its slices of the
caller's arrays (2-D copies: series-, draw- and pair-fastest arrays), running
the sub-request and writing its slices of the outputs back.  Every output must
be bit-identical to the same request on one device -- the sub-requests run the
same kernels on the same pairs -- for every pairing, ragged lengths, the
per-pair inputs (FFBS uniforms, fitted-draw randomness), the IOHMM inputs
u [N, T, M] and the Tayal-lite out-of-sample arrays; a GRID request with fewer
series than shards splits its draws instead."""
import ctypes as C

import numpy as np
import pytest

from hhmm_amd import _abi, synth

pytestmark = pytest.mark.gpu


@pytest.fixture
def devset(engine):
    def use(ords):
        arr = (C.c_int32 * len(ords))(*ords)
        assert engine.hhmm_init_devices(arr, len(ords)) == 0, engine.hhmm_last_error().decode()
        got = (C.c_int32 * 8)()
        assert engine.hhmm_device_set(got, 8) == len(ords)
        assert list(got)[:len(ords)] == list(ords)
    yield use
    assert engine.hhmm_init(1) == 0


def _same(a, b, keys):
    for k in keys:
        x, y = np.asarray(a[k]), np.asarray(b[k])
        assert x.shape == y.shape, k
        assert np.array_equal(x, y, equal_nan=True), k


def _both(engine, model, data, draws, pars, **kw):
    import hhmm_amd
    one = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, device=0, return_status=True, **kw)
    many = hhmm_amd.gqs(model, data, draws, pars=pars, lib=engine, device=_abi.DEVICE_SET, return_status=True, **kw)
    _same(one, many, pars + ["pair_status"])
    assert one["status"] == many["status"]
    return one, many


@pytest.mark.parametrize("pairing", ["grid", "zip", "block"])
@pytest.mark.parametrize("shards", [2, 3])
def test_devset_hmm_family(engine, devset, pairing, shards):
    devset([0] * shards)
    N = 7
    S = {"grid": 5, "zip": 7, "block": 21}[pairing]
    data, draws = synth.hmm_multinom(N=N, S=S, T=130, K=4, L=9)
    data["T"] = np.random.default_rng(shards).integers(1, 131, N).astype(np.int32)
    P = {"grid": N * S, "zip": N, "block": S}[pairing]
    u = synth.ffbs_uniforms(P, 130)
    pars = ["loglik", "alpha_tk", "gamma_tk", "zstar_t", "logp_zstar", "z_ffbs"]
    _both(engine, "hmm-multinom", data, draws, pars, pairing=pairing, uniforms=u)


def test_devset_grid_splits_draws(engine, devset):
    """One series under 250 draws (C5's shape per GPU) over 3 shards: the
    draws are split, each shard's pairs are rows of S' at a pitch of S."""
    devset([0, 0, 0])
    data, draws = synth.GENERATORS["hhmm-tayal2009"](N=2, S=250, T=3000)
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]
    _both(engine, "hhmm-tayal2009", data, draws, pars)


def test_devset_iohmm_inputs_and_fitted_draws(engine, devset):
    devset([0, 0])
    N, S, T = 5, 6, 90
    data, draws = synth.iohmm_reg(N=N, S=S, T=T, K=4, M=4)
    data["T"] = np.array([90, 3, 57, 90, 1], dtype=np.int32)
    rng = np.random.default_rng(4)
    hr = rng.random((N * S, T, 3))
    pars = ["loglik", "gamma_tk", "zstar_t", "logp_zstar", "oblik_tk", "hatz_t", "hatx_t"]
    _both(engine, "iohmm-reg", data, draws, pars, hat_rand=hr)


def test_devset_tayal_lite_out_of_sample(engine, devset):
    devset([0, 0, 0])
    data, draws = synth.GENERATORS["hhmm-tayal2009-lite"](N=4, S=3, T=400)
    pars = ["loglik", "alpha_tk", "alpha_tk_oos", "zstar_t", "logp_zstar"]
    _both(engine, "hhmm-tayal2009-lite", data, draws, pars)


def test_devset_invalid_backpointer_status(engine, devset):
    """A flagged pair in the second shard: pair_status lands at its own index
    and the call returns the warning status, as on one device."""
    devset([0, 0])
    data, draws = synth.hmm_multinom(N=4, S=4, T=12, K=3, L=4)
    draws["phi_k"][:, :, 3] = 0.0
    draws["phi_k"] /= draws["phi_k"].sum(axis=2, keepdims=True)
    data["x"] = np.minimum(data["x"], 3)  # symbol 4 (probability 0 under every state) only in series 3
    data["x"][3, 7] = 4
    one, many = _both(engine, "hmm-multinom", data, draws, ["loglik", "zstar_t", "logp_zstar"], pairing="zip")
    assert many["status"] == 1 and many["pair_status"][3] == 1 and many["pair_status"][:3].sum() == 0


def test_devset_rejects_invisible_ordinal(engine):
    arr = (C.c_int32 * 2)(0, 64)
    assert engine.hhmm_init_devices(arr, 2) == _abi.ERR_NO_DEVICE
    assert b"not visible" in engine.hhmm_last_error()
    assert engine.hhmm_init(1) == 0
