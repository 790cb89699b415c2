"""Walk-forward batch assembly (tayal2009/test-strategy.R:45-59,
tayal2009/R/wf-trade.R:30-100): the reference's per-window Stan fits as one
ragged request with HHMM_PAIR_BLOCK pairing.

CPU: the task list, the per-window data (features -> in/out-of-sample legs ->
Tayal coding), and assemble/split checked with the oracle: the batched block
request equals every window evaluated on its own.  GPU: the engine's block
request against per-window oracle runs (windows built from synthetic ticks by
the GPU feature extractor).
"""
import pathlib

import numpy as np
import pytest

from hhmm_amd import features as F, synth, walkforward as W
from tolerances import compare_all

DATA = pathlib.Path("/root/reference/tayal2009/data")
PARS = ["loglik", "alpha_tk", "alpha_tk_oos", "zstar_t", "logp_zstar"]


def _windows(n, seed0=0, extract=None):
    """n synthetic windows: ticks -> legs -> in-sample span -> Tayal coding."""
    out = []
    for i in range(n):
        price, size, tm = F.synth_ticks(6000 + 997 * i, seed=seed0 + i)
        out.append(W.window_data(price, size, tm, "2007-05-01 09:30:00/2007-05-01 13:00:00", extract=extract))
    return out


def _draws(n, B):
    return [synth.GENERATORS["hhmm-tayal2009-lite"](N=1, S=B, T=4, seed=100 + i)[1] for i in range(n)]


def _per_window(oracle, windows, draws, pars):
    refs = []
    for w, d in zip(windows, draws):
        data = {"K": 4, "L": 9, "x": w["x"][None], "sign": w["sign"][None], "x_oos": w["x_oos"][None],
                "sign_oos": w["sign_oos"][None]}
        refs.append(oracle.gqs("hhmm-tayal2009-lite", data, d, pars=pars))
    return refs


def test_window_tasks_layout(tmp_path):
    for stock in ("A.TO", "B.TO"):
        (tmp_path / stock).mkdir()
        for day in range(1, 9):
            (tmp_path / stock / f"2007.05.{day:02d}.{stock}.RData").write_bytes(b"")
    (tmp_path / "LICENSE.md").write_text("")
    tasks = W.window_tasks(tmp_path)
    assert len(tasks) == 2 * (8 - 6 + 1)
    t0 = tasks[0]
    assert [f.name[:10] for f in t0["files"]] == [f"2007.05.0{d}" for d in range(1, 7)]
    assert t0["ins"] == "2007-05-01 09:30:00/2007-05-05 16:30:00"
    assert t0["oos"] == "2007-05-06 09:30:00/2007-05-06 16:30:00"


@pytest.mark.skipif(not DATA.exists(), reason="reference tick data not present (GPU box)")
def test_reference_task_list_has_204_windows(oracle):
    """12 stocks x (22 - 6 + 1) windows (test-strategy.R:45-59); the first
    task's in/out-of-sample data through the oracle's extractor."""
    tasks = W.window_tasks(DATA)
    assert len(tasks) == 204 and len({t["stock"] for t in tasks}) == 12
    w = W.load_window(tasks[0], extract=oracle.extract_features)
    assert w["x"].size > 1000 and w["x_oos"].size > 100
    for k in ("x", "x_oos"):
        assert w[k].min() >= 1 and w[k].max() <= 9
    for k in ("sign", "sign_oos"):
        assert set(np.unique(w[k])) <= {1, 2}


def test_window_data_split_and_coding(oracle):
    price, size, tm = F.synth_ticks(20000, seed=5)
    ins = "2007-05-01 09:30:00/2007-05-01 20:00:00"
    w = W.window_data(price, size, tm, ins, extract=oracle.extract_features)
    legs = oracle.extract_features(price, size, tm)
    when = tm[F.index_ticks(legs, price)]
    inside = np.flatnonzero(F.xts_window(when, ins))
    assert w["x"].size == inside.size and w["x_oos"].size == legs["feature"].size - inside[-1] - 1
    f = np.concatenate([w["x"] + 9 * (w["sign"] - 1), w["x_oos"] + 9 * (w["sign_oos"] - 1)])
    assert np.array_equal(f, legs["feature"][inside[0]:])


def test_block_request_equals_per_window_fits_oracle(oracle):
    windows = _windows(5, extract=oracle.extract_features)
    draws = _draws(5, 8)
    data, dr = W.assemble(windows, draws)
    got = oracle.gqs("hhmm-tayal2009-lite", data, dr, pars=PARS, pairing="block")
    per = W.split(got, data)
    refs = _per_window(oracle, windows, draws, PARS)
    for g, r in zip(per, refs):
        compare_all(g, r, PARS)


@pytest.mark.gpu
def test_block_request_engine_vs_per_window_oracle(engine, oracle):
    import hhmm_amd
    windows = _windows(12, seed0=40)  # legs from the GPU extractor
    draws = _draws(12, 16)
    data, dr = W.assemble(windows, draws)
    got = hhmm_amd.gqs("hhmm-tayal2009-lite", data, dr, pars=PARS, pairing="block", lib=engine)
    per = W.split(got, data)
    refs = _per_window(oracle, windows, draws, PARS)
    for g, r in zip(per, refs):
        compare_all(g, r, PARS)
