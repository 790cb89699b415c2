"""CPU: the oracle reproduces the committed golden fixtures bit-for-bit
(tests/golden/make_golden.py documents how they were made and cross-checked)."""
import pathlib

import numpy as np
import pytest

from hhmm_amd import synth

GOLDEN = pathlib.Path(__file__).resolve().parent / "golden"
MODELS = sorted(p.stem for p in GOLDEN.glob("*.npz"))


def load(model):
    z = np.load(GOLDEN / f"{model}.npz", allow_pickle=False)
    data = {k[6:]: z[k] for k in z.files if k.startswith("data__")}
    draws = {k[7:]: z[k] for k in z.files if k.startswith("draws__")}
    outs = {k[5:]: z[k] for k in z.files if k.startswith("out__")}
    for k in ("K", "L", "M", "G"):
        if k in data:
            data[k] = int(data[k])
    return data, draws, outs


def test_every_model_has_a_fixture():
    assert set(MODELS) == set(synth.GENERATORS)


@pytest.mark.parametrize("model", MODELS)
def test_oracle_reproduces_golden(oracle, model):
    data, draws, outs = load(model)
    pars = [k for k in outs if k != "pair_status"]
    got = oracle.gqs(model, data, draws, pars=pars, variant="cr", return_status=True)
    for k, v in outs.items():
        a = np.asarray(got[k])
        same = (a == v) | (np.isnan(a) & np.isnan(v))
        assert same.all(), f"{model}:{k} drifted from the golden fixture"
