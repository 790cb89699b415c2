#!/usr/bin/env python3
"""Generates tests/golden/<model>.npz: small seeded inputs and the oracle's
outputs for every Stan program on the path (data, draws and every declared
TP/GQ output, plus pair_status).

The reference ships no fixtures and cannot run here, so
these vectors come from the C oracle (correctly rounded log) and are only
written after the independent pure-Python transcription
(tests/oracle_numpy.py, host libm) agrees with them: bit-exact Viterbi
paths and statuses, floats within 1e-12 relative (the two differ only by the
log's last-ulp rounding).  Re-run after an intentional oracle change:
    python tests/golden/make_golden.py
"""
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path[:0] = [str(REPO / "gsoc17-hhmm_amd"), str(REPO / "oracle"), str(REPO / "tests")]

import oracle_numpy as onp  # noqa: E402
import pyoracle  # noqa: E402
from hhmm_amd import synth  # noqa: E402

CASES = {
    "hmm": dict(N=2, S=3, T=16, K=3),
    "hmm-multinom": dict(N=2, S=3, T=16, K=4, L=9),
    "hmm-multinom-semisup": dict(N=2, S=3, T=16),
    "hhmm-tayal2009": dict(N=2, S=3, T=16),
    "hhmm-tayal2009-lite": dict(N=2, S=3, T=16, T_oos=12),
    "iohmm-reg": dict(N=2, S=3, T=16, K=3),
    "iohmm-mix": dict(N=2, S=3, T=16),
    "iohmm-hmix": dict(N=2, S=3, T=16),
    "iohmm-hmix-lite": dict(N=2, S=3, T=16),
}


def case_inputs(model):
    kw = dict(CASES[model])
    data, draws = synth.GENERATORS[model](seed=20170601, **kw)
    if model in ("hmm-multinom", "hhmm-tayal2009", "iohmm-hmix"):
        data["T"] = np.array([16, 9], dtype=np.int32)  # one ragged series
    return data, draws


def main():
    for model in CASES:
        data, draws = case_inputs(model)
        pars = synth.PARS[model]
        out = pyoracle.gqs(model, data, draws, pars=pars, variant="cr", return_status=True)
        rows = onp.run(model, data, draws)
        for p, r in enumerate(rows):
            assert int(out["pair_status"][p]) == r["pair_status"]
            for k in pars:
                a = np.asarray(out[k][p])
                b = np.asarray(r[k])
                if a.ndim:
                    a = a[: b.shape[0]]
                if k == "zstar_t":
                    assert np.array_equal(a, b), (model, k)
                else:
                    m = np.isfinite(b)
                    assert np.array_equal(np.isnan(a), np.isnan(b)), (model, k)
                    assert np.all(np.abs(a[m] - b[m]) <= 1e-12 * np.maximum(np.abs(b[m]), 1.0)), (model, k)
        blob = {}
        for k, v in data.items():
            blob["data__" + k] = np.asarray(v)
        for k, v in draws.items():
            blob["draws__" + k] = np.asarray(v)
        for k in pars + ["pair_status"]:
            blob["out__" + k] = np.asarray(out[k])
        np.savez_compressed(HERE / f"{model}.npz", **blob)
        print("wrote", model)


if __name__ == "__main__":
    main()
