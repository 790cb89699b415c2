#!/usr/bin/env python3
"""Worst case of the IOHMM log-space fallback (hhmm_iolog.hip): every
pair of a batch saturated (w_km scaled x400, so the linear sweep lists every pair
and the log-space kernel re-runs them all), against the same batch unsaturated.

  python tools/iolog_worst.py > gpurun_out/TAG/iolog_worst.json

Cases: the C3 shape (iohmm-reg, 1250 series x 4000 draws, T = 300, the bench's
C3 outputs), the C4 shape (iohmm-hmix, 16 x 4096, T = 10^4, loglik + gamma), and
one long series (iohmm-reg, 1 series x 64 draws, T = 10^5).  Each request runs
once untimed and twice timed with HIP events on resident buffers (tests/devrun)."""
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gsoc17-hhmm_amd"), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hhmm_amd  # noqa: E402
from hhmm_amd import synth  # noqa: E402
from devrun import DeviceRequest  # noqa: E402

CASES = [
    ("c3_shape", "iohmm-reg", dict(N=1250, S=4000, T=300, K=4, M=4), ["loglik", "gamma_tk", "zstar_t", "logp_zstar"]),
    ("c4_shape", "iohmm-hmix", dict(N=16, S=4096, T=10_000, K=4, L=3, M=4), ["loglik", "gamma_tk"]),
    ("long_series", "iohmm-reg", dict(N=1, S=64, T=100_000, K=4, M=4), ["loglik", "gamma_tk"]),
]


def timed(r, reps=2):
    r.run()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ms = []
    for _ in range(reps):
        ev[0].record()
        r.run()
        ev[1].record()
        torch.cuda.synchronize()
        ms.append(ev[0].elapsed_time(ev[1]))
    return min(ms)


def main():
    lib = hhmm_amd.load_library()
    out = {"library": lib.hhmm_version().decode(), "cases": {}}
    for name, model, kw, pars in CASES:
        data, draws = synth.GENERATORS[model](**kw)
        res = {}
        for scale in (1.0, 400.0):
            d = dict(draws)
            d["w_km"] = draws["w_km"] * scale
            r = DeviceRequest(lib, model, data, d, pars)
            ms = timed(r)
            ll = r.out["loglik"]
            res[f"w_x{int(scale)}"] = {"ms": ms, "finite_loglik": int(torch.isfinite(ll).sum()), "pairs": r.P}
            del r
            torch.cuda.empty_cache()
        res["rerun_over_linear"] = res["w_x400"]["ms"] / res["w_x1"]["ms"]
        out["cases"][name] = {"model": model, "shape": kw, "outputs": pars, **res}
        print(name, json.dumps(res), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
