#!/usr/bin/env python3
"""How often does the engine's Viterbi (correctly rounded log, bit-exact with
the `cr` oracle) differ from Stan-with-glibc semantics (the oracle's `libm`
build, which calls the host's glibc log exactly where Stan does)?

Runs a C2-shaped slice (hmm-multinom K=4, L=9, T=1000, zip) on the GPU and
through both oracle builds, and reports per-pair mismatch rates of zstar_t
and logp_zstar against each.  Writes one JSON line.

  python tools/glibc_viterbi_rate.py [--pairs 16384]
"""
import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gsoc17-hhmm_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (its HIP runtime first)

import hhmm_amd  # noqa: E402
import pyoracle  # noqa: E402
from hhmm_amd import _abi, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=16384)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    lib = hhmm_amd.load_library()
    data, draws = synth.hmm_multinom(N=a.pairs, S=a.pairs, T=a.T, K=4, L=9, seed=synth.SEED + 77)
    pars = ["zstar_t", "logp_zstar"]
    got = hhmm_amd.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", lib=lib,
                       flags=_abi.FLAG_VIT_LANES)
    res = {"pairs": a.pairs, "T": a.T, "model": "hmm-multinom K=4 L=9 zip (C2 slice)"}
    for variant in ("cr", "libm"):
        ref = pyoracle.gqs("hmm-multinom", data, draws, pars=pars, pairing="zip", nthreads=threads,
                           variant=variant)
        zdiff = (got["zstar_t"] != ref["zstar_t"]).any(axis=1)
        ldiff = got["logp_zstar"].view(np.int64) != ref["logp_zstar"].view(np.int64)
        steps = int((got["zstar_t"] != ref["zstar_t"]).sum())
        res[variant] = {"pairs_zstar_differ": int(zdiff.sum()), "pairs_logp_zstar_differ": int(ldiff.sum()),
                        "steps_zstar_differ": steps, "pair_rate_zstar": float(zdiff.mean()),
                        "pair_rate_logp_zstar": float(ldiff.mean())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
