#!/usr/bin/env python3
"""Time one request at several batch sizes (pairs) of a BASELINE config shape, to
see whether a kernel is latency-bound (time flat in the pair count until the
chip fills) or throughput-bound (time proportional to pairs).

  python tools/occupancy_probe.py --model iohmm-hmix --series 16 --draws 1024,2048,4096,8192,16384 \
      --T 10000 --pars loglik,gamma_tk,z_ffbs

Prints one JSON line per size: pairs, waves, ms (median of --rounds).
"""
import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gsoc17-hhmm_amd"), str(ROOT / "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import hhmm_amd  # noqa: E402
from devrun import DeviceRequest  # noqa: E402
from hhmm_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="iohmm-hmix")
    ap.add_argument("--series", type=int, default=16)
    ap.add_argument("--draws", default="1024,2048,4096,8192")
    ap.add_argument("--T", type=int, default=10000)
    ap.add_argument("--pars", default="loglik,gamma_tk,z_ffbs")
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    lib = hhmm_amd.load_library()
    pars = a.pars.split(",")
    for S in (int(v) for v in a.draws.split(",")):
        data, draws = synth.GENERATORS[a.model](N=a.series, S=S, T=a.T)
        uu = synth.ffbs_uniforms(a.series * S, a.T) if "z_ffbs" in pars else None
        r = DeviceRequest(lib, a.model, data, draws, pars, flags=a.flags, uniforms=uu)
        r.run()
        ts = []
        for _ in range(a.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        P = a.series * S
        print(json.dumps({"model": a.model, "pairs": P, "waves": (P + 63) // 64, "T": a.T,
                          "ms": float(np.median(ts)), "ns_per_pair_step": float(np.median(ts)) * 1e6 / (P * a.T)}),
              flush=True)
        del r


if __name__ == "__main__":
    main()
