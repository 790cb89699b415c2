#!/usr/bin/env python3
"""Interleaved A/B timing of libhhmm variants on one bench.py workload (c3,
c4, c5, n1), in ONE process on ONE device (cross-box numbers are not
comparable):

  python tools/ab_workload.py --workload c3 NAME=path/to/libhhmm.so[@VAR=VAL,...] [NAME=...] [--rounds 5] [--steps 3]

(@VAR=VAL sets environment variables around that variant's requests: the HHMM_PROBE_* knobs;
#FLAGS, after the path, gives that variant's request flags instead of --flags)

Every variant gets the same synthetic request (bench.prepare_other); rounds
run A B C A B C ..., each round `steps` back-to-back requests timed with HIP
events.  After the warm-up the variants' outputs are compared with the first
variant's (integer outputs bit for bit, float outputs to 1e-12 relative).
"""
import argparse
import json
import os
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "gsoc17-hhmm_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import hhmm_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--workload", default="c3", choices=["c1", "c3", "c4", "c5", "n1", "n2"])
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pars", default=None)
    ap.add_argument("--flags", type=int, default=0)
    ap.add_argument("--seed", type=int, default=bench.synth.SEED)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    runs = {}
    envs = {}
    for v in a.variants:
        name, path = v.split("=", 1)
        va = a
        if "#" in path:  # NAME=lib.so#FLAGS: this variant's request flags (hhmm_request.flags)
            path, fl = path.split("#", 1)
            va = argparse.Namespace(**vars(a))
            va.flags = int(fl, 0)
        if "@" in path:  # NAME=lib.so@VAR=VAL,VAR=VAL: environment set around this variant's requests
            path, ev = path.split("@", 1)
            envs[name] = dict(kv.split("=", 1) for kv in ev.split(","))
        runs[name] = bench.prepare_other(va, hhmm_amd.load_library(path), dev, 0)

    def step(n):
        env = envs.get(n, {})
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            runs[n]["step"]()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    ref = None
    for n, w in runs.items():
        step(n)
        torch.cuda.synchronize()
        outs = {k: t.cpu() for k, t in w["outs"].items()}
        if ref is None:
            ref = outs
            continue
        for k, t in outs.items():
            if t.dtype == torch.int32:
                ok = bool(torch.equal(t, ref[k]))
            else:
                d = (t - ref[k]).abs() / ref[k].abs().clamp_min(1e-300)
                ok = bool(torch.nan_to_num(d, nan=0.0).max() <= 1e-12)
            print(f"{n}: {k} matches the first variant: {ok}", flush=True)
    times = {n: [] for n in runs}
    for _ in range(a.rounds):
        for n, w in runs.items():
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(a.steps):
                step(n)
            ev[1].record()
            torch.cuda.synchronize()
            times[n].append(ev[0].elapsed_time(ev[1]) / a.steps)
    out = {n: {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))} for n, t in times.items()}
    print(json.dumps({"workload": a.workload, "ms_per_request": out}), flush=True)


if __name__ == "__main__":
    main()
