#!/usr/bin/env python3
"""Interleaved A/B timing of the C2 request's schedules in ONE process on ONE
device with one library (bench.DeviceRun's prepared requests):

  python tools/ab_sched.py [--lib path/to/libhhmm.so] [--rounds 7] [--steps 3] two vfb fused split
  python tools/ab_sched.py --lib new=lib/libhhmm.so --lib base=lib/variants/libhhmm_base.so new:vfb base:vfb

(a schedule may name its library: NAME:schedule with --lib NAME=path; a bare
schedule runs on the first library; NAME:schedule@VAR=VAL,... sets environment
variables around that schedule's launches, e.g. the HHMM_PROBE_* knobs)

Rounds run A B C A B C ...; each round times `steps` back-to-back requests
with HIP events on the launch stream (ms per request: median and min over
rounds).  Before timing, every schedule's outputs are compared bit for bit
with the first one's (gamma, loglik, zstar, logp_zstar on the whole batch).
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
    ap.add_argument("schedules", nargs="+")
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    libs = {}
    for spec in a.lib or ["default=" + str(hhmm_amd.api.LIB_PATH)]:
        name, path = spec.split("=", 1)
        libs[name] = hhmm_amd.load_library(path)
        assert libs[name].hhmm_init(1) == 0
    first = next(iter(libs))
    x, draws = bench.make_batch(a.pairs, a.T, 9000, dev)
    runs = {n: bench.DeviceRun(lib, x, draws, a.pairs, a.T, dev) for n, lib in libs.items()}

    def split(nm):
        """NAME:schedule@VAR=VAL,... -> (library, schedule, environment around its launches)"""
        env = {}
        if "@" in nm:
            nm, ev = nm.split("@", 1)
            env = dict(kv.split("=", 1) for kv in ev.split(","))
        ln, sc = nm.split(":", 1) if ":" in nm else (first, nm)
        return ln, sc, env

    def launch(nm):
        ln, sc, env = split(nm)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            runs[ln].launch(sc)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    s0 = torch.cuda.current_stream()
    ref = None
    same = {}
    for nm in a.schedules:
        run = runs[split(nm)[0]]
        for v in run.out.values():
            v.zero_()
        launch(nm)
        torch.cuda.synchronize()
        snap = {k: v.clone() for k, v in run.out.items()}
        if ref is None:
            ref = snap
        else:
            same[nm] = all(torch.equal(snap[k], ref[k]) for k in ref)
        del snap
    times = {nm: [] for nm in a.schedules}
    for _ in range(a.rounds):
        for nm in a.schedules:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s0)
            for _ in range(a.steps):
                launch(nm)
            e1.record(s0)
            torch.cuda.synchronize()
            times[nm].append(e0.elapsed_time(e1) / a.steps)
    out = {"pairs": a.pairs, "T": a.T, "rounds": a.rounds, "steps": a.steps,
           "bit_identical_to_first": same,
           "ms": {nm: {"median": float(np.median(t)), "min": float(np.min(t)), "all": [round(v, 3) for v in t]}
                  for nm, t in times.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
