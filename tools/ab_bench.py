#!/usr/bin/env python3
"""Interleaved A/B timing of libhhmm variants in ONE process on ONE device
(cdna_hip_programming.md §5.4 rule 24: cross-box numbers are not comparable).

  python tools/ab_bench.py NAME=path/to/libhhmm.so[@VAR=VAL,...] [NAME=...] [--rounds 5] [--pairs 1000000] [--T 1000]

(@VAR=VAL sets environment variables around that variant's launches, e.g. the
HHMM_PROBE_*_LDS_KB occupancy probes of hhmm_hmm.h)

Each variant runs the bench.py C2 step (fb_kernel, then viterbi_kernel, then
the two concurrently on two streams as bench.py does: "pair") on
the same resident inputs; rounds are interleaved A B C A B C ...; per-kernel
HIP-event times are reported as median / min over rounds.  Variants also
cross-check each other's outputs (gamma within 1e-12, zstar exact).
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    libs = {}
    envs = {}
    for v in a.variants:
        name, path = v.split("=", 1)
        if "@" in path:  # NAME=lib.so@VAR=VAL,VAR=VAL: environment set around this variant's launches
            path, ev = path.split("@", 1)
            envs[name] = dict(kv.split("=", 1) for kv in ev.split(","))
        libs[name] = hhmm_amd.load_library(path)
    x, draws = bench.make_batch(a.pairs, a.T, 9000, dev)
    # one set of output and workspace buffers for every variant: separate
    # allocations measured up to 20% apart for the SAME library (r05g: a copy of
    # the first-loaded build timed 6.79 vs 8.34 ms on fb_kernel)
    runs = {}
    for n, lib in libs.items():
        runs[n] = bench.DeviceRun(lib, x, draws, a.pairs, a.T, dev, share=next(iter(runs.values()), None))
    times = {n: {"fb": [], "vit": [], "pair": [], "step": [], "split": []} for n in runs}
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()

    def pair(run):
        """bench.py's step: viterbi on a side stream beside fb, forked and joined"""
        fork = torch.cuda.Event()
        fork.record(s0)
        s1.wait_event(fork)
        with torch.cuda.stream(s1):
            run.launch("viterbi")
        run.launch("fb")
        join = torch.cuda.Event()
        join.record(s1)
        s0.wait_event(join)
    ref = None
    for r in range(a.rounds + 1):
        for n, run in runs.items():
            for k in set().union(*envs.values()) if envs else ():
                os.environ.pop(k, None)
            os.environ.update(envs.get(n, {}))
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            ev[0].record()
            run.launch("fb")
            ev[1].record()
            run.launch("viterbi")
            ev[2].record()
            torch.cuda.synchronize()
            if r == 0:  # warm-up round; compare outputs
                g = run.out["gamma_tk"][:, :, :4096].cpu()
                z = run.out["zstar_t"][:, :4096].cpu()
                if ref is None:
                    ref = (g, z)
                else:
                    dg = float((g - ref[0]).abs().max())
                    same = bool(torch.equal(z, ref[1]))
                    print(f"{n}: max |dgamma| vs first variant {dg:.3e}, zstar identical {same}", flush=True)
                continue
            times[n]["fb"].append(ev[0].elapsed_time(ev[1]))
            times[n]["vit"].append(ev[1].elapsed_time(ev[2]))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s0)
            pair(run)
            e1.record(s0)
            torch.cuda.synchronize()
            times[n]["pair"].append(e0.elapsed_time(e1))
            for req in ("step", "split"):  # one library request each (side stream inside)
                torch.cuda.synchronize()
                e0.record(s0)
                run.launch(req)
                e1.record(s0)
                torch.cuda.synchronize()
                times[n][req].append(e0.elapsed_time(e1))
                if r == 1 and req == "split":
                    g = run.out["gamma_tk"][:, :, :4096].cpu()
                    z = run.out["zstar_t"][:, :4096].cpu()
                    run.launch("step")
                    torch.cuda.synchronize()
                    same_g = bool(torch.equal(g, run.out["gamma_tk"][:, :, :4096].cpu()))
                    same_z = bool(torch.equal(z, run.out["zstar_t"][:, :4096].cpu()))
                    print(f"{n}: split vs step outputs identical: gamma {same_g}, zstar {same_z}", flush=True)
    out = {}
    for n, t in times.items():
        out[n] = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))} for k, v in t.items()}
        print(n, json.dumps(out[n]), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
