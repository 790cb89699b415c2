#!/usr/bin/env python3
"""Probe: do fb_kernel (HBM-bound) and viterbi_kernel (VALU-bound) overlap
when launched on two streams?  Times, on the bench's C2 batch, the
sequential step (one stream) against the two-stream step, interleaved.

  python tools/concurrency_probe.py [--rounds 6] [--pairs 1000000] [--T 1000]
"""
import argparse
import json
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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = hhmm_amd.load_library()
    x, draws = bench.make_batch(a.pairs, a.T, 9000, dev)
    run = bench.DeviceRun(lib, x, draws, a.pairs, a.T, dev)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    res = {"seq": [], "two_stream": [], "two_stream_vit_first": []}

    def seq():
        run.launch("fb")
        run.launch("viterbi")

    def two(vit_first=False):
        e = torch.cuda.Event()
        e.record(s0)
        s1.wait_event(e)
        if vit_first:
            with torch.cuda.stream(s1):
                run.launch("viterbi")
            run.launch("fb")
        else:
            run.launch("fb")
            with torch.cuda.stream(s1):
                run.launch("viterbi")
        j = torch.cuda.Event()
        j.record(s1)
        s0.wait_event(j)

    modes = {"seq": seq, "two_stream": two, "two_stream_vit_first": lambda: two(True)}
    for r in range(a.rounds + 1):
        for name, fn in modes.items():
            torch.cuda.synchronize()
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            t0.record(s0)
            fn()
            t1.record(s0)
            torch.cuda.synchronize()
            if r:
                res[name].append(t0.elapsed_time(t1))
    out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))} for k, v in res.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
