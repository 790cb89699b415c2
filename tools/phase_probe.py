#!/usr/bin/env python3
"""Phase probe of the C2 step on one device (HIP events, median of rounds):
the forward-backward request (gamma + loglik), its forward sweep alone
(loglik only: the FB_FWD kernel), the Viterbi request, and the two
requests concurrently on two streams (bench.py's schedule).

  python tools/phase_probe.py [--rounds 5] [--pairs 1000000] [--T 1000]
"""
import argparse
import ctypes as C
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "gsoc17-hhmm_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import hhmm_amd  # noqa: E402
from hhmm_amd import _abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=1000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = hhmm_amd.load_library()
    x, draws = bench.make_batch(a.pairs, a.T, 9000, dev)
    run = bench.DeviceRun(lib, x, draws, a.pairs, a.T, dev)
    # forward sweep only: the fb request with loglik alone
    r, res, ws = run.reqs["fb"]
    fwd = _abi.Request.from_buffer_copy(r)
    fwd.outputs = _abi.OUT["loglik"]
    fres = _abi.Result.from_buffer_copy(res)
    fres.gamma_tk = None
    run.reqs["fwd"] = (fwd, fres, ws)
    # Viterbi forward only: logp_zstar without the path (no backtrack)
    r, res, ws = run.reqs["viterbi"]
    vf = _abi.Request.from_buffer_copy(r)
    vf.outputs = _abi.OUT["logp_zstar"]
    vres = _abi.Result.from_buffer_copy(res)
    vres.zstar_t = None
    run.reqs["vit_fwd"] = (vf, vres, ws)
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s0)
        fn()
        e1.record(s0)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def concurrent():
        fork = torch.cuda.Event()
        fork.record(s0)
        s1.wait_event(fork)
        with torch.cuda.stream(s1):
            run.launch("viterbi")
        run.launch("fb")
        join = torch.cuda.Event()
        join.record(s1)
        s0.wait_event(join)

    cases = {"fb": lambda: run.launch("fb"), "fwd_only": lambda: run.launch("fwd"),
             "viterbi": lambda: run.launch("viterbi"), "vit_fwd": lambda: run.launch("vit_fwd"),
             "concurrent": concurrent, "library_step": lambda: run.launch("step"),
             "sequential": lambda: (run.launch("fb"), run.launch("viterbi"))}
    t = {k: [] for k in cases}
    for i in range(a.rounds + 1):
        for k, fn in cases.items():
            ms = timed(fn)
            if i:
                t[k].append(ms)
    print(json.dumps({k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v))} for k, v in t.items()}))


if __name__ == "__main__":
    main()
