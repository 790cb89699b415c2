#!/usr/bin/env python3
"""C2 placement probe: does the phased sweep's time depend
on where its output and workspace buffers sit?

In ONE process on ONE device: one C2 batch (x, draws), then several complete
sets of output + workspace buffers, each allocated in a different order and
behind a different padding allocation.  Every set runs the same C2 request
("step" = the library default, the phased sweep vfb_kernel) and, with
--fb, the forward-backward alone; rounds interleave the sets A B C ... and
time each with HIP events.  Prints each set's buffer addresses (and their
residues mod 4 KiB / 2 MiB / 256 MiB / 1 GiB) and the per-set median.

  python tools/placement_probe.py [--sets 4] [--rounds 5] [--steps 3] [--fb]
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

ORDERS = [
    ("gamma", "zstar", "ws", "small"),
    ("ws", "gamma", "zstar", "small"),
    ("zstar", "small", "ws", "gamma"),
    ("small", "gamma", "ws", "zstar"),
    ("gamma", "ws", "zstar", "small"),
    ("ws", "zstar", "small", "gamma"),
]
PAD_MB = [0, 2, 6, 258, 1030, 34]


class Shared:
    """What bench.DeviceRun(share=...) reads: .out and ._ws."""

    def __init__(self, P, T, ws_bytes, order, pad_mb, dev):
        K = bench.K
        self.pad = torch.empty(pad_mb << 20, dtype=torch.uint8, device=dev) if pad_mb else None
        self.out, self._ws = {}, {}
        for what in order:
            if what == "gamma":
                self.out["gamma_tk"] = torch.empty((K, T, P), dtype=torch.float64, device=dev)
            elif what == "zstar":
                self.out["zstar_t"] = torch.empty((T, P), dtype=torch.int32, device=dev)
            elif what == "ws":
                self._ws[ws_bytes] = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
            else:
                self.out["loglik"] = torch.empty(P, dtype=torch.float64, device=dev)
                self.out["logp_zstar"] = torch.empty(P, dtype=torch.float64, device=dev)
                self.out["pair_status"] = torch.zeros(P, dtype=torch.int32, device=dev)

    def addresses(self):
        bufs = {k: v.data_ptr() for k, v in self.out.items() if k in ("gamma_tk", "zstar_t")}
        bufs["ws"] = next(iter(self._ws.values())).data_ptr()
        return {k: {"addr": hex(a), "mod4K": a % 4096, "mod2M": a % (2 << 20), "mod256M": a % (256 << 20),
                    "mod1G": a % (1 << 30)} for k, a in bufs.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--T", type=int, default=1000)
    ap.add_argument("--fb", action="store_true")
    ap.add_argument("--names", default="step")
    ap.add_argument("--libs", default=None,
                    help="NAME=path,...: library variants, each timed on every set (default: the in-tree build)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    libs = {"tree": hhmm_amd.load_library()}
    if a.libs:
        libs = {kv.split("=", 1)[0]: hhmm_amd.load_library(kv.split("=", 1)[1]) for kv in a.libs.split(",")}
    lib = next(iter(libs.values()))
    x, draws = bench.make_batch(a.pairs, a.T, 9000, dev)
    import ctypes as C
    from hhmm_amd import _abi
    ws_need = 0
    for flags in (0, _abi.FLAG_VFB_OFF):
        q = _abi.Request()
        q.abi_version, q.model, q.pairing, q.device, q.flags = (_abi.ABI_VERSION, _abi.MODELS["hmm-multinom"],
                                                               _abi.PAIR_ZIP, -1, flags)
        q.data.n_series, q.data.T_max, q.data.K, q.data.L = a.pairs, a.T, bench.K, bench.L
        q.draws.n_draws = a.pairs
        for o in ("loglik", "gamma_tk", "zstar_t", "logp_zstar"):
            q.outputs |= _abi.OUT[o]
        ws = C.c_size_t(0)
        assert lib.hhmm_workspace_size(C.byref(q), C.byref(ws)) == 0
        ws_need = max(ws_need, int(ws.value))
    sets, runs, tags = [], [], []
    for i in range(a.sets):
        sh = Shared(a.pairs, a.T, ws_need, ORDERS[i % len(ORDERS)], PAD_MB[i % len(PAD_MB)], dev)
        sets.append(sh)
        for ln, lb in libs.items():
            runs.append(bench.DeviceRun(lb, x, draws, a.pairs, a.T, dev, share=sh))
            tags.append(f"set{i}/{ln}")
        print(json.dumps({"set": i, "order": ORDERS[i % len(ORDERS)], "pad_mb": PAD_MB[i % len(PAD_MB)],
                          "addresses": sh.addresses()}), flush=True)
    torch.cuda.synchronize()
    names = a.names.split(",") + (["fb"] if a.fb else [])
    s0 = torch.cuda.current_stream()
    g0 = None
    for i, run in enumerate(runs):  # warm-up + cross-check: every set and library computes the same outputs
        for nm in names:
            run.launch(nm)
        torch.cuda.synchronize()
        g = (run.out["gamma_tk"][:, :8, :4096].cpu(), run.out["zstar_t"][:8].cpu())
        if g0 is None:
            g0 = g
        assert torch.equal(g[0], g0[0]) and torch.equal(g[1], g0[1]), f"{tags[i]} differs"
    times = {(i, nm): [] for i in range(len(runs)) for nm in names}
    for _ in range(a.rounds):
        for i, run in enumerate(runs):
            for nm in names:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s0)
                for _ in range(a.steps):
                    run.launch(nm)
                e1.record(s0)
                torch.cuda.synchronize()
                times[(i, nm)].append(e0.elapsed_time(e1) / a.steps)
    out = {f"{tags[i]}:{nm}": {"median_ms": float(np.median(t)), "min_ms": float(np.min(t))}
           for (i, nm), t in times.items()}
    print(json.dumps({"probe": "placement", "pairs": a.pairs, "T": a.T, "ms": out}), flush=True)
    for ln in libs:
        for nm in names:
            med = [float(np.median(times[(i, nm)])) for i in range(len(runs)) if tags[i].endswith("/" + ln)]
            print(json.dumps({"lib": ln, "name": nm, "spread_pct": 100.0 * (max(med) - min(med)) / min(med),
                              "mean_ms": float(np.mean(med)), "medians": med}), flush=True)


if __name__ == "__main__":
    main()
