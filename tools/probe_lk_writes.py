#!/usr/bin/env python3
"""Probe (run under rocprofv3 --pmc WRITE_SIZE): the large-K T-scan sweep's
write traffic against the pair count's alignment.  One request per S in
argv (hmm-multinom, K = 23, L = 9, one series under S draws, T = 2e5,
loglik + gamma), each run twice (warm-up, measured), so that a per-dispatch
WRITE_SIZE of lk_fb_kernel can be compared with the gamma bytes S*T*K*8
(+ checkpoints).  Usage: python tools/probe_lk_writes.py 250 256"""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "gsoc17-hhmm_amd"), str(ROOT / "tests")]

import torch  # noqa: E402

import hhmm_amd  # noqa: E402
from devrun import DeviceRequest  # noqa: E402
from hhmm_amd import synth  # noqa: E402

lib = hhmm_amd.load_library()
T = 200_000
for s in sys.argv[1:]:
    S = int(s)
    data, draws = synth.hmm_multinom(N=1, S=S, T=T, K=23, L=9)
    r = DeviceRequest(lib, "hmm-multinom", data, draws, ["loglik", "gamma_tk"])
    r.run()
    r.run()
    print(f"S={S} T={T} gamma bytes {S * T * 23 * 8 / 1e9:.3f} GB, ckpt {S * T * 23 * 8 / 8 / 1e9:.3f} GB "
          f"(x2 runs)", flush=True)
    del r
    torch.cuda.empty_cache()
