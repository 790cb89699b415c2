#!/usr/bin/env python3
"""Host copy rates on the GPU box (the host pipeline's staging copies): numpy
copies between pageable and pinned (torch pin_memory = hipHostMalloc) buffers,
1 and N threads, each 1 GiB, best of 3.  Prints one JSON line."""
import json
import os
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

N = 1 << 30


def rate(dst, src, nt):
    parts = np.array_split(np.arange(dst.size), nt)
    sl = [(p[0], p[-1] + 1) for p in parts if p.size]
    best = 1e9
    with ThreadPoolExecutor(nt) as ex:
        for _ in range(3):
            t0 = time.perf_counter()
            list(ex.map(lambda ab: np.copyto(dst[ab[0]:ab[1]], src[ab[0]:ab[1]]), sl))
            best = min(best, time.perf_counter() - t0)
    return dst.nbytes / best / 1e9


def main():
    pa = np.ones(N, dtype=np.uint8)
    pb = np.ones(N, dtype=np.uint8)
    pin = torch.ones(N, dtype=torch.uint8, pin_memory=True).numpy()
    out = {"cpus_affinity": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    for nt in (1, 4, 16):
        out[f"pageable_to_pageable_{nt}"] = rate(pb, pa, nt)
        out[f"pinned_to_pageable_{nt}"] = rate(pb, pin, nt)
        out[f"pageable_to_pinned_{nt}"] = rate(pin, pa, nt)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
