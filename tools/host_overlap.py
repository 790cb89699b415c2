#!/usr/bin/env python3
"""Overlap of hhmm_run's host pipeline in a rocprofv3 trace.

  rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d DIR -o trace -- \
      python3 bench.py --workload c2-host ...
  python tools/host_overlap.py DIR OUT.json

Reads every *kernel_trace.csv and *memory_copy_trace.csv under DIR and reports,
for the copies and kernels of the run: total busy time per engine class
(host-to-device copies, device-to-host copies, kernels), the union of all
three, and how much of the kernels' and the uploads' time lies under a
download (the pipeline's claim: the download stream stays busy while the next
chunk uploads and computes).  A serial request would show no such overlap.
"""
import csv
import glob
import json
import pathlib
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


def rows(d, pat):
    out = []
    for f in glob.glob(str(pathlib.Path(d) / "**" / pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def direction(r):
    for k in ("Direction", "Kind", "Operation"):
        v = (r.get(k) or "").upper()
        if "HOST_TO_DEVICE" in v or "H2D" in v or "HOSTTODEVICE" in v:
            return "h2d"
        if "DEVICE_TO_HOST" in v or "D2H" in v or "DEVICETOHOST" in v:
            return "d2h"
    return "other"


def main():
    d, dst = sys.argv[1], sys.argv[2]
    krows = rows(d, "*kernel_trace.csv")
    ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in krows]
    cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), direction(r)) for r in rows(d, "*memory_copy_trace.csv")]
    # uploads: SDMA copies from the pinned slots (memory-copy trace); downloads on
    # this stack: blit kernels (__amd_rocclr_copyBuffer) writing the pinned slots
    h2d_all = [[a, b] for a, b, k in cp if k == "h2d" and b - a > 100_000]
    d2h_all = [[a, b] for a, b, n in ker if "copyBuffer" in n and b - a > 100_000]
    hk = sorted([[a, b] for a, b, n in ker if "hhmm::" in n])
    # one window per hhmm_run call: hhmm kernels closer than 40 ms
    wins = []
    for a, b in hk:
        if wins and a - wins[-1][1] < 40_000_000:
            wins[-1][1] = max(wins[-1][1], b)
            wins[-1][2] += 1
        else:
            wins.append([a, b, 1])
    per = []
    for a, b, nk in wins:
        lo, hi = a - 60_000_000, b + 60_000_000  # the call's first upload and last download
        clip = lambda iv: [[max(x, lo), min(y, hi)] for x, y in iv if y > lo and x < hi]  # noqa: E731
        h2d, d2h = union(clip(h2d_all)), union(clip(d2h_all))
        kk = union([[x, y] for x, y in hk if x >= a and y <= b])
        allu = union(h2d + d2h + kk)
        per.append({
            "hhmm_kernels": nk,
            "span_ms": (allu[-1][1] - allu[0][0]) / 1e6 if allu else 0.0,
            "h2d_busy_ms": length(h2d) / 1e6, "d2h_busy_ms": length(d2h) / 1e6, "kernel_busy_ms": length(kk) / 1e6,
            "union_busy_ms": length(allu) / 1e6,
            "serial_sum_ms": (length(h2d) + length(d2h) + length(kk)) / 1e6,
            "kernel_under_d2h_ms": length(intersect(kk, d2h)) / 1e6,
            "h2d_under_d2h_ms": length(intersect(h2d, d2h)) / 1e6,
        })
    out = {"trace_dir": d, "calls": per,
           "note": "one entry per hhmm_run call (hhmm kernels within 40 ms); downloads are blit kernels "
                   "(__amd_rocclr_copyBuffer) on this stack, uploads SDMA copies; a serial call shows no "
                   "kernel or upload time under a download"}
    pathlib.Path(dst).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
