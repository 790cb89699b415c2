#!/usr/bin/env python3
"""Per-variant kernel durations from a rocprofv3 kernel trace of tools/ab_bench.py
(several libhhmm builds in one process): every hhmm kernel's dispatches grouped by
Kernel_Id (each loaded library registers its own), in dispatch order.

  python tools/trace_by_variant.py gpurun_out/TAG/trace [name-filter]
"""
import collections
import csv
import glob
import statistics
import sys


def main():
    rows = []
    for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    filt = sys.argv[2] if len(sys.argv) > 2 else "hhmm::"
    rows = [r for r in rows if filt in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[(r["Kernel_Name"].split("(")[0], int(r["Kernel_Id"]))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for (name, kid), d in sorted(by.items()):
        print(f"{name[:60]:60s} id {kid:5d} n {len(d):3d} median {statistics.median(d):8.3f} ms "
              f"min {min(d):8.3f}  [{' '.join(f'{x:.2f}' for x in d[:12])}]")


if __name__ == "__main__":
    main()
