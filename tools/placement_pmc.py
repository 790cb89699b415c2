#!/usr/bin/env python3
"""Per-allocation-set counters of tools/placement_probe.py under rocprofv3 --pmc.

  rocprofv3 --pmc C1 C2 ... --output-format csv -d DIR -o pmc -- python3 tools/placement_probe.py --sets S --fb ...
  python tools/placement_pmc.py DIR S OUT.json

The probe launches every set's requests in a fixed order (warm-up: set 0..S-1,
then rounds of set 0..S-1), so the i-th dispatch of a kernel belongs to set
i % S.  Prints, per kernel and set, the mean of every counter over its
dispatches (and the mean dispatch duration when the trace has it)."""
import collections
import csv
import glob
import json
import pathlib
import sys


def main():
    d, S, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = []
    for f in glob.glob(str(pathlib.Path(d) / "**" / "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter
    for r in rows:
        k = r["Kernel_Name"]
        short = next((n for n in ("vfb_kernel", "fb_kernel", "viterbi_kernel") if f"::{n}<" in k), None)
        if short is None:
            continue
        per[(short, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for short in ("vfb_kernel", "fb_kernel", "viterbi_kernel"):
        ds = sorted(i for (s, i) in per if s == short)
        if not ds:
            continue
        sets = collections.defaultdict(lambda: collections.defaultdict(list))
        for n, i in enumerate(ds):
            for c, v in per[(short, i)].items():
                sets[n % S][c].append(v)
        out[short] = {f"set{s}": {c: sum(v) / len(v) for c, v in sorted(cs.items())} for s, cs in sorted(sets.items())}
        out[short]["dispatches"] = len(ds)
    pathlib.Path(dst).write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
