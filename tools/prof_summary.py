#!/usr/bin/env python3
"""Summarise rocprofv3 output into profiles/ (committed evidence).

  python tools/prof_summary.py TAG gpurun_out/prof_TAG ['{"pairs": 1000000, "T": 1000}']

Writes profiles/TAG_kernel_stats.csv (per-kernel calls / total / avg / min / max
duration from the --kernel-trace --stats pass; SQLite .db or CSV input),
profiles/TAG_pmc.csv (per-kernel averages of every PMC counter collected in the
separate --pmc passes) and, when FETCH_SIZE / WRITE_SIZE are present,
profiles/TAG_pmc.json with HBM bytes per launch of each libhhmm kernel.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reads exactly half
of the bytes of wide coalesced streaming reads; the corrected figure doubles
it.  Both raw and corrected values are recorded.
"""
import csv
import glob
import json
import os
import pathlib
import sqlite3
import statistics
import sys
from collections import defaultdict

ROOT = pathlib.Path(__file__).resolve().parent.parent


def run_src(d):
    """The libhhmm build (source hash) the profiled run loaded: the "library"
    field of bench.py's JSON line(s) in the run's logs under `d`, or None."""
    srcs = set()
    for path in glob.glob(str(pathlib.Path(d) / "**" / "*.log"), recursive=True):
        for ln in open(path, errors="replace"):
            ln = ln.strip()
            if ln.startswith("{") and '"library"' in ln:
                try:
                    srcs.add(json.loads(ln)["library"].split(" src ")[-1])
                except Exception:
                    pass
    if len(srcs) > 1:
        raise SystemExit(f"{d}: runs of different builds {sorted(srcs)}")
    return srcs.pop() if srcs else None


def short(name):
    if "hhmm::" in name:
        return name.split("(")[0].replace("void ", "")
    return None


def kernel_rows_from_db(path):
    db = sqlite3.connect(path)
    rows = defaultdict(list)
    for name, dur in db.execute("select name, duration from kernels"):
        rows[name].append(dur)
    return rows


def kernel_rows_from_csv(path):
    rows = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("kernel_name") or r.get("Name")
            s, e = r.get("Start_Timestamp"), r.get("End_Timestamp")
            if name and s and e:
                rows[name].append(int(e) - int(s))
    return rows


def main():
    tag, d = sys.argv[1], pathlib.Path(sys.argv[2])
    out = ROOT / "profiles"
    out.mkdir(exist_ok=True)
    rows = None
    dbs = glob.glob(str(d / "**" / "*.db"), recursive=True)
    csvs = glob.glob(str(d / "**" / "*kernel_trace.csv"), recursive=True)
    if csvs:
        rows = kernel_rows_from_csv(csvs[0])
    elif dbs:
        rows = kernel_rows_from_db(dbs[0])
    if rows:
        with open(out / f"{tag}_kernel_stats.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "share_of_hhmm_time"])
            tot = sum(sum(v) for k, v in rows.items() if short(k))
            for k, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
                if not short(k):
                    continue
                w.writerow([short(k), len(v), sum(v), round(statistics.mean(v)), min(v), max(v),
                            round(sum(v) / tot, 4)])
        print("wrote", out / f"{tag}_kernel_stats.csv")

    # PMC passes: counter_collection.csv per pass
    pmc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(str(d / "pmc*" / "**" / "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", "")
                if not short(name):
                    continue
                ctr = r.get("Counter_Name")
                val = float(r.get("Counter_Value", "nan"))
                pmc[short(name)][(ctr, r.get("Dispatch_Id"))].append(val)
    if pmc:
        agg = {}
        for k, d2 in pmc.items():
            per = defaultdict(list)
            for (ctr, disp), vals in d2.items():
                per[ctr].append(sum(vals))  # sum over dimensions (XCD/SE instances)
            agg[k] = {c: statistics.mean(v) for c, v in per.items()}
        with open(out / f"{tag}_pmc.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "counter", "mean_per_dispatch"])
            for k, cs in agg.items():
                for c, v in sorted(cs.items()):
                    w.writerow([k, c, v])
        print("wrote", out / f"{tag}_pmc.csv")
        summ = {}
        for k, cs in agg.items():
            if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
                fetch_kb = cs.get("FETCH_SIZE", float("nan"))
                write_kb = cs.get("WRITE_SIZE", float("nan"))
                summ[k] = {"fetch_size_kb_raw": fetch_kb, "write_size_kb": write_kb,
                           "hbm_bytes_per_launch_raw": (fetch_kb + write_kb) * 1024,
                           "hbm_bytes_per_launch": (2 * fetch_kb + write_kb) * 1024,
                           "correction": "FETCH_SIZE doubled (gfx950, MI355X_MICROARCH.md §HBM)"}
        if summ:
            src = run_src(d)
            for v in summ.values():
                v["src"] = src
            (out / f"{tag}_pmc_traffic.json").write_text(json.dumps(summ, indent=1))
            print("wrote", out / f"{tag}_pmc_traffic.json")
            # the bench's roofline.traffic: HBM bytes per launch of each bench kernel,
            # keyed by its short name, for the batch shape the PMC passes ran
            shape = {}
            if len(sys.argv) > 3:
                shape = json.loads(sys.argv[3])
            bp = out / "bench_traffic.json"
            old = json.loads(bp.read_text()) if bp.exists() else {}
            bt = {"source": f"profiles/{tag}_pmc_traffic.json", "src": src, **shape, "kernels": {}}
            if "workloads" in old:  # the evidence workloads' per-step totals (tools/workload_pmc.py)
                bt["workloads"] = old["workloads"]
            for k, v in summ.items():
                base = k.split("::")[-1].split("<")[0]
                bt["kernels"][base] = {"template": k, "hbm_bytes_per_launch": v["hbm_bytes_per_launch"]}
            (out / "bench_traffic.json").write_text(json.dumps(bt, indent=1))
            print("wrote", out / "bench_traffic.json")


if __name__ == "__main__":
    main()
