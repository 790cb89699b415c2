#!/usr/bin/env python3
"""Summarise tools/pmc_workloads.sh output into profiles/ (committed evidence).

  python tools/workload_pmc.py TAG gpurun_out/pmcw_TAG

For every workload directory: per-kernel calls / average duration (kernel
trace) and per-dispatch PMC means (HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE,
the gfx950 correction of MI355X_MICROARCH.md §HBM; VALU and f64-MFMA
instruction counts), then per-STEP totals (each run is 1 warm-up + 1 timed
step, so a kernel's dispatches per step = calls / 2).  Writes
profiles/TAG_workloads_pmc.json and merges the per-step totals into
profiles/bench_traffic.json["workloads"], which bench.py reads for the
`traffic` and VALU / MFMA roofline fields of the evidence lines.
"""
import csv
import glob
import json
import pathlib
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
    return name.split("(")[0].replace("void ", "") if "hhmm::" in name else None


def trace(d):
    rows = defaultdict(list)
    for path in glob.glob(str(d / "trace" / "**" / "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r.get("Kernel_Name", ""))
                if k:
                    rows[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return rows


def pmc(d):
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for path in glob.glob(str(d / "pmc*" / "**" / "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = short(r.get("Kernel_Name", ""))
                if k:
                    per[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: {c: statistics.mean(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def main():
    tag, base = sys.argv[1], pathlib.Path(sys.argv[2])
    out = {}
    for d in sorted(p for p in base.iterdir() if p.is_dir()):
        tr, pm = trace(d), pmc(d)
        ks = {}
        step = defaultdict(float)
        for k, durs in tr.items():
            per_step = len(durs) / 2.0
            c = pm.get(k, {})
            hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in c and "WRITE_SIZE" in c else None
            ks[k] = {"calls_per_step": per_step, "avg_ns": statistics.mean(durs),
                     "hbm_bytes_per_dispatch": hbm, **{f"pmc_{n}": v for n, v in sorted(c.items())}}
            step["kernel_ns"] += per_step * statistics.mean(durs)
            if hbm is not None:
                step["hbm_bytes"] += per_step * hbm
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_SALU"):
                if n in c:
                    step[n] += per_step * c[n]
        out[d.name] = {"kernels": ks, "per_step": dict(step), "src": run_src(d)}
    prof = ROOT / "profiles"
    (prof / f"{tag}_workloads_pmc.json").write_text(json.dumps(out, indent=1))
    bt_path = prof / "bench_traffic.json"
    bt = json.loads(bt_path.read_text()) if bt_path.exists() else {}
    wl = bt.setdefault("workloads", {})
    for w, v in out.items():
        ps = v["per_step"]
        wl[w] = {"source": f"profiles/{tag}_workloads_pmc.json", "src": v["src"],
                 "hbm_bytes_per_step": ps.get("hbm_bytes"), "valu_insts_per_step": ps.get("SQ_INSTS_VALU"),
                 "mfma_f64_insts_per_step": ps.get("SQ_INSTS_VALU_MFMA_F64"),
                 # MOPS: f64 MFMA work in units of 512 FLOP (a v_mfma_f64_16x16x4 counts 4, a
                 # v_mfma_f64_4x4x4_16b 1), whatever the instruction mix
                 "mfma_f64_mops_per_step": ps.get("SQ_INSTS_VALU_MFMA_MOPS_F64"),
                 "kernel_ns_per_step": ps.get("kernel_ns")}
    bt_path.write_text(json.dumps(bt, indent=1))
    print(json.dumps({w: v["per_step"] for w, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
