#!/usr/bin/env python3
"""The C2 bench line against the rocprofv3 kernel trace of the SAME process
(VERDICT r4 item 2): `bench.py --gpus 1 --steps K --warmup W` run as
`rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o trace -- python3 bench.py ...`.

  python tools/trace_vs_line.py gpurun_out/TAG/bench_traced.json gpurun_out/TAG/trace TAG [OUT.json]

The bench launches the roofline kernel W times (warm-up), K times (the timed
steps, each bracketed by HIP events on the launch stream: the line's
roofline.duration_ms is their mean) and then the other schedules once each
after the timed region.  The dominant kernel's dispatches in the trace are
therefore [W warm-up][K timed][rest]; this script takes the K timed ones,
recomputes the roofline fraction from their mean duration, and writes one
JSON object with both figures and their ratio to OUT.json (default
gpurun_out/TAG/trace_vs_line.json; copy it into profiles/ to commit it), replacing
the file, never appending to it.
"""
import csv
import glob
import json
import pathlib
import statistics
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent


def main():
    line_path, trace_dir, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    line = None
    for ln in open(line_path):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    if line is None:
        sys.exit("no JSON line in " + line_path)
    rf = line["roofline"]
    kern = rf["kernel"]
    W, K = line["warmup"], line["steps"]
    files = glob.glob(str(pathlib.Path(trace_dir) / "**" / "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    disp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                  for r in rows if kern + "<" in r["Kernel_Name"] or r["Kernel_Name"].endswith(kern))
    if len(disp) < W + K:
        sys.exit(f"{len(disp)} dispatches of {kern}, expected at least {W + K}")
    timed = [d / 1e6 for _, d in disp[W:W + K]]
    mean_ms = statistics.fmean(timed)
    B = rf["algorithmic_bytes_per_series_timestep"]
    units = line["config"]["pairs_per_gpu"] * line["config"]["T"]
    frac_trace = B * units / (mean_ms * 1e-3) / (rf["peak"] * 1e9)
    out = {
        "tag": tag,
        "kernel": kern,
        "library": line.get("library"),
        "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps %d --warmup %d" % (K, W),
        "dispatches": len(disp),
        "timed_dispatch_ms": timed,
        "trace_mean_ms": mean_ms,
        "trace_median_ms": statistics.median(timed),
        "trace_min_ms": min(timed),
        "all_dispatch_mean_ms": statistics.fmean(d / 1e6 for _, d in disp),
        "line_duration_ms": rf["duration_ms"],
        "line_frac": rf["frac"],
        "trace_frac": frac_trace,
        "frac_ratio_line_over_trace": rf["frac"] / frac_trace,
        "line_ms_per_step": line["ms_per_step"],
        "line_value": line["value"],
    }
    dst = pathlib.Path(sys.argv[4]) if len(sys.argv) > 4 else ROOT / "gpurun_out" / tag / "trace_vs_line.json"
    dst.parent.mkdir(parents=True, exist_ok=True)
    tmp = dst.with_suffix(".tmp")
    tmp.write_text(json.dumps(out, indent=1) + "\n")
    json.loads(tmp.read_text())
    tmp.replace(dst)
    print(json.dumps({k: v for k, v in out.items() if k != "timed_dispatch_ms"}, indent=1))


if __name__ == "__main__":
    main()
