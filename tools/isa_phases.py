#!/usr/bin/env python3
"""Per-phase instruction breakdown of a kernel's main loop, from a hipcc `-g -S`
assembly file (where the VALU of the VALU-bound sweeps goes).

  hipcc -O3 -g ... --cuda-device-only -S -o k.s hhmm_io_reg_lo.hip
  python tools/isa_phases.py k.s 'iohmm_reg_kernelILi4ELi4ELi1ELb1E' [source dir, default csrc]

The main loop is the largest backward branch of the kernel; every instruction
in it is attributed to the source function its `.loc` line falls in (the
innermost inlined function: dev_cr_exp, softmax_cr_log, io_emission, ...),
and counted by class (f64 VALU, other VALU, SALU, LDS, VMEM).  Static counts of
one loop iteration (the t == 0 and store branches included): compare the VALU
total with the dynamic SQ_INSTS_VALU per wave-step of the PMC passes.
"""
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_stats import classify  # noqa: E402

FUNC_RE = re.compile(r"^[A-Za-z_][\w:<>,\s\*&]*?\b(~?\w+)\s*\([^;]*$")


def function_index(path):
    """line -> name of the function whose definition starts last at or before it."""
    idx, cur = [], None
    try:
        lines = open(path, errors="replace").read().split("\n")
    except OSError:
        return lambda ln: None
    for i, s in enumerate(lines, 1):
        if s and not s[0].isspace() and not s.startswith(("#", "/", "*", "}", "{")):
            m = FUNC_RE.match(s)
            if m and m.group(1) not in ("if", "for", "while", "switch", "return", "sizeof"):
                cur = m.group(1)
        idx.append(cur)
    return lambda ln: idx[ln - 1] if 0 < ln <= len(idx) else None


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2])
    text = open(path).read()
    files = {}
    for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', text, re.M):
        d, f = m.group(2), m.group(3)
        files[int(m.group(1))] = f if os.path.isabs(f) else os.path.join(d, f)
    srcdir = sys.argv[3] if len(sys.argv) > 3 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gsoc17-hhmm_amd", "csrc")
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", text, re.S):
        name, body = m.group(1), m.group(2)
        if not pat.search(name) or name.startswith("_ZL"):
            continue
        lines = body.split("\n")
        labels = {}
        insts = []  # (line index, op, loc)
        loc = (0, 0)
        for i, ln in enumerate(lines):
            s = ln.strip()
            if not s or s.startswith(";"):
                continue
            if s.startswith(".loc"):
                p = s.split()
                loc = (int(p[1]), int(p[2]))
                continue
            if s.endswith(":") and not s.startswith("."):
                continue
            if re.match(r"^\.LBB\w+:", s):
                labels[s.split(":")[0]] = len(insts)
                continue
            if s.startswith("."):
                continue
            insts.append((s.split()[0], s, loc))
        loops = []
        for k, (op, s, _) in enumerate(insts):
            if op.startswith("s_cbranch") or op == "s_branch":
                tgt = s.split()[-1]
                if tgt in labels and labels[tgt] <= k:
                    loops.append((k - labels[tgt] + 1, labels[tgt], k))
        if not loops:
            print(f"{name}: no loop")
            continue
        # outermost loops (not inside a larger one), largest first
        outer = [(n, a, b) for n, a, b in loops
                 if not any(a2 <= a and b <= b2 and (a2, b2) != (a, b) for _, a2, b2 in loops)]
        outer = sorted(set(outer), reverse=True)[:int(os.environ.get("ISA_LOOPS", "3"))]
        fidx = {}
        print(f"{name}: {len(insts)} instructions; outermost loops (static, one iteration):")
        for n, a, b in outer:
            per = collections.defaultdict(collections.Counter)
            tot = collections.Counter()
            for op, _, (fno, line) in insts[a:b + 1]:
                f = files.get(fno, "?")
                full = f if os.path.isabs(f) else os.path.join(srcdir, f)
                if full not in fidx:
                    fidx[full] = function_index(full)
                fn = fidx[full](line) or "?"
                key = f"{os.path.basename(f)}:{fn}"
                c = classify(op)
                c = "valu" if c.startswith("valu") else c
                per[key][c] += 1
                tot[c] += 1
            print(f"  loop [{a}, {b}] = {n} instructions  {dict(tot)}")
            for key, c in sorted(per.items(), key=lambda kv: -kv[1]["valu"]):
                if c["valu"] + c["salu"] == 0:
                    continue
                print(f"     {key:53s} valu {c['valu']:5d}  salu {c['salu']:4d}  lds {c['lds']:3d}  "
                      f"vmem {c['vmem']:3d}  other {sum(c.values()) - c['valu'] - c['salu'] - c['lds'] - c['vmem']:4d}")


if __name__ == "__main__":
    main()
