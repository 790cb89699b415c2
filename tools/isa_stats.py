#!/usr/bin/env python3
"""Static instruction mix of gfx950 kernels in a hipcc `-S` assembly file.

  hipcc -O3 ... --cuda-device-only -S -o k.s hhmm_io_mix_lo.hip
  python tools/isa_stats.py k.s 'iohmm_mix_kernelILi4ELi4ELb1'

Prints, per matching kernel: total instructions, VALU / SALU / VMEM / LDS
counts, v_readlane / v_writelane (SGPR spills live in VGPR lanes), f64 ops,
s_nop, and the register metadata (vgpr, sgpr spill count).
"""
import collections
import re
import sys


def classify(op):
    if op.startswith("v_readlane") or op.startswith("v_writelane"):
        return op.split("_b")[0]
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_") or op.startswith("scratch_"):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


def main():
    path, pat = sys.argv[1], re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    text = open(path).read()
    meta = {}
    for m in re.finditer(r"\.name:\s+(\S+)\n(?:.*\n)*?.*?\.sgpr_spill_count:\s+(\d+)\n(?:.*\n)*?.*?\.vgpr_count:\s+(\d+)",
                         text):
        meta[m.group(1)] = (int(m.group(2)), int(m.group(3)))
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end", text, re.S):
        name, body = m.group(1), m.group(2)
        if not pat.search(name) or name.startswith("_ZL"):
            continue
        c = collections.Counter()
        for ln in body.split("\n"):
            ln = ln.strip()
            if not ln or ln[0] in ";." or ln.endswith(":"):
                continue
            c[classify(ln.split()[0])] += 1
        sp, vg = meta.get(name, (None, None))
        print(f"{name}: total={sum(c.values())} vgpr={vg} sgpr_spill={sp}")
        print("   ", dict(sorted(c.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__":
    main()
