#!/usr/bin/env python3
"""Per-phase instruction breakdown of a kernel's main loop, from a hipcc `-g -S`
assembly file (where the VALU of the VALU-bound sweeps goes).

  hipcc -O3 -g ... --cuda-device-only -S -o k.s hhmm_io_reg_lo.hip
  python tools/isa_phases.py k.s 'iohmm_reg_kernelILi4ELi4ELi1ELb1E' [source dir, default csrc]

Loops are the natural loops of the kernel's control-flow graph (basic blocks,
dominators, back edges); every instruction in a loop body is attributed to
the source function its `.loc` line falls in (the innermost inlined function:
dev_cr_exp, softmax_cr_log, io_emission, ...) and counted by class (VALU, SALU,
LDS, VMEM).  Static counts with every block of the body once (rare branches
such as t == 0 included): compare the VALU total with the dynamic SQ_INSTS_VALU
per wave-step of the PMC passes.
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
        # basic blocks: split at labels and after branches / s_endpgm
        blocks = []  # [label, [(op, text, loc)], succ labels]
        cur = [None, []]
        loc = (0, 0)
        order = []

        def close(fall):
            if cur[1] or cur[0] is not None:
                blocks.append({"label": cur[0], "insts": cur[1], "fall": fall})

        for ln in lines:
            s2 = ln.strip()
            if not s2 or s2.startswith(";"):
                continue
            if s2.startswith(".loc"):
                p2 = s2.split()
                loc = (int(p2[1]), int(p2[2]))
                continue
            m2 = re.match(r"^(\.LBB\w+):", s2)
            if m2:
                close(True)
                cur = [m2.group(1), []]
                continue
            if s2.startswith(".") or s2.endswith(":"):
                continue
            op = s2.split()[0]
            cur[1].append((op, s2, loc))
            if op.startswith("s_cbranch") or op in ("s_branch", "s_endpgm", "s_setpc_b64"):
                close(op.startswith("s_cbranch"))
                cur = [None, []]
        close(False)
        idx = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
        succ = []
        for i, b in enumerate(blocks):
            sc = []
            last = b["insts"][-1] if b["insts"] else None
            if last and (last[0].startswith("s_cbranch") or last[0] == "s_branch"):
                tgt = last[1].split()[-1]
                if tgt in idx:
                    sc.append(idx[tgt])
            if b["fall"] and i + 1 < len(blocks):
                sc.append(i + 1)
            succ.append(sc)
        n_b = len(blocks)
        pred = [[] for _ in range(n_b)]
        for i, sc in enumerate(succ):
            for j in sc:
                pred[j].append(i)
        # blocks reachable from the entry only (cold tails after s_endpgm are not)
        reach, stack = {0}, [0]
        while stack:
            x = stack.pop()
            for y in succ[x]:
                if y not in reach:
                    reach.add(y)
                    stack.append(y)
        succ = [[y for y in sc if y in reach] if i in reach else [] for i, sc in enumerate(succ)]
        pred = [[q for q in ps if q in reach] for ps in pred]
        # dominators (iterative; entry = block 0)
        full = set(reach)
        dom = [full.copy() for _ in range(n_b)]
        dom[0] = {0}
        changed = True
        while changed:
            changed = False
            for i in range(1, n_b):
                if i not in reach:
                    continue
                ps = [dom[q] for q in pred[i]]
                nd = (set.intersection(*ps) if ps else set()) | {i}
                if nd != dom[i]:
                    dom[i], changed = nd, True
        loops = []  # (size, header, body)
        for u in range(n_b):
            for h in succ[u]:
                if h in dom[u]:  # back edge u -> h
                    body, stack = {h, u}, ([u] if u != h else [])
                    while stack:
                        x = stack.pop()
                        for q in pred[x]:
                            if q not in body:
                                body.add(q)
                                stack.append(q)
                    loops.append((sum(len(blocks[i]["insts"]) for i in body), h, frozenset(body)))
        if not loops:
            print(f"{name}: no loop")
            continue
        # merge back edges into one loop per header; outermost first
        by_h = {}
        for n2, h, body in loops:
            by_h[h] = by_h.get(h, frozenset()) | body
        lps = sorted(((sum(len(blocks[i]["insts"]) for i in b), h, b) for h, b in by_h.items()), reverse=True)
        fidx = {}
        total = sum(len(b["insts"]) for b in blocks)
        print(f"{name}: {total} instructions, {n_b} blocks; loops (static instructions of the body, "
              f"every block once):")
        for n2, h, body in lps[:int(os.environ.get("ISA_LOOPS", "3"))]:
            per = collections.defaultdict(collections.Counter)
            tot = collections.Counter()
            for i in sorted(body):
                for op, _, (fno, line) in blocks[i]["insts"]:
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
            inner = sum(1 for _, h2, b2 in lps if b2 < body)
            print(f"  loop at block {h} ({blocks[h]['label']}): {n2} instructions in {len(body)} blocks, "
                  f"{inner} inner loops  {dict(tot)}")
            for key, c in sorted(per.items(), key=lambda kv: -kv[1]["valu"]):
                if c["valu"] + c["salu"] == 0:
                    continue
                print(f"     {key:53s} valu {c['valu']:5d}  salu {c['salu']:4d}  lds {c['lds']:3d}  "
                      f"vmem {c['vmem']:3d}  other {sum(c.values()) - c['valu'] - c['salu'] - c['lds'] - c['vmem']:4d}")


if __name__ == "__main__":
    main()
