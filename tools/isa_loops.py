#!/usr/bin/env python3
"""Loops of one kernel in a hipcc --save-temps .s listing: every backward
branch (s_cbranch/s_branch to an earlier label) is a loop; prints its label
range, instruction count by class (VALU, SALU, branch, memory) and the VALU
opcodes it issues most.  With a listing built with -g, each loop is labelled by
the source lines its instructions come from (the most frequent ones).
Usage: isa_loops.py listing.s kernel_symbol [--json out.json]"""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    files = {}
    lines, on = [], False
    for ln in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]*)"', ln)
        if m:
            files[m.group(1)] = m.group(2).split("/")[-1]
        if ln.startswith(sym + ":"):
            on = True
        elif on and ln.startswith(".Lfunc_end"):
            break
        if on:
            lines.append(ln.rstrip())
    labels = {}
    body, locs = [], []  # opcode, source line of each instruction
    cur = None
    for ln in lines:
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = len(body)
            continue
        s = ln.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
        if not s or s.startswith((";", ".")):
            continue
        body.append(s.split()[0])
        locs.append(cur)
    raw = [ln.strip() for ln in lines]
    loops = []
    idx = 0
    for ln in raw:
        if re.match(r"^\.LBB\w+:", ln) or not ln or ln.startswith((";", ".")):
            continue
        op = ln.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = ln.split()[1]
            if tgt in labels and labels[tgt] <= idx:
                loops.append((labels[tgt], idx, tgt))
        idx += 1
    print(f"{sym}: {len(body)} instructions, {len(loops)} loops")
    rows = []
    for a, b, tgt in sorted(set(loops)):
        ops = body[a:b + 1]
        cls = collections.Counter("valu" if o.startswith("v_") else "salu" if o.startswith("s_") and not o.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop")) else "branch" if o.startswith(("s_cbranch", "s_branch")) else "mem" if o.startswith(("global_", "scratch_", "buffer_", "ds_", "flat_", "s_load", "s_buffer")) else "other" for o in ops)
        top = collections.Counter(o for o in ops if o.startswith("v_")).most_common(8)
        src = [l for l, _ in collections.Counter(x for x in locs[a:b + 1] if x and not x.startswith(("__clang", "amd_"))).most_common(6)]
        print(f"  loop {tgt} [{a}..{b}] {len(ops)} insts {dict(cls)}" + (f" src {src}" if src else ""))
        print("     ", ", ".join(f"{o}:{n}" for o, n in top))
        rows.append(dict(label=tgt, first=a, last=b, insts=len(ops), classes=dict(cls), top_valu=dict(top),
                         source_lines=src, nops=sum(1 for o in ops if o == "s_nop")))
    if out_json:
        import json
        json.dump(dict(listing=path, kernel=sym, instructions=len(body), loops=rows), open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
