#!/usr/bin/env python3
"""Loops of one kernel in an llvm-objdump -d listing of a code object (e.g. a
scene plugin dumped with RM_PLUGIN_DUMP): every backward branch is a loop;
prints its instruction range and VALU/SALU counts, and with --dump N the
instructions of loop N.  Usage: co_loops.py listing.s kernel [--dump N]"""
import collections
import re
import sys

path, sym = sys.argv[1], sys.argv[2]
dump = int(sys.argv[sys.argv.index("--dump") + 1]) if "--dump" in sys.argv else None
ins, on, base = [], False, None
for ln in open(path):
    m = re.match(r"^([0-9a-f]+) <(\w+)>:", ln)
    if m:
        on = m.group(2) == sym
        if on:
            base = int(m.group(1), 16)
        continue
    if not on:
        continue
    m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-F]+):\s*([0-9A-F ]+)(<.*>)?", ln)
    if m:
        ins.append((int(m.group(2), 16), m.group(1), m.group(4) or ""))
addr = {a: i for i, (a, _, _) in enumerate(ins)}
loops = set()
for i, (a, t, x) in enumerate(ins):
    op = t.split()[0]
    if (op.startswith("s_cbranch") or op == "s_branch") and x:
        m = re.search(r"\+0x([0-9a-f]+)>", x)
        tgt = base + int(m.group(1), 16)
        if tgt in addr and addr[tgt] <= i:
            loops.add((addr[tgt], i))
for n, (a, b) in enumerate(sorted(loops)):
    c = collections.Counter(ins[k][1].split()[0] for k in range(a, b + 1))
    v = sum(k for o, k in c.items() if o.startswith("v_"))
    s = sum(k for o, k in c.items() if o.startswith("s_"))
    print(n, a, b, b - a + 1, "valu", v, "salu", s, c.most_common(5))
    if dump == n:
        print("\n".join(ins[k][1] for k in range(a, b + 1)))
