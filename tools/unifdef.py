#!/usr/bin/env python3
"""Resolve the preprocessor conditionals of given macros in a source file (a
minimal unifdef): every #if / #ifdef / #ifndef / #elif / #else / #endif whose
condition depends only on the listed macros keeps its taken branch, and the
`#ifndef X / #define X v / #endif` default blocks of listed macros go.  Used to
retire measured-and-rejected variant switches from the kernel sources with
their default behaviour (tools/; not product).
Usage: unifdef.py FILE NAME=VALUE|NAME=undef ... (rewrites FILE in place)"""
import re
import sys


def evaluate(expr, known):
    """Python value of a #if expression, or None if it names an unknown macro."""
    e = re.sub(r"//.*", "", expr)
    e = re.sub(r"/\*.*?\*/", "", e)
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)",
               lambda m: "1" if (m.group(1) or m.group(2)) in known and known[m.group(1) or m.group(2)] is not None
               else ("0" if (m.group(1) or m.group(2)) in known else "UNKNOWN"), e)
    for name in re.findall(r"[A-Za-z_]\w*", e):
        if name in ("UNKNOWN",):
            return None
        if name not in known:
            return None
        v = known[name]
        e = re.sub(rf"\b{name}\b", "0" if v is None else str(v), e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    try:
        return bool(eval(e, {}, {}))
    except Exception:  # noqa: BLE001
        return None


def main():
    path = sys.argv[1]
    known = {}
    for a in sys.argv[2:]:
        k, v = a.split("=", 1)
        known[k] = None if v == "undef" else int(v)
    lines = open(path).read().split("\n")
    out = []
    stack = []  # per open conditional: (resolved?, keep current branch?, any branch taken, parent emitting)
    emitting = True
    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(ifndef|ifdef|if|elif|else|endif)\b(.*)", s)
        if m:
            kw, rest = m.group(1), m.group(2).strip()
            if kw == "ifndef":
                name = rest.split()[0]
                # a default block: #ifndef X / #define X v / #endif
                if name in known and i + 2 < len(lines) and re.match(rf"#\s*define\s+{name}\b", lines[i + 1].strip()) \
                        and lines[i + 2].strip().startswith("#endif"):
                    i += 3
                    continue
                cond = None if name not in known else known[name] is None
                kw2 = "if"
            elif kw == "ifdef":
                name = rest.split()[0]
                cond = None if name not in known else known[name] is not None
                kw2 = "if"
            else:
                kw2 = kw
                cond = evaluate(rest, known) if kw in ("if", "elif") else None
            if kw2 == "if":
                if cond is None:
                    stack.append([False, True, False, emitting])
                    if emitting:
                        out.append(ln)
                else:
                    stack.append([True, cond, cond, emitting])
                    emitting = emitting and cond
            elif kw2 == "elif":
                top = stack[-1]
                if not top[0]:
                    if top[3]:
                        out.append(ln)
                else:
                    if cond is None:
                        raise SystemExit(f"{path}:{i + 1}: #elif on an unknown condition after a resolved #if")
                    take = (not top[2]) and cond
                    top[1] = take
                    top[2] = top[2] or take
                    emitting = top[3] and take
            elif kw2 == "else":
                top = stack[-1]
                if not top[0]:
                    if top[3]:
                        out.append(ln)
                else:
                    take = not top[2]
                    top[1] = take
                    top[2] = True
                    emitting = top[3] and take
            else:  # endif
                top = stack.pop()
                if not top[0]:
                    if top[3]:
                        out.append(ln)
                emitting = top[3]
            i += 1
            continue
        if emitting:
            out.append(ln)
        i += 1
    if stack:
        raise SystemExit(f"{path}: unbalanced conditionals")
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
