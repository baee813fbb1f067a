#!/usr/bin/env python3
"""Check the register discipline of k_map's and k_agg's hand-counted asm loads.

k_map streams its input with inline-asm `buffer_load_dwordx4` and hand-placed `s_waitcnt
vmcnt(N)`.  The compiler believes an asm output is ready as soon as the asm statement ends, so a
register copy between a load and its wait (e.g. to reconcile a loop-carried value's registers at
the loop header) would read data that has not landed yet.  Every such load and wait carries a tag
in an assembly comment:

    buffer_load_dwordx4 v[14:17], v4, s[12:15], 0 offen ; wcg-load A0
    s_waitcnt vmcnt(2) ; wcg-wait A v[14:17] v[6:9]

(a quantised wait is one asm statement - a chain of scalar compares around several s_waitcnt -
whose last line carries the tag; the tag names the registers the whole statement holds)

A value can only move to a different register through a copy, so requiring that every load of a
tag writes the same registers, and that every wait of a set names exactly those registers
(A0/A1 for set A, B0/B1 for set B, ...), rules such copies out without any control-flow analysis.

k_agg's batch walk (wcg_agg.h) uses the same tags: sets A and B of three global_load_dwordx4
each (A0, A1, A2), and waits naming all three registers.

Usage: check_inflight.py FILE.s KERNEL_SYMBOL      (exit status 1 on a violation)
"""
import re
import sys


def kernel_lines(text, sym):
    lines = text.splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end + 1]


def check(text, sym):
    loads, waits, errors = {}, [], []
    for ln in kernel_lines(text, sym):
        m = re.search(r"(?:buffer|global)_load_dwordx4\s+(v\[\d+:\d+\]).*wcg-load\s+(\w+)", ln)
        if m:
            loads.setdefault(m.group(2), set()).add(m.group(1))
            continue
        m = re.search(r"wcg-wait\s+(\w)((?:\s+v\[\d+:\d+\])+)", ln)
        if m:
            waits.append((m.group(1),) + tuple(m.group(2).split()))
    if not loads or not waits:
        errors.append("no tagged loads/waits found (kernel not built from wcg_map.h?)")
    for tag, regs in sorted(loads.items()):
        if len(regs) != 1:
            errors.append(f"loads tagged {tag} write different registers: {sorted(regs)}")
    for w in waits:
        s = w[0]
        for tag, r in ((s + str(i), r) for i, r in enumerate(w[1:])):
            if loads.get(tag) != {r}:
                errors.append(f"wait of set {s} names {r}, loads tagged {tag} write {sorted(loads.get(tag, []))}")
    return sorted(set(errors)), loads, waits


def main():
    errors, loads, waits = check(open(sys.argv[1]).read(), sys.argv[2])
    for e in errors:
        print("violation:", e)
    print(f"{len(loads)} load tags, {len(waits)} waits, {len(errors)} violation(s)")
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main())
