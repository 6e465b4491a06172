#!/usr/bin/env python3
"""Compare deSAMBA SAM outputs read by read (test/dev tool).

Groups consecutive records by QNAME (one group per input read, in input order) and
reports: reads compared, full-record mismatches, primary-RNAME (taxid) mismatches,
mapped-flag mismatches.  Usage: samcmp.py A.sam B.sam [--show N]
"""
import sys


def groups(path):
    """One group per input read: a primary/unmapped record (flag without 0x900) followed by
    its supplementary (0x800) and secondary (0x100) records."""
    out = []
    with open(path, "rb") as f:
        for line in f:
            fl = line.split(b"\t")
            name, flag = fl[0], int(fl[1])
            if out and (flag & 0x900) and out[-1][0] == name:
                out[-1][1].append(line)
            else:
                out.append((name, [line]))
    return out


def primary_key(g):
    f = g[1][0].split(b"\t")
    return f[2], int(f[1]) & 4


def compare(a, b, show=0):
    ga, gb = groups(a), groups(b)
    n = min(len(ga), len(gb))
    full = tax = mapped = 0
    bad = []
    for i in range(n):
        if ga[i][0] != gb[i][0]:
            raise SystemExit(f"read order differs at {i}: {ga[i][0]} vs {gb[i][0]}")
        if ga[i][1] != gb[i][1]:
            full += 1
            bad.append(i)
        ka, kb = primary_key(ga[i]), primary_key(gb[i])
        if ka[0] != kb[0]:
            tax += 1
        if ka[1] != kb[1]:
            mapped += 1
    res = dict(reads_a=len(ga), reads_b=len(gb), compared=n, full_mismatch=full,
               taxid_mismatch=tax, mapped_mismatch=mapped, bad=bad)
    for i in bad[:show]:
        print("----", ga[i][0].decode())
        for l in ga[i][1]:
            print("A", l.decode().rstrip()[:160])
        for l in gb[i][1]:
            print("B", l.decode().rstrip()[:160])
    return res


if __name__ == "__main__":
    show = 0
    if "--show" in sys.argv:
        show = int(sys.argv[sys.argv.index("--show") + 1])
    r = compare(sys.argv[1], sys.argv[2], show)
    r["bad"] = r["bad"][:50]
    print(r)
