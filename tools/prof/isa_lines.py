#!/usr/bin/env python3
"""Attribute the static instructions of one kernel in a `hipcc -g -S` device assembly file to
source lines (.loc), optionally only inside [first, last) of its own line range: which source
lines the VALU instruction stream is spent on.
usage: isa_lines.py <file.s> <kernel-name-substring> [top=40]"""
import collections, re, sys


def main(path, sub, top=40):
    s = open(path).read().split("\n")
    files = {}
    for l in s:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
    start = next(i for i, l in enumerate(s) if re.match(r"^\S*%s\S*:" % re.escape(sub), l))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    cur = "?"
    by_line = collections.Counter()
    by_line_mad = collections.Counter()
    for l in s[start:end]:
        t = l.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = "%s:%s" % (files.get(m.group(1), m.group(1)), m.group(2))
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("s_"):
            continue
        by_line[cur] += 1
        if op == "v_mad_u64_u32":
            by_line_mad[cur] += 1
    tot = sum(by_line.values())
    print("vector instructions", tot, "mads", sum(by_line_mad.values()))
    for k, v in by_line.most_common(top):
        print("%6d %6d  %s" % (v, by_line_mad[k], k))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
