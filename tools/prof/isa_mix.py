#!/usr/bin/env python3
"""Instruction mix of one kernel in a device assembly file (hipcc --cuda-device-only -S).
usage: isa_mix.py <file.s> <kernel-name-substring> [top]"""
import collections, re, sys


def main(path, sub, top=40):
    s = open(path).read()
    m = re.search(r"^(\S*%s\S*):" % re.escape(sub), s, re.M)
    i = m.start()
    j = s.index(".Lfunc_end", i)
    c = collections.Counter()
    for l in s[i:j].split("\n"):
        l = l.strip()
        if not l or l.startswith((".", ";")) or l.endswith(":") or ":" in l.split()[0]:
            continue
        c[l.split()[0]] += 1
    print(m.group(1), "total", sum(c.values()))
    for k, v in c.most_common(top):
        print("%6d %s" % (v, k))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
