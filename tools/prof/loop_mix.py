#!/usr/bin/env python3
"""Static VALU instruction mix of a kernel's loop bodies in a `hipcc --cuda-device-only -S` file.

Blocks are attributed to loops by the compiler's comments ("Loop Header: Depth=", "in Loop: Header=BBx_y");
prints every loop's blocks with their instruction counts so the common path of a hot loop can be chosen
(exceptional paths such as a doubling are separate blocks), and with --blocks the opcode mix of the chosen
blocks.
usage: loop_mix.py <file.s> <kernel-substring> [--blocks BB1,BB2,...] [--json]"""
import collections
import json
import re
import sys


def blocks_of(path, sub):
    s = open(path).read().split("\n")
    start = next(i for i, l in enumerate(s) if re.match(r"^\S*%s\S*:" % re.escape(sub), l))
    end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
    blocks = collections.OrderedDict()
    cur, loop = "entry", None
    blocks[cur] = {"loop": None, "ops": collections.Counter()}
    for l in s[start + 1:end]:
        m = re.match(r"^(\.LBB\w+):\s*(;.*)?$", l)
        if m:
            cur = m.group(1)[1:]
            c = m.group(2) or ""
            h = re.search(r"Header=(BB\w+)", c)
            loop = h.group(1) if h else (cur if "Loop Header" in c else None)
            blocks[cur] = {"loop": loop, "ops": collections.Counter()}
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        blocks[cur]["ops"][t.split()[0]] += 1
    return blocks


def main():
    path, sub = sys.argv[1], sys.argv[2]
    bl = blocks_of(path, sub)
    sel = None
    if "--blocks" in sys.argv:
        sel = sys.argv[sys.argv.index("--blocks") + 1].split(",")
    if sel is None:
        for name, b in bl.items():
            n = sum(b["ops"].values())
            v = sum(c for o, c in b["ops"].items() if o.startswith("v_"))
            mad = b["ops"].get("v_mad_u64_u32", 0)
            print("%-12s loop=%-10s instr=%5d valu=%5d mad=%5d" % (name, b["loop"], n, v, mad))
        return
    mix = collections.Counter()
    for name in sel:
        mix.update(bl[name]["ops"])
    valu = {o: c for o, c in mix.items() if o.startswith("v_")}
    if "--json" in sys.argv:
        print(json.dumps({"blocks": sel, "valu_total": sum(valu.values()), "valu": dict(sorted(valu.items(), key=lambda x: -x[1])),
                          "other": {o: c for o, c in mix.items() if not o.startswith("v_")}}))
    else:
        print("valu total", sum(valu.values()))
        for o, c in sorted(valu.items(), key=lambda x: -x[1]):
            print("%6d %s" % (c, o))


if __name__ == "__main__":
    main()
