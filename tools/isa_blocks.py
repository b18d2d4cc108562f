#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a gfx950 .s file.

usage: isa_blocks.py file.s mangled_kernel_name [min_instructions]
"""
import re
import sys
from collections import Counter


def main():
    path, name = sys.argv[1], sys.argv[2]
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    s = open(path).read()
    i = s.find("\n" + name + ":")
    if i < 0:
        sys.exit("kernel not found")
    j = s.find("s_endpgm", i)
    blocks, cur = [], ["entry", []]
    for ln in s[i:j].split("\n")[2:]:
        t = ln.strip()
        if re.match(r"^\.LBB\S+:", t):
            blocks.append(cur)
            cur = [t.split(":")[0], []]
            continue
        if not t or t.startswith((";", ".")):
            continue
        cur[1].append(t.split()[0])
    blocks.append(cur)
    for b, ins in blocks:
        if len(ins) < lo:
            continue
        c = Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        mem = sum(v for k, v in c.items() if k.startswith(("global_", "ds_", "buffer_", "flat_",
                                                             "s_load", "scratch")))
        br = [x for x in ins if x.startswith("s_cbranch") or x == "s_branch"]
        top = ", ".join("%s %d" % kv for kv in c.most_common(6))
        print("%-12s %5d valu %5d mem %3d wait %3d %-16s | %s" % (b, len(ins), valu, mem,
                                                                   c["s_waitcnt"], br[-1] if br else "", top))


if __name__ == "__main__":
    main()
