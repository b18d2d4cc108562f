#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 counter_collection CSVs: median counter
values per dispatch of the kernels matching a substring, plus the effective
clock (GRBM_GUI_ACTIVE / 8 XCDs / duration) and the stall split."""
import collections
import csv
import sys


def load(paths, match):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if match not in k:
                continue
            key = (p, r["Dispatch_Id"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k][key] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return acc, dur


def main():
    match = sys.argv[1]
    acc, dur = load(sys.argv[2:], match)
    for k, cs in acc.items():
        d = sorted(dur[k].values())
        dmed = d[len(d) // 2]
        print("kernel:", k[:90], "dispatches", len(d), "median ns", dmed)
        m = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}  # median dispatch
        for c in sorted(m):
            print("  %-24s %.4g" % (c, m[c]))
        if "GRBM_GUI_ACTIVE" in m:
            print("  eff clock GHz          %.3f" % (m["GRBM_GUI_ACTIVE"] / 8 / dmed))
        if "SQ_WAVE_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
            print("  VALU active / wave cyc %.3f" % (m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]))
        if "SQ_WAIT_ANY" in m and "SQ_ACTIVE_INST_ANY" in m:
            tot = m["SQ_WAIT_ANY"] + m["SQ_WAIT_INST_ANY"] + m["SQ_ACTIVE_INST_ANY"]
            print("  wait_any %.3f wait_inst %.3f active %.3f" % (
                m["SQ_WAIT_ANY"] / tot, m["SQ_WAIT_INST_ANY"] / tot, m["SQ_ACTIVE_INST_ANY"] / tot))


if __name__ == "__main__":
    main()
