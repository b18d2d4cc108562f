#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of `bench.py` into its phases and summarise
the dominant kernel: warmup, timed region (W builds in flight) and the
isolated launches bench.py makes after the timed region.

usage: prof_summary.py run_kernel_trace.csv --steps K --warmup W [--isolated 5]
"""
import argparse
import csv
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--steps", type=int, required=True)
    p.add_argument("--warmup", type=int, required=True)
    p.add_argument("--isolated", type=int, default=10)
    p.add_argument("--kernel", default="k_entries_fixed")
    a = p.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    w, k = a.warmup, a.steps
    timed, iso = dur[w:w + k], dur[w + k:w + k + a.isolated]
    out = {"kernel": a.kernel, "launches": len(dur),
           "timed_region_mean_ms": round(sum(timed) / max(len(timed), 1), 4),
           "isolated_mean_ms": round(sum(iso) / max(len(iso), 1), 4) if iso else None,
           "all_mean_ms": round(sum(dur) / max(len(dur), 1), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
