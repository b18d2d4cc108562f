#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of `bench.py` into its phases and summarise
the dominant kernel: clock pre-warm + warmup, timed region (builds in flight)
and the isolated launches bench.py makes after the timed region.  The trace is
split from its end (ISO isolated launches last, the K timed ones before them),
so the pre-warm's variable build count does not shift the phases.

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
    k, m = a.steps, a.isolated
    iso = dur[len(dur) - m:] if m else []
    timed = dur[len(dur) - m - k:len(dur) - m]
    out = {"kernel": a.kernel, "launches": len(dur),
           "before_timed_region": len(dur) - m - k,
           "timed_region_mean_ms": round(sum(timed) / max(len(timed), 1), 4),
           "isolated_mean_ms": round(sum(iso) / max(len(iso), 1), 4) if iso else None,
           "all_mean_ms": round(sum(dur) / max(len(dur), 1), 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
