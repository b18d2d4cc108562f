#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of `bench.py` into its phases and summarise
the dominant kernel: clock pre-warm + warmup, timed region (builds in flight,
no timing events), the contended pass after it (the same steps with the timing
events on), the single builds without events and the isolated launches with
them.  The trace is split from its end (ISO isolated launches last, the
untimed single builds, the contended pass and the K timed ones before them),
so the pre-warm's variable build count does not shift the phases.

usage: prof_summary.py run_kernel_trace.csv --steps K --warmup W [--isolated 10]
       [--single 50] [--contended min(K, 60 * inflight)]
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
    p.add_argument("--single", type=int, default=50)
    p.add_argument("--inflight", type=int, default=3)
    p.add_argument("--contended", type=int, default=None)
    p.add_argument("--kernel", default="k_entries_fixed")
    a = p.parse_args()
    if a.contended is None:
        a.contended = min(a.steps, 60 * a.inflight)
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    k, m, sb, cp = a.steps, a.isolated, a.single, a.contended
    n = len(dur)
    iso = dur[n - m:] if m else []
    single = dur[n - m - sb:n - m]
    cont = dur[n - m - sb - cp:n - m - sb]
    timed = dur[n - m - sb - cp - k:n - m - sb - cp]

    def mean(x):
        return round(sum(x) / max(len(x), 1), 4) if x else None

    out = {"kernel": a.kernel, "launches": n,
           "before_timed_region": n - m - sb - cp - k,
           "timed_region_mean_ms": mean(timed),
           "contended_pass_mean_ms": mean(cont),
           "single_builds_mean_ms": mean(single),
           "isolated_mean_ms": mean(iso),
           "all_mean_ms": mean(dur)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
