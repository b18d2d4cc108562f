#!/usr/bin/env python3
"""Which hardware queue each kernel ran on and how much the in-flight builds
overlapped, from a rocprofv3 kernel trace (run_kernel_trace.csv):

    python3 tools/queue_map.py <trace dir> [<trace dir> ...]

Per trace: kernel counts per Queue_Id, the mean k_entries_fixed duration in
the last 400 launches before the isolated ones, and the fraction of that
window with >= 2 leaf kernels running at once (three builds in flight should
keep it high; builds sharing a queue serialise and it falls)."""
import collections
import csv
import os
import sys


def analyse(d):
    path = os.path.join(d, "run_kernel_trace.csv")
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    per_q = collections.defaultdict(collections.Counter)
    for r in rows:
        per_q[r["Queue_Id"]][r["Kernel_Name"].split("(")[0][:40]] += 1
    print("== %s: %d dispatches" % (d, len(rows)))
    for q in sorted(per_q, key=int):
        print("  queue %s: %s" % (q, ", ".join("%s x%d" % (k, c) for k, c in per_q[q].most_common(6))))
    ef = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"]) for r in rows
          if "k_entries_fixed" in r["Kernel_Name"]]
    # the bench's last 60 (ISO) launches are isolated / single builds: skip them
    win = ef[-460:-60] if len(ef) > 460 else ef
    t0, t1 = win[0][0], win[-1][1]
    ev = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
    cur, last, two = 0, t0, 0
    for t, dlt in ev:
        if cur >= 2:
            two += t - last
        cur += dlt
        last = t
    mean = sum(e - s for s, e, _ in win) / len(win) / 1e3
    print("  window: %d leaf launches in %.2f ms = %.4f ms per launch; mean duration %.1f us; "
          ">= 2 leaf kernels running %.0f %% of the time; queues %s" % (
              len(win), (t1 - t0) / 1e6, (t1 - t0) / 1e6 / len(win), mean, 100 * two / (t1 - t0),
              sorted(set(q for _, _, q in win), key=int)))


for d in sys.argv[1:]:
    analyse(d)
