"""Summary of a tools/wg_trace JSON: dispatch ramp, per-CU finish order and
spacing, the workgroups' shader clock (s_memtime cycles / 100 MHz wall clock)."""
import collections
import json
import sys

import numpy as np


def summary(path):
    d = json.load(open(path))
    w = np.array(d["wg"], dtype=np.float64)
    xcc, cu, s, l, e, c0, c2, f = w.T
    t0 = s.min()
    s, l, e, f = (s - t0) / 100.0, (l - t0) / 100.0, (e - t0) / 100.0, (f - t0) / 100.0  # us
    mhz = (c2 - c0) / np.maximum(e - s, 1e-9)
    byc = collections.defaultdict(list)
    for i in range(len(w)):
        byc[(xcc[i], cu[i])].append(l[i])
    per_cu = collections.Counter(len(v) for v in byc.values())
    ranks = np.array([sorted(v) for v in byc.values() if len(v) == max(per_cu)])
    # residency: the most workgroups of one CU alive at the same instant
    # (start <= t < end), over every CU
    alive = collections.defaultdict(list)
    for i in range(len(w)):
        alive[(xcc[i], cu[i])].append((s[i], e[i]))
    conc = []
    for iv in alive.values():
        ev = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv], key=lambda x: (x[0], x[1]))
        cur = best = 0
        for _, dlt in ev:
            cur += dlt
            best = max(best, cur)
        conc.append(best)
    return {
        "file": path, "warm": d.get("warm"), "contended": d.get("contended"),
        "kernel_ms": d["kernel_ms"], "workgroups": int(len(w)), "lpl": d.get("lpl"),
        "workgroups_per_cu": dict(sorted((int(k), v) for k, v in per_cu.items())),
        "max_concurrent_per_cu": int(max(conc)) if conc else None,
        "cus_reaching_max": int(sum(1 for c in conc if c == max(conc))) if conc else None,
        "start_us_quantiles": [round(float(np.percentile(s, q)), 1) for q in (0, 25, 50, 75, 100)],
        "start_us_max": round(float(s.max()), 1),
        "end_us_max": round(float(e.max()), 1),
        "per_cu_leaf_end_us_by_rank": ranks.mean(0).round(1).tolist() if len(ranks) else None,
        "first_block_us": [round(float(np.percentile(f - s, q)), 1) for q in (0, 50, 100)],
        "subtree_us_median": round(float(np.median(e - l)), 1),
        "shader_mhz_median": round(float(np.median(mhz)), 0),
        "shader_mhz_by_xcc": [round(float(np.median(mhz[xcc == x])), 0) for x in range(8)],
    }


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(json.dumps(summary(p)))
