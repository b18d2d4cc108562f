#!/usr/bin/env python3
"""HBM traffic per launch of one kernel from tools/gpu_pmc.sh's rocprofv3 --pmc
passes (counter_collection CSVs under DIR), corrected as MI355X_MICROARCH.md's
HBM section prescribes for gfx950: FETCH_SIZE (KB) x 1024 x 2 for 16-B/lane
streaming reads (tallied at 64 B per 128-B request), WRITE_SIZE (KB) x 1024.

usage: traffic_json.py DIR KERNEL_SUBSTRING LABEL ALG_BYTES > out.json"""
import collections
import csv
import glob
import json
import sys


def main():
    d, match, label, alg = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    acc = collections.defaultdict(list)
    for p in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if match in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: sum(v) / len(v) for k, v in acc.items()}
    rd = c["FETCH_SIZE"] * 1024 * 2
    wr = c["WRITE_SIZE"] * 1024
    print(json.dumps({
        "kernel": label,
        "source": "rocprofv3 --kernel-trace --pmc, separate passes (tools/gpu_pmc.sh), mean over dispatches",
        "counters": c,
        "correction": "FETCH_SIZE (KB) x 1024 x 2: gfx950 tallies 128-B requests of 16-B/lane streaming "
                      "reads at 64 B (MI355X_MICROARCH.md HBM section); WRITE_SIZE (KB) x 1024 exact for "
                      "16-B stores",
        "hbm_read_bytes_per_launch": rd,
        "hbm_write_bytes_per_launch": wr,
        "hbm_bytes_per_launch": rd + wr,
        "algorithmic_bytes_per_launch": alg}, indent=1))


if __name__ == "__main__":
    main()
