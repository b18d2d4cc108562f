#!/usr/bin/env python3
"""Collect the JSON result lines of a tools/gpu_run.sh call into one profiles/
file: every line of gpurun_out/<TAG>/<step>.out that parses as a JSON object,
tagged with the step it came from, plus the exit status the runner expected
for the wcorrupt / corrupt steps (they must exit 1).

    python3 tools/collect_lines.py gpurun_out/r05a profiles/multirank_r05.jsonl "<runner command>"
"""
import glob
import json
import os
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    cmd = sys.argv[3] if len(sys.argv) > 3 else ""
    out = [json.dumps({"source": "tools/gpu_run.sh", "command": cmd, "dir": src})]
    for f in sorted(glob.glob(os.path.join(src, "*.out"))):
        step = os.path.basename(f)[:-4]
        for line in open(f, errors="replace"):
            line = line.strip()
            if not line.startswith("{"):
                continue
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if not isinstance(d, dict) or "metric" not in d:
                continue
            d = dict({"step": step}, **d)
            if step.startswith(("wcorrupt", "corrupt")) or step.endswith("_corrupt"):
                d["expected_exit"] = 1
            out.append(json.dumps(d))
    with open(dst, "w") as fh:
        fh.write("\n".join(out) + "\n")
    print("%d lines -> %s" % (len(out) - 1, dst))


if __name__ == "__main__":
    main()
