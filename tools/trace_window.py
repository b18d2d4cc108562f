"""Timeline of the last `span_us` of a rocprofv3 run: kernel and memory-copy
records in start order with durations and the idle gaps between them.
usage: trace_window.py <dir with *_kernel_trace.csv / *_memory_copy_trace.csv> [span_us]"""
import csv
import glob
import os
import sys


def rows(pattern, kind):
    out = []
    for p in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(p)):
            name = r.get("Kernel_Name") or r.get("Direction") or r.get("Operation") or kind
            if kind == "A":  # host API call (--hip-runtime-trace): thread and function
                name = "t%s %s" % (str(r.get("Thread_Id", ""))[-3:], r.get("Function", ""))
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name[:60]))
    return out


def main(d, span_us=6000.0):
    ev = rows(os.path.join(d, "**", "*kernel_trace.csv"), "K") + \
        rows(os.path.join(d, "**", "*memory_copy_trace.csv"), "C")
    # host API calls (when traced) are listed but do not count as device busy
    api = rows(os.path.join(d, "**", "*hip_api_trace.csv"), "A")
    if not ev:
        ev = rows(os.path.join(d, "*kernel_trace.csv"), "K") + rows(os.path.join(d, "*memory_copy_trace.csv"), "C")
    ev.sort()
    end = max(e[1] for e in ev)
    win = [e for e in ev + api if e[0] >= end - span_us * 1000 and e[0] <= end]
    win.sort()
    t0 = win[0][0]
    busy_end = t0
    for s, e, k, n in win:
        if k == "A":
            print("%9.1f %8.1f %s           %s" % ((s - t0) / 1000, (e - s) / 1000, k, n))
            continue
        gap = max(0, s - busy_end) / 1000
        print("%9.1f %8.1f %s gap %6.1f  %s" % ((s - t0) / 1000, (e - s) / 1000, k, gap, n))
        busy_end = max(busy_end, e)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 6000.0)
