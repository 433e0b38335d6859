#!/usr/bin/env python3
"""Timeline of the last host-API call in a rocprofv3 trace (kernels + memory copies):
usage: host_timeline.py <rocprof output dir> [--last-ms 10]
Prints each kernel / copy of the final call window with start offset, duration and gap."""
import csv
import glob
import sys


def rows(d, pat):
    f = glob.glob(d + f"/**/*{pat}.csv", recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    d = sys.argv[1]
    win = float(sys.argv[2]) if len(sys.argv) > 2 else 6.0
    ev = []
    for r in rows(d, "kernel_trace"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]))
    for r in rows(d, "memory_copy_trace"):
        n = f"C {r.get('Direction', '')} {int(r.get('Size', 0) or 0) / 1e6:.2f}MB"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n))
    ev.sort()
    end = max(e[1] for e in ev)
    # the last call: events after the largest idle gap within the final window
    tail = [e for e in ev if e[0] >= end - win * 1e6]
    gaps = [(tail[i + 1][0] - max(x[1] for x in tail[:i + 1]), i + 1) for i in range(len(tail) - 1)]
    start = max(gaps)[1] if gaps and max(gaps)[0] > 200e3 else 0
    call = tail[start:]
    t0 = call[0][0]
    busy_end = t0
    for s, e, n in call:
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - busy_end) / 1e3:7.1f}  {n}")
        busy_end = max(busy_end, e)
    print(f"call span {(busy_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
