#!/usr/bin/env python3
"""Busy vs idle time of the GPU in a rocprofv3 kernel trace (kernel_trace.csv): over the
last ``--tail`` fraction of kernels (the timed decode steps), report span, summed kernel
time, idle gaps between consecutive kernels, and per-kernel averages."""
import argparse
import csv
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=float, default=0.3)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows))
    ks = ks[int(len(ks) * (1 - a.tail)):]
    span = ks[-1][1] - ks[0][0]
    busy = sum(e - s for s, e, _ in ks)
    gaps = [max(0, ks[i + 1][0] - ks[i][1]) for i in range(len(ks) - 1)]
    print(f"kernels {len(ks)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us ({100*busy/span:.1f}%)  "
          f"gap median {statistics.median(gaps)/1e3:.2f} us  mean {statistics.mean(gaps)/1e3:.2f} us")
    per = {}
    for s, e, n in ks:
        per.setdefault(n, []).append(e - s)
    print(f"{'kernel':70s} {'n':>5s} {'avg_us':>8s} {'sum_us':>9s}")
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:70s} {len(v):5d} {statistics.mean(v)/1e3:8.2f} {sum(v)/1e3:9.1f}")


if __name__ == "__main__":
    main()
