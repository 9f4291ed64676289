#!/usr/bin/env python3
"""Idle gap between consecutive kernels of a rocprofv3 kernel trace (csv), grouped by the
(predecessor -> successor) kernel pair, over the decode steps of a bench run (kernels after the
last ``--after`` dispatch, default: the last flash-prefill). Tells where the per-step GPU idle
time of the decode loop goes. usage: gap_pairs.py kernel_trace.csv [--after NAME]"""
import argparse
import collections
import csv
import statistics
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--after", default="flash_prefill")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    last = max((i for i, k in enumerate(ks) if a.after in k[2]), default=-1)
    ks = ks[last + 1:]
    span = ks[-1][1] - ks[0][0]
    busy = sum(e - s for s, e, _ in ks)
    pairs = collections.defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
        pairs[(n0[:40], n1[:40])].append(max(0, s1 - e0) / 1e3)
    gap_tot = sum(sum(v) for v in pairs.values())
    print(f"kernels {len(ks)}  span {span / 1e3:.1f} us  busy {busy / 1e3:.1f} us ({100 * busy / span:.1f}%)  "
          f"idle {gap_tot:.1f} us")
    print(f"{'predecessor':40s} {'successor':40s} {'n':>5s} {'med_us':>7s} {'mean_us':>7s} {'sum_us':>9s}")
    for (p, q), v in sorted(pairs.items(), key=lambda kv: -sum(kv[1]))[:20]:
        print(f"{p:40s} {q:40s} {len(v):5d} {statistics.median(v):7.2f} {statistics.mean(v):7.2f} {sum(v):9.1f}")


if __name__ == "__main__":
    main()
