#!/usr/bin/env python3
"""Where in a decode step the GPU idles: split a rocprofv3 kernel trace (csv) into steps at each
``embed_kernel`` after the last flash prefill, and print every gap above ``--min-us`` with its
position in the step (dispatch index and the kernels around it).
usage: step_gaps.py kernel_trace.csv [--min-us 5]"""
import argparse
import collections
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from prof_summary import short  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-us", type=float, default=5.0)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    last = max((i for i, k in enumerate(ks) if "flash_prefill" in k[2]), default=-1)
    ks = ks[last + 1:]
    steps, cur = [], []
    for k in ks:
        if "embed_kernel" in k[2] and cur:
            steps.append(cur)
            cur = []
        cur.append(k)
    steps.append(cur)
    where = collections.defaultdict(list)
    for si, st in enumerate(steps):
        for i, ((s0, e0, n0), (s1, e1, n1)) in enumerate(zip(st, st[1:])):
            g = (s1 - e0) / 1e3
            if g >= a.min_us:
                where[(i, n0[:28], n1[:28])].append(g)
        if si < 3:
            print(f"step {si}: {len(st)} kernels, span {(st[-1][1] - st[0][0]) / 1e3:.1f} us, "
                  f"busy {sum(e - s for s, e, _ in st) / 1e3:.1f} us")
    print(f"{'idx':>4} {'pred':28s} {'succ':28s} {'n':>4} {'mean_us':>8} {'sum_us':>9}")
    for (i, n0, n1), v in sorted(where.items(), key=lambda kv: -sum(kv[1]))[:25]:
        print(f"{i:4d} {n0:28s} {n1:28s} {len(v):4d} {sum(v) / len(v):8.1f} {sum(v):9.1f}")


if __name__ == "__main__":
    main()
