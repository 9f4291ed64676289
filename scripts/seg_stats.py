#!/usr/bin/env python3
"""Per-segment kernel breakdown of a rocprofv3 kernel trace (CSV or rocpd .db): a new segment starts at every
dispatch of a marker kernel (default embed_kernel = one forward). usage: seg_stats.py csv [marker] [min_us]"""
import collections
import csv
import re
import sys


def short(name):
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    m = re.match(r"([A-Za-z_0-9:]+)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or ""))[:70] if m else n[:70]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "embed_kernel"
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 1000
    if path.endswith(".db"):  # rocprofv3 >= 7 default output (rocpd sqlite)
        import sqlite3
        con = sqlite3.connect(path)
        rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
                for n, s, e in con.execute("select name, start, end from kernels")]
    else:
        rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    segs, cur = [], []
    for r in rows:
        if marker in r["Kernel_Name"] and cur:
            segs.append(cur)
            cur = []
        cur.append(r)
    segs.append(cur)
    for s in segs:
        agg, n = collections.defaultdict(float), collections.Counter()
        for r in s:
            k = short(r["Kernel_Name"])
            agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            n[k] += 1
        tot = sum(agg.values())
        if tot < min_us:
            continue
        span = (int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3
        print(f"segment: {len(s)} kernels, span {span:.0f} us, kernel sum {tot:.0f} us")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:8]:
            print(f"   {k:70s} {n[k]:5d} {v:9.1f} us {v / n[k]:8.1f} avg")


if __name__ == "__main__":
    main()
