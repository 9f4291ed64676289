#!/usr/bin/env python3
"""Per-kernel stats of a rocprofv3 --kernel-trace CSV, split into the window after the last
dispatch of a marker kernel (default: the flash prefill = the decode window).
usage: kstats.py run_kernel_trace.csv [marker] [top]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "flash_prefill"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = max((i for i, r in enumerate(rows) if marker in r["Kernel_Name"]), default=-1)
    for title, sel in (("after last " + marker, rows[last + 1:]), ("whole run", rows)):
        agg = collections.defaultdict(list)
        for r in sel:
            agg[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        tot = sum(sum(v) for v in agg.values())
        if not sel:
            continue
        span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
        print(f"# {title}: {len(sel)} dispatches, {tot / 1e3:.2f} ms kernel time, span {span / 1e3:.2f} ms "
              f"(GPU busy {100 * tot / max(span, 1e-9):.1f}%)")
        print(f"{'kernel':90s} {'calls':>6} {'avg_us':>9} {'total_ms':>9} {'%':>6}")
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
            print(f"{k[:90]:90s} {len(v):6d} {sum(v) / len(v):9.2f} {sum(v) / 1e3:9.3f} {100 * sum(v) / tot:6.2f}")
        print()


if __name__ == "__main__":
    main()
