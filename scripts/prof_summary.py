#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv (short names, calls, avg/min us, share)."""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)<([^>]*)>", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.search(r"::(\w+_kernel)\(", name)
    if m:
        return m.group(1)
    if "at::native" in name:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(\w+)", name)
        return "torch::" + (m.group(1) if m else "op")
    return name[:60]


def main(path: str, top: int = 25) -> None:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':60s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'total_ms':>9s} {'%':>6s}")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{short(r['Name']):60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} "
              f"{float(r['MinNs'])/1e3:9.2f} {float(r['TotalDurationNs'])/1e6:9.3f} "
              f"{100*float(r['TotalDurationNs'])/tot:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
