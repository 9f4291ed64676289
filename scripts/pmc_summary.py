#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per kernel (first dispatch of each kernel dropped) over one or
more pass directories (each holding a *counter_collection.csv).
usage: pmc_summary.py DIR [DIR ...]  -> one JSON line per kernel"""
import collections
import csv
import glob
import json
import sys


def main():
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            seen = collections.Counter()
            rows = list(csv.DictReader(open(p)))
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            names = {}
            for r in rows:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                names[key] = r["Kernel_Name"]
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            for key in sorted(per, key=lambda k: int(k)):
                k = names[key]
                seen[k] += 1
                if seen[k] == 1:
                    continue
                for c, v in per[key].items():
                    vals[k][c].append(v)
    for k, cs in vals.items():
        print(json.dumps({"kernel": k[:120], **{c: sum(v) / len(v) for c, v in sorted(cs.items())}}))


if __name__ == "__main__":
    main()
