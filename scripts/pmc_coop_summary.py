"""Aggregate rocprofv3 counter_collection.csv of scripts/coop_pmc.py: per shape (8 launches
in order qkv, o, down, gate_up; the first 2 of each skipped as cold), mean counters per
dispatch and derived ratios."""
import collections
import csv
import glob
import sys

SHAPES = ["qkv", "o", "down", "gate_up"]
per_file = collections.defaultdict(lambda: collections.OrderedDict())
for f in sorted(glob.glob(sys.argv[1] + "/g*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "gemv" not in r["Kernel_Name"]:
            continue
        d = per_file[f].setdefault(int(r["Dispatch_Id"]), {
            "name": r["Kernel_Name"].split("<")[1].split(">")[0], "vgpr": r.get("VGPR_Count"),
            "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
agg = [collections.defaultdict(list) for _ in SHAPES]
for f, ds in per_file.items():
    for i, d in enumerate(ds.values()):
        g, j = divmod(i, 8)
        if g < len(SHAPES) and j >= 2:
            for k, v in d.items():
                agg[g][k].append(v)
for name, a in zip(SHAPES, agg):
    if not a:
        continue
    med = lambda xs: sorted(xs)[len(xs) // 2]
    print(f"{name:8s} cfg<{a['name'][0]}> vgpr={a['vgpr'][0]} dur_us~{med(a['dur']):.1f}")
    vals = {k: sum(v) / len(v) for k, v in a.items() if k not in ("name", "vgpr", "dur")}
    for k in sorted(vals):
        print(f"    {k:32s} {vals[k]:16.0f}")
    wc = vals.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_VALU"):
            if k in vals:
                print(f"    {k + ' / wave_cycles':44s} {vals[k] / wc:8.3f}")
    if vals.get("SQ_INSTS_LDS"):
        print(f"    {'LDS bank conflicts / LDS inst':44s} {vals.get('SQ_LDS_BANK_CONFLICT', 0) / vals['SQ_INSTS_LDS']:8.3f}")
