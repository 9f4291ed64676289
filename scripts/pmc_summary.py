"""Aggregate rocprofv3 counter_collection.csv files: per gemv dispatch, counters summed over
instances; dispatches grouped in order (6 per M value in scripts/gemv_pmc.py)."""
import csv, glob, sys, collections
rows = collections.OrderedDict()
for f in sorted(glob.glob(sys.argv[1] + "/g*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "gemv_packed" not in r["Kernel_Name"]:
            continue
        key = (f, int(r["Dispatch_Id"]))
        d = rows.setdefault(key, {"name": r["Kernel_Name"].split("<")[1].split(">")[0], "vgpr": r["VGPR_Count"],
                                  "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
by_file = collections.defaultdict(list)
for (f, _), d in rows.items():
    by_file[f].append(d)
Ms = [1, 16, 32, 64]
merged = [dict() for _ in Ms]
for f, ds in by_file.items():
    for i, d in enumerate(ds):
        g = i // 6
        if g < len(Ms) and i % 6 >= 2:  # skip the first 2 (cold) of each group
            for k, v in d.items():
                if isinstance(v, float) and k != "dur":
                    merged[g][k] = merged[g].get(k, 0) + v / 4
            merged[g]["name"] = d["name"]; merged[g]["vgpr"] = d["vgpr"]
            merged[g].setdefault("durs", []).append(d["dur"])
for M, d in zip(Ms, merged):
    print(f"M={M:2d} cfg<{d.get('name')}> vgpr={d.get('vgpr')} dur_us~{sorted(d.get('durs',[0]))[len(d.get('durs',[0]))//2]:.1f}")
    for k in sorted(k for k in d if k not in ("name", "vgpr", "durs")):
        print(f"    {k:36s} {d[k]:16.0f}")
