#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv files) + derived
ratios. usage: pmc_hot_summary.py DIR [DIR ...]  (each DIR one rocprofv3 -d output)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per-dispatch values]
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(lambda: defaultdict(float))
            for r in csv.DictReader(open(f)):
                per[(r["Kernel_Name"], r.get("Dispatch_Id", r.get("Correlation_Id")))][r["Counter_Name"]] += float(r["Counter_Value"])
            for (k, _), cs in per.items():
                for c, v in cs.items():
                    vals[k][c].append(v)
    for k, cs in sorted(vals.items()):
        short = k.replace("(anonymous namespace)::", "").split("(")[0].strip()[-100:]
        print(short)
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        for c in sorted(avg):
            print(f"    {c:36s} {avg[c]:18.0f}")
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg and avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"] > 0:
            print(f"    {'L2 hit rate':36s} {avg['TCC_HIT_sum'] / (avg['TCC_HIT_sum'] + avg['TCC_MISS_sum']):18.3f}")
        if "SQ_INSTS_LDS" in avg and avg["SQ_INSTS_LDS"] and "SQ_LDS_BANK_CONFLICT" in avg:
            print(f"    {'LDS bank-conflict cycles / LDS inst':36s} {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_INSTS_LDS']:18.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and avg.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs; MFMA-busy cycles over all 1024 SIMDs
            # (16 per v_mfma_f32_16x16x32_bf16: SQ_INSTS_MFMA x 16 == SQ_VALU_MFMA_BUSY_CYCLES)
            gpu_cyc = avg["GRBM_GUI_ACTIVE"] / 8
            print(f"    {'GPU-active cycles (per XCD)':36s} {gpu_cyc:18.0f}")
            print(f"    {'MFMA utilisation (1024 SIMDs)':36s} {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (gpu_cyc * 1024):18.3f}")
        if "FETCH_SIZE" in avg and avg.get("GRBM_GUI_ACTIVE"):
            us = avg["GRBM_GUI_ACTIVE"] / 8 / 1.9e3  # ~1.9 GHz under load
            print(f"    {'fabric fetch GB/s (FETCH_SIZE, ~1.9 GHz)':36s} {avg['FETCH_SIZE'] * 1024 / us / 1e3:18.1f}")


if __name__ == "__main__":
    main()
