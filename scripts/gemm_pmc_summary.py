#!/usr/bin/env python3
"""Summarise rocprofv3 passes over scripts/gemm_pmc_probe.py: every GEMM dispatch is attributed to
its (impl, shape) block (blocks are separated by the probe's 1-element fill kernel; segments with
no GEMM kernel are dropped), counters are averaged over the block's dispatches (the first one,
cold instruction cache, skipped), durations come from a --kernel-trace pass.

usage: gemm_pmc_summary.py PROBE_LOG OUT_DIR [OUT_DIR ...]   -> one JSON line per block
Derived per block: clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA busy share, L2 hit rate,
L2->CU read bytes (TCP_TCC_READ_REQ x 128 B) per CU per second, HBM-side read bytes
(TCC_EA0_RDREQ x 64 B, halved by the counter on gfx950: MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import json
import sys

GEMM_TAGS = ("gemm_sk", "gemm_wr", "Cijk", "gemm_kernel", "gemv")


def is_gemm(name: str) -> bool:
    return any(t in name for t in GEMM_TAGS)


def segments(rows):
    """rows: dispatch dicts sorted by id -> list of per-block lists of GEMM dispatches."""
    segs, cur = [], []
    for r in rows:
        if "FillFunctor" in r["Kernel_Name"] or "fill" in r["Kernel_Name"].lower():
            if cur:
                segs.append(cur)
            cur = []
        elif is_gemm(r["Kernel_Name"]):
            cur.append(r)
    if cur:
        segs.append(cur)
    return segs


def main():
    blocks = None
    for ln in open(sys.argv[1]):
        if ln.startswith('{"blocks"'):
            blocks = json.loads(ln)["blocks"]
    assert blocks, "no block list in the probe log"
    res = [dict(b, counters={}, dur_us=None, kernels=set()) for b in blocks]
    for d in sys.argv[2:]:
        for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            disp = collections.OrderedDict()
            for r in csv.DictReader(open(f)):
                k = int(r["Dispatch_Id"])
                e = disp.setdefault(k, {"Kernel_Name": r["Kernel_Name"], "Grid_Size": r.get("Grid_Size"), "c": {}})
                e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            rows = [disp[k] for k in sorted(disp)]
            segs = segments(rows)
            assert len(segs) == len(res), (f, len(segs), len(res))
            for b, seg in zip(res, segs):
                use = seg[1:] if len(seg) > 1 else seg
                for cn in use[0]["c"]:
                    b["counters"][cn] = sum(x["c"].get(cn, 0.0) for x in use) / len(use)
                b["kernels"].update(x["Kernel_Name"][:90] for x in seg)
        for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
            rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
            segs = segments(rows)
            assert len(segs) == len(res), (f, len(segs), len(res))
            for b, seg in zip(res, segs):
                use = seg[1:] if len(seg) > 1 else seg
                ds = sorted((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3 for x in use)
                b["dur_us"] = ds[len(ds) // 2]
    for b in res:
        c, t = b["counters"], b["dur_us"]
        out = {k: b[k] for k in ("impl", "shape", "M", "N", "K", "plan")}
        out["kernels"] = sorted(b["kernels"])
        out["dur_us"] = t
        if t:
            out["tflops"] = round(2.0 * b["M"] * b["N"] * b["K"] / t / 1e6, 1)
        if t and "GRBM_GUI_ACTIVE" in c:
            out["clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (t * 1e3), 3)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # MFMA busy cycles summed over SIMDs vs 1024 SIMDs x active cycles (per XCD count / 8)
            out["mfma_busy_pct"] = round(100.0 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8), 1)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
            out["l2_hit_pct"] = round(100.0 * c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 1)
        if t and "TCP_TCC_READ_REQ_sum" in c:
            out["l2_to_cu_GBps_per_cu_at128B"] = round(c["TCP_TCC_READ_REQ_sum"] * 128 / (t * 1e-6) / 256 / 1e9, 1)
            out["l2_to_cu_MB_at128B"] = round(c["TCP_TCC_READ_REQ_sum"] * 128 / 1e6, 1)
        if t and "TCC_EA0_RDREQ_sum" in c:
            out["hbm_read_MB_x2"] = round(c["TCC_EA0_RDREQ_sum"] * 64 * 2 / 1e6, 1)
            out["hbm_read_TBps_x2"] = round(c["TCC_EA0_RDREQ_sum"] * 128 / (t * 1e-6) / 1e12, 2)
        out["counters"] = {k: round(v, 1) for k, v in sorted(c.items())}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
