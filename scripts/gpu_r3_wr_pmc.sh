#!/bin/bash
# PMC counters of the W-in-registers GEMM at M=16384 N=K=4096 (bn 256, p 2, grid 512)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wrpmc
export TMPDIR=/tmp
export WR_ONLY=256,1,512
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/wrpmc/p$i -o run --output-format csv -- python3 scripts/gemm_wr_probe.py 16384,4096,4096 > gpurun_out/wrpmc/p$i.log 2>&1 || { tail -5 gpurun_out/wrpmc/p$i.log; exit 3; }
done
python3 - << 'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/wrpmc/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gemm_wr" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: sum(v) / len(v) for k, v in acc.items()})
PY
