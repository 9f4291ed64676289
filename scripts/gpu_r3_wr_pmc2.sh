#!/bin/bash
# PMC counters of gemm_wr at the 7B qkv decode shape (M=512, bn 192, grid 256), one pass per group
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/wrpmc2
export TMPDIR=/tmp
export WR_ONLY=192,1,256
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "GRBM_GUI_ACTIVE TA_BUSY_avr SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d gpurun_out/wrpmc2/p$i -o run --output-format csv -- python3 scripts/gemm_wr_probe.py 512,12288,4096 > gpurun_out/wrpmc2/p$i.log 2>&1 || { tail -5 gpurun_out/wrpmc2/p$i.log; exit 3; }
done
python3 - << 'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/wrpmc2/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gemm_wr" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f, {k: round(sum(v) / len(v), 1) for k, v in acc.items()})
PY
