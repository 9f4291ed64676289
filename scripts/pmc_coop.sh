#!/bin/bash
# PMC counters (one group per rocprofv3 run, kernel-trace only) for the coop GEMV at M=64.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
python csrc/build.py > /dev/null || exit 2
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM" \
           "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" \
           "TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCC_HIT TCC_MISS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcc/g$i -o run -- python3 scripts/coop_pmc.py > gpurun_out/pmcc_g$i.log 2>&1 || { echo "group $i failed"; tail -3 gpurun_out/pmcc_g$i.log; }
done
ls -R gpurun_out/pmcc | head -30
