#!/bin/bash
# PMC counters (one group per rocprofv3 run, kernel-trace only) for the GEMV shapes.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
python csrc/build.py > /dev/null || exit 2
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES" \
           "TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY" \
           "TCC_HIT TCC_MISS TCC_EA0_RDREQ"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run -- python3 scripts/gemv_pmc.py > gpurun_out/pmc_g$i.log 2>&1 || { echo "group $i failed"; tail -5 gpurun_out/pmc_g$i.log; }
done
ls -R gpurun_out/pmc | head
