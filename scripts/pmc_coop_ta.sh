#!/bin/bash
# TA / L1 / L2-latency counters of the coop GEMV at M=$M (default 64): is the kernel bound by
# the texture-address path, by L2 latency or by neither? One counter group per rocprofv3 run.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
rm -rf gpurun_out/pmct
i=0
for grp in "TA_TA_BUSY TA_BUFFER_TOTAL_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ" \
           "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmct/g$i -o run -- python3 scripts/coop_pmc.py > gpurun_out/pmct_g$i.log 2>&1 || { echo "group $i failed"; tail -3 gpurun_out/pmct_g$i.log; exit 1; }
done
python3 scripts/pmc_coop_summary.py gpurun_out/pmct
