#!/bin/bash
# rocprofv3 counter passes (one run each, no tracing domains) over scripts/pmc_hot.py
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM \
    -d gpurun_out/pmc/p1 -o run --output-format csv -- python3 scripts/pmc_hot.py > gpurun_out/pmc/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    -d gpurun_out/pmc/p2 -o run --output-format csv -- python3 scripts/pmc_hot.py > gpurun_out/pmc/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE \
    -d gpurun_out/pmc/p3 -o run --output-format csv -- python3 scripts/pmc_hot.py > gpurun_out/pmc/p3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE \
    -d gpurun_out/pmc/p4 -o run --output-format csv -- python3 scripts/pmc_hot.py > gpurun_out/pmc/p4.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o run -- python3 scripts/pmc_hot.py > gpurun_out/pmc/kt.log 2>&1
echo "rc=$?"
