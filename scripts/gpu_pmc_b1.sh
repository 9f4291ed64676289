#!/bin/bash
# rocprofv3 counter passes (one run each, no tracing domains) over scripts/pmc_b1.py
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
rm -rf gpurun_out/pmcb1 && mkdir -p gpurun_out/pmcb1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE \
    -d gpurun_out/pmcb1/p1 -o run --output-format csv -- python3 scripts/pmc_b1.py > gpurun_out/pmcb1/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT \
    -d gpurun_out/pmcb1/p2 -o run --output-format csv -- python3 scripts/pmc_b1.py > gpurun_out/pmcb1/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
    -d gpurun_out/pmcb1/p3 -o run --output-format csv -- python3 scripts/pmc_b1.py > gpurun_out/pmcb1/p3.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmcb1/kt -o run -- python3 scripts/pmc_b1.py > gpurun_out/pmcb1/kt.log 2>&1
echo "rc=$?"
