#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters in this run).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
python csrc/build.py > gpurun_out/build.log 2>&1 || exit 2
OUT=${PROF_OUT:-gpurun_out/prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py ${BENCH_ARGS:---steps 16 --warmup 2} > gpurun_out/prof_bench.log 2>&1; rc=$?
tail -3 gpurun_out/prof_bench.log
find $OUT -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -30 "{}"'
exit $rc
