#!/bin/bash
# rocprofv3 kernel traces of the bench at two batch sizes (kernel-trace + stats only, no PMC).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in ${BATCHES:-1 64}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b$B -o run -- \
      python3 bench.py --batch $B --steps 16 --warmup 2 > gpurun_out/prof_b$B.log 2>&1 || { tail -20 gpurun_out/prof_b$B.log; exit 1; }
  tail -1 gpurun_out/prof_b$B.log | cut -c1-200
  f=$(find gpurun_out/prof_b$B -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_gaps.py "$f" --tail 0.3 > gpurun_out/prof_b$B.gaps.txt || exit 1
  head -12 gpurun_out/prof_b$B.gaps.txt
done
