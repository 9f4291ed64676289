#!/bin/bash
# gemm_sk phase stamps at 128 rows (the mid-batch decode regime), tuned-plan configs
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r3_sk128_stamps.txt
: > $O
# M N K bn grid dp split reps bm
for cfg in "128 12288 4096 128 256 1 6 6 128" "128 12288 4096 128 256 1 2 6 128" "128 22016 4096 128 256 1 1 6 128" \
           "128 4096 11008 128 256 1 6 6 128" "128 4096 4096 128 256 1 6 6 128"; do
  timeout -k 10 120 python scripts/gemm_stamps.py $cfg >> $O 2>&1 || { echo "FAILED $cfg"; tail -5 $O; exit 3; }
done
grep -v amdgpu.ids $O
