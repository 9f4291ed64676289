#!/bin/bash
# gemm_sk phase stamps for stream-K decompositions at M = 512 (where does stream-K lose?)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r3_sk_stamps.txt
: > $O
# M N K bn grid dp split reps bm
for cfg in "512 12288 4096 256 256 1 0 6 256" "512 12288 4096 256 256 0 0 6 256" "512 22016 4096 256 256 1 0 6 256" \
           "512 4096 11008 256 256 1 0 6 256" "512 4096 11008 256 256 1 4 6 256" "512 4096 4096 256 256 1 0 6 256"; do
  timeout -k 10 120 python scripts/gemm_stamps.py $cfg >> $O 2>&1 || { echo "FAILED $cfg"; tail -5 $O; exit 3; }
done
grep -v amdgpu.ids $O
