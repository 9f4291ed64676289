#!/bin/bash
# TTFT sweep + headline-bench kernel trace in one call
set -o pipefail
cd "$(dirname "$0")/.."
rm -rf gpurun_out/ttft gpurun_out/pb
bash scripts/gpu_ttft.sh && bash scripts/gpu_prof_bench.sh
