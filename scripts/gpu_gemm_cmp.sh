#!/bin/bash
# decode-size gemm_sk vs coop GEMV, and gemm_sk vs hipBLASLt at decode/prefill M
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/cmp
timeout -k 10 300 python -u scripts/gemm_vs_coop.py llama2-7b 32,64,96,128 > gpurun_out/cmp/coop.jsonl 2> gpurun_out/cmp/coop.err &&
timeout -k 10 300 python -u scripts/gemm_vs_hipblaslt.py > gpurun_out/cmp/blas.jsonl 2> gpurun_out/cmp/blas.err
echo "rc=$?"
