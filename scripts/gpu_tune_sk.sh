#!/bin/bash
# autotune gemm_sk decompositions with the engine's epilogues, then the headline bench on the new table
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/tune
rm -f llm_sharding_amd/ops/gemm_sk_tuning.json
timeout -k 10 800 python -u scripts/tune_gemm_sk.py --models llama2-7b,llama2-70b \
    > gpurun_out/tune/tune.jsonl 2> gpurun_out/tune/tune.err &&
cp llm_sharding_amd/ops/gemm_sk_tuning.json gpurun_out/tune/ &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tune/bench.log 2>&1
echo "rc=$?"
