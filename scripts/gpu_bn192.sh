#!/bin/bash
# BN=192 gemm_sk: numerics tests, then the autotuner with 192 candidates and the headline bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/b192
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/b192/pytest.log 2>&1 &&
rm -f llm_sharding_amd/ops/gemm_sk_tuning.json &&
timeout -k 10 500 python -u scripts/tune_gemm_sk.py --models llama2-7b,llama2-70b \
    > gpurun_out/b192/tune.jsonl 2> gpurun_out/b192/tune.err &&
cp llm_sharding_amd/ops/gemm_sk_tuning.json gpurun_out/b192/ &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b192/bench.log 2>&1
echo "rc=$?"
