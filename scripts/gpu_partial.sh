#!/bin/bash
# EPI_PARTIAL + resid_rmsnorm_partials: numerics, engine vs golden, retune with partial candidates, bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/part
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/part/pytest.log 2>&1 &&
rm -f llm_sharding_amd/ops/gemm_sk_tuning.json &&
timeout -k 10 600 python -u scripts/tune_gemm_sk.py --models llama2-7b,llama2-70b \
    > gpurun_out/part/tune.jsonl 2> gpurun_out/part/tune.err &&
cp llm_sharding_amd/ops/gemm_sk_tuning.json gpurun_out/part/ &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/part/bench.log 2>&1
echo "rc=$?"
