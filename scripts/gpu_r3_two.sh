#!/bin/bash
# gemm_sk two-contributor split-K without the last arriver's slab store: tests, M=512 re-tune, headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_two_test.log 2>&1 || { tail -30 gpurun_out/r3_two_test.log; exit 3; }
tail -1 gpurun_out/r3_two_test.log
cp llm_sharding_amd/ops/gemm_sk_tuning.json gpurun_out/r3_two_tuning.json
timeout -k 10 600 python scripts/tune_gemm_sk.py --rows ${ROWS:-512} --out gpurun_out/r3_two_tuning.json \
    > gpurun_out/r3_two_tune.jsonl 2>&1 || { tail -20 gpurun_out/r3_two_tune.jsonl; exit 5; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_two_tune.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["shape"], d["M"], d["best_us"], d["best"], d.get("partial", {}) and d["partial"].get("best"), d.get("partial", {}) and d["partial"].get("fused_us"))
PY
cp gpurun_out/r3_two_tuning.json llm_sharding_amd/ops/gemm_sk_tuning.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_two_bench.log 2>&1 || { tail -20 gpurun_out/r3_two_bench.log; exit 6; }
tail -1 gpurun_out/r3_two_bench.log | cut -c1-400
