#!/bin/bash
# coop EPI_PARTIAL: numerics, then fused vs partial timing for the residual decode projections.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "partials or coop or big_batch" > gpurun_out/r3_partial_test.log 2>&1 || { tail -30 gpurun_out/r3_partial_test.log; exit 3; }
tail -1 gpurun_out/r3_partial_test.log
cp llm_sharding_amd/ops/gemv_tuning.json gpurun_out/r3_gemv_tuning_partial.json
timeout -k 10 400 python scripts/tune_coop_partial.py --models ${MODELS:-llama2-7b} --rows ${ROWS:-32,48,64,96,128} \
    --tune-file gpurun_out/r3_gemv_tuning_partial.json > gpurun_out/r3_coop_partial.jsonl 2>&1 || { tail -20 gpurun_out/r3_coop_partial.jsonl; exit 4; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_coop_partial.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["shape"], d["M"], "fused", d["fused_us"], d["fused_cfg"], "partial", d["partial_best"])
PY
