#!/bin/bash
# re-decide coop partial entries after the epilogue fix; engine decode tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
cp llm_sharding_amd/ops/gemv_tuning.json gpurun_out/r3_gemv_tuning_partial2.json
timeout -k 10 400 python scripts/tune_coop_partial.py --rows 32,48,64,96,128 --tune-file gpurun_out/r3_gemv_tuning_partial2.json \
    > gpurun_out/r3_coop_partial2.jsonl 2>&1 || { tail -20 gpurun_out/r3_coop_partial2.jsonl; exit 4; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_coop_partial2.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["shape"], d["M"], "fused", d["fused_us"], d["fused_cfg"], "partial", d["partial_best"])
PY
cp gpurun_out/r3_gemv_tuning_partial2.json llm_sharding_amd/ops/gemv_tuning.json
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_full_depth_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_engine_test.log 2>&1 || { tail -30 gpurun_out/r3_engine_test.log; exit 3; }
tail -1 gpurun_out/r3_engine_test.log
