#!/bin/bash
# gemm_sk with non-temporal weight DMA at decode sizes: tests, re-tune the 7B decode shapes, headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py tests/test_attn_gqa_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_nt_test.log 2>&1 || { tail -30 gpurun_out/r3_nt_test.log; exit 3; }
tail -2 gpurun_out/r3_nt_test.log
timeout -k 10 300 python scripts/attn_gqa_bench.py > gpurun_out/r3_gqa_bench2.jsonl 2>&1 || { tail -20 gpurun_out/r3_gqa_bench2.jsonl; exit 4; }
timeout -k 10 600 python scripts/tune_gemm_sk.py --rows 256,384,512,640,768,1024 --no-partial > gpurun_out/r3_tune_nt.jsonl 2>&1 || { tail -20 gpurun_out/r3_tune_nt.jsonl; exit 5; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_tune_nt.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["shape"], d["M"], d["best_us"], d["best"])
PY
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_bench_nt.log 2>&1 || { tail -20 gpurun_out/r3_bench_nt.log; exit 6; }
tail -1 gpurun_out/r3_bench_nt.log
