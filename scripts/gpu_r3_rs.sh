#!/bin/bash
# gemm_sk role-split rings (nb = 4): numerics, then a tuning sweep over nb 0 / 4 at the 7B decode sizes.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_rs_test.log 2>&1 || { tail -30 gpurun_out/r3_rs_test.log; exit 3; }
tail -2 gpurun_out/r3_rs_test.log
timeout -k 10 900 python scripts/tune_gemm_sk.py --rows ${ROWS:-256,512,1024} --no-partial --nbs 0,4 \
    --out gpurun_out/r3_rs_tuning.json > gpurun_out/r3_rs_tune.jsonl 2>&1 || { tail -20 gpurun_out/r3_rs_tune.jsonl; exit 5; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_rs_tune.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        b0 = min((r for r in d["all"] if r[4] == 0), default=None)
        b4 = min((r for r in d["all"] if r[4] == 4), default=None)
        print(d["shape"], d["M"], "nb0", b0, "nb4", b4)
PY
