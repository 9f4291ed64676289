#!/bin/bash
# skinny_gemm.hip: numerics vs fp32, then the 7B decode-projection sweep (gemv / coop / skinny) at 32-128 rows.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_skinny_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r3_skinny_test.log 2>&1 || { tail -30 gpurun_out/r3_skinny_test.log; exit 3; }
tail -2 gpurun_out/r3_skinny_test.log
timeout -k 10 600 python scripts/bench_kernels.py --only gemv --models ${MODELS:-llama2-7b} --rows ${ROWS:-32,64,128} \
    --out gpurun_out/r3_skinny_sweep.json > gpurun_out/r3_skinny_sweep.jsonl 2>&1 || { tail -20 gpurun_out/r3_skinny_sweep.jsonl; exit 4; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_skinny_sweep.jsonl"):
    if not l.startswith("{"):
        continue
    d = json.loads(l)
    best = {}
    for r in d["all"]:
        if r[1] not in best or r[0] < best[r[1]][0]:
            best[r[1]] = r
    print(d["shape"], d["M"], {k: (v[0], round(d["N"] * d["K"] * 2 / v[0] / 1e6, 2), v[2:]) for k, v in best.items()})
PY
timeout -k 10 300 python scripts/skinny_ablate.py 128 4096 4096 4 4 2 4  128 12288 4096 3 4 3 1  128 12288 4096 6 4 2 2  128 4096 11008 4 4 2 4 \
    > gpurun_out/r3_skinny_ablate2.jsonl 2>&1 || { tail -20 gpurun_out/r3_skinny_ablate2.jsonl; exit 5; }
cat gpurun_out/r3_skinny_ablate2.jsonl
