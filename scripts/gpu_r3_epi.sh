#!/bin/bash
# coop epilogue with static quad reads: kernel tests, stamps, 7B decode sweep (re-tune into gpurun_out), bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "coop or gemv or qkv" \
    > gpurun_out/r3_epi_test.log 2>&1 || { tail -30 gpurun_out/r3_epi_test.log; exit 3; }
tail -1 gpurun_out/r3_epi_test.log
if [ -f llm_sharding_amd/_native/liblsa_coop_stamps.so ]; then
  timeout -k 10 300 python scripts/coop_stamps.py 64 128 > gpurun_out/r3_coop_stamps2.txt 2>&1 || { tail -20 gpurun_out/r3_coop_stamps2.txt; exit 4; }
  grep -E "M=|tile|epi " gpurun_out/r3_coop_stamps2.txt
fi
cp llm_sharding_amd/ops/gemv_tuning.json gpurun_out/r3_gemv_tuning_epi.json
timeout -k 10 600 python scripts/bench_kernels.py --only gemv --models llama2-7b --rows ${ROWS:-32,64,128} --tune \
    --tune-file gpurun_out/r3_gemv_tuning_epi.json --out gpurun_out/r3_epi_sweep.json > gpurun_out/r3_epi_sweep.jsonl 2>&1 \
    || { tail -20 gpurun_out/r3_epi_sweep.jsonl; exit 5; }
python - << 'PY'
import json
for l in open("gpurun_out/r3_epi_sweep.jsonl"):
    if l.startswith("{"):
        d = json.loads(l); print(d["shape"], d["M"], d["best_us"], d["best_algo"], d["best_cfg"], d["best_TBps"])
PY
cp gpurun_out/r3_gemv_tuning_epi.json llm_sharding_amd/ops/gemv_tuning.json
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r3_epi_bench.log 2>&1 || { tail -20 gpurun_out/r3_epi_bench.log; exit 6; }
tail -1 gpurun_out/r3_epi_bench.log | cut -c1-900
