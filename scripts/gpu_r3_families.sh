#!/bin/bash
# Round 3 final kernels on the other model families (one GPU, 512 sequences; 70B: 128 sequences, all 80 layers)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/fam
for m in llama3.2-3b llama2-13b gpt2-xl; do
  timeout -k 10 400 python -u bench.py --model $m --steps 20 --warmup 5 --mid-batch 0 > gpurun_out/fam/$m.log 2>&1 || { tail -20 gpurun_out/fam/$m.log; exit 3; }
  echo "$m $(tail -1 gpurun_out/fam/$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["b1_p50_tpot_ms"])')"
done
timeout -k 10 600 python -u bench.py --model llama2-70b --batch 128 --steps 10 --warmup 3 --mid-batch 0 > gpurun_out/fam/llama2-70b.log 2>&1 || { tail -20 gpurun_out/fam/llama2-70b.log; exit 4; }
echo "llama2-70b $(tail -1 gpurun_out/fam/llama2-70b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["b1_p50_tpot_ms"])')"
