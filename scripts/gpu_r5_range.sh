#!/bin/bash
# round-5 operating range on the final kernels: Llama-3.2-3B / 13B / GPT-2 XL at 512 sequences,
# long-context decode (32 x 4k, 64 x 2k), 1024 x 128, and the serving load test
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r5_range
mkdir -p $out
rm -f $out/*
line() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["p50_tpot_ms"], d.get("b1_p50_tpot_ms"), d.get("ttft_ms"), d.get("mem_peak_gb"))'; }
for m in llama3.2-3b llama2-13b gpt2-xl; do
  timeout -k 10 300 python3 -u bench.py --model $m --steps 20 --warmup 5 --ttft-lens 0 --extras= > $out/$m.log 2>&1 || { tail -20 $out/$m.log; exit 2; }
  echo "$m: $(grep '^{' $out/$m.log | tail -1 | line)"
done
for cfg in "32 4000" "64 2000" "1024 128"; do
  set -- $cfg
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --latency-steps 0 --ttft-lens 0 --extras= --batch $1 --prompt-len $2 > $out/b$1_p$2.log 2>&1 || { tail -20 $out/b$1_p$2.log; exit 3; }
  echo "batch $1 prompt $2: $(grep '^{' $out/b$1_p$2.log | tail -1 | line)"
done
timeout -k 10 300 python3 -u serve.py --model llama2-7b --requests 1024 --prompt-len 128 --max-new-tokens 128 --batch 512 \
    --max-seq 320 --microbatches 1 > $out/serve.log 2>&1 || { tail -20 $out/serve.log; exit 4; }
grep '^{' $out/serve.log | tail -1
