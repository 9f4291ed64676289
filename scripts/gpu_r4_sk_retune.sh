#!/bin/bash
# gemm_sk re-tune at the headline rows with pure stream-K candidates, then headline A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_sk
mkdir -p $out
rm -f $out/*
cp llm_sharding_amd/ops/gemm_sk_tuning.json $out/old.json
cp llm_sharding_amd/ops/gemm_sk_tuning.json $out/tuning.json
timeout -k 10 600 python3 scripts/tune_gemm_sk.py --rows 448,512 --models llama2-7b --out $out/tuning.json \
    > $out/tune.jsonl 2> $out/tune.err || { tail -20 $out/tune.err; exit 2; }
for i in 1 2; do
  cp $out/old.json llm_sharding_amd/ops/gemm_sk_tuning.json
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 0 > $out/b_old.log 2>&1 || { tail -20 $out/b_old.log; exit 3; }
  echo "old $(grep '^\[bench\] load' $out/b_old.log)"
  cp $out/tuning.json llm_sharding_amd/ops/gemm_sk_tuning.json
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 0 > $out/b_new.log 2>&1 || { tail -20 $out/b_new.log; exit 4; }
  echo "new $(grep '^\[bench\] load' $out/b_new.log)"
done
