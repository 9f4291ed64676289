#!/bin/bash
# re-tune the 7B decode projections at 32-128 rows with the ring-depth-4 coop configs, then the
# batch-128 step on the old and the re-tuned table
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_retune
mkdir -p $out
rm -f $out/*
timeout -k 10 200 python3 bench.py --batch 128 --steps 32 --warmup 8 --latency-steps 0 --mid-batch 0 > $out/mid_old.log 2>&1 || { tail -20 $out/mid_old.log; exit 3; }
echo "old $(grep '^\[bench\] load' $out/mid_old.log)"
timeout -k 10 700 python3 scripts/bench_kernels.py --only gemv --models llama2-7b --rows 128,64,32 --tune \
    --tune-file $out/tuning.json --out $out/sweep.json > $out/sweep.jsonl 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 4; }
cp $out/tuning.json llm_sharding_amd/ops/gemv_tuning.json
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --batch 128 --steps 32 --warmup 8 --latency-steps 0 --mid-batch 0 > $out/mid_new.log 2>&1 || { tail -20 $out/mid_new.log; exit 5; }
  echo "new $(grep '^\[bench\] load' $out/mid_new.log)"
done
