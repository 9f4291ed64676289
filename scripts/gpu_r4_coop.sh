#!/bin/bash
# coop GEMV with 3 / 6 / 1-wave workgroups (no split for 768-tile qkv): fp32 tests, re-tune the
# 7B decode projections at 32-128 rows, batch-128 step A/B (old table vs re-tuned table)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/r4_coop
mkdir -p $out
rm -f $out/*
timeout -k 10 120 python3 scripts/probes/gemv_rows_diag.py > $out/diag.jsonl 2> $out/diag.err || { tail -20 $out/diag.err; exit 1; }
cat $out/diag.jsonl
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_wr_gpu.py -q --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1; rc=$?
tail -8 $out/pytest.log
grep -q "Timeout\|Fatal\|core dumped" $out/pytest.log && exit 2
timeout -k 10 200 python3 bench.py --batch 128 --steps 32 --warmup 8 --latency-steps 0 --mid-batch 0 > $out/mid_old.log 2>&1 || { tail -20 $out/mid_old.log; exit 3; }
echo "old $(grep '^\[bench\] load' $out/mid_old.log)"
timeout -k 10 600 python3 scripts/bench_kernels.py --only gemv --models llama2-7b --rows 128,64,32 --tune \
    --tune-file $out/tuning.json --out $out/sweep.json > $out/sweep.jsonl 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 4; }
cp $out/tuning.json llm_sharding_amd/ops/gemv_tuning.json
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --batch 128 --steps 32 --warmup 8 --latency-steps 0 --mid-batch 0 > $out/mid_new.log 2>&1 || { tail -20 $out/mid_new.log; exit 5; }
  echo "new $(grep '^\[bench\] load' $out/mid_new.log)"
done
