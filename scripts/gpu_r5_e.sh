#!/bin/bash
# Round 5: gemm_sk re-tune on the new main loop at the headline rows, qkv gemm_sk-vs-gemm_wr check,
# then headline A/B of the old vs new tuning table (alternating).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_e}
mkdir -p $out
rm -rf $out/*
cp llm_sharding_amd/ops/gemm_sk_tuning.json $out/old.json
cp llm_sharding_amd/ops/gemm_sk_tuning.json $out/tuning.json
timeout -k 10 900 python3 scripts/tune_gemm_sk.py --rows 384,448,512 --models llama2-7b --out $out/tuning.json \
    > $out/tune.jsonl 2> $out/tune.err || { tail -20 $out/tune.err; exit 2; }
cp $out/tuning.json llm_sharding_amd/ops/gemm_sk_tuning.json
LSA_GEMM_WR=0 timeout -k 10 200 python3 scripts/gemm_vs_hipblaslt.py 384,512 > $out/gemm_nowr.jsonl 2>&1 || { tail -5 $out/gemm_nowr.jsonl; exit 3; }
timeout -k 10 200 python3 scripts/gemm_vs_hipblaslt.py 384,512 > $out/gemm_wr.jsonl 2>&1 || { tail -5 $out/gemm_wr.jsonl; exit 3; }
grep qkv $out/gemm_nowr.jsonl $out/gemm_wr.jsonl | cut -c1-220
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then cp $out/old.json llm_sharding_amd/ops/gemm_sk_tuning.json; else cp $out/tuning.json llm_sharding_amd/ops/gemm_sk_tuning.json; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 0 > $out/b_${v}_$i.log 2>&1 || { tail -20 $out/b_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^\[bench\] load' $out/b_${v}_$i.log)"
  done
done
cp $out/tuning.json llm_sharding_amd/ops/gemm_sk_tuning.json
