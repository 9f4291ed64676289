#!/bin/bash
# Round 5 (new gemm_sk main loop): Llama-2-70B stage (70B projection GEMMs vs fp32, one 10-layer
# stage of the 8-stage plan, 8 x 512-row micro-batches, under rocprofv3 kernel stats) and the
# batch-1 TTFT / decode latency sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_f}
mkdir -p $out
rm -rf $out/*
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -k llama70b -q --timeout 120 --timeout-method thread \
    > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 2; }
tail -1 $out/pytest.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
    python3 -u bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 10 --warmup 3 \
    --latency-steps 8 > $out/stage.log 2>&1 || { tail -20 $out/stage.log; exit 3; }
grep '^{' $out/stage.log | tail -1
f=$(find $out/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 12 > $out/kstats_70b.txt
head -12 $out/kstats_70b.txt
rm -f "$f"
timeout -k 10 500 python3 -u scripts/latency_sweep.py --lengths 8,128,256,512,1024,2048,4096 > $out/sweep.jsonl 2> $out/sweep.err || { tail -20 $out/sweep.err; exit 4; }
cat $out/sweep.jsonl
