#!/bin/bash
# Round 4: fused QKV + attention at batch 1 - stamps + isolated A/B, tests, decode A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_qa2
rm -f gpurun_out/r4_qa2/stamps.jsonl gpurun_out/r4_qa2/ab.txt
for T in 150 400; do
  timeout -k 10 120 python3 scripts/probes/qa_stamps.py $T >> gpurun_out/r4_qa2/stamps.jsonl 2> gpurun_out/r4_qa2/err.log || { tail -20 gpurun_out/r4_qa2/err.log; exit 1; }
done
cat gpurun_out/r4_qa2/stamps.jsonl
timeout -k 10 300 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_qa2/pytest.log 2>&1 || { tail -30 gpurun_out/r4_qa2/pytest.log; exit 2; }
tail -1 gpurun_out/r4_qa2/pytest.log
for qa in 0 1 0 1; do
  LSA_QKV_ATTN=$qa timeout -k 10 200 python3 bench.py --batch 1 --steps 128 --warmup 16 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_qa2/b1.log 2>&1 || exit 3
  echo "qkv_attn=$qa $(grep '^\[bench\] load' gpurun_out/r4_qa2/b1.log)" | tee -a gpurun_out/r4_qa2/ab.txt
done
