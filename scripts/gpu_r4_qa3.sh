#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_qa3
rm -f gpurun_out/r4_qa3/*
timeout -k 10 120 python3 scripts/probes/qa_stamps.py 150 > gpurun_out/r4_qa3/stamps.jsonl 2> gpurun_out/r4_qa3/err.log || { tail -20 gpurun_out/r4_qa3/err.log; exit 1; }
cat gpurun_out/r4_qa3/stamps.jsonl
timeout -k 10 300 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_qa3/pytest.log 2>&1 || { tail -30 gpurun_out/r4_qa3/pytest.log; exit 2; }
tail -1 gpurun_out/r4_qa3/pytest.log
for qa in 0 1 0 1; do
  LSA_QKV_ATTN=$qa timeout -k 10 200 python3 bench.py --batch 1 --steps 128 --warmup 16 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_qa3/b1.log 2>&1 || exit 3
  echo "qkv_attn=$qa $(grep '^\[bench\] load' gpurun_out/r4_qa3/b1.log)" | tee -a gpurun_out/r4_qa3/ab.txt
done
