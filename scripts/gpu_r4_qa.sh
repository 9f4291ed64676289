#!/bin/bash
# Round 4: fused QKV + attention (qkv_attn.hip): GPU tests, then batch-1 A/B and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_qa
timeout -k 10 600 python -u -m pytest tests/test_qkv_attn_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/r4_qa/pytest.log 2>&1 || { tail -30 gpurun_out/r4_qa/pytest.log; exit 1; }
tail -2 gpurun_out/r4_qa/pytest.log
for qa in 0 1 0 1; do
  LSA_QKV_ATTN=$qa timeout -k 10 200 python3 bench.py --batch 1 --steps 128 --warmup 16 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_qa/b1.log 2>&1 || exit 2
  echo "qkv_attn=$qa $(grep '^\[bench\] load' gpurun_out/r4_qa/b1.log)" | tee -a gpurun_out/r4_qa/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_qa/p1 -o run -- \
    python3 bench.py --batch 1 --steps 64 --warmup 8 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_qa/prof.log 2>&1 || exit 3
f=$(find gpurun_out/r4_qa/p1 -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats.py $f flash_prefill 12 > gpurun_out/r4_qa/b1_kstats.txt
rm -rf gpurun_out/r4_qa/p1
head -16 gpurun_out/r4_qa/b1_kstats.txt
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_qa/pytest_sk.log 2>&1 || { tail -30 gpurun_out/r4_qa/pytest_sk.log; exit 4; }
tail -2 gpurun_out/r4_qa/pytest_sk.log
