#!/bin/bash
# GPU tests (optionally filtered by PYTEST_K) + one short bench per batch size in BATCHES.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
test -f llm_sharding_amd/_native/liblsa_kernels.so || exit 2
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
      > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for B in ${BATCHES:-1 64}; do
  timeout -k 10 300 python bench.py --batch $B --steps 32 --warmup 4 ${BENCH_EXTRA:-} > gpurun_out/bench_b$B.log 2>&1 || { tail -20 gpurun_out/bench_b$B.log; exit 1; }
  grep "^\[bench\] load" gpurun_out/bench_b$B.log
done
