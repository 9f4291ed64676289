#!/bin/bash
# One GPU session: build, GPU tests, smoke, short bench. Each GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
test -f llm_sharding_amd/_native/liblsa_kernels.so && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 32 --warmup 4} > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 4; }
tail -4 gpurun_out/bench.log
