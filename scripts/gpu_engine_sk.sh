set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eng_pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/eng_bench512.log 2>&1 && \
timeout -k 10 200 python -u bench.py --batch 256 --streams 2 --latency-steps 0 > gpurun_out/eng_bench256x2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --batch 1024 --latency-steps 0 > gpurun_out/eng_bench1024.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/eng_prof -o run -- python3 bench.py --steps 10 --warmup 3 --latency-steps 8 > gpurun_out/eng_prof.log 2>&1
echo rc=$?
