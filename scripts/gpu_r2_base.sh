set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2_base_pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py > gpurun_out/r2_base_bench.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_base_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r2_base_prof.log 2>&1
echo rc=$?
