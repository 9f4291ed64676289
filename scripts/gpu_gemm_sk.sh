set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gsk_pytest.log 2>&1 && \
timeout -k 10 500 python -u scripts/bench_gemm_sk.py 512,1024 --configs 256:256:1:0:1,256:256:1:0:2,256:256:1:0:3,256:256:1:0:4,128:256:1:0:1,128:256:1:0:2,128:256:1:0:4,256:256:1:0:0,128:256:1:0:0 > gpurun_out/gsk_bench7.jsonl 2> gpurun_out/gsk_bench7.err
echo rc=$?
