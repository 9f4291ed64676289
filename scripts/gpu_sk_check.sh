set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/chk
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/chk/pytest.log 2>&1 &&
timeout -k 10 400 python -u scripts/gemm_vs_coop.py llama2-7b 32,64,96,128 > gpurun_out/chk/coop.jsonl 2> gpurun_out/chk/coop.err
echo rc=$?
