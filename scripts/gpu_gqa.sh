set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gqa
timeout -k 10 300 python -u -m pytest tests/test_attn_gqa_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gqa/pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/attn_gqa_bench.py > gpurun_out/gqa/bench.jsonl 2> gpurun_out/gqa/bench.err
echo rc=$?
