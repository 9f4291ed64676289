set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/flash2 && mkdir -p gpurun_out/flash2
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "prefill or multistage" -x -q --timeout 200 --timeout-method thread > gpurun_out/flash2/pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/prefill_attn_bench.py > gpurun_out/flash2/roofline.jsonl 2> gpurun_out/flash2/roofline.err &&
timeout -k 10 300 python -u scripts/latency_sweep.py --lengths 128,512,2048,4096 --repeats 3 --decode-steps 16 --decode-batches 1 > gpurun_out/flash2/sweep.log 2>&1
echo rc=$?
