set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/flash && mkdir -p gpurun_out/flash
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_attn_gqa_gpu.py -k "prefill or gqa or mfma" -x -q --timeout 200 --timeout-method thread > gpurun_out/flash/pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/prefill_attn_bench.py > gpurun_out/flash/roofline.jsonl 2> gpurun_out/flash/roofline.err &&
timeout -k 10 200 python -u scripts/attn_gqa_bench.py > gpurun_out/flash/gqa.jsonl 2> gpurun_out/flash/gqa.err &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES \
    -d gpurun_out/flash/pmc -o run --output-format csv -- python3 scripts/pmc_hot.py > gpurun_out/flash/pmc.log 2>&1
echo rc=$?
