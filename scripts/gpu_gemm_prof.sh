set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gprof
timeout -k 10 60 rocprofv3 -L > gpurun_out/gprof/counters.txt 2>&1 || true
for cfg in "512 12288 4096 256 256 1 2" "16384 12288 4096 256 256 1 0"; do
  tag=$(echo $cfg | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/gprof/p1_$tag -o run -- python3 scripts/gemm_probe.py $cfg 10 > gpurun_out/gprof/p1_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/gprof/p2_$tag -o run -- python3 scripts/gemm_probe.py $cfg 10 > gpurun_out/gprof/p2_$tag.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/gprof/p3_$tag -o run -- python3 scripts/gemm_probe.py $cfg 10 > gpurun_out/gprof/p3_$tag.log 2>&1 || true
done
echo rc=$?
