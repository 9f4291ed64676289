#!/bin/bash
# Round 4: batch-1 decode kernel timeline (per-kernel time + inter-kernel gaps) and the
# 128-row decode step, for the latency work.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_b1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_b1/p1 -o run -- \
    python3 bench.py --batch 1 --steps 64 --warmup 8 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_b1/b1.log 2>&1 || exit 1
f=$(find gpurun_out/r4_b1/p1 -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats.py $f flash_prefill 30 > gpurun_out/r4_b1/b1_kstats.txt
python3 scripts/gap_pairs.py $f > gpurun_out/r4_b1/b1_gaps.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_b1/p128 -o run -- \
    python3 bench.py --batch 128 --steps 32 --warmup 8 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_b1/b128.log 2>&1 || exit 2
f=$(find gpurun_out/r4_b1/p128 -name '*kernel_trace.csv' | head -1)
python3 scripts/kstats.py $f flash_prefill 30 > gpurun_out/r4_b1/b128_kstats.txt
python3 scripts/gap_pairs.py $f > gpurun_out/r4_b1/b128_gaps.txt
rm -rf gpurun_out/r4_b1/p1 gpurun_out/r4_b1/p128

timeout -k 10 300 python3 scripts/mall_probe.py > gpurun_out/r4_b1/mall_probe.jsonl 2> gpurun_out/r4_b1/mall_probe.err || exit 3
cat gpurun_out/r4_b1/mall_probe.jsonl
for pf in "" "34,0,32" "34,64,32" "34,128,64" "34,64,16" ; do
  LSA_MALL_PF="$pf" timeout -k 10 200 python3 bench.py --batch 1 --steps 256 --warmup 16 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_b1/pf.log 2>&1 || exit 4
  echo "pf=[$pf] $(grep '^\[bench\] load' gpurun_out/r4_b1/pf.log)" | tee -a gpurun_out/r4_b1/pf_ab.txt
done
for cfg in "256 2" "512 2" "384 2" "128 4"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --batch $1 --streams $2 --latency-steps 0 --mid-batch 0 > gpurun_out/r4_b1/st.log 2>&1 || exit 5
  echo "batch=$1 streams=$2 $(grep '^\[bench\] load' gpurun_out/r4_b1/st.log)" | tee -a gpurun_out/r4_b1/streams_ab.txt
done
