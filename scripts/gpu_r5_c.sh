#!/bin/bash
# Round 5: IPC ring cost A/B (uncached vs coarse-grained buffers), batch-1 kernel trace, PMC passes
# over the four 512-row Llama-2-7B projection GEMMs (ours vs hipBLASLt).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_c}
mkdir -p $out
rm -rf $out/*
for alloc in uncached coarse; do
  port=$((29600 + RANDOM % 1000))
  (LSA_IPC_ALLOC=$alloc timeout -k 10 120 python3 scripts/ipc_ring_check.py --rank 1 --port $port > $out/ipc_${alloc}_r1.log 2>&1) &
  LSA_IPC_ALLOC=$alloc timeout -k 10 120 python3 scripts/ipc_ring_check.py --rank 0 --port $port > $out/ipc_${alloc}_r0.log 2>&1
  r0=$?
  wait $!
  r1=$?
  [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { tail -5 $out/ipc_${alloc}_r*.log; exit 3; }
  grep -h '^{' $out/ipc_${alloc}_r*.log
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/prof_b1 -o run -- \
    python3 -u bench.py --steps 4 --warmup 2 --latency-steps 32 --mid-batch 0 > $out/prof_b1.log 2>&1 || { tail -20 $out/prof_b1.log; exit 6; }
f=$(find $out/prof_b1 -name "*kernel_trace.csv" | head -1)
python3 scripts/kstats.py "$f" flash_prefill 14 > $out/kstats_b1.txt
head -10 $out/kstats_b1.txt
rm -f "$f"
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
P="python3 scripts/gemm_pmc_probe.py --rows 512 --launches 6"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o run -- $P > $out/probe_kt.log 2>&1 \
    || { tail -20 $out/probe_kt.log; exit 5; }
i=0
for pmc in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o run -- $P > $out/probe_pmc$i.log 2>&1 \
      || { echo "pmc pass $i failed"; tail -8 $out/probe_pmc$i.log; break; }
done
python3 scripts/gemm_pmc_summary.py $out/probe_kt.log $out/kt $out/pmc1 $out/pmc2 $out/pmc3 > $out/gemm_pmc.jsonl 2> $out/gemm_pmc.err
cut -c1-400 $out/gemm_pmc.jsonl
tail -3 $out/gemm_pmc.err
# the CU-mask probe whose teardown crashed under rocprofv3 in round 4 (streams now destroyed)
CUMASK_TRACE=8,16,24,32,64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/masked -o run -- \
    python3 scripts/cumask_probe.py > $out/masked.log 2>&1
echo "cumask probe exit $?"
grep '^{' $out/masked.log | head -3
