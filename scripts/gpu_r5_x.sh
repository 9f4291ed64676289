#!/bin/bash
# Round 5: PMC passes over the four 128-row Llama-2-7B decode projections: the coop GEMV (the
# engine's path at 17-128 rows), the MFMA GEMM path and hipBLASLt on the same operands.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_x}
mkdir -p $out
rm -rf $out/*
P="python3 scripts/gemm_pmc_probe.py --rows 128 --launches 6 --impls coop,ours,blas"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/kt -o run -- $P > $out/probe_kt.log 2>&1 \
    || { tail -20 $out/probe_kt.log; exit 5; }
i=0
for pmc in "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc$i -o run -- $P > $out/probe_pmc$i.log 2>&1 \
      || { echo "pmc pass $i failed"; tail -8 $out/probe_pmc$i.log; exit 6; }
done
python3 scripts/gemm_pmc_summary.py $out/probe_kt.log $out/kt $out/pmc1 $out/pmc2 $out/pmc3 > $out/gemm_pmc.jsonl 2> $out/gemm_pmc.err
cut -c1-600 $out/gemm_pmc.jsonl
tail -3 $out/gemm_pmc.err
find $out -name "*.csv" -size +20M -delete
