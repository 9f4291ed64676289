#!/bin/bash
# counter passes over skinny_gemm (o, M=128) vs its no-weight-load build vs gemv_coop: does A hit L2?
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
D=gpurun_out/skpmc
rm -rf $D && mkdir -p $D
run() {  # tag, counters..., -- args
  local tag=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  timeout -s KILL 90 rocprofv3 --pmc "${ctr[@]}" -d $D/$tag -o run --output-format csv -- python3 scripts/skinny_pmc.py "$@" > $D/$tag.log 2>&1
}
for V in "skinny 128 4096 4096 4 4 2 4" "abl2 128 4096 4096 4 4 2 4" "coop 128 4096 4096 1 4 2 4 2"; do
  T=$(echo $V | cut -d' ' -f1)
  run ${T}_tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum -- $V &&
  run ${T}_tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum -- $V &&
  run ${T}_sq SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -- $V || { echo "fail $T"; tail -5 $D/*.log; exit 3; }
done
python - << 'PY'
import csv, glob, os, collections
D = "gpurun_out/skpmc"
for tag in sorted(os.listdir(D)):
    p = glob.glob(os.path.join(D, tag, "**", "*counter_collection.csv"), recursive=True)
    if not p:
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p[0])):
        if "skinny" in r["Kernel_Name"] or "coop" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(tag, {k: round(sum(v) / len(v)) for k, v in agg.items()})
PY
