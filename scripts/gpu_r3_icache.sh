#!/bin/bash
# Instruction-cache counters on the coop kernel (qkv M=128): production vs exit-after-main-loop build.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
D=gpurun_out/icache
rm -rf $D && mkdir -p $D
timeout -s KILL 60 rocprofv3 -L > $D/avail.txt 2>&1 || true
grep -o -E "SQC_[A-Z_]+|SQ_IFETCH[A-Z_]*|SQ_INSTS_[A-Z_]+|SQ_WAIT_[A-Z_]+" $D/avail.txt | sort -u > $D/names.txt || true
cat $D/names.txt | tr '\n' ' '
echo
C=$(grep -E "^SQC_ICACHE_(REQ|HITS|MISSES|MISSES_DUPLICATE)$" $D/names.txt | tr '\n' ' ')
echo "counters: $C"
[ -n "$C" ] || exit 0
for V in prod main_loop; do
  timeout -s KILL 90 rocprofv3 --pmc $C SQ_WAVES SQ_IFETCH -d $D/$V -o run --output-format csv -- python3 scripts/coop_pmc_one.py $V > $D/$V.log 2>&1 || { tail -5 $D/$V.log; exit 3; }
done
python - << 'PY'
import csv, glob, collections
for v in ("prod", "main_loop"):
    p = glob.glob(f"gpurun_out/icache/{v}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in agg.items()})
PY
