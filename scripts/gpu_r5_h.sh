#!/bin/bash
# Round 5: A/B of the gemm_sk main-loop change where 256 x 256 tiles run (7B prefill-sized M = 2048,
# Llama-2-70B projections at 512 rows, the 70B stage step, TTFT at 2048), new vs the previous loop
# (LSA_KERNELS_SO=scripts/probes/bin/liblsa_kernels_base.so: same build otherwise), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_h}
mkdir -p $out
rm -rf $out/*
BASE=$GRAFT_REPO_ROOT/scripts/probes/bin/liblsa_kernels_base.so
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
    timeout -k 10 240 python3 scripts/gemm_vs_hipblaslt.py 2048 > $out/g7_${v}_$i.jsonl 2>&1 || { tail -5 $out/g7_${v}_$i.jsonl; exit 3; }
    timeout -k 10 300 python3 scripts/gemm_vs_hipblaslt.py 512 llama2-70b > $out/g70_${v}_$i.jsonl 2>&1 || { tail -5 $out/g70_${v}_$i.jsonl; exit 3; }
  done
done
for v in new base new base; do
  if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
  timeout -k 10 300 python3 bench.py --model llama2-70b --stage-layers 10 --microbatches 8 --steps 6 --warmup 2 \
      --latency-steps 0 > $out/s70_$v.log 2>&1 || { tail -20 $out/s70_$v.log; exit 4; }
  echo "70B stage $v: $(grep '^\[bench\] load' $out/s70_$v.log)"
  timeout -k 10 200 python3 -u scripts/latency_sweep.py --lengths 2048 --decode-batches 1 --decode-steps 16 > $out/ttft_$v.jsonl 2> $out/ttft_$v.err || { tail -5 $out/ttft_$v.err; exit 5; }
  echo "ttft $v: $(tail -1 $out/ttft_$v.jsonl | cut -c1-120)"
done
unset LSA_KERNELS_SO
python3 - << 'PY'
import json, glob, collections, os
out = "gpurun_out/" + os.environ.get("LSA_OUT", "r5_h")
res = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/g*_*_*.jsonl")):
    tag, v = os.path.basename(f).split("_")[:2]
    for ln in open(f):
        if ln.startswith("{"):
            d = json.loads(ln)
            res[(tag, d["shape"], d["M"], v)].append(d["ours_us"])
            res[(tag, d["shape"], d["M"], "hipblaslt")].append(d["hipblaslt_us"])
for k, ts in sorted(res.items()):
    print(*k, ts)
PY
