#!/bin/bash
# Round 5: gemm_sk main loop with compile-time stage conditions - numerics (GPU tests of every
# gemm_sk geometry + engine paths), then per-shape and bench A/B against the previous build
# (LSA_KERNELS_SO=scripts/probes/bin/liblsa_kernels_base.so), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
out=gpurun_out/${LSA_OUT:-r5_d}
mkdir -p $out
rm -rf $out/*
timeout -k 10 600 python -u -m pytest tests/test_gemm_sk_gpu.py tests/test_engine_gpu.py tests/test_full_depth_gpu.py \
    tests/test_kernels_gpu.py tests/test_gemm_wr_gpu.py -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > $out/pytest.log 2>&1
rc=$?
tail -6 $out/pytest.log
grep -q "Timeout\|Fatal Python\|core dumped" $out/pytest.log && exit 2
[ $rc -eq 0 ] || exit 2
BASE=$GRAFT_REPO_ROOT/scripts/probes/bin/liblsa_kernels_base.so
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
    timeout -k 10 240 python3 scripts/gemm_vs_hipblaslt.py 384,512,768 > $out/gemm_${v}_$i.jsonl 2>&1 || { tail -5 $out/gemm_${v}_$i.jsonl; exit 3; }
  done
done
for i in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export LSA_KERNELS_SO=$BASE; else unset LSA_KERNELS_SO; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --latency-steps 0 > $out/bench_${v}_$i.log 2>&1 || { tail -20 $out/bench_${v}_$i.log; exit 4; }
    echo "$v $i: $(grep '^{' $out/bench_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
unset LSA_KERNELS_SO
python3 - << 'PY'
import json, glob, collections
out = "gpurun_out/" + __import__("os").environ.get("LSA_OUT", "r5_d")
res = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/gemm_*_*.jsonl")):
    v = f.split("/gemm_")[1].split("_")[0]
    for ln in open(f):
        if ln.startswith("{"):
            d = json.loads(ln)
            res[(d["shape"], d["M"], v)].append(d["ours_us"])
for (shape, M, v), ts in sorted(res.items()):
    print(shape, M, v, ts)
PY
