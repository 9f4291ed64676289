#!/bin/bash
# The one GPU-box runner (replaces the per-experiment scripts/gpu_*.sh wrappers of rounds 1-5; their
# index, with the commit that holds each one, is scripts/RUNS.md).
#
#   gpurun --timeout 900 -- 'bash scripts/gpu.sh TASK [ARGS] [+ TASK [ARGS] ...]'
#
# Steps separated by "+" run in order, each under its own time limit; the chain stops at the first
# step that fails, times out or faults (no retries). Everything a step writes goes under
# gpurun_out/$RUN/ (RUN defaults to the first task's name).
#
# tasks:
#   tests [PYTEST ARGS]          GPU suite (pytest -m gpu -x, per-test thread timeout), e.g. tests -k gemm
#   smoke                        __graft_entry__.smoke()
#   bench [BENCH ARGS]           python bench.py ARGS (default: the driver's --steps 20 --warmup 5)
#   ab ROUNDS ENV_A ENV_B [ARGS] bench.py alternated A / B ROUNDS times (ENV_x: "K=V K2=V2" or "-")
#   trace [BENCH ARGS]           rocprofv3 --kernel-trace --stats over bench.py (no PMC in the same run)
#   pmc COUNTERS SCRIPT [ARGS]   one rocprofv3 --pmc pass (COUNTERS comma-separated) over a python script
#   py SCRIPT [ARGS]             a python probe script
#   exe BINARY [ARGS]            a prebuilt probe binary (probe_bin/...)
#   record                       record the full-depth tripwire fixture -> $OUT/full_depth_7b.json
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
RUN=${RUN:-${1:-run}}
OUT=gpurun_out/$RUN
mkdir -p "$OUT"
test -f llm_sharding_amd/_native/liblsa_kernels.so || { echo "kernel library not built"; exit 2; }
LIMIT=${STEP_LIMIT:-600}
n=0

step() {
  local task=$1; shift
  n=$((n + 1))
  local log=$OUT/$n-$task.log
  local rc=0
  case $task in
    tests)
      timeout -k 10 "$LIMIT" python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
          -p no:cacheprovider -rs "$@" > "$log" 2>&1 || rc=$? ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || rc=$? ;;
    bench)
      [ $# -eq 0 ] && set -- --steps 20 --warmup 5
      timeout -k 10 "$LIMIT" python -u bench.py "$@" --json-out "$OUT/$n-bench.json" > "$log" 2>&1 || rc=$? ;;
    ab)
      local rounds=$1 ea=$2 eb=$3; shift 3
      for r in $(seq 1 "$rounds"); do
        for tag in A B; do
          local ev=$ea; [ $tag = B ] && ev=$eb; [ "$ev" = "-" ] && ev=""
          env $ev timeout -k 10 "$LIMIT" python -u bench.py "$@" --json-out "$OUT/$n-ab-$tag$r.json" \
              > "$OUT/$n-ab-$tag$r.log" 2>&1 || { rc=$?; break 2; }
          echo "$tag$r ($ev): $(grep '^\[bench\] load' "$OUT/$n-ab-$tag$r.log")" | tee -a "$log"
        done
      done ;;
    trace)
      [ $# -eq 0 ] && set -- --steps 20 --warmup 5
      timeout -k 10 "$LIMIT" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace$n" -o run -- python3 bench.py "$@" \
          > "$log" 2>&1 || rc=$? ;;
    pmc)
      local ctr=$1; shift
      timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } --output-format csv -d "$OUT/pmc$n" -o run -- python3 "$@" > "$log" 2>&1 || rc=$? ;;
    py)
      timeout -k 10 "$LIMIT" python -u "$@" > "$log" 2>&1 || rc=$? ;;
    exe)
      timeout -k 10 "$LIMIT" "$@" > "$log" 2>&1 || rc=$? ;;
    record)
      rm -f "$OUT/full_depth_7b.json"
      LSA_FULL_DEPTH_FIXTURE="$OUT/full_depth_7b.json" LSA_RECORD_FULL_DEPTH=1 timeout -k 10 400 \
          python -u -m pytest tests/test_full_depth_gpu.py -v -s --timeout 300 --timeout-method thread \
          -p no:cacheprovider > "$log" 2>&1 || rc=$? ;;
    *)
      echo "unknown task $task"; return 2 ;;
  esac
  echo "== step $n: $task $* -> rc $rc ($log)"
  tail -4 "$log"
  return $rc
}

args=("$@")
cur=()
for a in "${args[@]}" +; do
  if [ "$a" = "+" ]; then
    [ ${#cur[@]} -gt 0 ] && { step "${cur[@]}" || exit $?; }
    cur=()
  else
    cur+=("$a")
  fi
done
