set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/stamps.log
for cfg in "512 4096 4096 128 256 1 0" "512 4096 4096 128 256 1 4" "512 4096 4096 256 256 1 8" "512 4096 11008 128 256 1 0" "512 12288 4096 192 256 1 3" "512 22016 4096 192 256 1 6"; do
  timeout -k 10 60 python -u scripts/gemm_stamps.py $cfg 5 >> gpurun_out/stamps.log 2>&1 || exit 1
done
echo rc=$?
