set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
timeout -k 10 300 python -u scripts/sk_ablate.py 512 4096 4096 128 0  512 12288 4096 192 3  2048 12288 4096 256 3  16384 12288 4096 256 0 > gpurun_out/abl/abl3.jsonl 2> gpurun_out/abl/abl3.err
echo rc=$?
