set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
rm -f gpurun_out/abl/abl4.jsonl
timeout -k 10 300 python -u scripts/sk_ablate.py 512 12288 4096 192 3  2048 12288 4096 256 3  16384 12288 4096 256 0 > gpurun_out/abl/abl4.jsonl 2> gpurun_out/abl/abl4.err
echo rc=$?
