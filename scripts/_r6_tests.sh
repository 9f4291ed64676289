set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
export LSA_FULL_DEPTH_FIXTURE=gpurun_out/r6/full_depth_7b.json
rm -f $LSA_FULL_DEPTH_FIXTURE
LSA_RECORD_FULL_DEPTH=1 timeout -k 10 400 python -u -m pytest tests/test_full_depth_gpu.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/fd_record.log 2>&1 || { tail -30 gpurun_out/r6/fd_record.log; exit 1; }
tail -3 gpurun_out/r6/fd_record.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=15 --timeout 300 --timeout-method thread -p no:cacheprovider -rs > gpurun_out/r6/gpu_tests.log 2>&1; rc=$?
tail -40 gpurun_out/r6/gpu_tests.log
exit $rc
