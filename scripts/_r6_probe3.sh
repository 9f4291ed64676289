set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r6
export TMPDIR=/tmp
timeout -k 10 180 ./probe_bin/pk_hazard_probe > gpurun_out/r6/pk_hazard2.txt 2>&1 || { tail -5 gpurun_out/r6/pk_hazard2.txt; exit 1; }
tail -2 gpurun_out/r6/pk_hazard2.txt
rm -f gpurun_out/r6/full_depth_7b.json gpurun_out/r6/full_depth_7b_slp.json
LSA_FULL_DEPTH_FIXTURE=gpurun_out/r6/full_depth_7b.json LSA_RECORD_FULL_DEPTH=1 timeout -k 10 400 python -u -m pytest tests/test_full_depth_gpu.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/fd_record.log 2>&1 || { tail -30 gpurun_out/r6/fd_record.log; exit 2; }
LSA_KERNELS_SO=probe_bin/liblsa_kernels_slp.so LSA_FULL_DEPTH_FIXTURE=gpurun_out/r6/full_depth_7b_slp.json LSA_RECORD_FULL_DEPTH=1 timeout -k 10 400 python -u -m pytest tests/test_full_depth_gpu.py -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6/fd_record_slp.log 2>&1 || { tail -30 gpurun_out/r6/fd_record_slp.log; exit 3; }
grep "greedy tokens" gpurun_out/r6/fd_record.log gpurun_out/r6/fd_record_slp.log
