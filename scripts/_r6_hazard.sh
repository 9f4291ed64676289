set -o pipefail
cd /root/repo
mkdir -p gpurun_out/r6
timeout -k 10 120 ./probe_bin/pk_hazard_probe > gpurun_out/r6/pk_hazard.txt 2>&1; rc=$?
tail -5 gpurun_out/r6/pk_hazard.txt
exit $rc
