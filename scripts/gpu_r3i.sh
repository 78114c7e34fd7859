# round 3: partition profile at C4 (kernel stats) and C5 (phase timers)
set -o pipefail
mkdir -p gpurun_out/r3i
export TMPDIR=/tmp
CFG=c4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pp -o p -- python3 scripts/partition_prof.py > gpurun_out/r3i/c4.log 2>&1 || { tail -20 gpurun_out/r3i/c4.log; exit 1; }
grep -v "^partition_device: round" gpurun_out/r3i/c4.log | tail -8
f=$(find /tmp/pp -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r3i/c4_kernel_stats.csv; cut -d, -f1-4 gpurun_out/r3i/c4_kernel_stats.csv | head -16
CFG=c5 timeout -k 10 700 python3 -u scripts/partition_prof.py > gpurun_out/r3i/c5.log 2>&1; rc=$?
grep -v "^partition_device: round" gpurun_out/r3i/c5.log | tail -8; exit $rc
