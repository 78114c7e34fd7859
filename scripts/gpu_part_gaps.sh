#!/bin/bash
# C4 device partition: plain timing (library phase timers), then a kernel trace
# reduced on the box to busy time, idle gaps and per-kernel sums (scripts/part_gaps.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-partgaps}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/partition_prof.py > $OUT/plain.log 2>&1 || { tail -5 $OUT/plain.log; exit 1; }
grep -E "partition |partition_device: n=" $OUT/plain.log
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/pg -o pg -- \
  python3 -u scripts/partition_prof.py > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 scripts/part_gaps.py $(find /tmp/pg -name "*kernel_trace.csv" | head -1) > $OUT/gaps.txt
cat $OUT/gaps.txt
