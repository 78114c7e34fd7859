#!/bin/bash
# Device partition iteration: parity tests, C4 timing twice, then the idle-gap trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-partiter}
mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/gpu_part_ab.sh $(basename $OUT) $2 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/pg -o pg -- \
  python3 -u scripts/partition_prof.py > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
python3 scripts/part_gaps.py $(find /tmp/pg -name "*kernel_trace.csv" | head -1) > $OUT/gaps.txt
cat $OUT/gaps.txt
