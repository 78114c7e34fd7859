#!/bin/bash
# GPU: rocprofv3 kernel trace of the C3 multilevel bench (one timed step).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3prof}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "rc=$rc"; cat $OUT/bench.json
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -12 $OUT/kernel_stats.csv | cut -c1-220
exit $rc
