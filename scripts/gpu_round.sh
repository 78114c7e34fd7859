#!/bin/bash
# GPU: parity tests, C3 kernel profile, C2 bench (1 step) with kernel timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-round}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3trace -o c3 -- \
  python3 bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit $?
cat $OUT/c3.json
find $OUT/c3trace -name "*kernel_stats.csv" -exec cp {} $OUT/c3_kernel_stats.csv \;
cut -d, -f1-5 $OUT/c3_kernel_stats.csv | head -8
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || exit $?
cat $OUT/c2.json
