#!/bin/bash
# GPU: parity tests, then the C3 (multilevel) bench with end-to-end embed timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-c3}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
GE_PROFILE_PARTITION=1 timeout -k 10 900 python bench.py --workload c3 "$@" > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?
echo "bench c3 rc=$rc"; cat $OUT/bench_c3.json; tail -5 $OUT/bench_c3.err
exit $rc
