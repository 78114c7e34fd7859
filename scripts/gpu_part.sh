#!/bin/bash
# Device partition: parity tests, then C3 (vs host path) and C4 timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-part}
mkdir -p $OUT
export GE_PROFILE_PARTITION=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_partition_device.py > $OUT/tests.log 2>&1; rc=$?
tail -25 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/partition_dev_check.py 1000000 8000000 --host > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
cat $OUT/c3.json; grep partition $OUT/c3.err
timeout -k 10 400 python -u scripts/partition_dev_check.py 10000000 80000000 > $OUT/c4.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
cat $OUT/c4.json; grep partition $OUT/c4.err
