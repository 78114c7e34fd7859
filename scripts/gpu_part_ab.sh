#!/bin/bash
# Device partition: parity tests, then C4 timing A/B (env switch given as $2, e.g.
# GE_PART_BLIT_EXPORT=1) with the library's phase timers, twice each, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-partab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_partition_device.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/tests.log 2>&1; rc=$?
tail -2 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  timeout -k 10 200 python3 -u scripts/partition_prof.py > $OUT/new_$k.log 2>&1 || { tail -5 $OUT/new_$k.log; exit 1; }
  echo "new: $(grep -E 'partition_device: n=' $OUT/new_$k.log)"
  if [ -n "$2" ]; then
    timeout -k 10 200 env $2 python3 -u scripts/partition_prof.py > $OUT/old_$k.log 2>&1 || { tail -5 $OUT/old_$k.log; exit 1; }
    echo "old: $(grep -E 'partition_device: n=' $OUT/old_$k.log)"
  fi
done
