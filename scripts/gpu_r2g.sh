#!/bin/bash
# GPU: radius-step tests (repeated) + embed goldens, then the C4 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02g}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_radius.py tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_dropin.py -k "radius or embed or transport or dropin" > $OUT/radius.log 2>&1; rc=$?
echo "radius rc=$rc"; tail -4 $OUT/radius.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench_c4.json; tail -3 $OUT/bench_c4.err
exit $rc
