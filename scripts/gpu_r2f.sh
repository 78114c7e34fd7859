#!/bin/bash
# GPU: device graph tests, C4 parity test, the whole GPU suite, C4 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02f}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_graph.py "tests/test_gpu_configs.py::test_c4_level0_sampled_aggregates" -s \
  > $OUT/tests_new.log 2>&1; rc=$?
echo "new tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed|\[ *[0-9.]+s\]" $OUT/tests_new.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $OUT/gpu_tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -4 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench_c4.json; tail -3 $OUT/bench_c4.err
exit $rc
