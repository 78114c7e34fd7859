#!/bin/bash
# GPU: multilevel parity tests (sweeps / grouped rows), then the per-rank rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02i}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_degenerate.py tests/test_gpu_dist.py -k "faml or embed or transport" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/scale_sim.py > $OUT/scale.jsonl 2> $OUT/scale.err; rc=$?
cat $OUT/scale.jsonl | cut -c1-250; exit $rc
