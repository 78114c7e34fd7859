#!/bin/bash
# Quick GPU iteration: parity tests + bench (no profiling).  Usage: bash scripts/gpu_quick.sh tag [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
exit $rc
