#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel trace + PMC passes.
# Usage: bash scripts/gpu_check.sh [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rocminfo 2>/dev/null | grep -m3 -E "Marketing Name|gfx950" > $OUT/devinfo.txt
lscpu | grep -E "Model name|^CPU\(s\)" > $OUT/host.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench.json; tail -3 $OUT/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1; rc=$?
echo "rocprof trace rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1; rc=$?
echo "pmc fetch rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_write.log 2>&1; rc=$?
echo "pmc write rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ -n "$FAST_CHECK" ]; then
  timeout -k 10 400 python scripts/fast_vs_strict.py $FAST_CHECK > $OUT/fast_vs_strict.jsonl 2>&1; rc=$?
  echo "fast_vs_strict rc=$rc"; tail -3 $OUT/fast_vs_strict.jsonl
fi
exit $rc
