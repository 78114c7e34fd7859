#!/bin/bash
# Round evidence: GPU suite, smoke, the default bench (C4), rocprof kernel stats of
# the same command, FETCH / WRITE PMC passes restricted to the dominant kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r03final3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
lscpu | grep -E "Model name|^CPU\(s\)|Core\(s\) per socket|Socket\(s\)" > $OUT/host.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  > $OUT/gpu_tests.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -3 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c4 -- \
  python3 bench.py --no-cpu-baseline --no-end-to-end > $OUT/trace.log 2>&1; rc=$?
echo "trace rc=$rc"
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $OUT/rocprof_kernel_stats_c4.csv; rm -rf $OUT/trace
[ $rc -eq 0 ] || exit $rc
head -6 $OUT/rocprof_kernel_stats_c4.csv | cut -d, -f1-5
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-include-regex "faml_sym_repulse" --output-format csv -d $OUT/pmc_$c -o p -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $OUT/pmc_$c.log 2>&1 || { tail -5 $OUT/pmc_$c.log; exit 1; }
  cp $(find $OUT/pmc_$c -name "*counter_collection.csv" | head -1) $OUT/pmc_${c}_c4.csv; rm -rf $OUT/pmc_$c
done
echo done
