#!/bin/bash
# One GPU session producing the round's evidence under gpurun_out/$TAG:
#   parity tests; rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE PMC
#   passes for the C2 and C3 workloads (copied into profiles/$TAG so the benches
#   of this same session read them); then the C2 and C3 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
PROF=profiles/$TAG
mkdir -p $OUT $PROF
export TMPDIR=/tmp
rocminfo 2>/dev/null | grep -m3 -E "Marketing Name|gfx950" > $OUT/devinfo.txt
lscpu | grep -E "Model name|^CPU\(s\)" > $OUT/host.txt
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
prof() {  # name, rocprof args, bench args
  local name=$1; shift; local rp=$1; shift
  timeout -k 10 600 rocprofv3 $rp --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py --no-cpu-baseline "$@" > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; return 1; }
  echo "$name ok"
}
prof c2_trace "--kernel-trace --stats" --steps 3 --warmup 1 &&
prof c2_fetch "--pmc FETCH_SIZE" --steps 1 --warmup 0 &&
prof c2_write "--pmc WRITE_SIZE" --steps 1 --warmup 0 &&
prof c3_trace "--kernel-trace --stats" --workload c3 --steps 1 --warmup 0 &&
prof c3_fetch "--pmc FETCH_SIZE" --workload c3 --steps 1 --warmup 0 &&
prof c3_write "--pmc WRITE_SIZE" --workload c3 --steps 1 --warmup 0 || exit 1
for w in c2 c3; do
  cp $(find $OUT/${w}_trace -name "*kernel_stats.csv" | head -1) $OUT/rocprof_kernel_stats_$w.csv
  cp $(find $OUT/${w}_fetch -name "*counter_collection.csv" | head -1) $PROF/pmc_fetch_$w.csv
  cp $(find $OUT/${w}_write -name "*counter_collection.csv" | head -1) $PROF/pmc_write_$w.csv
  cp $PROF/pmc_fetch_$w.csv $PROF/pmc_write_$w.csv $OUT/
done
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -5 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 900 python bench.py --workload c3 --steps 3 --warmup 1 --end-to-end > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
