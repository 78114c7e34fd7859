#!/bin/bash
# Round evidence for one workload: the bench line (same flags as the driver), the
# rocprofv3 kernel stats of the same workload/steps, and FETCH_SIZE / WRITE_SIZE PMC
# passes (one counter group per run).  Summaries land in gpurun_out/$TAG/$W/summary
# (raw traces are deleted: gpurun copies back at most 64 MiB); copy them into
# profiles/$TAG afterwards.
# usage: bash scripts/gpu_bench.sh TAG WORKLOAD [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}; W=${2:-c4}; shift 2
OUT=gpurun_out/$TAG/$W
PROF=$OUT/summary
mkdir -p $OUT $PROF
export TMPDIR=/tmp
lscpu | grep -E "Model name|^CPU\(s\)|Socket|Core\(s\)" > $OUT/host.txt
timeout -k 10 900 python3 bench.py --workload $W --steps 20 --warmup 5 "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json; tail -4 $OUT/bench.err; cp $OUT/bench.json $PROF/bench_$W.json
prof() {  # name, rocprof args
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py --workload $W --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.log; return 1; }
  echo "$name ok"
}
prof trace --kernel-trace --stats &&
prof fetch --pmc FETCH_SIZE --kernel-include-regex "faml_|rows_kernel|heavy_|fa_repulse|fa_grouped" &&
prof write --pmc WRITE_SIZE --kernel-include-regex "faml_|rows_kernel|heavy_|fa_repulse|fa_grouped" || exit 1
cp $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $PROF/rocprof_kernel_stats_$W.csv
cp $(find $OUT/fetch -name "*counter_collection.csv" | head -1) $PROF/pmc_fetch_$W.csv
cp $(find $OUT/write -name "*counter_collection.csv" | head -1) $PROF/pmc_write_$W.csv
cp $OUT/bench.json $PROF/bench_$W.json
cp $OUT/host.txt $PROF/host.txt
rm -rf $OUT/trace $OUT/fetch $OUT/write
head -6 $PROF/rocprof_kernel_stats_$W.csv | cut -d, -f1-4
