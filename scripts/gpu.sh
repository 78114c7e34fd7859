#!/bin/bash
# One entry point for GPU sessions under gpurun (replaces the per-experiment
# gpu_*.sh scripts of rounds 1-3).  Steps run in order; each has its own time
# limit and the first failure ends the call (no GPU step after a fault or timeout).
#
# usage: bash scripts/gpu.sh TAG STEP [STEP ...]       (outputs in gpurun_out/TAG)
#   tests            the whole -m gpu suite                  -> tests.log
#   tests:EXPR       a -k selection of it                    -> tests.log
#   smoke            __graft_entry__.smoke()                 -> smoke.log
#   bench:W[:ARGS]   bench.py --workload W --steps 20 --warmup 5 [ARGS, commas = spaces]
#                                                            -> bench_W.json
#   trace:W          rocprofv3 --kernel-trace --stats of bench W (steps 20, no baseline)
#                                                            -> rocprof_kernel_stats_W.csv
#   pmc:W:CTRS[:RE]  one rocprofv3 --pmc pass (CTRS comma-separated, within one pass's
#                    per-block limits) over bench W (3 steps), dispatches matching RE
#                    (default: the multilevel / single-level repulsion and row kernels)
#                                                            -> pmc_<CTRS>_W.csv (+ summary)
#   c5[:ARGS]        scripts/c5_attraction.py [ARGS]  (configs[4] attraction pass)
#                                                            -> c5_attraction.json
#   pmc5:CTRS[:ARGS] one --pmc pass over c5_attraction.py (2 passes + 1 warmup) [ARGS,
#                    commas = spaces], attraction kernels only -> pmc_<CTRS>[_args]_c5.csv
#   py:SCRIPT[:ARGS] python -u SCRIPT [ARGS, commas = spaces] -> SCRIPT-name.log
#   env:K=V          export K=V for the following steps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
lscpu | grep -E "Model name|^CPU\(s\)|Core\(s\) per socket|Socket\(s\)" > $OUT/host.txt
DEFAULT_RE="faml_sym_repulse|faml_big_repulse|rows_kernel|heavy_|fa_repulse|fa_grouped"

fail() { echo "step '$1' failed (rc $2)"; tail -15 "$3"; exit "$2"; }

for step in "$@"; do
  IFS=: read -r kind a b c <<< "$step"
  case $kind in
    tests)
      sel=()
      [ -n "$a" ] && sel=(-k "$a")
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 \
        --timeout-method thread -p no:cacheprovider "${sel[@]}" > $OUT/tests.log 2>&1 \
        || fail "$step" $? $OUT/tests.log
      tail -2 $OUT/tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
        || fail "$step" $? $OUT/smoke.log
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 900 python -u bench.py --workload $a --steps 20 --warmup 5 ${b//,/ } \
        > $OUT/bench_$a.json 2> $OUT/bench_$a.err || fail "$step" $? $OUT/bench_$a.err
      cat $OUT/bench_$a.json ;;
    trace)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$a \
        -o t -- python3 bench.py --workload $a --steps 20 --warmup 5 --no-cpu-baseline \
        --no-end-to-end > $OUT/trace_$a.log 2>&1 || fail "$step" $? $OUT/trace_$a.log
      cp "$(find $OUT/trace_$a -name '*kernel_stats.csv' | head -1)" $OUT/rocprof_kernel_stats_$a.csv
      rm -rf $OUT/trace_$a
      head -6 $OUT/rocprof_kernel_stats_$a.csv | cut -d, -f1-5 ;;
    pmc)
      name=${b//,/_}
      timeout -s KILL 600 rocprofv3 --pmc ${b//,/ } --kernel-include-regex "${c:-$DEFAULT_RE}" \
        --output-format csv -d $OUT/pmc_$name -o p -- python3 bench.py --workload $a --steps 3 \
        --warmup 1 --no-cpu-baseline --no-end-to-end > $OUT/pmc_${name}_$a.log 2>&1 \
        || fail "$step" $? $OUT/pmc_${name}_$a.log
      cp "$(find $OUT/pmc_$name -name '*counter_collection.csv' | head -1)" $OUT/pmc_${name}_$a.csv
      rm -rf $OUT/pmc_$name
      python3 scripts/pmc_summary.py $OUT/pmc_${name}_$a.csv "" > $OUT/pmc_${name}_$a.txt 2>&1
      cat $OUT/pmc_${name}_$a.txt ;;
    c5)
      timeout -k 10 600 python -u scripts/c5_attraction.py ${a//,/ } > $OUT/c5_attraction.json \
        2> $OUT/c5_attraction.err || fail "$step" $? $OUT/c5_attraction.err
      cat $OUT/c5_attraction.json ;;
    pmc5)
      name=${a//,/_}${b:+_${b//[^a-z0-9]/}}
      timeout -s KILL 600 rocprofv3 --pmc ${a//,/ } --kernel-include-regex "rows_kernel|heavy_" \
        --output-format csv -d $OUT/pmc5_$name -o p -- python3 scripts/c5_attraction.py --steps 2 \
        --warmup 1 ${b//,/ } > $OUT/pmc_${name}_c5.log 2>&1 || fail "$step" $? $OUT/pmc_${name}_c5.log
      cp "$(find $OUT/pmc5_$name -name '*counter_collection.csv' | head -1)" $OUT/pmc_${name}_c5.csv
      rm -rf $OUT/pmc5_$name
      python3 scripts/pmc_summary.py $OUT/pmc_${name}_c5.csv "" > $OUT/pmc_${name}_c5.txt 2>&1
      cat $OUT/pmc_${name}_c5.txt ;;
    py)
      log=$OUT/$(basename $a .py).log
      timeout -k 10 1200 python -u $a ${b//,/ } > $log 2>&1 || fail "$step" $? $log
      tail -25 $log ;;
    env)
      export "$a" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG: done"
