#!/bin/bash
# Development loop: the GPU test suite (or a -k selection), then short bench lines.
# usage: bash scripts/gpu_iter.sh TAG "pytest -k expr or ''" [bench workloads...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; SEL=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$SEL" ]; then K=(-k "$SEL"); else K=(); fi
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
  -m gpu tests "${K[@]}" > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $OUT/tests.log | head -20; exit $rc; }
for w in "$@"; do
  timeout -k 10 600 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end \
    > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { tail -5 $OUT/bench_$w.err; exit 1; }
  python - $OUT/bench_$w.json <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
print(sys.argv[1], "value", round(b["value"], 4), "ms/step", round(b["ms_per_step"], 2),
      "rep ms", round(b["roofline"]["avg_launch_ms"], 3), "frac", round(b["roofline"]["frac"], 4))
PY
done
