#!/bin/bash
# GPU: gather-copy + C4 parity tests; C2 bench with / without the gather copy;
# attraction-kernel PMC at C2; C5 attraction pass with / without the copy.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02e}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_degenerate.py -k gather "tests/test_gpu_configs.py::test_c4_level0_sampled_aggregates" \
  "tests/test_gpu_configs.py::test_c2_full_size_iteration_sampled_rows" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed|\[ " $OUT/tests.log | tail -15
[ $rc -eq 0 ] || exit $rc
for g in 1 0; do
  GE_GATHER_COPY=$g timeout -k 10 300 python bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline \
    > $OUT/c2_copy$g.json 2> $OUT/c2_copy$g.err || { tail -5 $OUT/c2_copy$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c2_copy$g.json'));a=d['roofline_attraction'];print('copy=$g', d['ms_per_step'], a['avg_launch_ms'], a['frac'])"
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "FaRows" --output-format csv -d $OUT/pmc_$c -o p -- \
    python3 bench.py --workload c2 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_$c.log 2>&1 || { tail -5 $OUT/pmc_$c.log; exit 1; }
  cp $(find $OUT/pmc_$c -name "*counter_collection.csv" | head -1) $OUT/pmc_${c}_c2.csv; rm -rf $OUT/pmc_$c
done
python3 - $OUT <<'PY'
import csv, sys, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f"{sys.argv[1]}/pmc_{c}_c2.csv")):
        v[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
    for k, x in v.items():
        print(c, k, len(x), sum(x) / len(x))
PY
for g in 1 0; do
  GE_GATHER_COPY=$g timeout -k 10 400 python -u scripts/c5_attraction.py --steps 5 --warmup 2 \
    > $OUT/c5_copy$g.json 2> $OUT/c5_copy$g.err || { tail -5 $OUT/c5_copy$g.err; exit 1; }
  echo "c5 copy=$g"; cat $OUT/c5_copy$g.json
done
