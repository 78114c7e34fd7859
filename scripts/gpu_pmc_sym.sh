#!/bin/bash
# PMC of the symmetric repulsion kernel at one workload: SQ issue / wait counters in
# one pass (<= 8 SQ, <= 2 GRBM counters), restricted to faml_sym_repulse dispatches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmcsym}; W=${2:-c4}; mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "faml_sym_repulse" --output-format csv -d $OUT/p1 -o p1 -- \
  python3 bench.py --workload $W --steps 2 --warmup 0 --no-cpu-baseline --no-end-to-end > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
f=$(find $OUT/p1 -name "*counter_collection.csv" | head -1)
cp $f $OUT/pmc_sym_$W.csv
python3 - "$f" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    v[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(k, len(x), sum(x) / len(x))
PY
rm -rf $OUT/p1
