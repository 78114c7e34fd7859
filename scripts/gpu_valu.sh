#!/bin/bash
# GPU: VALU issue evidence for the strict repulsion kernel (C2, one step):
# available counters, then one rocprofv3 --pmc pass per counter.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-valu}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -oE "\b(SQ_[A-Z0-9_]*VALU[A-Z0-9_]*|GRBM_GUI_ACTIVE|SQ_WAVES|SQ_BUSY_CYCLES|SQ_WAVE_CYCLES|SQ_INSTS_VALU_[A-Z0-9_]*|SQ_INST_CYCLES_VALU|SQ_ACTIVE_INST_ANY)\b" $OUT/avail.txt | sort -u > $OUT/counters.txt
cat $OUT/counters.txt | tr '\n' ' '; echo
for c in GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_BUSY_CYCLES; do
  grep -qx "$c" $OUT/counters.txt || { echo "skip $c"; continue; }
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o $c -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "${@:2}" > $OUT/$c.log 2>&1 || { echo "$c failed"; tail -3 $OUT/$c.log; exit 1; }
  f=$(find $OUT/$c -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$c" <<'PY'
import csv, sys
f, c = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f)):
    if "fa_repulse" in r["Kernel_Name"]:
        print(c, r["Counter_Value"], "grid", r["Grid_Size"], "dur_ns", int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
PY
done
