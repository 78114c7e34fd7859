#!/bin/bash
# GPU: kernel-trace stats of the C2 (1 step) and C3 (1 step) benches -> $OUT/*_stats.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-kt}; mkdir -p $OUT
export TMPDIR=/tmp
for w in c2 c3; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w -o $w -- \
    python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$w.json 2> $OUT/$w.err || exit 1
  python3 - "$OUT" "$w" <<'PY'
import csv, glob, sys
out, w = sys.argv[1], sys.argv[2]
f = glob.glob(f"{out}/{w}/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]:
    print(w, r["Name"][:70], r["Calls"], "%.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
