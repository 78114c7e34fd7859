#!/bin/bash
# rocprofv3 kernel stats of the device partition (C3 and C4 LCCs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-partprof}
mkdir -p $OUT
export TMPDIR=/tmp GE_PROFILE_PARTITION=1
for w in "c3 1000000 8000000" "c4 10000000 80000000"; do
  set -- $w
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o $1 -- \
    python3 scripts/partition_dev_check.py $2 $3 > $OUT/$1.log 2>&1 || { tail -5 $OUT/$1.log; exit 1; }
  f=$(find $OUT/$1 -name "*kernel_stats.csv" | head -1)
  cp $f $OUT/kstats_$1.csv
  head -14 $OUT/kstats_$1.csv | cut -d, -f1-8
  grep partition_device $OUT/$1.log
done
