#!/bin/bash
# Interleaved A/B of one environment switch on the C4 bench (one box, same process
# image): bash scripts/ab_env.sh TAG VAR "V1 V2 ..." [ROUNDS [WORKLOAD]]
# ("-" as a value leaves VAR unset).  Per run: ms per step, the repulsion launch and
# the attraction pass (HIP events) -> gpurun_out/TAG/ab_VAR.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=$1; VAR=$2; VALS=$3; ROUNDS=${4:-2}; W=${5:-c4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for v in $VALS; do
    if [ "$v" = "-" ]; then unset $VAR; else export $VAR=$v; fi
    tagv=$(basename "$(dirname "$v")")_$(basename "$v")  # a path value names its directory
    f=$OUT/ab_${VAR}_${tagv}_$r.json
    timeout -k 10 400 python -u bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline \
      --no-end-to-end > $f 2> $OUT/ab_${VAR}_${tagv}_$r.err || { tail -5 $OUT/ab_${VAR}_${tagv}_$r.err; exit 1; }
    python3 -c "
import json; d = json.load(open('$f'))
print('$VAR=$v', round(d['ms_per_step'], 2), round(d['roofline']['avg_launch_ms'], 2),
      round(d['roofline_attraction']['avg_launch_ms'], 3))" | tee -a $OUT/ab_$VAR.log
  done
done
unset $VAR
