#!/bin/bash
# C4 bench with 2 / 3 symmetric-kernel blocks per CU, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-symblocks}; mkdir -p $OUT
for k in 1 2; do for b in 2 3; do
  GE_FAML_SYM_BLOCKS=$b timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-end-to-end > $OUT/b${b}_$k.json 2> $OUT/b${b}_$k.err || { tail -5 $OUT/b${b}_$k.err; exit 1; }
  python3 -c "import json,sys; b=json.load(open('$OUT/b${b}_$k.json')); print('blocks/CU $b', round(b['ms_per_step'],2), 'ms/step', round(b['roofline']['avg_launch_ms'],2), 'ms sym')"
done; done
