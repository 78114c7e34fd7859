#!/bin/bash
# C4 device partition with GE_PART_MID_BLOCKS = 512 / 1024 / 2048, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-midblocks}; mkdir -p $OUT
for k in 1 2; do for b in 512 1024 2048; do
  GE_PART_MID_BLOCKS=$b timeout -k 10 200 python3 -u scripts/partition_prof.py > $OUT/m${b}_$k.log 2>&1 || { tail -5 $OUT/m${b}_$k.log; exit 1; }
  echo "mid blocks $b: $(grep -E 'partition_device: n=' $OUT/m${b}_$k.log | grep -oE 'merges [0-9.]+s')"
done; done
