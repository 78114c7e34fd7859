#!/bin/bash
# GPU: symmetric-kernel occupancy variants (no LDS prefetch, 5 / 6 waves per SIMD)
# against the default build on the C4 level-0 bench; parity of the variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02l}
mkdir -p $OUT
export TMPDIR=/tmp
for v in default np5 np6; do
  if [ $v != default ]; then export GE_LIB_PATH=graph-embed_amd/variants/$v/libge.so; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py -k "symmetric or faml_golden" > $OUT/t_$v.log 2>&1 || { tail -5 $OUT/t_$v.log; exit 1; }
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-end-to-end \
    > $OUT/c4_$v.json 2> $OUT/c4_$v.err || { tail -5 $OUT/c4_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c4_$v.json'));r=d['roofline'];print('$v', d['value'], d['ms_per_step'], r['avg_launch_ms'])"
done
