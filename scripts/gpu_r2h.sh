#!/bin/bash
# GPU: symmetric-kernel parity tests, then C4 level-0 timing with paired steps
# (default build) and single steps (variant build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02h}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity.py tests/test_degenerate.py -k "faml or embed" > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
for v in paired single; do
  if [ $v = single ]; then export GE_LIB_PATH=graph-embed_amd/variants/single/libge.so; fi
  timeout -k 10 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-end-to-end \
    > $OUT/c4_$v.json 2> $OUT/c4_$v.err || { tail -5 $OUT/c4_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c4_$v.json'));r=d['roofline'];print('$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'])"
done
