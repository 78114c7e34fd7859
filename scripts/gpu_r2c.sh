#!/bin/bash
# GPU: device radius step tests + embed goldens, then C4 end-to-end with per-level
# embed timing (device radius step, then host radius step) and a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_radius.py tests/test_gpu_parity.py -k "radius or embed" > $OUT/radius_tests.log 2>&1; rc=$?
echo "radius tests rc=$rc"; tail -22 $OUT/radius_tests.log
[ $rc -eq 0 ] || exit $rc
GE_PROFILE_EMBED=1 timeout -k 10 400 python bench.py --steps 2 --warmup 0 --no-cpu-baseline \
  > $OUT/c4_dev.json 2> $OUT/c4_dev.err; rc=$?
echo "c4 device radius rc=$rc"; grep -E "embed:|LCC" $OUT/c4_dev.err; python -c "import json;d=json.load(open('$OUT/c4_dev.json'));print(d['embed_seconds_end_to_end'], d['setup_seconds'])"
[ $rc -eq 0 ] || exit $rc
GE_RADIUS_HOST=1 GE_PROFILE_EMBED=1 timeout -k 10 400 python bench.py --steps 2 --warmup 0 --no-cpu-baseline \
  > $OUT/c4_host.json 2> $OUT/c4_host.err; rc=$?
echo "c4 host radius rc=$rc"; grep -E "embed:" $OUT/c4_host.err; python -c "import json;d=json.load(open('$OUT/c4_host.json'));print(d['embed_seconds_end_to_end'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c4 -- \
  python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > $OUT/trace.log 2>&1; rc=$?
echo "trace rc=$rc"
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1); cp "$f" $OUT/c4_kernel_stats.csv
cut -d, -f1-5 $OUT/c4_kernel_stats.csv | head -30
exit $rc
