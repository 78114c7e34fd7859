# round 3: the whole GPU suite (durations), smoke, then the default bench line
set -o pipefail
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --durations=30 --timeout 990 --timeout-method thread -p no:cacheprovider > gpurun_out/r3h/gpu_tests.log 2>&1; rc=$?
tail -45 gpurun_out/r3h/gpu_tests.log
[ $rc = 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3h/smoke.log 2>&1 || { cat gpurun_out/r3h/smoke.log; exit 1; }
cat gpurun_out/r3h/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3h/bench_c4.json 2> gpurun_out/r3h/bench_c4.err || { tail -20 gpurun_out/r3h/bench_c4.err; exit 1; }
cat gpurun_out/r3h/bench_c4.json
