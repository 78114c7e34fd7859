mkdir -p gpurun_out/seg4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/seg4/tests.log 2>&1; rc=$?; tail -3 gpurun_out/seg4/tests.log; [ $rc -eq 0 ] || exit $rc
export GE_ROWS_STATS=1
GE_TUNE_GRAPHS=star_rand,rmat GE_TUNE_CONFIGS="1,32,512" GE_TUNE_ENVS=";GE_ROWS_SEGMENTS=0" timeout -k 10 200 python scripts/rows_tune.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --workload c3 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/seg4/c3.json 2> gpurun_out/seg4/c3.err; rc=$?; cut -c1-330 gpurun_out/seg4/c3.json; exit $rc
