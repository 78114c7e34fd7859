# round 3: C5 graph (device vs host, LCC), then the C5 multilevel test
set -o pipefail
mkdir -p gpurun_out/r3g
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/c5_graph_check.py > gpurun_out/r3g/c5graph.log 2>&1 || { cat gpurun_out/r3g/c5graph.log; exit 1; }
cat gpurun_out/r3g/c5graph.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -k "c5_level0" -x -v -s --timeout 990 --timeout-method thread -p no:cacheprovider > gpurun_out/r3g/c5.log 2>&1; rc=$?; grep -v "^  " gpurun_out/r3g/c5.log | tail -30; exit $rc
