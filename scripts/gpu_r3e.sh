# round 3: split aggregates across ranks (transport ranks on one GPU) + C5 multilevel test
set -o pipefail
mkdir -p gpurun_out/r3e
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3e/dist.log 2>&1 || { tail -40 gpurun_out/r3e/dist.log; exit 1; }
tail -2 gpurun_out/r3e/dist.log
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -k "c5_level0" -x -v -s --timeout 990 --timeout-method thread -p no:cacheprovider > gpurun_out/r3e/c5.log 2>&1; rc=$?; grep -v "^  " gpurun_out/r3e/c5.log | tail -25; exit $rc
