mkdir -p gpurun_out/c8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c8/tests.log 2>&1; rc=$?; tail -3 gpurun_out/c8/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/coarse_tune.py 2>&1 | grep us/iter
