mkdir -p gpurun_out/t3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "replay or tiles" > gpurun_out/t3/tests.log 2>&1; rc=$?; tail -3 gpurun_out/t3/tests.log; exit $rc
