mkdir -p gpurun_out/c5a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c5a/tests.log 2>&1; rc=$?; tail -3 gpurun_out/c5a/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c5_attraction.py --n 1000000 --draws 8000000 2>&1 | grep -v amdgpu.ids
