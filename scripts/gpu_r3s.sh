mkdir -p gpurun_out/r3s
timeout -k 10 300 python -u -m pytest tests/test_partition_device.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3s/part_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/partition_prof.py > gpurun_out/r3s/part.log 2>&1
