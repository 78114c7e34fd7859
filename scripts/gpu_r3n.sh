mkdir -p gpurun_out/r3r
timeout -k 10 300 python -u -m pytest tests/test_partition_device.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3r/part_tests.log 2>&1 || exit 1
GE_PROFILE_ROUNDS=1 timeout -k 10 200 python -u scripts/partition_prof.py > gpurun_out/r3r/part.log 2> gpurun_out/r3r/rounds.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_part -o part -- python3 $GRAFT_REPO_ROOT/scripts/partition_prof.py > $GRAFT_REPO_ROOT/gpurun_out/r3r/prof.log 2>&1 || exit 1
f=$(find /tmp/prof_part -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/scripts/trace_buckets.py $f "rebuild_global,scan_mid,scan_big_kernel<1024>,rebuild_block,scan_small,mark_dirty" > $GRAFT_REPO_ROOT/gpurun_out/r3r/buckets.log 2>&1
