set -o pipefail
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lone or symmetric" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b/lone.log 2>&1 || { tail -30 gpurun_out/r3b/lone.log; exit 1; }
tail -2 gpurun_out/r3b/lone.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_radius.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b/radius.log 2>&1 || { tail -30 gpurun_out/r3b/radius.log; exit 1; }
tail -2 gpurun_out/r3b/radius.log
SAVE_LEVEL=gpurun_out/r3b/c4_level0.npz NS=1,8 timeout -k 10 300 python -u scripts/scale_sim.py > gpurun_out/r3b/sim_base.log 2>&1 || exit 1
cat gpurun_out/r3b/sim_base.log
for k in 1 3; do GE_FAML_LONE=$k NS=1,8 timeout -k 10 300 python -u scripts/scale_sim.py > gpurun_out/r3b/sim_lone$k.log 2>&1 || exit 1; echo lone$k; cat gpurun_out/r3b/sim_lone$k.log; done
timeout -k 10 950 python -u -m pytest tests/test_gpu_configs.py -k "c5_level0" -x -v -s --timeout 940 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b/c5.log 2>&1; rc=$?; tail -30 gpurun_out/r3b/c5.log; exit $rc
