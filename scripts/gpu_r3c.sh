# round 3: sym2 (producer/adder sweeps) parity + C4 one-GPU shares, C5 multilevel test
set -o pipefail
mkdir -p gpurun_out/r3c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "workgroup or symmetric or lone" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c/par.log 2>&1 || { tail -40 gpurun_out/r3c/par.log; exit 1; }
tail -2 gpurun_out/r3c/par.log
GE_FAML_SYM2=1 NS=1,8 timeout -k 10 300 python -u scripts/scale_sim.py > gpurun_out/r3c/sim_sym2.log 2>&1 || { cat gpurun_out/r3c/sim_sym2.log; exit 1; }
cat gpurun_out/r3c/sim_sym2.log
for b in 3; do GE_FAML_SYM_BLOCKS=$b NS=8 timeout -k 10 300 python -u scripts/scale_sim.py > gpurun_out/r3c/sim_b$b.log 2>&1 || exit 1; echo bpc$b; cat gpurun_out/r3c/sim_b$b.log; done
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py -k "c5_level0" -x -v -s --timeout 990 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c/c5.log 2>&1; rc=$?; grep -v "^  " gpurun_out/r3c/c5.log | tail -25; exit $rc
