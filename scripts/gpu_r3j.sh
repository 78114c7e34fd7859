# round 3: sweep hand-over sub-tiles (16/32/64 columns): parity, C4 level 0, shares
set -o pipefail
mkdir -p gpurun_out/r3j
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "symmetric or faml" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j/par.log 2>&1 || { tail -40 gpurun_out/r3j/par.log; exit 1; }
tail -2 gpurun_out/r3j/par.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k "c4_level0" -x -q --timeout 280 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j/c4.log 2>&1 || { tail -40 gpurun_out/r3j/c4.log; exit 1; }
tail -2 gpurun_out/r3j/c4.log
for w in 16 32 64; do GE_FAML_SYM_SUB=$w NS=1,2,4,8 timeout -k 10 400 python -u scripts/scale_sim.py > gpurun_out/r3j/sim_$w.log 2>&1 || { cat gpurun_out/r3j/sim_$w.log; exit 1; }; echo sub$w; cut -c1-400 gpurun_out/r3j/sim_$w.log | grep -v amdgpu; done
