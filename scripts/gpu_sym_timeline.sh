# Device partition parity + C4 timing, then symmetric repulsion timelines of one C4
# launch (scripts/sym_timeline.py) and the one-GPU rehearsal of N-GPU shares.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_partition_device.py > gpurun_out/part_par.log 2>&1 || { tail -30 gpurun_out/part_par.log; exit 1; }
tail -2 gpurun_out/part_par.log
GE_PROFILE_PARTITION=0 GE_PROGRESS=0 timeout -k 10 200 python -u scripts/partition_prof.py > gpurun_out/part_c4.log 2>&1 || exit 1
cat gpurun_out/part_c4.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" GE_SYM_STAMPS=gpurun_out/stamps_$tag.bin timeout -k 10 200 python -u scripts/sym_timeline.py > gpurun_out/sym_tl_$tag.json 2>gpurun_out/sym_tl_$tag.err || exit 1
}
run b3 GE_FAML_SYM_BLOCKS=3
run b4 GE_FAML_SYM_BLOCKS=4
run nowait_b4 GE_FAML_SYM_BLOCKS=4 GE_SYM_NOWAIT=1 ITERS=1
run b2 GE_FAML_SYM_BLOCKS=2
GE_FAML_SYM_BLOCKS=3 NS=1,4,8 timeout -k 10 300 python -u scripts/scale_sim.py > gpurun_out/scale_sim_b3.log 2>&1 || exit 1
