# Symmetric repulsion: parity of the sweep kernels, then per-unit timelines of one
# C4 launch (scripts/sym_timeline.py) and the one-GPU rehearsal of N-GPU shares.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_parity.py -k "symmetric or faml" > gpurun_out/sym_par.log 2>&1 || { tail -30 gpurun_out/sym_par.log; exit 1; }
tail -2 gpurun_out/sym_par.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" GE_SYM_STAMPS=gpurun_out/stamps_$tag.bin timeout -k 10 200 python -u scripts/sym_timeline.py > gpurun_out/sym_tl_$tag.json 2>gpurun_out/sym_tl_$tag.err || exit 1
}
run pf
NS=1,8 timeout -k 10 300 python -u scripts/scale_sim.py > gpurun_out/scale_sim_pf.log 2>&1 || exit 1
