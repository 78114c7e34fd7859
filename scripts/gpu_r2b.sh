#!/bin/bash
# GPU: new parity tests first (multi-rank libge, overflow, P^T A P), then the
# whole GPU suite, then a short C4 bench and a 2-rank bench rehearsal (gloo).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dist.py tests/test_degenerate.py "tests/test_gpu_parity.py::test_ptap_golden" \
  > $OUT/new_tests.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -25 $OUT/new_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $OUT/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -8 $OUT/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?
echo "bench rc=$rc"; cat $OUT/bench_c4.json; tail -4 $OUT/bench_c4.err
[ $rc -eq 0 ] || exit $rc
GE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload c3 --steps 5 --warmup 1 \
  > $OUT/bench_c3_2rank.json 2> $OUT/bench_c3_2rank.err; rc=$?
echo "2-rank rc=$rc"; cat $OUT/bench_c3_2rank.json; tail -4 $OUT/bench_c3_2rank.err
exit $rc
