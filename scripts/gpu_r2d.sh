#!/bin/bash
# GPU: drop-in tests (embedVia via the C++ driver), then PMC of the symmetric kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 800 --timeout-method thread -p no:cacheprovider \
  tests/test_dropin.py > $OUT/dropin.log 2>&1; rc=$?
echo "dropin rc=$rc"; tail -12 $OUT/dropin.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_sym.sh ${1:-r02d}/pmcsym c4
