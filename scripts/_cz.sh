set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5q
export MODES=persistent
for v in ${VARS:-main dc1 dc2}; do
  if [ $v = main ]; then unset GE_LIB_PATH; else export GE_LIB_PATH=graph-embed_amd/variants/$v/libge.so; fi
  echo "== $v" | tee -a gpurun_out/r5q/coarse.log
  timeout -k 10 300 python -u scripts/coarsest_time.py 1068 20000 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r5q/coarse.log || exit 1
done
