cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4abt; export TMPDIR=/tmp
for v in cur r03; do
  unset GE_LIB_PATH
  [ $v = r03 ] && export GE_LIB_PATH=graph-embed_amd/variants/r03/libge.so
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4abt/t_$v -o t -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-end-to-end > gpurun_out/r4abt/$v.log 2>&1 || exit 1
  cp "$(find gpurun_out/r4abt/t_$v -name '*kernel_stats.csv' | head -1)" gpurun_out/r4abt/stats_$v.csv
  rm -rf gpurun_out/r4abt/t_$v
done
