cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r04c5; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/c5_attraction.py > gpurun_out/r04c5/c5_attraction.json 2> gpurun_out/r04c5/c5_attraction.err || { tail -5 gpurun_out/r04c5/c5_attraction.err; exit 1; }
cat gpurun_out/r04c5/c5_attraction.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 500 rocprofv3 --pmc $c --kernel-include-regex "rows_kernel|heavy_" --output-format csv -d gpurun_out/r04c5/p_$c -o p -- python3 scripts/c5_attraction.py --steps 2 --warmup 1 > gpurun_out/r04c5/p_$c.log 2>&1 || { tail -5 gpurun_out/r04c5/p_$c.log; exit 1; }
  cp "$(find gpurun_out/r04c5/p_$c -name '*counter_collection.csv' | head -1)" gpurun_out/r04c5/pmc_${c}_c5.csv; rm -rf gpurun_out/r04c5/p_$c
  python3 scripts/pmc_summary.py gpurun_out/r04c5/pmc_${c}_c5.csv ""
done
