mkdir -p gpurun_out/r3m
for n in 130 1068; do
  timeout -k 10 120 python -u scripts/coarsest_time.py $n 20000 >> gpurun_out/r3m/sweep.log 2>&1 || exit 1
  echo tree >> gpurun_out/r3m/sweep.log
  GE_PERSIST_TREE=1 timeout -k 10 120 python -u scripts/coarsest_time.py $n 20000 >> gpurun_out/r3m/sweep.log 2>&1 || exit 1
done
