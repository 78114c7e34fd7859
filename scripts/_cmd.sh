mkdir -p gpurun_out/d2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "shards or dropin" > gpurun_out/d2/tests.log 2>&1; rc=$?; tail -3 gpurun_out/d2/tests.log; [ $rc -eq 0 ] || exit $rc
GE_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/d2/bench2.json 2> gpurun_out/d2/bench2.err; rc=$?
cut -c1-400 gpurun_out/d2/bench2.json; tail -3 gpurun_out/d2/bench2.err; exit $rc
