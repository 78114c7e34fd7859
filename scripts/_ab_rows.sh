cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4ab3
for i in 1 2; do
  for v in cur handf r03; do
    unset GE_SYM_HAND_F GE_LIB_PATH
    [ $v = handf ] && export GE_SYM_HAND_F=1
    [ $v = r03 ] && export GE_LIB_PATH=graph-embed_amd/variants/r03/libge.so
    timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-end-to-end > gpurun_out/r4ab3/b_${v}_${i}.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/r4ab3/b_${v}_${i}.json'));print('$v', round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],2), round(d['roofline_attraction']['avg_launch_ms'],3), d['level_rate'])"
  done
done
