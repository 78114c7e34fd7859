set -o pipefail
B="bench:c4:--no-cpu-baseline,--no-end-to-end"
bash scripts/ab_env.sh r5f_ab GE_LIB_PATH "- graph-embed_amd/variants/rcp/libge.so" 2 && \
bash scripts/gpu.sh r5f_base env:GE_ROWS_XCD=0 env:GE_FAML_PULL=0 $B && \
bash scripts/gpu.sh r5f_xcd env:GE_FAML_PULL=0 $B && \
bash scripts/gpu.sh r5f_c5 c5 && \
bash scripts/gpu.sh r5f_c5bfs c5:--relabel,bfs && \
bash scripts/gpu.sh r5f_c5noxcd env:GE_ROWS_XCD=0 c5 && \
bash scripts/gpu.sh r5f_c2sim env:WORKLOAD=c2 py:scripts/scale_sim.py
