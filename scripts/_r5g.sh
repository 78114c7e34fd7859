set -o pipefail
bash scripts/gpu.sh r5g_tr trace:c4 && \
bash scripts/gpu.sh r5g_tr0 env:GE_ROWS_XCD=0 env:GE_FAML_PULL=0 trace:c4 && \
bash scripts/gpu.sh r5g_trp env:GE_ROWS_XCD=0 trace:c4 && \
bash scripts/gpu.sh r5g_t tests
