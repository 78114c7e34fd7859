# round 3: LDS-by-component records; sym vs sym2 timings and SQ counters on C4 (one GPU)
set -o pipefail
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for v in sym sym2; do
  if [ $v = sym2 ]; then export GE_FAML_SYM2=1; fi
  NS=1 ITERS=2 timeout -s KILL 240 rocprofv3 --kernel-include-regex "faml_sym" --pmc $C --output-format csv -d /tmp/pmc_$v -o p -- python3 scripts/scale_sim.py > gpurun_out/r3d/pmc_$v.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py /tmp/pmc_$v faml_sym gpurun_out/r3d/pmc_$v.json || exit 1
done
