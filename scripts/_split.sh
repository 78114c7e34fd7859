# SURVEY 8(e) split rehearsal (scripts/scale_sim.py SPLIT_MIN) + C2 trace/PMC + C5 attraction.
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04split; mkdir -p $O; export TMPDIR=/tmp
for k in 30000 15000; do
  NS=8 SPLIT_MIN=$k timeout -k 10 400 python -u scripts/scale_sim.py > $O/scale_split_$k.log 2>&1 \
    || { tail -8 $O/scale_split_$k.log; exit 1; }
  python3 -c "
import json
for l in open('$O/scale_split_$k.log'):
    if l.startswith('{'):
        d=json.loads(l); print($k, d['N'], round(d['max_ms'],2), 'rep', [round(x,2) for x in d['repulse_ms_by_rank']], 'rows', [round(x,2) for x in d['rows_ms_by_rank']], d.get('split_aggregates'), d.get('exchange_ms_priced'))
"
done
bash scripts/gpu.sh r04h trace:c2 pmc:c2:FETCH_SIZE pmc:c2:WRITE_SIZE && bash scripts/_c5.sh
