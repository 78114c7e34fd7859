mkdir -p gpurun_out/r3r
timeout -k 10 300 python -u -m pytest tests/test_partition_device.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3r/part_tests.log 2>&1 || exit 1
GE_PROFILE_ROUNDS=1 timeout -k 10 200 python -u scripts/partition_prof.py > gpurun_out/r3r/part.log 2> gpurun_out/r3r/rounds.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_part -o part -- python3 $GRAFT_REPO_ROOT/scripts/partition_prof.py > $GRAFT_REPO_ROOT/gpurun_out/r3r/prof.log 2>&1 || exit 1
f=$(find /tmp/prof_part -name "*kernel_trace.csv" | head -1)
python3 $GRAFT_REPO_ROOT/scripts/trace_buckets.py $f "rebuild_global,scan_mid,scan_huge_part,rebuild_block,scan_small,mark_dirty" > $GRAFT_REPO_ROOT/gpurun_out/r3r/buckets.log 2>&1
python3 - "$f" > $GRAFT_REPO_ROOT/gpurun_out/r3r/stats.log 2>&1 <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(int); cnt = defaultdict(int)
first = last = None
for r in csv.DictReader(open(sys.argv[1])):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    tot[r["Kernel_Name"][:70]] += e - s; cnt[r["Kernel_Name"][:70]] += 1
    first = s if first is None else min(first, s); last = e if last is None else max(last, e)
print("kernel time total %.3f s, span %.3f s" % (sum(tot.values()) / 1e9, (last - first) / 1e9))
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:25]:
    print("%8.3f s %8d  %s" % (v / 1e9, cnt[k], k))
PY
