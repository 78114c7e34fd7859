"""Sum kernel durations of a rocprofv3 kernel_trace.csv by dispatch-order buckets
(per kernel name, the k-th dispatch of a once-per-round kernel is round k)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
names = sys.argv[2].split(",")
per = defaultdict(list)
with open(path) as f:
    for r in csv.DictReader(f):
        nm = r["Kernel_Name"]
        for key in names:
            if key in nm:
                per[key].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
edges = [0, 10, 100, 1000, 3000, 10000, 10**9]
for key in names:
    v = sorted(per[key])
    calls_per_round = 2 if "scan" in key or "resolve" in key or "filter" in key else 1
    out = []
    for lo, hi in zip(edges[:-1], edges[1:]):
        seg = v[lo * calls_per_round:hi * calls_per_round]
        if seg:
            out.append(f"rounds[{lo},{hi}) {sum(d for _, d in seg) / 1e6:.1f} ms")
    print(key, len(v), "; ".join(out))
