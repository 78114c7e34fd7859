"""Attraction pass timeline from a rocprofv3 kernel_trace.csv of the C4 bench.

Per attraction pass (the row kernels between two multilevel repulsion launches):
every row-kernel dispatch's start / end relative to the pass's first row-kernel
start, grouped by (kernel, grid); the median over the passes is printed, plus the
median pass span (first start to last end).
usage: python scripts/rows_timeline.py kernel_trace.csv
"""
import csv
import statistics
import sys
from collections import defaultdict

ROWS = ("tile_rows_kernel", "heavy_chain_kernel", "heavy_finish_kernel", "classed_rows_kernel")
REP = "faml_sym_repulse"

ev = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        nm = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
        if REP in nm:
            ev.append((s, e, "rep", grid))
        else:
            for k in ROWS:
                if k in nm:
                    ev.append((s, e, k, grid))
ev.sort()
passes, cur = [], []
for x in ev:
    if x[2] == "rep":
        if cur:
            passes.append(cur)
        cur = []
    else:
        cur.append(x)
if cur:
    passes.append(cur)
passes = [p for p in passes if len(p) >= 2]
rel = defaultdict(lambda: ([], []))
spans = []
for p in passes:
    t0 = min(x[0] for x in p)
    spans.append((max(x[1] for x in p) - t0) / 1e3)
    for s, e, k, g in p:
        rel[(k, g)][0].append((s - t0) / 1e3)
        rel[(k, g)][1].append((e - t0) / 1e3)
print(f"passes {len(passes)}  median span {statistics.median(spans):.1f} us")
for (k, g), (ss, es) in sorted(rel.items(), key=lambda kv: statistics.median(kv[1][0])):
    print(f"{k:22s} grid {g:>10s}  n={len(ss):3d}  start {statistics.median(ss):8.1f}  "
          f"end {statistics.median(es):8.1f} us")
