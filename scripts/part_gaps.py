"""Busy time vs idle gaps of the device partition in a rocprofv3 kernel_trace.csv.

Restricted to the round loop (first classify_scan_kernel .. last dispatch).  Reports
the span, the union of kernel intervals, the idle time split by the kernel that
follows the gap (a gap before the round's first classify_scan_kernel is the host
synchronisation + bookkeeping; the others are dispatch latency between queued
kernels), and per-kernel sums."""
import csv
import sys
from collections import defaultdict


def short(nm):
    nm = nm.replace("ge::(anonymous namespace)::", "").replace("void ", "")
    return nm.split("(")[0]


rows = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
rows.sort()
first = next(i for i, r in enumerate(rows) if r[2].startswith("classify_scan_kernel"))
rows = rows[first:]
span = rows[-1][1] - rows[0][0]
busy = 0
cur_s, cur_e = rows[0][0], rows[0][1]
gap_before = defaultdict(float)
ngap = defaultdict(int)
per = defaultdict(float)
cnt = defaultdict(int)
prev_end = rows[0][1]
for s, e, nm in rows:
    per[nm] += e - s
    cnt[nm] += 1
    if s > cur_e:
        busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    if s > prev_end:
        gap_before[nm] += s - prev_end
        ngap[nm] += 1
    prev_end = max(prev_end, e)
busy += cur_e - cur_s
print(f"dispatches {len(rows)}  span {span / 1e9:.3f} s  busy {busy / 1e9:.3f} s  idle {(span - busy) / 1e9:.3f} s")
print("idle before kernel (s, count, mean us):")
for nm, g in sorted(gap_before.items(), key=lambda x: -x[1])[:16]:
    print(f"  {g / 1e9:8.3f} {ngap[nm]:8d} {g / max(ngap[nm], 1) / 1e3:8.1f}  {nm}")
print("kernel time (s, calls, mean us):")
for nm, t in sorted(per.items(), key=lambda x: -x[1])[:24]:
    print(f"  {t / 1e9:8.3f} {cnt[nm]:8d} {t / cnt[nm] / 1e3:8.1f}  {nm}")
