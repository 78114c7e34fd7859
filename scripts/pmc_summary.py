"""Sums rocprofv3 --pmc counter CSVs per kernel (kernels whose name contains a
pattern) into one small JSON line -- totals, dispatch count and the per-dispatch
average of every counter; the raw directory can then be removed.
usage: python scripts/pmc_summary.py <rocprof out dir or csv> [<name pattern>] [<out.json>]"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    tot, disp = {}, {}
    paths = [d] if os.path.isfile(d) else glob.glob(
        os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for path in paths:
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if pat not in name:
                    continue
                key = name.split("(")[0]
                c = row["Counter_Name"]
                tot.setdefault(key, {}).setdefault(c, 0.0)
                tot[key][c] += float(row["Counter_Value"])
                disp.setdefault(key, set()).add(row.get("Dispatch_Id"))
    out = {k: dict(v, dispatches=len(disp[k]),
                   per_dispatch={c: x / len(disp[k]) for c, x in v.items()})
           for k, v in tot.items()}
    s = json.dumps(out)
    print(s)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
