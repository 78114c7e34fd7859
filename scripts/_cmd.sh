export TMPDIR=/tmp
mkdir -p gpurun_out/c5
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --output-format csv -d gpurun_out/c5/pmc_$c -o c5 -- python3 -u scripts/c5_attraction.py --steps 2 --warmup 1 > gpurun_out/c5/pmc_$c.json 2> gpurun_out/c5/pmc_$c.err || exit 1
  find gpurun_out/c5/pmc_$c -name "*counter_collection.csv" -exec cp {} gpurun_out/c5/pmc_$c.csv \;
  rm -rf gpurun_out/c5/pmc_$c
done
python3 - <<'PY'
import csv
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = {}
    for r in csv.DictReader(open(f"gpurun_out/c5/pmc_{c}.csv")):
        if "rows_kernel" in r["Kernel_Name"] or "finish" in r["Kernel_Name"]:
            vals.setdefault(r["Kernel_Name"][:40], []).append(float(r["Counter_Value"]))
    for k, v in vals.items():
        print(c, k, [round(x * 1024 / 1e9, 2) for x in v], "GB (x1024)")
PY
