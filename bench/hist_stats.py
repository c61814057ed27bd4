"""Per-kernel totals of the histogram kernels in rocprofv3 kernel_stats CSVs (bench/exp_hist.sh)."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    path = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    tot = 0.0
    print("==", d)
    for r in rows:
        if "hist_" in r["Name"] or "partition" in r["Name"] or "split" in r["Name"]:
            ms = float(r["TotalDurationNs"]) / 1e6
            tot += ms
            print(f"{ms:8.2f} ms {int(r['Calls']):4d} {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][24:90]}")
    print(f"{tot:8.2f} ms total")
