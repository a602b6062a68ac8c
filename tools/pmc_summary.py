"""Summarise rocprofv3 --pmc CSVs under gpurun_out/pmc for one kernel."""
import csv
import glob
import sys
from collections import defaultdict

kern = sys.argv[1] if len(sys.argv) > 1 else "rollout_kernel"
vals = defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        if kern in row.get("Kernel_Name", ""):
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
