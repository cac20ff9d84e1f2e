"""Summarise tools/pmc_kernels.sh output: mean counter value per kernel."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc") + "/g*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if k.startswith("__amd") or "elementwise" in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):.4g}")
