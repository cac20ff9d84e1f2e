"""Per-kernel means of every counter in one or more rocprofv3 PMC runs (CSV output):

    python tools/pmc_table.py gpurun_out/<dir>/pmc/g*/run_counter_collection.csv
"""
import collections
import csv
import sys


def main():
    for path in sys.argv[1:]:
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        dur = collections.defaultdict(float)
        seen = collections.defaultdict(set)
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1][:34]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            key = r.get("Dispatch_Id") or r.get("Correlation_Id")
            if key not in seen[k]:
                seen[k].add(key)
                dur[k] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(path)
        for k, v in sorted(agg.items(), key=lambda kv: -dur[kv[0]]):
            n = len(seen[k])
            vals = " ".join(f"{a}={b / n:.4g}" for a, b in v.items())
            print(f"  {k:34s} n={n:3d} us={dur[k] / n / 1e3:7.1f} {vals}")


if __name__ == "__main__":
    main()
