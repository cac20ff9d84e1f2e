"""Effective clock per kernel from a rocprofv3 PMC run with GRBM_GUI_ACTIVE (GPU-busy cycles):
counter cycles divided by the dispatch's duration.  Comparing a kernel isolated against the
same kernel inside the pipeline separates "runs at a lower clock" (the device idles between
bursts and does not boost) from "does more work / waits longer".

    python tools/pmc_clock.py gpurun_out/<dir>/g1/run_counter_collection.csv [COUNTER]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    counter = sys.argv[2] if len(sys.argv) > 2 else "GRBM_GUI_ACTIVE"
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
        a = agg[name]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
        a[2] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print(f"{'kernel':40s} {'calls':>6s} {'mean_us':>9s} {counter + ' / ns':>22s}")
    for name, (n, c, ns) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        print(f"{name[:40]:40s} {n:6d} {ns / n / 1e3:9.1f} {c / max(ns, 1):22.3f}")


if __name__ == "__main__":
    main()
