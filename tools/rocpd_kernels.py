"""Per-kernel summary of a rocprofv3 SQLite output (``--kernel-trace`` writes a rocpd database):
calls, total / mean / min microseconds per kernel, plus (``--timeline``) the dispatch sequence
with the idle gap before each kernel — what `--stats` prints, for the output format this
image's rocprofv3 writes.

    python tools/rocpd_kernels.py gpurun_out/<dir>/prof/run_results.db [--timeline N]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--timeline", type=int, default=0, help="print the last N dispatches with gaps")
    ap.add_argument("--match", default="", help="only kernels whose name contains this")
    args = ap.parse_args()
    cur = sqlite3.connect(args.db).cursor()
    rows = cur.execute(
        "select s.display_name, d.start, d.end, d.grid_size_x, d.workgroup_size_x from rocpd_kernel_dispatch d "
        "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
    rows = [r for r in rows if args.match in r[0]]
    agg = collections.OrderedDict()
    for name, st, en, *_ in rows:
        a = agg.setdefault(name, [0, 0.0, float("inf")])
        a[0] += 1
        a[1] += (en - st) / 1e3
        a[2] = min(a[2], (en - st) / 1e3)
    total = sum(a[1] for a in agg.values())
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'mean_us':>9s} {'min_us':>9s} {'pct':>6s}")
    for name, (n, tot, mn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{name[:70]:70s} {n:6d} {tot:10.1f} {tot / n:9.1f} {mn:9.1f} {100 * tot / total:6.1f}")
    if args.timeline:
        print()
        prev = None
        for name, st, en, gx, wx in rows[-args.timeline:]:
            gap = (st - prev) / 1e3 if prev is not None else 0.0
            print(f"gap {gap:8.1f} us  run {(en - st) / 1e3:8.1f} us  grid {gx // max(wx, 1):6d}x{wx:<5d} {name[:60]}")
            prev = en


if __name__ == "__main__":
    main()
