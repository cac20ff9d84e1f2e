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
    ap.add_argument("--per", default="aes128_cbc_decrypt",
                    help="--busy: the window runs from this kernel's first dispatch to its last, one step each")
    ap.add_argument("--busy", action="store_true",
                    help="also the device's busy time: the union of kernel (and memory-copy) intervals against "
                         "the sum of kernel durations (concurrency makes per-kernel durations overlap)")
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
    if args.busy:
        busy(cur, rows, args.per)
    if args.timeline:
        print()
        prev = None
        for name, st, en, gx, wx in rows[-args.timeline:]:
            gap = (st - prev) / 1e3 if prev is not None else 0.0
            print(f"gap {gap:8.1f} us  run {(en - st) / 1e3:8.1f} us  grid {gx // max(wx, 1):6d}x{wx:<5d} {name[:60]}")
            prev = en


def _union(iv):
    tot, end = 0, None
    for st, en in sorted(iv):
        if end is None or st > end:
            tot += en - st
            end = en
        elif en > end:
            tot += en - end
            end = en
    return tot


def busy(cur, rows, per):
    marks = [(st, en) for name, st, en, *_ in rows if per in name]
    if len(marks) < 2:
        return
    t0, t1 = marks[0][0], marks[-1][1]  # steady state: first to last dispatch of `per`
    clip = [(max(st, t0), min(en, t1)) for _, st, en, *_ in rows if en > t0 and st < t1]
    try:
        copies = [(max(st, t0), min(en, t1)) for st, en in
                  cur.execute("select start, end from rocpd_memory_copy").fetchall() if en > t0 and st < t1]
    except sqlite3.Error:
        copies = []
    n = len(marks)
    ksum, ku, cu = sum(en - st for st, en in clip), _union(clip), _union(clip + copies)
    print(f"\nsteady window {(t1 - t0) / 1e3:.1f} us over {n} '{per}' dispatches ({(t1 - t0) / 1e3 / n:.1f} us each): "
          f"kernels sum {ksum / 1e3 / n:.1f} us, union {ku / 1e3 / n:.1f} us per step "
          f"(device busy {100 * ku / (t1 - t0):.1f} %, mean kernel concurrency {ksum / max(ku, 1):.2f}); "
          f"with DMA copies {cu / 1e3 / n:.1f} us per step ({100 * cu / (t1 - t0):.1f} %)")


if __name__ == "__main__":
    main()
