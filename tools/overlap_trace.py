"""Concurrency of RCCL and the transmux in a rocprofv3 kernel trace (rocpd database) of
``tools/overlap_n8.py``: busy time of the RCCL kernels, of the decrypt kernel and of every
kernel, and how much of the RCCL busy time ran while a decrypt grid was resident.

    python tools/overlap_trace.py run_results.db
"""
import json
import sqlite3
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    cur = sqlite3.connect(sys.argv[1]).cursor()
    rows = cur.execute("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d "
                       "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    rccl = union([(s, e) for n, s, e in rows if "rccl" in n.lower() or "nccl" in n.lower()])
    aes = union([(s, e) for n, s, e in rows if "aes128" in n])
    every = union([(s, e) for _, s, e in rows])
    both = intersect(rccl, aes)
    print(json.dumps({"kernels": len(rows), "rccl_kernels": sum(1 for n, *_ in rows if "rccl" in n.lower()),
                      "rccl_busy_ms": round(length(rccl) / 1e6, 3), "decrypt_busy_ms": round(length(aes) / 1e6, 3),
                      "device_busy_ms": round(length(every) / 1e6, 3),
                      "rccl_beside_decrypt_ms": round(length(both) / 1e6, 3),
                      "rccl_beside_decrypt_share": round(length(both) / max(1, length(rccl)), 3)}))


if __name__ == "__main__":
    main()
