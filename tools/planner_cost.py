"""Host cost of the replicated control plane at N ranks (round-3 VERDICT item 4).

Every rank runs, each round, ``ingest_control`` (all ranks' cache deltas into the native
``Directory`` + the round's want rows) and ``plan_round`` (deterministic holder / CDN-seed
choice) over ALL ranks' wants (``agent/node.py:launch_round``).  This times exactly those
two native calls on synthetic messages shaped like the bench's steady state:

* every rank wants the same ``W`` new segments per round (player ``w`` plays the same slice
  on every rank, ``bench.py``), none resident yet: the planner seeds each from the CDN on
  one rank and forwards it to the others in the same round (CDN dedup);
* every rank announces ``W`` adds (last round's segments, now resident) and ``W`` removes
  (ring eviction of the oldest ones), so the directory holds a steady window of
  ``--resident`` segments per rank.

    python tools/planner_cost.py [--world 8] [--wants 256 512 1024] [--rounds 300]

Prints one JSON line per (world, wants): microseconds per round for each call, the
message size in int64 words, and whether it fits the shared-memory control slot.
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np

from hlsjs_p2p_wrapper_amd.agent.node import HDR, MAGIC
from hlsjs_p2p_wrapper_amd.ops._native import runtime
from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm

SEG = 3_000_000  # 1080p 6 Mb/s x 4 s


def _msg(rt, rank: int, rnd: int, wants: np.ndarray, adds: np.ndarray, rms: np.ndarray) -> np.ndarray:
    hdr = np.zeros(HDR, dtype=np.int64)
    hdr[0] = MAGIC
    hdr[1] = rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD | rt.FLAG_CDN_DEDUP
    hdr[2], hdr[3], hdr[4] = len(wants), len(adds), len(rms)
    hdr[6] = rnd
    return np.concatenate([hdr, wants.reshape(-1), adds.reshape(-1), rms.reshape(-1)])


def _keys(sn0: int, n: int) -> np.ndarray:
    k = np.zeros((n, 4), dtype=np.int64)
    k[:, 0] = 7  # swarm id
    k[:, 3] = np.arange(sn0, sn0 + n)
    return k


def run(world: int, W: int, rounds: int, resident: int) -> dict:
    rt = runtime()
    d = rt.Directory()
    # steady state: every rank holds the last `resident` segments
    warm = _keys(0, resident)
    adds0 = np.concatenate([warm, np.full((resident, 1), SEG, dtype=np.int64)], axis=1)
    for r in range(world):
        d.apply(r, np.ascontiguousarray(adds0), np.zeros((0, 4), dtype=np.int64))
    t_ing = t_plan = 0.0
    words = 0
    rows_out = 0
    sn = resident
    for rnd in range(rounds):
        new = _keys(sn, W)
        wants = np.concatenate([new, np.full((W, 1), SEG, dtype=np.int64),
                                np.arange(W, dtype=np.int64)[:, None] + rnd * W], axis=1)
        prev = _keys(sn - W, W)  # fetched last round: now resident everywhere
        adds = np.concatenate([prev, np.full((W, 1), SEG, dtype=np.int64)], axis=1)
        rms = _keys(sn - resident - W, W) if sn - resident - W >= 0 else np.zeros((0, 4), dtype=np.int64)
        parts = [_msg(rt, r, rnd, wants, adds, rms) for r in range(world)]
        words = max(words, len(parts[0]))
        t0 = time.perf_counter()
        all_wants, flags, _, _ = rt.ingest_control(d, parts, MAGIC, HDR)
        t1 = time.perf_counter()
        plan, _, _ = rt.plan_round_for(d, all_wants, flags, world, rnd % world)  # as agent/node.py calls it
        t2 = time.perf_counter()
        if rnd >= rounds // 10:  # skip the first tenth (allocator / cache warm-up)
            t_ing += t1 - t0
            t_plan += t2 - t1
        rows_out = len(plan)
        sn += W
    n = rounds - rounds // 10
    return {"world": world, "wants_per_rank": W, "resident_per_rank": resident, "rounds": n,
            "ingest_control_us": round(t_ing / n * 1e6, 1), "plan_round_us": round(t_plan / n * 1e6, 1),
            "total_us": round((t_ing + t_plan) / n * 1e6, 1), "plan_rows_this_rank": rows_out,
            "msg_words": int(words), "fits_shm_slot": bool(words <= DistComm.SHM_SLOT_WORDS)}


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--world", type=int, nargs="+", default=[8])
    p.add_argument("--wants", type=int, nargs="+", default=[256, 512, 1024])
    p.add_argument("--rounds", type=int, default=300)
    p.add_argument("--resident", type=int, default=2700, help="segments held per rank (8 GB / 3 MB)")
    a = p.parse_args()
    for w in a.world:
        for k in a.wants:
            print(json.dumps(run(w, k, a.rounds, a.resident)), flush=True)


if __name__ == "__main__":
    main()
