"""Host cost of one rank's swarm rounds at N ranks, measured in isolation (no peers, no GPU).

At N=8 the rank's Python host path (control message, planning, the P2P phase's layout and
posting, deliveries, deferred-check bookkeeping) has to fit inside the step the PCIe link
sets (~1.7 ms for 256 segments), and a rehearsal with 8 ranks sharing one box's CPUs cannot
tell its real cost (every figure is inflated by contention, ``profiles/r6_n8``).  Here rank 0
runs alone: a fake communicator answers its control all-gather with the messages of N-1
synthetic peers shaped like the bench's steady state -- every rank wants the same ``W`` new
segments per round (each player plays the same slice on every rank), announces the previous
round's segments as added and the oldest as removed -- so the native planner seeds ``W/N``
of them on rank 0 and forwards each to the other N-1 ranks, and rank 0 receives the rest
from the N-1 seeders.  The data plane is a no-op (the bytes are not the point) and every
received row is checked by a fake consumer that reports it passed one round later, as the
fleet's transmux does.

    PYTHONPATH=. python tools/round_replay.py [--world 8] [--wants 256] [--rounds 200] [--profile out.txt]

Prints one JSON line: host microseconds per round for each node phase, launch and complete
totals, and the plan's shape (CDN rows, sends, receives per round).
"""
from __future__ import annotations

import argparse
import cProfile
import json
import os
import pstats
import time

import numpy as np

os.environ.setdefault("HLSP2P_AUDIT", "0")

from hlsjs_p2p_wrapper_amd.agent.node import CHECK_WORD, HDR, MAGIC, SwarmNode  # noqa: E402
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop  # noqa: E402
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin  # noqa: E402
from hlsjs_p2p_wrapper_amd.ops._native import runtime  # noqa: E402
from hlsjs_p2p_wrapper_amd.parallel.comm import SwarmComm  # noqa: E402


class FakePeers(SwarmComm):
    """Rank 0 of ``world``: the other ranks' control messages are synthesized each round.

    Every peer wants what rank 0 wants this round (same keys and sizes, its own want ids),
    announces the segments wanted the round before as added (every rank received all of them)
    and those ``keep`` rounds old as removed (its ring), and echoes rank 0's consistency and
    counter words, so the planner's replicas and CDN balance see agreeing, even peers."""

    def __init__(self, world: int, keep: int = 8, churn: int = 0) -> None:
        self.rank, self.world_size = 0, world
        self.keep = keep
        # churn (BASELINE config 3): every `churn` rounds the next peer goes offline for `churn`
        # rounds (masked in the control plane: it neither serves nor receives P2P and fetches
        # its wants from the CDN), then one all-online period -- bench.py's --churn rotation
        self.churn = churn
        self.rounds = 0
        self.rt = runtime()
        self.held: list = []  # per round: (keys [n, 4], sizes [n]) every fake peer holds after it
        self.want_id = 1 << 40
        self.exchanges = 0
        # each peer's cumulative CDN bytes (header word 7, the planner's CDN balance): what it
        # seeded to this rank -- a seeder sends every segment it fetched to all wanters -- read
        # from the node's last posted plan when the caller sets `node`
        self.node = None
        self.cdn = np.zeros(world, dtype=np.int64)
        self._credited = -1

    def _credit_seeders(self) -> None:
        h = getattr(self.node, "_last_posted", None) if self.node is not None else None
        if h is None or h.plan is None or h.round == self._credited:
            return
        self._credited = h.round
        recv = h.plan[1]
        if len(recv):
            np.add.at(self.cdn, recv[:, 5], recv[:, 4])

    def allgather_control(self, msg):
        msg = np.asarray(msg, dtype=np.int64)
        if msg.size < HDR or msg[0] != MAGIC:  # a barrier / other collective: echo
            return [msg.copy() for _ in range(self.world_size)]
        self._credit_seeders()
        nw = int(msg[2])
        rows = msg[HDR:HDR + 6 * nw].reshape(nw, 6)
        flags = self.rt.FLAG_ONLINE | self.rt.FLAG_UPLOAD | self.rt.FLAG_DOWNLOAD | self.rt.FLAG_CDN_DEDUP
        none = np.zeros((0, 5), dtype=np.int64)
        adds = np.concatenate([self.held[-1][0], self.held[-1][1][:, None]], axis=1) if self.held else none
        rms = self.held[-1 - self.keep][0] if len(self.held) > self.keep else none[:, :4]
        self.held.append((rows[:, :4].copy(), rows[:, 4].copy()))
        if len(self.held) > self.keep + 1:
            self.held.pop(0)
        parts = [msg.copy()]
        off = (self.rounds // self.churn) % (self.world_size + 1) if self.churn > 0 else -1
        self.rounds += 1
        for r in range(1, self.world_size):
            hdr = np.zeros(HDR, dtype=np.int64)
            f = flags & ~self.rt.FLAG_ONLINE if r == off else flags
            hdr[0], hdr[1], hdr[2], hdr[3], hdr[4] = MAGIC, f, nw, len(adds), len(rms)
            hdr[6:10] = msg[6:10]  # round, p2p / upload counters: even peers
            if self.node is not None:
                hdr[7] = self.cdn[r]
            hdr[CHECK_WORD:CHECK_WORD + 3] = msg[CHECK_WORD:CHECK_WORD + 3]  # the replicas agree
            w = rows.copy()
            w[:, 5] = self.want_id + np.arange(nw)
            self.want_id += nw
            parts.append(np.concatenate([hdr, w.reshape(-1), adds.reshape(-1), rms.reshape(-1)]))
        return parts

    def exchange(self, sends, recvs) -> None:  # the bytes are not measured here
        self.exchanges += 1

    def exchange_spans(self, *cols) -> None:  # the native RCCL plane's entry (device runs)
        self.exchanges += 1


class Consumer:
    """The fleet's part in a round: deliveries in, deferred checks reported passed one round
    later (after the 'transmux')."""

    def __init__(self, node: SwarmNode) -> None:
        self.node = node
        self.pending: list = []
        self.delivered = 0

    def deliver(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect=None):
        self.delivered += len(tok)
        if expect is not None:
            chk = np.asarray(expect) >= 0
            if chk.any():
                self.pending.append((eids[chk], tok[chk]))

    def fail(self, tok, status):
        raise RuntimeError(f"request failed: {status[:4]}")

    def report(self) -> None:
        items, self.pending = self.pending, []
        for eids, tok in items:
            self.node.verify_done(eids, np.ones(len(eids), dtype=bool), tok)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--wants", type=int, default=256, help="segments per rank and round (4 players x 64)")
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--lag", type=int, default=2, help="rounds in flight (the bench's lag-2 pipeline)")
    ap.add_argument("--churn", type=int, default=0, help="peers go offline in rotation every N rounds")
    ap.add_argument("--seg-duration", type=float, default=0.1, help="seconds per synthetic segment (its size)")
    ap.add_argument("--device", default="cpu", help="cpu, or cuda (the node's arena and kernels on the GPU)")
    ap.add_argument("--profile", default=None, help="write a cProfile of the timed rounds here")
    args = ap.parse_args()
    clear_origins()
    new_event_loop("virtual")
    W = args.wants
    n_seg = (args.rounds + args.warmup + args.lag + 2) * W
    # tiny segments: the per-byte work (the CPU stand-in's CRC and copies, device work on a GPU)
    # stays out of the figures, which are per-row host cost
    origin = SyntheticHlsOrigin("http://cdn.replay/vod/", renditions=[Rendition(8_000, 160, 90, audio_kbps=8)],
                                segment_duration=args.seg_duration, num_segments=n_seg, encrypted=False, pool_size=8,
                                pin_memory=args.device != "cpu")
    seg_len = int(max(origin.pools[0].lengths))
    comm = FakePeers(args.world, churn=args.churn)
    node = SwarmNode(comm, device=args.device, cache_bytes=64 * W * (seg_len + 512) + (64 << 20), auto_tick=False,
                     max_wants_per_round=W)
    node.verify_deferred = True
    comm.node = node
    node._grow_crc(1 << 17)  # tiny segments fill the ring with more entries than its sizing assumes
    node.divergence_check = False  # the fake peers echo rank 0's check words; nothing to compare
    sink = Consumer(node)
    node.set_bulk_sink(sink)
    urls = [origin.base_url + origin.segment_path(0, sn) for sn in range(n_seg)]
    sn = 0
    hs = []
    prof = cProfile.Profile() if args.profile else None
    t_launch = t_complete = 0.0
    cdn_rows = send_rows = recv_rows = 0

    def step(timed: bool) -> None:
        nonlocal sn, t_launch, t_complete, cdn_rows, send_rows, recv_rows
        keys = np.zeros((W, 4), dtype=np.int64)
        keys[:, 0] = 5
        keys[:, 3] = np.arange(sn, sn + W)
        node.request_batch(keys, urls[sn:sn + W], None, np.arange(sn, sn + W, dtype=np.int64))
        sn += W
        t0 = time.perf_counter()
        h = node.launch_round()
        t1 = time.perf_counter()
        hs.append(h)
        t2 = t1
        if len(hs) > args.lag:
            node.complete_round(hs.pop(0))
            t2 = time.perf_counter()
        node.loop.run_until(lambda: False, timeout_ms=0)
        sink.report()
        if timed:
            t_launch += t1 - t0
            t_complete += t2 - t1
            if h.plan is not None:
                send_rows += len(h.plan[0])
                recv_rows += len(h.plan[1])
            cdn_rows += 0 if h.cdn is None else len(h.cdn[0])

    for _ in range(args.warmup):
        step(False)
    node.timer.reset()
    if prof is not None:
        prof.enable()
    t0 = time.perf_counter()
    for _ in range(args.rounds):
        step(True)
    wall = time.perf_counter() - t0
    for h in hs:  # drain the rounds still in flight (outside the figures)
        node.complete_round(h)
    if args.device != "cpu":
        import torch

        torch.cuda.synchronize()
    if prof is not None:
        prof.disable()
        with open(args.profile, "w") as f:
            st = pstats.Stats(prof, stream=f)
            st.sort_stats("tottime").print_stats(40)
    R = args.rounds
    phases = {k: round(v * 1e6 / R, 1) for k, v in sorted(node.timer.total.items()) if not k.startswith("dev_")}
    print(json.dumps({"world": args.world, "wants": W, "rounds": R, "seg_bytes": seg_len,
                      "launch_us": round(t_launch * 1e6 / R, 1), "complete_us": round(t_complete * 1e6 / R, 1),
                      "round_total_us": round(wall * 1e6 / R, 1), "phases_us": phases,
                      "per_round": {"cdn": cdn_rows / R, "send": send_rows / R, "recv": recv_rows / R},
                      "delivered": sink.delivered, "crc_failures": node.stats["crc_failures"],
                      "p2p_segments": node.stats["p2p_segments"], "cdn_segments": node.stats["cdn_segments"]}))
    clear_origins()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
