"""N=8 exchange vs. the persistent decrypt grid, rehearsed on one MI355X.

At N=8 a rank receives 7/8 of its fragments from peers: per round ~7 x 32 x 3 MB over RCCL,
posted on the node stream while the previous step's transmux batch (AES-CBC decrypt with the
fused receive CRC, then the demux) runs on the default stream, and the next batch is queued
right behind it.  Round 3 measured (``profiles/r3_rccl_overlap``) that RCCL makes progress
beside the decrypt grid but most of a round queues until the grid drains.  This tool times
that cadence for each mitigation, one option per run:

  base        CU reserve 8 (round 4's default; 64 since this rehearsal), RCCL on a default-priority stream
  prio        the RCCL stream at the highest stream priority
  rN          CU reserve N (the decrypt grid leaves N CUs free; r16, r32, r64, ...)
  split       every transmux batch as two launches of half the segments (RCCL kernels can
              dispatch between the two decrypt grids)
  a+b         options combined (prio+split, r32+split, ...)

Per option (median of --iters), from a common start event:
  rccl_alone_us / tm_alone_us      one exchange round / one transmux batch, alone
  cadence: batch A, then the exchange round R, then batch B (A and B on one stream, R on
  another, enqueued in that order): rccl_done_us, a_done_us, b_done_us, total_us
  serial_us = rccl_alone + 2 x tm_alone;  saved = 1 - total / serial
  steady_step_us (--steady K): the bench's pipeline for K steps -- round t+2 posted, then
  batch t, which consumes round t's deliveries (its stream waits on round t's end event) --
  total time / K: the device time per step when exchange and transmux overlap in steady
  state; steady_saved = 1 - steady_step / (rccl_alone + tm_alone)

A one-rank communicator sends to itself: the same ncclGroupStart / ncclSend x 7 + ncclRecv x 7
/ ncclGroupEnd path as a round between peers, but an HBM-to-HBM copy (more CU work per byte
than an xGMI-bound transfer), so the contention measured here is an upper bound.

    PYTHONPATH=. python tools/overlap_n8.py --options base,prio,r16,r32,split,prio+split
"""
import argparse
import json
import zlib

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.net.origin import PRESET_1080P_6M, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import aes, crc, tsdemux
from hlsjs_p2p_wrapper_amd.ops._native import device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=7)
    ap.add_argument("--per-peer", type=int, default=32, help="3 MB segments per peer and round")
    ap.add_argument("--segs", type=int, default=256, help="segments per transmux batch (64 in flight x 4 players)")
    ap.add_argument("--options", default="base,prio,r16,r32,split,prio+split")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--steady", type=int, default=0, help="also time K steps of the bench's lag-2 pipeline")
    ap.add_argument("--only-steady", action="store_true", help="time the steady pipeline only (A/B runs)")
    ap.add_argument("--repeat", type=int, default=1, help="run the option list this many times, interleaved")
    args = ap.parse_args()
    cuda = torch.device("cuda", 0)
    dev = device()
    comm = dev.RcclComm(dev.rccl_unique_id(), 1, 0, 0)
    seg_bytes = 3 << 20
    per = args.per_peer * seg_bytes
    # the round: one contiguous buffer + one CRC trailer per peer pair, every pair to self
    sbuf = torch.randint(0, 256, (args.peers * per,), dtype=torch.uint8, device=cuda)
    rbuf = torch.empty_like(sbuf)
    strl = torch.randint(0, 1 << 30, (args.peers * args.per_peer,), dtype=torch.int32, device=cuda)
    rtrl = torch.empty_like(strl)
    tb = 4 * args.per_peer
    sp = np.array([sbuf.data_ptr() + i * per for i in range(args.peers)] +
                  [strl.data_ptr() + i * tb for i in range(args.peers)], dtype=np.int64)
    rp = np.array([rbuf.data_ptr() + i * per for i in range(args.peers)] +
                  [rtrl.data_ptr() + i * tb for i in range(args.peers)], dtype=np.int64)
    sz = np.array([per] * args.peers + [tb] * args.peers, dtype=np.int64)
    peers = np.zeros(2 * args.peers, dtype=np.int64)
    lo, hi = torch.cuda.Stream.priority_range()
    streams = {"default": torch.cuda.Stream(), "high": torch.cuda.Stream(priority=min(lo, hi))}
    s_tm = torch.cuda.Stream()

    # the transmux batch: AES-128 segments with the receive CRC fused into the decrypt
    pool_n = 64
    origin = SyntheticHlsOrigin("http://cdn.ov8/", renditions=PRESET_1080P_6M, num_segments=pool_n, encrypted=True,
                                pool_size=pool_n, pin_memory=True, seed=5, register=False)
    pool = origin.pools[0]
    host = pool.data.numpy()
    src = pool.data.to(cuda)
    offs = np.array([pool.offsets[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    lens = np.array([pool.lengths[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    crcs = np.array([zlib.crc32(host[o:o + n].tobytes()) for o, n in zip(offs, lens)], dtype=np.int64)
    enc = np.ones(args.segs, dtype=np.uint8)
    drk = np.tile(aes.round_keys_le(origin.key), (args.segs, 1)).astype(np.uint32)
    iv = np.tile(np.frombuffer(origin.iv, dtype=np.uint8), (args.segs, 1))
    td0, isb = aes.device_tables(cuda)
    cw, ctab = crc.fused_consts(cuda)
    keep = []
    state = {"split": False, "rccl": streams["default"]}

    def batch():
        parts = [slice(0, args.segs)] if not state["split"] else \
            [slice(0, args.segs // 2), slice(args.segs // 2, args.segs)]
        with torch.cuda.stream(s_tm):
            for p in parts:
                keep.append(dev.transmux_launch(src, offs[p], lens[p], enc[p], drk[p], iv[p], td0, isb,
                                                tsdemux.DEFAULT_MAX_PES, crcs[p], cw, ctab))

    def rround():
        comm.exchange(sp, sz, peers, rp, sz, peers, state["rccl"].cuda_stream)

    def timed(steps):
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        s_tm.wait_event(start)
        for s in streams.values():
            s.wait_event(start)
        ends = {}
        for name, fn, stream in steps:
            fn()
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            ends[name] = e
        torch.cuda.synchronize()
        for k in keep:  # every fused verify passed (the bytes are the pool's own)
            if k[3] is not None:
                assert bool(k[3][1].numpy().all()), "fused CRC verify failed"
        keep.clear()
        return {k: start.elapsed_time(e) * 1e3 for k, e in ends.items()}

    def steady(rs, k, lag=2):
        """k steps of the bench's pipeline; returns the total device time in us."""
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        s_tm.wait_event(start)
        rs.wait_event(start)
        done = []
        for t in range(k + lag):
            if t < k:
                rround()
                e = torch.cuda.Event()
                e.record(rs)
                done.append(e)
            if t >= lag:
                s_tm.wait_event(done[t - lag])  # batch t-lag decrypts round t-lag's deliveries
                batch()
        end = torch.cuda.Event(enable_timing=True)
        end.record(s_tm)
        torch.cuda.synchronize()
        keep.clear()
        return start.elapsed_time(end) * 1e3

    out = {"peers": args.peers, "per_peer": args.per_peer, "round_MB": round(args.peers * per / 1e6, 1),
           "segs": args.segs, "rccl_version": int(dev.rccl_version()), "priority_range": [lo, hi], "runs": []}
    for _ in range(2):  # warm-up (RCCL channels, allocator, code objects)
        timed([("r", rround, streams["default"])])
        timed([("t", batch, s_tm)])
    for opt in args.options.split(",") * args.repeat:
        parts = opt.split("+")
        state["split"] = "split" in parts
        state["rccl"] = streams["high" if "prio" in parts else "default"]
        reserve = [int(p[1:]) for p in parts if p[:1] == "r" and p[1:].isdigit()]
        dev.set_cu_reserve(reserve[0] if reserve else 8)
        rs = state["rccl"]
        med = lambda xs: round(float(np.median(xs)), 1)  # noqa: E731
        st = []
        for _ in range(args.iters if args.steady else 0):
            st.append(steady(rs, args.steady) / args.steady)
        if args.only_steady:
            row = {"option": opt, "cu_reserve": dev.cu_reserve(), "steady_step_us": med(st),
                   "steady_all_us": [round(x, 1) for x in st]}
            out["runs"].append(row)
            print(json.dumps(row), flush=True)
            continue
        ra, ta, cad = [], [], []
        for _ in range(args.iters):
            ra.append(timed([("r", rround, rs)])["r"])
            ta.append(timed([("t", batch, s_tm)])["t"])
            cad.append(timed([("a", batch, s_tm), ("r", rround, rs), ("b", batch, s_tm)]))
        row = {"option": opt, "cu_reserve": dev.cu_reserve(), "rccl_alone_us": med(ra), "tm_alone_us": med(ta),
               "rccl_done_us": med([c["r"] for c in cad]), "a_done_us": med([c["a"] for c in cad]),
               "b_done_us": med([c["b"] for c in cad]), "total_us": med([max(c.values()) for c in cad])}
        row["serial_us"] = round(row["rccl_alone_us"] + 2 * row["tm_alone_us"], 1)
        row["saved"] = round(1 - row["total_us"] / row["serial_us"], 3)
        if st:
            row["steady_step_us"] = med(st)
            row["steady_saved"] = round(1 - row["steady_step_us"] / (row["rccl_alone_us"] + row["tm_alone_us"]), 3)
        out["runs"].append(row)
        print(json.dumps(row), flush=True)
    dev.set_cu_reserve(8)
    comm.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
