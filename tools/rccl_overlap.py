"""Does RCCL make progress while a decrypt batch holds the GPU?  

One process, a one-rank native RCCL communicator (`kernels/rccl_comm.cpp`): a round of
--msgs x 3 MB self-exchange (the same ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd
path as a round between peers, RCCL kernels included) on one stream, and a transmux batch
(AES-128-CBC + TS demux of --segs 3 MB segments, `transmux_launch`) on another.  For each
CU reserve (the CUs the persistent decrypt grid leaves free, `set_cu_reserve`) it times:

  rccl_alone_us        the exchange alone
  transmux_alone_us    the batch alone
  both: rccl_done_us / transmux_done_us / total_us, from a common start event, with the
  batch enqueued FIRST — so an RCCL round that cannot find a CU finishes only after the
  decrypt grid drains (rccl_done_us ~ transmux_done_us), one that can finishes near its
  alone time.

    PYTHONPATH=. python tools/rccl_overlap.py [--segs 128] [--msgs 64] [--reserves 0,8,16]
"""
import argparse
import json

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.net.origin import PRESET_1080P_6M, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux
from hlsjs_p2p_wrapper_amd.ops._native import device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=128)
    ap.add_argument("--msgs", type=int, default=64)
    ap.add_argument("--reserves", default="0,8,16")
    ap.add_argument("--iters", type=int, default=5)
    args = ap.parse_args()
    cuda = torch.device("cuda", 0)
    dev = device()
    comm = dev.RcclComm(dev.rccl_unique_id(), 1, 0, 0)
    # the RCCL round: msgs x 3 MB to self
    seg_bytes = 3 << 20
    sbuf = torch.randint(0, 256, (args.msgs * seg_bytes,), dtype=torch.uint8, device=cuda)
    rbuf = torch.empty_like(sbuf)
    sp = np.array([sbuf.data_ptr() + i * seg_bytes for i in range(args.msgs)], dtype=np.int64)
    rp = np.array([rbuf.data_ptr() + i * seg_bytes for i in range(args.msgs)], dtype=np.int64)
    sz = np.full(args.msgs, seg_bytes, dtype=np.int64)
    peers = np.zeros(args.msgs, dtype=np.int64)
    s_rccl, s_tm = torch.cuda.Stream(), torch.cuda.Stream()

    def rccl_round():
        comm.exchange(sp, sz, peers, rp, sz, peers, s_rccl.cuda_stream)

    # the transmux batch
    pool_n = min(args.segs, 64)
    origin = SyntheticHlsOrigin("http://cdn.ov/", renditions=PRESET_1080P_6M, num_segments=pool_n, encrypted=True,
                                pool_size=pool_n, pin_memory=True, seed=5, register=False)
    pool = origin.pools[0]
    src = pool.data.to(cuda)
    offs = np.array([pool.offsets[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    lens = np.array([pool.lengths[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    enc = np.ones(args.segs, dtype=np.uint8)
    drk = np.tile(aes.round_keys_le(origin.key), (args.segs, 1)).astype(np.uint32)
    iv = np.tile(np.frombuffer(origin.iv, dtype=np.uint8), (args.segs, 1))
    td0, isb = aes.device_tables(cuda)
    keep = []

    def transmux():
        with torch.cuda.stream(s_tm):
            keep.append(dev.transmux_launch(src, offs, lens, enc, drk, iv, td0, isb, tsdemux.DEFAULT_MAX_PES))

    def timed(fn_list):
        """Start event on the current stream, both streams wait on it, run, per-stream end events."""
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        ends = {}
        for name, fn, stream in fn_list:
            stream.wait_event(start)
            fn()
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            ends[name] = e
        torch.cuda.synchronize()
        keep.clear()
        return {k: start.elapsed_time(e) * 1e3 for k, e in ends.items()}

    out = {"msgs": args.msgs, "msg_bytes": seg_bytes, "segs": args.segs, "rccl_version": int(dev.rccl_version())}
    for _ in range(2):  # warm-up
        timed([("r", rccl_round, s_rccl)])
        timed([("t", transmux, s_tm)])
    rows = []
    for reserve in [int(x) for x in args.reserves.split(",")]:
        dev.set_cu_reserve(reserve)
        ra, ta, both = [], [], []
        for _ in range(args.iters):
            ra.append(timed([("r", rccl_round, s_rccl)])["r"])
            ta.append(timed([("t", transmux, s_tm)])["t"])
            both.append(timed([("t", transmux, s_tm), ("r", rccl_round, s_rccl)]))
        rows.append({
            "cu_reserve": reserve,
            "rccl_alone_us": round(float(np.median(ra)), 1),
            "transmux_alone_us": round(float(np.median(ta)), 1),
            "both_rccl_done_us": round(float(np.median([b["r"] for b in both])), 1),
            "both_transmux_done_us": round(float(np.median([b["t"] for b in both])), 1),
            "both_total_us": round(float(np.median([max(b.values()) for b in both])), 1),
        })
    dev.set_cu_reserve(8)
    out["runs"] = rows
    comm.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
