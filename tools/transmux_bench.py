"""Isolated timing of one transmux batch on the MI355X: AES-128-CBC decrypt (aes_cbc.hip) +
the four-kernel TS demux (ts_demux.hip), as one ``transmux_launch``.  Batches of 1080p
6 Mb/s AES-128 segments (~3 MB), as a bench round delivers them.

(Round 3 also timed a fused decrypt + demux kernel, a one-pass demux and a scatter demux
against this sequence; all three were slower and were removed in round 4 -- their numbers
stay in profiles/r3_transmux_fused_vs_split.md and profiles/r3_scatter/.)

    PYTHONPATH=. python tools/transmux_bench.py [--segs 256] [--iters 10] [--verify]

``--verify`` also times the batch with every segment's ciphertext CRC checked by the decrypt
(the CRC fused into aes_cbc.hip, as the fleet's deferred receive verification runs it), and
adds the separate CRC kernel the node would otherwise run for comparison.
"""
import argparse
import json
import time
import zlib

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.net.origin import PRESET_1080P_6M, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux
from hlsjs_p2p_wrapper_amd.ops._native import device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--pool", type=int, default=64,
                    help="distinct segments (the batch cycles through them): 64 x 3 MB fits the 256 MB "
                         "Infinity Cache (MALL), 256 does not -- as in the pipeline, where every segment is new")
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--split", default="", help="split batches (decrypt on the current stream, demux on a second "
                                                 "one) with these CU reserves for the decrypt grid, e.g. 32,64,96")
    ap.add_argument("--overlap", default="", help="streams:reserve pairs, e.g. 1:0,2:0,2:64 -- consecutive batches "
                                                   "alternate over that many streams with the decrypt grid leaving "
                                                   "`reserve` CUs free (does batch k's demux overlap batch k+1's decrypt?)")
    args = ap.parse_args()
    cuda = torch.device("cuda", 0)
    dev = device()
    pool_n = min(args.segs, args.pool)
    origin = SyntheticHlsOrigin("http://cdn.tb/", renditions=PRESET_1080P_6M, num_segments=pool_n, encrypted=True,
                                pool_size=pool_n, pin_memory=True, seed=5, register=False)
    pool = origin.pools[0]
    src = pool.data.to(cuda)
    offs = np.array([pool.offsets[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    lens = np.array([pool.lengths[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    enc = np.ones(args.segs, dtype=np.uint8)
    drk = np.tile(aes.round_keys_le(origin.key), (args.segs, 1)).astype(np.uint32)
    iv = np.tile(np.frombuffer(origin.iv, dtype=np.uint8), (args.segs, 1))
    td0, isb = aes.device_tables(cuda)
    total = int(lens.sum())

    def launch(expect=None, cw=None, ctab=None, ds=0):
        return dev.transmux_launch(src, offs, lens, enc, drk, iv, td0, isb, tsdemux.DEFAULT_MAX_PES, expect, cw, ctab,
                                   ds)

    def timed(fn):
        keep = [fn() for _ in range(args.iters + 2)]  # warm the caching allocator: no hipMalloc in the timed loop
        torch.cuda.synchronize()
        keep = keep[:2]
        t0 = time.perf_counter()
        for _ in range(args.iters):
            keep.append(fn())
        torch.cuda.synchronize()  # wall clock: launches on several streams
        return (time.perf_counter() - t0) * 1e6 / args.iters, keep

    us, _ = timed(launch)
    out = {"segs": args.segs, "bytes": total, "us": round(us, 1), "us_per_seg": round(us / args.segs, 3),
           "GBps": round(total / (us * 1e-6) / 1e9, 1)}
    if args.verify:
        from hlsjs_p2p_wrapper_amd.ops import crc

        host = pool.data.numpy()
        expect = np.array([zlib.crc32(host[o:o + n].tobytes()) for o, n in zip(offs, lens)], dtype=np.int64)
        cw, ctab = crc.fused_consts(cuda)
        us_v, keep = timed(lambda: launch(expect, cw, ctab))
        ok = all(bool(k[3][1].numpy().all()) for k in keep)
        us_c, _ = timed(lambda: crc.crc32_batch(src, offs, lens, expect=(expect & 0xFFFFFFFF).tolist()))
        out.update(fused_us=round(us_v, 1), fused_us_per_seg=round(us_v / args.segs, 3), fused_all_ok=ok,
                   crc_kernel_us_per_seg=round(us_c / args.segs, 3),
                   separate_us_per_seg=round((us + us_c) / args.segs, 3))
    if args.split:
        ds = torch.cuda.Stream()
        base = dev.split_reserve()
        for r in [int(x) for x in args.split.split(",") if x]:
            dev.set_split_reserve(r)
            us_s, _ = timed(lambda: launch(ds=ds.cuda_stream))
            out[f"split_r{r}_us_per_seg"] = round(us_s / args.segs, 3)
            if args.verify:
                us_sv, keep = timed(lambda: launch(expect, cw, ctab, ds=ds.cuda_stream))
                out[f"split_r{r}_fused_us_per_seg"] = round(us_sv / args.segs, 3)
                out[f"split_r{r}_fused_ok"] = all(bool(k[3][1].numpy().all()) for k in keep)
        dev.set_split_reserve(base)
    for pair in [x for x in args.overlap.split(",") if x]:
        ns, res = (int(v) for v in pair.split(":"))
        streams = [torch.cuda.Stream() for _ in range(ns)]
        dev.set_cu_reserve(res)

        def alt(it=[0]):
            st = streams[it[0] % ns]
            it[0] += 1
            with torch.cuda.stream(st):
                return launch()

        us_o, _ = timed(lambda: alt())
        out[f"s{ns}_r{res}_us_per_seg"] = round(us_o / args.segs, 3)
        dev.set_cu_reserve(0)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
