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
    ap.add_argument("--sub", type=int, default=0,
                    help="launch the batch as back-to-back sub-batches of this many segments (0: one launch)")
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

    def launch_one(sl, expect=None, cw=None, ctab=None):
        return dev.transmux_launch(src, offs[sl], lens[sl], enc[sl], drk[sl], iv[sl], td0, isb, tsdemux.DEFAULT_MAX_PES,
                                   None if expect is None else expect[sl], cw, ctab)

    step = args.sub if 0 < args.sub < args.segs else args.segs
    slices = [slice(a, min(a + step, args.segs)) for a in range(0, args.segs, step)]

    def launch(expect=None, cw=None, ctab=None):
        outs = [launch_one(sl, expect, cw, ctab) for sl in slices]
        return outs[0] if len(outs) == 1 else outs

    def timed(fn):
        keep = [fn() for _ in range(args.iters + 2)]  # warm the caching allocator: no hipMalloc in the timed loop
        torch.cuda.synchronize()
        keep = keep[:2]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            keep.append(fn())
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / args.iters, keep

    us, _ = timed(launch)
    out = {"segs": args.segs, "sub": step, "bytes": total, "us": round(us, 1), "us_per_seg": round(us / args.segs, 3),
           "GBps": round(total / (us * 1e-6) / 1e9, 1)}
    if args.verify:
        from hlsjs_p2p_wrapper_amd.ops import crc

        host = pool.data.numpy()
        expect = np.array([zlib.crc32(host[o:o + n].tobytes()) for o, n in zip(offs, lens)], dtype=np.int64)
        cw, ctab = crc.fused_consts(cuda)
        us_v, keep = timed(lambda: launch(expect, cw, ctab))
        ok = all(bool(o[3][1].numpy().all()) for k in keep for o in (k if isinstance(k, list) else [k]))
        us_c, _ = timed(lambda: crc.crc32_batch(src, offs, lens, expect=(expect & 0xFFFFFFFF).tolist()))
        out.update(fused_us=round(us_v, 1), fused_us_per_seg=round(us_v / args.segs, 3), fused_all_ok=ok,
                   crc_kernel_us_per_seg=round(us_c / args.segs, 3),
                   separate_us_per_seg=round((us + us_c) / args.segs, 3))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
