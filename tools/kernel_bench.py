"""Per-kernel microbenchmark on one bench round's batch: 64 x ~3 MB AES-128 TS segments
(the 1080p 6 Mb/s config).  Times AES-CBC decrypt, TS demux (psi+scan+gather) and the MFMA
CRC with HIP events and reports us / GB/s of input.  Checks results against the host
oracles once.

    PYTHONPATH=. python tools/kernel_bench.py [--segs 64] [--iters 20]
"""
import argparse
import json

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.net.origin import PRESET_1080P_6M, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import aes, crc, segment, tsdemux


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda")
    origin = SyntheticHlsOrigin("http://cdn.kb/", renditions=PRESET_1080P_6M, num_segments=args.segs,
                                encrypted=True, pool_size=args.segs, pin_memory=True, seed=3)
    pool = origin.pools[0]
    offs = [int(o) for o in pool.offsets[:args.segs]]
    lens = [int(n) for n in pool.lengths[:args.segs]]
    src = pool.data.to(dev)
    total = sum(lens)
    keys = [origin.key] * args.segs
    ivs = [origin.iv] * args.segs
    dec = torch.empty_like(src)
    res = {}
    out_len = aes.cbc_decrypt_batch(src, offs, lens, keys, ivs, dec, offs)
    res["aes_us"] = timed(lambda: aes.cbc_decrypt_batch(src, offs, lens, keys, ivs, dec, offs), args.iters)
    # correctness vs host (first segment)
    ref = aes.cbc_decrypt(origin.key, origin.iv, pool.data[offs[0]:offs[0] + lens[0]].numpy())
    assert dec[offs[0]:offs[0] + len(ref)].cpu().numpy().tobytes() == ref.tobytes(), "AES mismatch"
    es = torch.empty_like(src)
    caps = lens
    r = tsdemux.demux_batch(dec, offs, out_len, es, offs, caps=caps)
    res["demux_us"] = timed(lambda: tsdemux.demux_batch(dec, offs, out_len, es, offs, caps=caps), args.iters)
    cpu = tsdemux.demux_batch(torch.from_numpy(ref.copy()), [0], [len(ref)], torch.empty(len(ref) + 256,
                                                                                           dtype=torch.uint8), [0])
    g, c = r.segment(0), cpu.segment(0)
    assert g["video_bytes"] == c["video_bytes"] and torch.equal(g["video"]["es"].cpu(), c["video"]["es"]), \
        "demux mismatch"
    res["crc_us"] = timed(lambda: crc.crc32_batch(src, offs, lens), args.iters)
    got = crc.crc32_batch(src, offs, lens)[0].cpu().numpy().view(np.uint32)
    assert int(got[0]) == crc.crc32(pool.data[offs[0]:offs[0] + lens[0]].numpy()), "CRC mismatch"
    # byte-moving rooflines on the same bytes: the batched K4 segment copy and torch's copy_
    cp = torch.empty_like(src)
    res["copy_us"] = timed(lambda: segment.copy_segments(src, cp, offs, offs, lens), args.iters)
    assert torch.equal(cp[offs[5]:offs[5] + lens[5]], src[offs[5]:offs[5] + lens[5]]), "copy mismatch"
    res["torch_copy_us"] = timed(lambda: cp.copy_(src), args.iters)
    for k in ("aes", "demux", "crc", "copy", "torch_copy"):
        res[f"{k}_GBps"] = round(total / (res[f"{k}_us"] * 1e-6) / 1e9, 1)
        res[f"{k}_us"] = round(res[f"{k}_us"], 1)
    res["bytes"] = total
    print(json.dumps(res))


if __name__ == "__main__":
    main()
