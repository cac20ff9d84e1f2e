"""Host-side cost of one batched launch (the per-round fixed overhead of the host path).

Times, in host microseconds per call, the pieces a round's launches are made of, on 64
tiny (30 KB) segments so device time is negligible:

    PYTHONPATH=. python tools/launch_overhead.py
"""
import json
import time

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import aes, crc, tsdemux
from hlsjs_p2p_wrapper_amd.ops.desc import pack_to_device


def per_call_us(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return round(dt / n * 1e6, 2)


def main():
    dev = torch.device("cuda")
    segs = 64
    origin = SyntheticHlsOrigin("http://cdn.lo/", renditions=[Rendition(60_000, 320, 180)], num_segments=segs,
                                encrypted=True, pool_size=segs, pin_memory=True, seed=3)
    pool = origin.pools[0]
    offs = [int(o) for o in pool.offsets[:segs]]
    lens = [int(n) for n in pool.lengths[:segs]]
    src = pool.data.to(dev)
    dec = torch.empty_like(src)
    keys, ivs = [origin.key] * segs, [origin.iv] * segs
    arrays = {k: np.arange(segs, dtype=np.int64) for k in ("a", "b", "c", "d", "e")}
    arrays["f"] = np.zeros((segs, 16), dtype=np.uint8)
    out_len = aes.cbc_decrypt_batch(src, offs, lens, keys, ivs, dec, offs)
    es = torch.empty_like(src)
    res = {
        "torch_empty_device": per_call_us(lambda: torch.empty(4096, dtype=torch.int64, device=dev)),
        "torch_empty_pinned": per_call_us(lambda: torch.empty(4096, dtype=torch.uint8, pin_memory=True)),
        "pack_to_device_6_arrays": per_call_us(lambda: pack_to_device(arrays, dev)),
        "event_record": per_call_us(lambda: torch.cuda.Event().record()),
        "aes_cbc_decrypt_batch_64": per_call_us(lambda: aes.cbc_decrypt_batch(src, offs, lens, keys, ivs, dec, offs)),
        "ts_demux_batch_64": per_call_us(lambda: tsdemux.demux_batch(dec, offs, out_len, es, offs, caps=lens)),
        "crc32_batch_64": per_call_us(lambda: crc.crc32_batch(src, offs, lens)),
    }
    print(json.dumps(res))


if __name__ == "__main__":
    main()
