#!/usr/bin/env python3
"""Is a hipGraph worth it for the per-round device chain?

1. Host time per call of the round's real launch paths, eager: ``ops.crc.crc32_batch``
   (native: descriptor block, one H2D, residue + combine kernels) and
   ``ops.aes.cbc_decrypt_batch`` (descriptor H2D + one decrypt kernel), on a small and on a
   bench-sized batch (64 x 3 MB segments).
2. The most a graph can save per launch: host time of a chain of ``K`` small kernels
   (``add_``, HIP's launch floor) launched eagerly vs replayed from one captured
   ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm).

The native launch paths stage descriptors through a fresh pinned block per call, which
stream capture does not permit (``hipHostMalloc`` is not capturable), so they cannot be
captured as they are; (2) bounds what restructuring them for capture could buy.
"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from hlsjs_p2p_wrapper_amd.ops import aes, crc  # noqa: E402


def host_us(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    host = (time.perf_counter() - t) / iters * 1e6
    torch.cuda.synchronize()
    return host


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for label, B, seg in (("small", 4, 64 << 10), ("bench", 64, 3_000_000)):
        seg = seg // 16 * 16
        buf = torch.randint(0, 256, (B * seg,), dtype=torch.int32).to(torch.uint8).to(dev)
        offs = [i * seg for i in range(B)]
        lens = [seg] * B
        keys = [bytes(range(16))] * B
        ivs = [bytes(16)] * B
        dst = torch.empty_like(buf)
        out[f"crc_eager_host_us_{label}"] = round(host_us(lambda: crc.crc32_batch(buf, offs, lens)), 2)
        out[f"aes_eager_host_us_{label}"] = round(
            host_us(lambda: aes.cbc_decrypt_batch(buf, offs, lens, keys, ivs, dst, offs)), 2)
        del buf, dst
    x = torch.zeros(1024, device=dev)
    for K in (1, 6, 12):
        def chain():
            for _ in range(K):
                x.add_(1.0)

        eager = host_us(chain)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            chain()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            chain()
        replay = host_us(g.replay)
        out[f"chain{K}_eager_host_us"] = round(eager, 2)
        out[f"chain{K}_graph_replay_host_us"] = round(replay, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
