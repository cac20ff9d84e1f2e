#!/usr/bin/env python3
"""Is a hipGraph worth it for the per-round device chain?  Host time per launch of the
round's kernels, eager vs replayed from a captured graph (``torch.cuda.CUDAGraph`` = a
hipGraph on ROCm).

Measured on a small and on a bench-sized batch (64 x 3 MB segments):
* ``crc``: ``ops.crc.crc32_batch`` (native: descriptor block, one H2D, residue + combine);
* ``aes``: ``ops.aes.cbc_decrypt_batch`` (descriptor H2D + one decrypt kernel);
* ``launch``: a bare elementwise kernel (``torch.Tensor.add_``), HIP's launch floor.

Each eager number is host time per call with the stream left to run (no sync inside the
loop); the graph number is host time per ``graph.replay()`` of the same sequence.
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


def graphed(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def main():
    dev = torch.device("cuda", 0)
    out = {}
    x = torch.zeros(1024, device=dev)
    out["launch_eager_us"] = host_us(lambda: x.add_(1.0))
    for label, B, seg in (("small", 4, 64 << 10), ("bench", 64, 3_000_000)):
        seg = seg // 16 * 16
        buf = torch.randint(0, 256, (B * seg,), dtype=torch.uint8, device=dev)
        offs = [i * seg for i in range(B)]
        lens = [seg] * B
        keys = [bytes(range(16))] * B
        ivs = [bytes(16)] * B
        dst = torch.empty_like(buf)

        def crc_fn():
            crc.crc32_batch(buf, offs, lens)

        def aes_fn():
            aes.cbc_decrypt_batch(buf, offs, lens, keys, ivs, dst, offs)

        for name, fn in (("crc", crc_fn), ("aes", aes_fn)):
            try:
                eager = host_us(fn)
                g = graphed(fn)
                replay = host_us(g.replay)
                out[f"{name}_{label}"] = {"eager_host_us": round(eager, 2), "graph_replay_host_us": round(replay, 2)}
            except Exception as e:  # capture refused: record why
                out[f"{name}_{label}"] = {"error": f"{type(e).__name__}: {e}"[:300]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
