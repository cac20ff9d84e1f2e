"""H2D strategy probe for the CDN phase (pinned host origin -> HBM arena).

Measures 64 x 3 MB (one bench round) pinned->device with: one large copy, per-segment
hipMemcpyAsync on 1/2/4 streams, and the native batched h2d (one stream).  Prints GB/s.
"""
import time

import torch

from hlsjs_p2p_wrapper_amd.ops._native import device as _dev


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    n, seg = 64, 3_000_000
    stride = (seg + 4095) // 4096 * 4096
    host = torch.empty(n * stride, dtype=torch.uint8, pin_memory=True)
    host.random_(0, 255)
    dev = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
    total = n * seg
    res = {}
    res["one_copy"] = n * stride / timeit(lambda: dev.copy_(host, non_blocking=True)) / 1e9
    for ns in (1, 2, 4, 8):
        streams = [torch.cuda.Stream() for _ in range(ns)]

        def run():
            cur = torch.cuda.current_stream()
            for s in streams:
                s.wait_stream(cur)
            for i in range(n):
                with torch.cuda.stream(streams[i % ns]):
                    dev[i * stride:i * stride + seg].copy_(host[i * stride:i * stride + seg], non_blocking=True)
            for s in streams:
                cur.wait_stream(s)

        res[f"per_seg_{ns}streams"] = total / timeit(run) / 1e9
    import numpy as np

    offs = np.arange(n, dtype=np.int64) * stride
    ptrs = host.data_ptr() + offs
    lens = np.full(n, seg, dtype=np.int64)
    alloc_same = np.full(n, host.data_ptr(), dtype=np.int64)
    alloc_each = ptrs.copy()  # distinct "allocations": no merging
    res["native_h2d_batch_64dma"] = total / timeit(
        lambda: _dev().h2d_batch(dev, offs, ptrs, lens, alloc_each, 4096)) / 1e9
    res["native_h2d_batch_merged"] = total / timeit(
        lambda: _dev().h2d_batch(dev, offs, ptrs, lens, alloc_same, 4096)) / 1e9
    print("dmas merged:", _dev().h2d_batch(dev, offs, ptrs, lens, alloc_same, 4096))
    for k, v in res.items():
        print(f"{k:24s} {v:8.2f} GB/s")


if __name__ == "__main__":
    main()
