"""Segment identity and batched copies.

* :func:`pack_keys` / :func:`wire_keys` — 16-byte segment keys and their 12-byte wire form
  (exactly ``SegmentView.toArrayBuffer()`` rows).  The 64-bit key hash of the native cache
  index and want table lives with them in C++ (K2, ``runtime/store.hpp`` SegKeyHash).
* :func:`copy_segments` — batched byte-range gather/scatter between buffers (K4).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from ._native import device as _dev
from .desc import pack_to_device


def pack_keys(levels, url_ids, sns, swarm: int = 0) -> np.ndarray:
    """``int32[n, 4]`` = (swarm, level, urlId, sn); columns 1..3 are the 12-byte wire key."""
    n = len(sns)
    out = np.empty((n, 4), dtype=np.uint32)
    out[:, 0] = swarm
    out[:, 1] = np.asarray(levels, dtype=np.int64) & 0xFFFFFFFF
    out[:, 2] = np.asarray(url_ids, dtype=np.int64) & 0xFFFFFFFF
    out[:, 3] = np.asarray(sns, dtype=np.int64) & 0xFFFFFFFF
    return out.view(np.int32)


def wire_keys(keys: np.ndarray) -> bytes:
    """12-byte little-endian ``[level, urlId, sn]`` rows (``SegmentView.toArrayBuffer``)."""
    k = np.ascontiguousarray(np.asarray(keys).view(np.uint32).reshape(-1, 4)[:, 1:]).astype("<u4")
    return k.tobytes()


def copy_segments(src: torch.Tensor, dst: torch.Tensor, src_offs: Sequence[int], dst_offs: Sequence[int],
                  lens: Sequence[int]) -> None:
    """``dst[do:do+n] = src[so:so+n]`` for every triple, one launch on device."""
    so = np.asarray(src_offs, dtype=np.int64)
    do = np.asarray(dst_offs, dtype=np.int64)
    n = np.asarray(lens, dtype=np.int64)
    if len(n) == 0:
        return
    if np.any(so + n > src.numel()) or np.any(do + n > dst.numel()) or np.any(n < 0):
        raise ValueError("copy_segments: out of bounds")
    if src.device.type == "cpu":
        s = src.numpy()
        d = dst.numpy()
        for a, b, c in zip(so.tolist(), do.tolist(), n.tolist()):
            d[b:b + c] = s[a:a + c]
        return
    chunks = (n + 65535) // 65536
    cp = np.zeros(len(n) + 1, dtype=np.int64)
    np.cumsum(chunks, out=cp[1:])
    t = pack_to_device({"so": so, "do": do, "n": n, "cp": cp}, src.device)
    _dev().segment_copy(src, dst, t["so"], t["do"], t["n"], t["cp"], int(cp[-1]))
