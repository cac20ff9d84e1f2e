"""Segment identity, range selection and batched copies.

* :func:`range_select`  — batched ``MediaMap.getSegmentList`` (K1, HIP kernel on a GPU).
* :func:`pack_keys` / :func:`wire_keys` / :func:`key_hash_host` — 16-byte segment keys, their
  12-byte wire form (exactly ``SegmentView.toArrayBuffer()`` rows) and the 64-bit hash the
  native cache index and want table use (K2, ``runtime/store.hpp`` SegKeyHash).
* :func:`copy_segments` — batched byte-range gather/scatter between buffers (K4).
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np
import torch

from ._native import device as _dev
from .desc import pack_to_device

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_G = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def key_hash_host(keys: np.ndarray) -> np.ndarray:
    """Host mirror of the device key hash (== C++ SegKeyHash)."""
    k = np.asarray(keys, dtype=np.int64).reshape(-1, 4).astype(np.uint64) & np.uint64(0xFFFFFFFF)
    a = (k[:, 0] << np.uint64(32)) | k[:, 1]
    b = (k[:, 2] << np.uint64(32)) | k[:, 3]
    with np.errstate(over="ignore"):
        return _mix64(a ^ _mix64(b + _G))


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


def range_select(starts: Sequence[Sequence[float]], queries: Sequence[Tuple[int, float, float]],
                 device: torch.device) -> Tuple[np.ndarray, np.ndarray]:
    """For each (track, begin, duration) query return [lo, hi) indices of fragments with
    ``begin <= start <= begin + duration`` (starts sorted per track)."""
    track_off = np.zeros(len(starts) + 1, dtype=np.int64)
    np.cumsum([len(s) for s in starts], out=track_off[1:])
    flat = np.concatenate([np.asarray(s, dtype=np.float64) for s in starts]) if starts else np.zeros(0)
    q = np.asarray(queries, dtype=np.float64).reshape(-1, 3)
    qt = q[:, 0].astype(np.int64)
    if device.type == "cpu":
        lo = np.full(len(q), -1, dtype=np.int64)
        hi = np.full(len(q), -1, dtype=np.int64)
        for i, (t, b, d) in enumerate(zip(qt, q[:, 1], q[:, 2])):
            if 0 <= t < len(starts):
                s = flat[track_off[t]:track_off[t + 1]]
                lo[i] = np.searchsorted(s, b, side="left")
                hi[i] = np.searchsorted(s, b + d, side="right")
        return lo, hi
    d = pack_to_device({"s": flat if flat.size else np.zeros(1), "to": track_off, "qt": qt,
                        "qb": np.ascontiguousarray(q[:, 1]), "qd": np.ascontiguousarray(q[:, 2])}, device)
    lo = torch.empty(len(q), dtype=torch.int64, device=device)
    hi = torch.empty(len(q), dtype=torch.int64, device=device)
    _dev().range_select(d["s"], d["to"], d["qt"], d["qb"], d["qd"], lo, hi)
    return lo.cpu().numpy(), hi.cpu().numpy()


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
