"""CRC-32 (zlib) integrity check of segment payloads on the MFMA cores.

Every segment that enters a node (CDN fetch or peer transfer) is checksummed on device;
peer transfers carry the sender's CRC and the receiver compares on device, so corrupted
bytes from a peer are caught before the player sees them (fault injection: §5.3).

Device path: ``kernels/crc32_mfma.hip`` (``v_mfma_i32_32x32x32_i8`` GF(2) products +
shift-operator combine).  CPU path: slice-by-8 host oracle (== ``zlib.crc32``).
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

from ._native import device as _dev
from ._native import runtime as _rt
from .desc import pack_to_device

_consts: Dict[tuple, tuple] = {}
_lock = threading.Lock()


# matrix-core path of the residue kernel: "fp4" (f8f6f4 MFMA, e2m1 operands, 32 MFMAs per
# 8 KB tile) or "i8" (v_mfma_i32_32x32x32_i8, 64 per tile); the B-fragment dtype selects it
MFMA_VARIANT = os.environ.get("HLSP2P_CRC_MFMA", "fp4")


def _device_consts(device: torch.device, variant: str):
    k = (str(device), variant)
    c = _consts.get(k)
    if c is None:
        if variant not in ("fp4", "i8"):
            raise ValueError(f"unknown CRC MFMA variant {variant!r}")
        rt = _rt()
        frags = rt.crc_mfma_weights_fp4() if variant == "fp4" else rt.crc_mfma_weights()
        w = torch.from_numpy(frags).to(device)
        t = torch.from_numpy(rt.crc_shift_tables().view(np.int32)).to(device)
        c = (w, t)
        with _lock:
            _consts[k] = c
    return c


def fused_consts(device: torch.device):
    """Device constants of the CRC fused into the AES decrypt (``kernels/aes_cbc.hip``
    ``AesCrc``; ``transmux_launch(..., expect, crc_w, crc_tables)``): the decrypt's B fragments (4 steps x
    64 lanes x 16 bytes) followed by the chunk fold's A fragments (64 steps), and the shift
    tables P_0..P_39, Q_0..Q_11."""
    k = (str(device), "chunk")
    c = _consts.get(k)
    if c is None:
        w = torch.from_numpy(_rt().crc_chunk_weights_fp4()).to(device)
        c = (w, _device_consts(device, "fp4")[1])
        with _lock:
            _consts[k] = c
    return c


def crc32_batch(buf: torch.Tensor, offs: Sequence[int], lens: Sequence[int],
                expect: Optional[Sequence[int]] = None,
                expect_dev: Optional[torch.Tensor] = None, scatter_to: Optional[torch.Tensor] = None,
                scatter_idx: Optional[Sequence[int]] = None,
                variant: Optional[str] = None,
                keys: Optional[np.ndarray] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """CRC-32 of ``buf[offs[i]:offs[i]+lens[i]]``.

    Returns ``(crc int32[B], ok uint8[B] | None)`` on ``buf.device``; ``ok`` is produced
    when expected values are given (host list ``expect`` or device tensor ``expect_dev``).
    With ``scatter_to`` (int32 table on ``buf.device``) the CRCs are also written to
    ``scatter_to[scatter_idx[i]]`` -- on the device by the combine kernel, whose index
    array rides the same descriptor H2D (no separate index copy / index_put launch).
    ``variant`` picks the residue kernel's matrix-core path (default :data:`MFMA_VARIANT`).

    ``keys`` (int64[B, 4] segment keys ``(swarm, level, urlId, sn)``): keyed mode -- the
    expected values and the scattered table entries are the CRCs bound to each segment's key,
    ``crc ^ key_digest(key)`` (computed in the combine kernel from the keys riding the
    descriptor block; :func:`key_digest` is the host twin).  A node's CRC table and the trailers
    it sends hold keyed values, so bytes that reach a peer under another key fail its check.
    The returned ``crc`` is always the plain CRC-32.
    """
    B = len(offs)
    o = np.asarray(offs, dtype=np.int64)
    n = np.asarray(lens, dtype=np.int64)
    if B == 0:
        z = torch.empty(0, dtype=torch.int32, device=buf.device)
        want_ok = expect is not None or expect_dev is not None
        return z, (torch.empty(0, dtype=torch.uint8, device=buf.device) if want_ok else None)
    sidx = None if scatter_to is None else np.asarray(scatter_idx, dtype=np.int64).reshape(-1)
    kk = None
    if keys is not None:
        kk = np.ascontiguousarray(np.asarray(keys, dtype=np.int64).reshape(-1, 4)[:, :4])
        if len(kk) != B:
            raise ValueError("crc32_batch: keys must be int64[B, 4]")
    if buf.device.type == "cpu":
        if np.any(o < 0) or np.any(n < 0) or np.any(o + n > buf.numel()):
            raise ValueError("crc32_batch: range out of bounds")
        if sidx is not None and (sidx.size != B or np.any(sidx < 0) or np.any(sidx >= scatter_to.numel())):
            raise ValueError("crc32_batch: scatter index out of range")
        crc = _rt().crc32_batch(buf.numpy(), o, n).view(np.int32)
        crc_t = torch.from_numpy(crc.copy())
        bound = crc if kk is None else crc ^ key_digest(kk)
        bound_t = crc_t if kk is None else torch.from_numpy(bound.copy())
        ok = None
        if expect_dev is not None:
            ok = (bound_t == expect_dev.to(torch.int32)).to(torch.uint8)
        elif expect is not None:
            exp = np.asarray(expect, dtype=np.uint32).view(np.int32)
            ok = torch.from_numpy((bound == exp).astype(np.uint8))
        if sidx is not None:
            scatter_to[torch.from_numpy(sidx)] = bound_t
        return crc_t, ok
    w, tables = _device_consts(buf.device, variant or MFMA_VARIANT)  # bounds / alignment: checked natively
    if expect_dev is None and expect is not None:
        expect_dev = torch.from_numpy(np.asarray(expect, dtype=np.uint32).view(np.int32).copy()).to(buf.device)
    # one native call: descriptor math, one staging H2D, residue + combine launches
    return _dev().crc32_launch(buf, o, n, w, tables, expect_dev, scatter_to, sidx, kk)


def key_digest(keys: np.ndarray) -> np.ndarray:
    """int32[n] digests of int64[n, 4] segment keys: the value a keyed CRC is XOR-ed with
    (``crc32_batch(..., keys=...)``; host twin of the combine kernel's ``key_digest``)."""
    k = np.ascontiguousarray(np.asarray(keys, dtype=np.int64).reshape(-1, 4)[:, :4])
    return _rt().key_digest(k).view(np.int32)


def _crc32_batch_py(buf: torch.Tensor, o: np.ndarray, n: np.ndarray, expect, expect_dev, scatter_to, sidx,
                    variant: Optional[str] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """The same device launch assembled in Python (kept as the reference for the native
    ``crc32_launch``; tests compare the two)."""
    B = len(o)
    groups = (n + 255) // 256
    tiles = (groups + 31) // 32
    tile_prefix = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(tiles, out=tile_prefix[1:])
    res_off = np.zeros(B, dtype=np.int64)
    if B > 1:
        np.cumsum(groups[:-1], out=res_off[1:])
    arrays = {"o": o, "n": n, "tp": tile_prefix, "ro": res_off}
    if expect is not None and expect_dev is None:
        arrays["ex"] = np.asarray(expect, dtype=np.uint32)
    if sidx is not None:
        arrays["si"] = sidx
    d = pack_to_device(arrays, buf.device)
    w, tables = _device_consts(buf.device, variant or MFMA_VARIANT)
    residues = torch.empty(max(1, int(groups.sum())), dtype=torch.int32, device=buf.device)
    crc = torch.empty(B, dtype=torch.int32, device=buf.device)
    exp_t = expect_dev if expect_dev is not None else d.get("ex")
    ok = torch.empty(B, dtype=torch.uint8, device=buf.device) if exp_t is not None else None
    _dev().crc32_batch(buf, d["o"], d["n"], d["tp"], d["ro"], w, tables, residues, crc, exp_t, ok,
                       int(tile_prefix[-1]), d.get("si"), scatter_to)
    return crc, ok


def crc32(data) -> int:
    """Host CRC-32 of bytes / numpy / CPU tensor (== zlib.crc32)."""
    if isinstance(data, torch.Tensor):
        data = data.detach().cpu().numpy()
    if isinstance(data, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(data, dtype=np.uint8)
    else:
        arr = np.asarray(data, dtype=np.uint8)
    return int(_rt().crc32(np.ascontiguousarray(arr)))


def to_u32(x: int) -> int:
    return int(x) & 0xFFFFFFFF
