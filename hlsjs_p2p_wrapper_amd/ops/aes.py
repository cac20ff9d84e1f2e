"""AES-128-CBC segment decryption.

HLS ``#EXT-X-KEY:METHOD=AES-128`` segments are AES-128-CBC with PKCS#7 padding; the IV
is the ``IV=`` attribute or, when absent, the media sequence number as a 128-bit
big-endian integer (RFC 8216 §5.2).  In the reference this runs inside hls.js after
``FRAG_LOADED``; here a whole batch of segments is decrypted by one launch of the CDNA4
kernel ``kernels/aes_cbc.hip``.  CPU tensors use the host oracle (``runtime/aes_host.cpp``).

Round keys (equivalent inverse cipher) are expanded once per key on the host and cached.
"""
from __future__ import annotations

import threading
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from ._native import device as _dev
from ._native import runtime as _rt
from .desc import pack_to_device

_key_cache: Dict[bytes, np.ndarray] = {}
_key_cache_le: Dict[bytes, np.ndarray] = {}
_tables: Dict[str, tuple] = {}
_lock = threading.Lock()


def iv_from_sn(sn: int) -> bytes:
    """Default HLS IV: the media sequence number, 128-bit big-endian."""
    return int(sn).to_bytes(16, "big")


def round_keys(key: bytes) -> np.ndarray:
    rk = _key_cache.get(key)
    if rk is None:
        if len(key) != 16:
            raise ValueError("AES-128 key must be 16 bytes")
        rk = _rt().expand_key_dec(key)
        with _lock:
            _key_cache[key] = rk
    return rk


def round_keys_le(key: bytes) -> np.ndarray:
    """Round keys as the kernel consumes them: uint32[44] byte-swapped to little-endian
    column words (state words are used as loaded)."""
    rk = _key_cache_le.get(key)
    if rk is None:
        rk = np.ascontiguousarray(round_keys(bytes(key)).astype(np.uint32).byteswap())
        with _lock:
            _key_cache_le[key] = rk
    return rk


def device_tables(device: torch.device):
    """(TdL int32[256], InvSbox uint8[256]) on ``device`` (cached)."""
    return _device_tables(device)


def _device_tables(device: torch.device):
    k = str(device)
    t = _tables.get(k)
    if t is None:
        td0, inv, _, _ = _rt().aes_tables()
        # the kernel works on little-endian column words: TdL = bswap(Td0)
        tdl = td0.astype(np.uint32).byteswap()
        t = (torch.from_numpy(tdl.view(np.int32).copy()).to(device), torch.from_numpy(inv.copy()).to(device))
        with _lock:
            _tables[k] = t
    return t


def cbc_decrypt_batch(src: torch.Tensor, src_offs: Sequence[int], nbytes: Sequence[int], keys: Sequence[bytes],
                      ivs: Sequence[bytes], dst: torch.Tensor, dst_offs: Sequence[int]) -> torch.Tensor:
    """Decrypt ``len(src_offs)`` segments; returns ``int64[B]`` plaintext lengths on
    ``src.device`` (``-1`` = bad PKCS#7 padding).  ``dst`` must not alias ``src``."""
    B = len(src_offs)
    nb = np.asarray(nbytes, dtype=np.int64)
    if B == 0:
        return torch.empty(0, dtype=torch.int64, device=src.device)
    if np.any(nb % 16) or np.any(nb < 16):
        raise ValueError("AES-CBC segments must be non-empty multiples of 16 bytes")
    if np.any(nb >= 1 << 31):
        raise ValueError("AES-CBC segments must be under 2 GiB (the kernel's buffer ranges)")
    so = np.asarray(src_offs, dtype=np.int64)
    do = np.asarray(dst_offs, dtype=np.int64)
    if np.any(so % 16) or np.any(do % 16):
        raise ValueError("segment offsets must be 16-byte aligned")
    if np.any(so + nb > src.numel()) or np.any(do + nb > dst.numel()):
        raise ValueError("segment range out of bounds")
    k0 = keys[0]
    if all(k is k0 or k == k0 for k in keys):  # one key per stream: expand / stack once
        drk = np.broadcast_to(round_keys(bytes(k0)).astype(np.uint32), (B, 44))
    else:
        drk = np.stack([round_keys(bytes(k)) for k in keys]).astype(np.uint32)
    iv = np.frombuffer(b"".join(bytes(v) for v in ivs), dtype=np.uint8).reshape(B, 16)
    if src.device.type == "cpu":
        out_len = np.zeros(B, dtype=np.int64)
        _rt().cbc_decrypt_batch(src.numpy(), dst.numpy(), so, do, nb, drk, iv, out_len)
        return torch.from_numpy(out_len)
    blk_prefix = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(nb // 16, out=blk_prefix[1:])
    # work unit: one wave-chunk of consecutive blocks of one segment
    chunk = _dev().aes_chunk_blocks()  # 64 lanes x the kernel's chains per lane
    units = (nb // 16 + chunk - 1) // chunk
    unit_prefix = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(units, out=unit_prefix[1:])
    drk_le = drk.byteswap()  # state words are used as loaded (little-endian) on device
    d = pack_to_device({"so": so, "do": do, "bp": blk_prefix, "pp": unit_prefix, "drk": drk_le, "iv": iv},
                       src.device)
    out_len = torch.empty(B, dtype=torch.int64, device=src.device)
    td0, isb = _device_tables(src.device)
    _dev().aes128_cbc_decrypt(src, dst, d["so"], d["do"], d["bp"], d["pp"], d["drk"], d["iv"], td0, isb, out_len,
                              int(unit_prefix[-1]))
    return out_len


def cbc_encrypt(key: bytes, iv: bytes, data) -> np.ndarray:
    """Host CBC encrypt + PKCS#7 (packager side)."""
    return _rt().cbc_encrypt(bytes(key), bytes(iv), np.ascontiguousarray(np.asarray(data, dtype=np.uint8)))


def cbc_decrypt(key: bytes, iv: bytes, data) -> Optional[np.ndarray]:
    return _rt().cbc_decrypt(bytes(key), bytes(iv), np.ascontiguousarray(np.asarray(data, dtype=np.uint8)))
