"""Warm restart of a peer's HBM segment cache.

The reference has no checkpointing: the cache lives inside the closed-source agent and
dies with the session (``lib/hlsjs-p2p-wrapper-private.js:105-113``).  A GPU peer's cache
can hold hundreds of GB of segments, so losing it on a process restart costs a full
re-fetch from the CDN.  :func:`save_cache` writes the resident segments, their keys and
their ingest CRCs to a safetensors file (no pickle: loading executes nothing from the
file).  :func:`load_cache` places them back into a node's arena in their original
eviction order and re-verifies every byte with the CRC kernel, dropping any segment that
fails.  The surviving entries are committed, so the next round announces them to the
swarm like freshly fetched segments.

File layout (tensors): ``keys`` int64[n,4], ``lens`` int64[n], ``crcs`` int32[n],
``offs`` int64[n] (byte offsets into ``data``, ALIGN-aligned), ``data`` uint8[total].
Metadata: ``format`` = ``hlsjs-p2p-cache/1``, ``align``.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

FORMAT = "hlsjs-p2p-cache/1"


def save_cache(node, path: str) -> Dict[str, int]:
    """Checkpoint ``node``'s resident segments to ``path`` (safetensors)."""
    from safetensors.torch import save_file

    from .node import ALIGN

    if node.is_cuda:
        torch.cuda.current_stream(node.device).wait_stream(node.stream)  # queued ingest finished
        torch.cuda.synchronize(node.device)
    ids, keys = node.store.resident()
    n = len(ids)
    if n:
        ent = node.store.entries(ids)
        offs_src, lens = ent[:, 0], ent[:, 1]
    else:
        offs_src = lens = np.zeros(0, dtype=np.int64)
    aligned = (lens + ALIGN - 1) // ALIGN * ALIGN
    offs = np.zeros(n, dtype=np.int64)
    if n > 1:
        offs[1:] = np.cumsum(aligned[:-1])
    total = int(aligned.sum()) if n else 0
    data = torch.zeros(max(total, 1), dtype=torch.uint8)
    if n:
        staged = torch.empty(max(total, 1), dtype=torch.uint8, device=node.device)
        from ..ops import segment as _seg

        _seg.copy_segments(node.arena, staged, offs_src, offs, lens)
        data.copy_(staged)
        if getattr(node, "ingest_crc", True):
            # the table holds keyed CRCs (crc ^ key digest): the file keeps plain CRC-32s
            crcs = node.crc_dev[torch.from_numpy(ids).to(node.device)].cpu()
            crcs = torch.from_numpy(crcs.numpy() ^ _crc_mod().key_digest(keys))
        else:  # a one-rank node keeps no CRC table: compute the CRCs the restore verifies
            from ..ops import crc as _crc

            crcs = _crc.crc32_batch(staged, offs.tolist(), lens.tolist())[0].cpu()
    else:
        crcs = torch.zeros(0, dtype=torch.int32)
    save_file({"keys": torch.from_numpy(np.ascontiguousarray(keys, dtype=np.int64)),
               "lens": torch.from_numpy(lens.astype(np.int64)),
               "offs": torch.from_numpy(offs),
               "crcs": crcs.to(torch.int32).contiguous(),
               "data": data}, path, metadata={"format": FORMAT, "align": str(ALIGN)})
    return {"segments": n, "bytes": int(lens.sum()) if n else 0}


def _crc_mod():
    from ..ops import crc as _crc

    return _crc


def load_cache(node, path: str) -> Dict[str, int]:
    """Restore a checkpoint into ``node`` (same or different process / device).  Entries
    that no longer fit the cache, or whose bytes fail their CRC, are skipped."""
    from safetensors import safe_open

    from ..ops import crc as _crc
    from ..ops import segment as _seg

    with safe_open(path, framework="pt") as f:
        meta = f.metadata() or {}
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a segment-cache checkpoint ({meta.get('format')!r})")
        keys = f.get_tensor("keys").numpy()
        lens = f.get_tensor("lens").numpy()
        offs = f.get_tensor("offs").numpy()
        crcs = f.get_tensor("crcs")
        data = f.get_tensor("data")
    n = len(lens)
    if n == 0:
        return {"restored": 0, "skipped": 0, "bad_crc": 0}
    st = node.store
    keep = []  # newest entries win if the cache is smaller than the checkpoint
    budget = node.cache_bytes
    for i in range(n - 1, -1, -1):
        a = st.aligned(int(lens[i]))
        if a > budget:
            break
        budget -= a
        keep.append(i)
    keep = keep[::-1]
    if not keep:
        return {"restored": 0, "skipped": n, "bad_crc": 0}
    k = np.ascontiguousarray(keys[keep])
    ln = np.ascontiguousarray(lens[keep])
    res = st.reserve_run(k, ln, node.round)
    if res is None:
        raise RuntimeError("segment cache has pinned entries in the way; restore before playback starts")
    _, ids, dst_offs = res
    node._grow_crc(int(ids.max()) + 1)
    # the node stream owns the CRC table (node.py's ownership rule): the restore runs on it,
    # so the table write below is ordered before the next round's trailer gathers
    with node._on_node_stream():
        src = data.to(node.device, non_blocking=False) if node.is_cuda else data
        _seg.copy_segments(src, node.arena, offs[keep], dst_offs, ln)
        expect = crcs[keep].to(node.device)
        _, ok = _crc.crc32_batch(node.arena, dst_offs.tolist(), ln.tolist(), expect_dev=expect)
        ok = ok.cpu().numpy().astype(bool)
        good, bad = ids[ok], ids[~ok]
        keyed = crcs[keep].numpy() ^ _crc.key_digest(k)  # the table holds CRCs bound to their keys
        node.crc_dev[torch.from_numpy(good).to(node.device)] = torch.from_numpy(keyed[ok]).to(node.device)
    if len(good):
        st.commit(good)
    if len(bad):
        st.drop(bad)
    return {"restored": int(len(good)), "skipped": n - len(keep), "bad_crc": int(len(bad))}
