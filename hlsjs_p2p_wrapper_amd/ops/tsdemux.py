"""MPEG-TS demux of segment batches.

Output per segment (identical for the gfx950 kernels and the host oracle):

* ES bytes per class at ``es_offs[i]`` of the ES buffer: video at 0, audio and id3 at the
  offsets the info row gives (``audio_es_offset`` / ``id3_es_offset``: packed back to back);
* ``pes[i, class, k] = (es_offset, pts, dts)`` for the k-th PES of each class;
* ``info[i]`` = status bits, PIDs, packet count, per-class byte and PES counts
  (slot names in :data:`INFO`).

Segment lengths may be a device tensor (the decrypt kernel's ``out_len``), so decrypt ->
demux needs no host round trip; ``caps`` (host upper bounds, e.g. ciphertext sizes)
size the grid.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence, Union

import numpy as np
import torch

from ._native import device as _dev
from ._native import runtime as _rt
from .desc import pack_to_device

PACKET = 188
CLASSES = ("video", "audio", "id3")
INFO = {"status": 0, "pmt_pid": 1, "video_pid": 2, "audio_pid": 3, "id3_pid": 4, "n_packets": 5,
        "video_bytes": 6, "audio_bytes": 7, "id3_bytes": 8, "n_video_pes": 9, "n_audio_pes": 10,
        "n_id3_pes": 11, "video_type": 12, "audio_type": 13, "payload_bytes": 14,
        "video_first_pts": 16, "audio_first_pts": 17, "id3_first_pts": 18,
        "video_last_pts": 19, "audio_last_pts": 20, "id3_last_pts": 21,
        "audio_es_offset": 22, "id3_es_offset": 23}
INFO_WORDS = 24
STATUS = {"bad_sync": 1, "no_pat": 2, "no_pmt": 4, "pes_overflow": 8, "pes_header_error": 16, "bad_length": 32}
DEFAULT_MAX_PES = 512


@dataclass
class DemuxResult:
    info: torch.Tensor        # int64[B, 16]
    pes: torch.Tensor         # int64[B, 3, max_pes, 3]
    es: torch.Tensor          # the ES buffer
    es_offs: np.ndarray       # host int64[B]

    def segment(self, i: int) -> dict:
        """Host view of segment ``i`` (syncs)."""
        info = self.info[i].cpu().numpy()
        pes = self.pes[i].cpu().numpy()
        out = {k: int(info[v]) for k, v in INFO.items()}
        base = int(self.es_offs[i])
        sizes = [out["video_bytes"], out["audio_bytes"], out["id3_bytes"]]
        starts = [base, base + out["audio_es_offset"], base + out["id3_es_offset"]]
        counts = [out["n_video_pes"], out["n_audio_pes"], out["n_id3_pes"]]
        for c, name in enumerate(CLASSES):
            out[name] = {"es": self.es[starts[c]:starts[c] + sizes[c]],
                         "pes": pes[c, :min(counts[c], pes.shape[1])]}
        return out


def demux_batch(buf: torch.Tensor, offs: Sequence[int], lens: Union[Sequence[int], torch.Tensor],
                es: torch.Tensor, es_offs: Sequence[int], caps: Optional[Sequence[int]] = None,
                max_pes: int = DEFAULT_MAX_PES) -> DemuxResult:
    B = len(offs)
    o = np.asarray(offs, dtype=np.int64)
    eo = np.asarray(es_offs, dtype=np.int64)
    if isinstance(lens, torch.Tensor):
        if caps is None:
            raise ValueError("caps (host upper bounds) are required when lens is a tensor")
        cap = np.asarray(caps, dtype=np.int64)
    else:
        cap = np.asarray(lens, dtype=np.int64)
    if np.any(o + cap > buf.numel()) or np.any(eo + cap > es.numel()):
        raise ValueError("demux_batch: range out of bounds")
    dev = buf.device
    if dev.type == "cpu":
        n = lens.numpy().astype(np.int64) if isinstance(lens, torch.Tensor) else cap
        n = np.minimum(np.maximum(n, 0), cap)
        info = np.zeros((B, INFO_WORDS), dtype=np.int64)
        pes = np.zeros((B, 3, max_pes, 3), dtype=np.int64)
        _rt().demux_batch(buf.numpy(), o, n, es.numpy(), eo, pes, info, max_pes)
        if isinstance(lens, torch.Tensor):
            bad = lens.numpy() < 0
            info[bad, 0] |= STATUS["bad_length"]
        return DemuxResult(torch.from_numpy(info), torch.from_numpy(pes), es, eo)
    if np.any(o % 16):
        raise ValueError("demux_batch: offsets must be 16-byte aligned on device")
    blocks = ((cap + PACKET - 1) // PACKET + 255) // 256
    blk_prefix = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(blocks, out=blk_prefix[1:])
    arrays = {"o": o, "bp": blk_prefix, "eo": eo}
    if not isinstance(lens, torch.Tensor):
        arrays["n"] = cap
    d = pack_to_device(arrays, dev)
    n_dev = lens if isinstance(lens, torch.Tensor) else d["n"]
    total_blocks = int(blk_prefix[-1])
    nb = max(1, total_blocks)
    meta = torch.empty(nb * 256, dtype=torch.int32, device=dev)
    pts_dts = torch.empty(nb * 256 * 2, dtype=torch.int64, device=dev)
    blk_sums = torch.empty(nb * 12 + B * 7, dtype=torch.int32, device=dev)  # sums|prefixes|totals|counters
    info = torch.empty((B, INFO_WORDS), dtype=torch.int64, device=dev)
    pes = torch.empty((B, 3, max_pes, 3), dtype=torch.int64, device=dev)
    _dev().ts_demux(buf, d["o"], n_dev, d["bp"], total_blocks, meta, pts_dts, blk_sums, es, d["eo"], pes, max_pes, info)
    return DemuxResult(info, pes, es, eo)


def mux_segment(duration: float = 4.0, fps: float = 25.0, target_bytes: int = 3_000_000, audio_kbps: int = 128,
                with_id3: bool = False, seed: int = 1, sn: int = 0, start_time: float = 0.0):
    """Synthetic MPEG-TS segment (PAT/PMT, H.264-like video PES, ADTS audio PES)."""
    return _rt().mux_segment(float(duration), float(fps), int(target_bytes), int(audio_kbps), bool(with_id3),
                             int(seed), int(sn), float(start_time))
