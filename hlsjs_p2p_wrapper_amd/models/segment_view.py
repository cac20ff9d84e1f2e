"""SegmentView — identity of one media segment ``(sn, trackView)`` plus its start ``time``.

Parity: ``lib/integration/mapping/segment-view.js:3-66`` (component C8).

The 12-byte binary wire/cache key is ``Uint32Array([level, urlId, sn])`` in little-endian
byte order (``:59-61``, ``:9-17``); ``time`` is not serialised in the binary form but does
survive a JSON round-trip (``test/segment-view.js:5-11``).  On the MI355X engine the same
12-byte layout is the row format of the ``int32[B,3]`` key tensors that the device hash
kernel (``ops.keys``) packs and hashes in batches, so ``toArrayBuffer()`` of a view and
row ``i`` of a packed key tensor are byte-identical.
"""
from __future__ import annotations

import struct
from typing import Any, Optional, Tuple

from .track_view import TrackView, _js_str

_KEY = struct.Struct("<III")
KEY_BYTES = _KEY.size  # 12


def _field(obj: Any, name: str) -> Any:
    if isinstance(obj, dict):
        return obj.get(name)
    return getattr(obj, name, None)


class SegmentView:
    """One media segment ``(sn, trackView)`` plus its start ``time``; 12-byte binary key."""

    __slots__ = ("sn", "trackView", "time")

    def __init__(self, obj: Any = None, *, sn: Any = None, trackView: Any = None,
                 time: Any = None) -> None:
        if obj is not None:
            sn = _field(obj, "sn")
            trackView = _field(obj, "trackView")
            time = _field(obj, "time")
        self.sn = sn
        # the reference deep-copies the track view (``segment-view.js:24``)
        self.trackView = TrackView(trackView)
        self.time = time

    @classmethod
    def _owning(cls, sn: Any, trackView: TrackView, time: Any) -> "SegmentView":
        """A view that takes ``trackView`` as is (no copy): for callers that just built that
        TrackView and hand it over (the P2P loader, once per fragment request)."""
        v = cls.__new__(cls)
        v.sn = sn
        v.trackView = trackView
        v.time = time
        return v

    # --- reference API -------------------------------------------------------
    @staticmethod
    def fromArrayBuffer(buf: Any) -> "SegmentView":
        """Inverse of :meth:`toArrayBuffer` (``segment-view.js:9-17``)."""
        mv = memoryview(_as_bytes(buf))
        level, url_id, sn = _KEY.unpack_from(mv, 0)
        return SegmentView(trackView=TrackView(level=level, urlId=url_id), sn=sn)

    def isEqual(self, segmentView: Optional["SegmentView"]) -> bool:
        """Same sn and track (``time`` ignored; ``False`` for a falsy argument)."""
        if not segmentView:
            return False
        return self.sn == segmentView.sn and self.trackView.isEqual(segmentView.trackView)

    def isInTrack(self, trackView: Optional[TrackView]) -> bool:
        """The segment belongs to ``trackView``."""
        return self.trackView.isEqual(trackView)

    def viewToString(self) -> str:
        """``"L{level}U{urlId}S{sn}"``."""
        return f"{self.trackView.viewToString()}S{_js_str(self.sn)}"

    def toArrayBuffer(self) -> bytes:
        """12-byte key ``<u32 level, u32 urlId, u32 sn>`` (``segment-view.js:59-61``)."""
        return _KEY.pack(_u32(self.trackView.level), _u32(self.trackView.urlId), _u32(self.sn))

    def getId(self) -> Any:
        """The sequence number."""
        return self.sn

    # --- python conveniences -------------------------------------------------
    from_array_buffer = fromArrayBuffer
    is_equal = isEqual
    is_in_track = isInTrack
    view_to_string = viewToString
    to_array_buffer = toArrayBuffer
    get_id = getId

    def key(self) -> Tuple[int, int, int]:
        """``(level, urlId, sn)`` as u32 — the cache/wire identity (time excluded)."""
        return (_u32(self.trackView.level), _u32(self.trackView.urlId), _u32(self.sn))

    def to_dict(self) -> dict:
        """``{"sn", "trackView"[, "time"]}`` (JSON form; ``time`` survives the round trip)."""
        d = {"sn": self.sn, "trackView": self.trackView.to_dict()}
        if self.time is not None:
            d["time"] = self.time
        return d

    toJSON = to_dict

    def __eq__(self, other: object) -> bool:  # deep equality (``should.eql``)
        return (isinstance(other, SegmentView) and self.sn == other.sn
                and self.trackView == other.trackView and self.time == other.time)

    def __hash__(self) -> int:
        return hash((self.sn, self.trackView.level, self.trackView.urlId))

    def __bool__(self) -> bool:
        return True

    def __repr__(self) -> str:
        return f"SegmentView(sn={self.sn!r}, trackView={self.trackView!r}, time={self.time!r})"


def _u32(v: Any) -> int:
    """``Uint32Array`` element conversion (ToUint32; ``undefined``/NaN → 0)."""
    if v is None:
        return 0
    try:
        f = float(v)
    except (TypeError, ValueError):
        return 0
    if f != f or f in (float("inf"), float("-inf")):
        return 0
    return int(f) & 0xFFFFFFFF


def _as_bytes(buf: Any) -> bytes:
    if isinstance(buf, (bytes, bytearray, memoryview)):
        return bytes(buf)
    if hasattr(buf, "numpy"):  # torch tensor
        buf = buf.detach().cpu().numpy()
    if hasattr(buf, "tobytes"):  # numpy
        return buf.tobytes()
    return bytes(buf)
