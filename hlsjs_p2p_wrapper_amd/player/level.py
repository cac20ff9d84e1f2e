"""Playlist data model: ``Level``, ``LevelDetails``, ``Fragment`` (hls.js shapes).

Fields are the ones the reference reads: ``levels[i].url[]`` (redundant
URLs), ``urlId``, ``details.live``, ``details.fragments[]`` with ``sn``, ``start``,
``duration``, ``level``, ``byteRangeStartOffset``/``EndOffset``, ``loaded``, and
``details.totalduration``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, List, Optional


@dataclass(slots=True)
class DecryptData:
    method: Optional[str] = None
    uri: Optional[str] = None
    iv: Optional[bytes] = None
    key: Optional[bytes] = None

    @property
    def needs_key(self) -> bool:
        return self.method == "AES-128" and self.uri is not None and self.key is None


# Bumped whenever a Fragment's ``start`` is REWRITTEN after construction: consumers that
# cache derived start-time arrays (models.media_map) compare generations instead of trusting
# list identity -- hls.js rewrites ``frag.start`` in place on PTS realignment.  Building
# fragments (a playlist parse or reload) does not bump it, so it never invalidates the start
# index of other levels.
_START_GENERATION = [0]


def fragment_generation() -> int:
    """Counter of post-construction ``Fragment.start`` rewrites in this process."""
    return _START_GENERATION[0]


class Fragment:
    """One media fragment (hls.js ``Fragment`` fields the reference reads).  A plain slotted
    class (a long DVR playlist holds 10^5..10^6 of these): field writes are slot stores with
    no Python hook; only ``start`` is a property, whose setter bumps the generation."""

    __slots__ = ("url", "sn", "_start", "duration", "level", "cc", "byteRangeStartOffset", "byteRangeEndOffset",
                 "decryptdata", "loaded", "loadCounter", "loadIdx", "autoLevel", "loader", "title",
                 "programDateTime")

    def __init__(self, url: str, sn: int, start: float, duration: float, level: int = 0, cc: int = 0,
                 byteRangeStartOffset: Optional[int] = None, byteRangeEndOffset: Optional[int] = None,
                 decryptdata: Optional[DecryptData] = None, loaded: int = 0, loadCounter: int = 0,
                 loadIdx: int = 0, autoLevel: bool = False, loader: Any = None, title: str = "",
                 programDateTime: Any = None) -> None:
        self.url = url
        self.sn = sn
        self._start = start
        self.duration = duration
        self.level = level
        self.cc = cc
        self.byteRangeStartOffset = byteRangeStartOffset
        self.byteRangeEndOffset = byteRangeEndOffset
        self.decryptdata = decryptdata
        self.loaded = loaded
        self.loadCounter = loadCounter
        self.loadIdx = loadIdx
        self.autoLevel = autoLevel
        self.loader = loader
        self.title = title
        self.programDateTime = programDateTime

    @property
    def start(self) -> float:
        return self._start

    @start.setter
    def start(self, value: float) -> None:
        self._start = value
        _START_GENERATION[0] += 1

    @property
    def end(self) -> float:
        return self.start + self.duration

    def iv_for_decrypt(self) -> Optional[bytes]:
        dd = self.decryptdata
        if dd is None or dd.method != "AES-128":
            return None
        if dd.iv is not None:
            return dd.iv
        return int(self.sn).to_bytes(16, "big")

    def __repr__(self) -> str:
        return f"Fragment(sn={self.sn}, level={self.level}, start={self.start:.3f}, dur={self.duration:.3f})"


@dataclass(eq=False)
class LevelDetails:
    url: str
    fragments: List[Fragment] = field(default_factory=list)
    live: bool = True
    startSN: int = 0
    endSN: int = 0
    targetduration: float = 0.0
    totalduration: float = 0.0
    version: int = 3
    averagetargetduration: float = 0.0
    endCC: int = 0
    PTSKnown: bool = False
    tload: float = 0.0

    def frag_by_sn(self, sn: int) -> Optional[Fragment]:
        i = sn - self.startSN
        if 0 <= i < len(self.fragments) and self.fragments[i].sn == sn:
            return self.fragments[i]
        for f in self.fragments:
            if f.sn == sn:
                return f
        return None


@dataclass(eq=False)
class Level:
    url: List[str]
    bitrate: int = 0
    width: int = 0
    height: int = 0
    name: str = ""
    codecs: str = ""
    audioCodec: Optional[str] = None
    videoCodec: Optional[str] = None
    details: Optional[LevelDetails] = None
    urlId: int = 0
    fragmentError: bool = False

    def __repr__(self) -> str:
        return f"Level(bitrate={self.bitrate}, urls={len(self.url)}, urlId={self.urlId})"
