"""Media element model — the ``<video>`` + MSE ``SourceBuffer`` the player drives.

The reference hands the real ``HTMLVideoElement`` to the peer agent
(``lib/hlsjs-p2p-wrapper-private.js:174-182``) so it can follow the playhead, and its
browser tests assert on ``currentTime``, ``timeupdate`` and ``seeked``
(``test/html/bundle.js:45-78``).  This is that element for a server-side MI355X peer:

* ``currentTime`` / ``paused`` / ``seeking`` / ``ended`` / ``buffered`` (TimeRanges) /
  ``readyState`` / ``playbackRate`` / ``duration`` and ``addEventListener`` for
  ``timeupdate``, ``playing``, ``waiting``, ``seeking``, ``seeked``, ``ended``;
* a playback clock on the event loop (``mode="realtime"``: advances with loop time while
  the playhead is inside a buffered range, stalls otherwise), or ``mode="drain"``: a
  consumer that takes buffered media as fast as it arrives (restream / edge-cache use
  and throughput benches);
* the SourceBuffer side: ``append(start, end, nbytes, data)`` merges buffered ranges;
  a back-buffer is evicted behind the playhead so memory stays bounded.
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional, Tuple

from ..net.event_loop import get_event_loop
from ..utils.events import EventEmitter


class TimeRanges:
    def __init__(self, ranges: Optional[List[Tuple[float, float]]] = None) -> None:
        self._r: List[Tuple[float, float]] = list(ranges or [])

    @property
    def length(self) -> int:
        return len(self._r)

    def start(self, i: int) -> float:
        return self._r[i][0]

    def end(self, i: int) -> float:
        return self._r[i][1]

    def __len__(self) -> int:
        return len(self._r)

    def __iter__(self):
        return iter(self._r)

    def __repr__(self) -> str:
        return f"TimeRanges({self._r})"


class MediaElement(EventEmitter):
    """``<video>`` + SourceBuffer model: playhead clock, buffered ranges, media events."""
    TICK_MS = 250.0
    GAP_TOLERANCE = 0.1  # seconds: adjacent appends closer than this merge

    def __init__(self, mode: str = "realtime", loop=None, back_buffer: float = 30.0) -> None:
        super().__init__()
        if mode not in ("realtime", "drain"):
            raise ValueError("mode must be 'realtime' or 'drain'")
        self.mode = mode
        self.loop = loop or get_event_loop()
        self.back_buffer = back_buffer
        self._ranges: List[Tuple[float, float]] = []
        self._time = 0.0
        self.paused = True
        self.seeking = False
        self.ended = False
        self.playbackRate = 1.0
        self.duration = float("nan")
        self.volume = 1.0
        self._last_tick: Optional[float] = None
        self._timer = None
        self._stalled = False
        self.bytes_appended = 0
        self.segments_appended = 0
        self.retained: List[Any] = []
        self.retain = False

    # ---------------------------------------------------------------- DOM-ish API
    def addEventListener(self, name: str, fn: Callable) -> None:
        """Subscribe to a media event (``timeupdate``, ``seeked``, ...)."""
        self.on(name, fn)

    def removeEventListener(self, name: str, fn: Callable) -> None:
        """Unsubscribe."""
        self.remove_listener(name, fn)

    @property
    def currentTime(self) -> float:
        """Playhead position in seconds (settable: seeks)."""
        return self._time

    @currentTime.setter
    def currentTime(self, t: float) -> None:
        self._time = max(0.0, float(t))
        self.seeking = True
        self.ended = False
        self.emit("seeking")
        self._check_seeked()

    @property
    def buffered(self) -> TimeRanges:
        """Buffered ranges as TimeRanges."""
        return TimeRanges(self._ranges)

    @property
    def readyState(self) -> int:
        """4 with > 0.5 s buffered ahead, 1 with any buffer, else 0."""
        return 4 if self._buffer_ahead(self._time) > 0.5 else (1 if self._ranges else 0)

    def play(self) -> None:
        """Start the playback clock (``play``)."""
        if not self.paused:
            return
        self.paused = False
        self._last_tick = self.loop.now()
        self._ensure_timer()
        self.emit("play")

    def pause(self) -> None:
        """Stop the playback clock."""
        self.paused = True
        self.emit("pause")

    # ---------------------------------------------------------------- SourceBuffer side
    def append(self, start: float, end: float, nbytes: int = 0, data: Any = None) -> None:
        """SourceBuffer append of media ``[start, end)`` (``nbytes`` counted, ranges merged)."""
        if end <= start:
            return
        self.bytes_appended += int(nbytes)
        self.segments_appended += 1
        if self.retain and data is not None:
            self.retained.append((start, end, data))
        rs = self._ranges
        rs.append((start, end))
        rs.sort()
        merged: List[Tuple[float, float]] = []
        for s, e in rs:
            if merged and s <= merged[-1][1] + self.GAP_TOLERANCE:
                merged[-1] = (merged[-1][0], max(merged[-1][1], e))
            else:
                merged.append((s, e))
        self._ranges = merged
        if self.mode == "drain" and not self.paused and not self.seeking:
            self._drain()
        self._check_seeked()

    def remove(self, start: float, end: float) -> None:
        """Drop buffered media in ``[start, end)``."""
        out = []
        for s, e in self._ranges:
            if e <= start or s >= end:
                out.append((s, e))
            else:
                if s < start:
                    out.append((s, start))
                if e > end:
                    out.append((end, e))
        self._ranges = out
        if self.retained:
            self.retained = [r for r in self.retained if r[1] <= start or r[0] >= end]

    def flush(self) -> None:
        """Drop all buffered media."""
        self._ranges = []
        self.retained = []

    # ---------------------------------------------------------------- playback clock
    def _buffer_ahead(self, t: float) -> float:
        for s, e in self._ranges:
            if s - self.GAP_TOLERANCE <= t < e:
                return e - t
        return 0.0

    def _range_end_at(self, t: float) -> Optional[float]:
        for s, e in self._ranges:
            if s - self.GAP_TOLERANCE <= t < e + 1e-9:
                return e
        return None

    def _ensure_timer(self) -> None:
        if self._timer is None:
            self._timer = self.loop.set_interval(self._tick, self.TICK_MS)

    def _drain(self) -> None:
        end = self._range_end_at(self._time)
        if end is not None and end > self._time:
            self._time = end
            self.emit("timeupdate")
            self._evict_back_buffer()

    def _tick(self) -> None:
        now = self.loop.now()
        last = self._last_tick if self._last_tick is not None else now
        self._last_tick = now
        if self.paused or self.seeking or self.ended:
            return
        if self.mode == "drain":
            self._drain()
            return
        ahead = self._buffer_ahead(self._time)
        if ahead <= 0:
            if not self._stalled:
                self._stalled = True
                self.emit("waiting")
            if self.duration == self.duration and self._time >= self.duration - 0.05:
                self.ended = True
                self.emit("ended")
            return
        if self._stalled:
            self._stalled = False
            self.emit("playing")
        dt = (now - last) / 1000.0 * self.playbackRate
        self._time = min(self._time + dt, self._time + ahead)
        self.emit("timeupdate")
        self._evict_back_buffer()

    def _evict_back_buffer(self) -> None:
        limit = self._time - self.back_buffer
        if self._ranges and self._ranges[0][0] < limit:
            self.remove(0.0, limit)

    def _check_seeked(self) -> None:
        if self.seeking and self._range_end_at(self._time) is not None:
            self.seeking = False
            self._last_tick = self.loop.now()
            self.emit("seeked")
            if self.mode == "drain" and not self.paused:
                self._drain()

    def stop(self) -> None:
        """Cancel the playback timer."""
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None

    def restart(self) -> None:
        """Restart the playback clock after :meth:`stop` (the engine re-attaching this element)
        unless playback is paused."""
        if not self.paused and self._timer is None:
            self._last_tick = self.loop.now()
            self._ensure_timer()


HTMLVideoElement = MediaElement
