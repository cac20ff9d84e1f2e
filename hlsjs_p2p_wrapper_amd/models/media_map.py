"""MediaMap — the peer agent's read-only view of the player's playlists.

Parity: ``lib/integration/mapping/media-map.js:4-88`` (component C9).

* ``getSegmentTime(sv)``   → ``sv.time``; throws if undefined (``:14-19``).
* ``getSegmentList(track, beginTime, duration)`` → the fragments of
  ``levels[track.level]`` with ``beginTime <= start <= beginTime + duration`` (closed on
  both ends), in playlist order, as ``SegmentView{sn, trackView: track, time: start}``.
  Throws if the level does not exist, warns and returns ``[]`` if it is not parsed yet
  (``:27-54``).  Like the reference it ignores ``track.urlId`` when picking the level.
* ``getTrackList()`` → level-major / urlId-minor ``TrackView`` list (``:60-73``).
* ``getSegmentDuration(sv)`` → duration of the *first* fragment of the segment's level
  (reference quirk kept on purpose, ``:81-87``; only the debug buffer display uses it).

Hot-path note (K1 in SURVEY §2.2): the reference does a linear scan per query.  HLS
fragment lists are sorted by ``start``, so the closed interval maps to one contiguous
index range; we cache a start-time array per ``details`` object and answer with two
binary searches (falling back to the literal scan if the list is ever unsorted); the cache
is dropped on any fragment-start rewrite (``player.level.fragment_generation``).
Batched multi-track queries (``getSegmentLists``) share that index.  The answer is always
consumed on the host (the agent's prefetch planning), so a device range-select launch plus
its D2H sync would cost more than the bisects; round 3 removed that kernel.
"""
from __future__ import annotations

import bisect
import logging
from typing import Any, List

from .segment_view import SegmentView
from .track_view import TrackView

log = logging.getLogger("hlsjs_p2p_wrapper_amd.media_map")


def _generation() -> int:
    """The engine's fragment-start mutation counter (player.level), 0 for engines without one."""
    try:
        from ..player.level import fragment_generation
    except ImportError:  # pragma: no cover - the bundled engine always has it
        return 0
    return fragment_generation()


class _StartIndex:
    """Start times of one fragment list, valid while the list object, its length, the
    fragment-start generation and its end points are unchanged."""
    __slots__ = ("frags_id", "n", "gen", "first", "last", "starts", "sorted")

    def __init__(self, fragments: List[Any]) -> None:
        self.frags_id = id(fragments)
        self.n = len(fragments)
        self.gen = _generation()
        self.starts = [f.start for f in fragments]
        s = self.starts
        self.first = fragments[0] if fragments else None
        self.last = fragments[-1] if fragments else None
        self.sorted = all(s[i] <= s[i + 1] for i in range(len(s) - 1))

    def valid_for(self, fragments: List[Any]) -> bool:
        # list identity and length catch replaced / grown playlists; the generation catches
        # in-place start rewrites (PTS realignment); the end points catch objects swapped in
        # without a start assignment
        n = len(fragments)
        return (self.frags_id == id(fragments) and self.n == n and self.gen == _generation()
                and (n == 0 or (fragments[0] is self.first and fragments[-1] is self.last)))


class MediaMap:
    """Segment/track queries over the engine's parsed playlists, for the peer agent."""
    def __init__(self, hls: Any) -> None:
        self.hls = hls
        self._idx: dict = {}

    def getSegmentTime(self, segmentView: SegmentView) -> Any:
        """Start time of the segment (raises when the view carries none)."""
        if segmentView.time is None:
            raise Exception("getSegmentTime: segmentView.time is undefined")
        return segmentView.time

    def _level(self, index: Any) -> Any:
        levels = self.hls.levels
        if levels is None:
            raise TypeError("Cannot read property of undefined (hls.levels)")
        if not isinstance(index, int) or index < 0 or index >= len(levels):
            return None
        return levels[index]

    def getSegmentList(self, trackView: TrackView, beginTime: float, duration: float) -> List[SegmentView]:
        """SegmentViews of ``trackView`` whose start lies in ``[beginTime, beginTime + duration]``
        (playlist order; ``[]`` while the level is unparsed, raises for a missing level)."""
        level = self._level(trackView.level)
        if not level:
            raise Exception("getSegmentList: level doesn't exist")
        details = getattr(level, "details", None)
        if not details:
            log.warning("getSegmentList: level not parsed yet")
            return []
        fragments = details.fragments
        end = beginTime + duration
        idx = self._idx.get(trackView.level)
        if idx is None or not idx.valid_for(fragments):
            idx = _StartIndex(fragments)
            self._idx[trackView.level] = idx
        if idx.sorted:
            lo = bisect.bisect_left(idx.starts, beginTime)
            hi = bisect.bisect_right(idx.starts, end)
            rng = range(lo, hi)
        else:
            rng = [i for i, s in enumerate(idx.starts) if beginTime <= s <= end]
        out = []
        for i in rng:
            f = fragments[i]
            out.append(SegmentView(sn=f.sn, trackView=trackView, time=f.start))
        return out

    # ------------------------------------------------------------------ batched (K1)
    def getSegmentLists(self, queries: List[Any]) -> List[List[SegmentView]]:
        """Batched ``getSegmentList`` over ``[(trackView, beginTime, duration), ...]``: the
        same semantics per query (closed interval, playlist order; unparsed level -> ``[]``,
        missing level -> raises), one cached start index per level for the whole batch."""
        return [self.getSegmentList(tv, begin, dur) for tv, begin, dur in queries]

    def fragment(self, segmentView: SegmentView) -> Any:
        """The playlist fragment behind a SegmentView (url / byte range for the agent's
        own prefetch requests), or None."""
        level = self._level(segmentView.trackView.level)
        details = getattr(level, "details", None) if level else None
        if not details or not details.fragments:
            return None
        frags = details.fragments
        i = int(segmentView.sn) - int(frags[0].sn)
        if 0 <= i < len(frags) and frags[i].sn == segmentView.sn:
            return frags[i]
        for f in frags:
            if f.sn == segmentView.sn:
                return f
        return None

    def getTrackList(self) -> List[TrackView]:
        """Every ``(level, urlId)`` track, redundant URLs included."""
        levels = self.hls.levels
        if not levels:
            return []
        tracks = []
        for i, level in enumerate(levels):
            for j in range(len(level.url)):
                tracks.append(TrackView(level=i, urlId=j))
        return tracks

    def getSegmentDuration(self, segmentView: SegmentView) -> Any:
        """Duration of the track's segments (the first fragment's)."""
        level = self._level(segmentView.trackView.level)
        for fragment in level.details.fragments:
            return fragment.duration
        raise Exception("All segments should have a duration")

    # python aliases
    get_segment_time = getSegmentTime
    get_segment_list = getSegmentList
    get_track_list = getTrackList
    get_segment_duration = getSegmentDuration
