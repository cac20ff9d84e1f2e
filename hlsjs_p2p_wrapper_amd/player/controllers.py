"""Player controllers: playlist / level / key / fragment loading and the stream loop.

These recreate the slice of hls.js the reference wrapper depends on:
``MANIFEST_LOADING`` → ``MANIFEST_LOADED`` → ``MANIFEST_PARSED``, level switching
(``LEVEL_SWITCH``, ``LEVEL_LOADING``/``LOADED`` with live reloads), key loading through
the *default* loader (never the P2P ``fLoader``, ``private.js:82-85``), fragment loading
through ``config.fLoader`` with the exact 10-argument call
(``p2p-loader-generator.js:52``), ``FRAG_LOAD_PROGRESS``/``FRAG_LOADED``, batched
decrypt+demux (:mod:`.transmux`), buffer append and ``FRAG_BUFFERED``.

Extension over hls.js: ``config.maxFragLoadsInFlight`` fragments may load concurrently
(1 = hls.js behaviour), so a serving deployment moves many segments per swarm round.
"""
from __future__ import annotations

import bisect
import logging
from typing import Any, Dict, List, Optional, Tuple

from .events import ErrorDetails, ErrorTypes, Events
from .level import _START_GENERATION, Fragment, Level, LevelDetails
from .playlist import PlaylistError, is_master, parse_master, parse_media
from ..parallel.fleet import RemoteSegment
from .transmux import TransmuxJob, pipeline_for

log = logging.getLogger("hlsjs_p2p_wrapper_amd.player")


def _loader_class(cfg, key: str):
    cls = cfg.get(key)
    return cls if cls is not None else cfg.get("loader")


# ---------------------------------------------------------------------------- playlists
class PlaylistLoader:
    def __init__(self, hls) -> None:
        self.hls = hls
        self.loaders: Dict[str, Any] = {}
        hls.on(Events.MANIFEST_LOADING, self.onManifestLoading)
        hls.on(Events.LEVEL_LOADING, self.onLevelLoading)

    def destroy(self) -> None:
        for l in self.loaders.values():
            l.destroy()
        self.loaders.clear()

    def _load(self, kind: str, url: str, ctx: dict) -> None:
        cfg = self.hls.config
        old = self.loaders.pop(kind, None)
        if old is not None:
            old.abort()
        loader = _loader_class(cfg, "pLoader")(cfg)
        self.loaders[kind] = loader
        if kind == "manifest":
            timeout = cfg.manifestLoadingTimeOut
            retry, delay = cfg.manifestLoadingMaxRetry, cfg.manifestLoadingRetryDelay
        else:
            timeout, retry, delay = cfg.levelLoadingTimeOut, cfg.levelLoadingMaxRetry, cfg.levelLoadingRetryDelay
        loader.load(url, "text", lambda e, s: self._success(kind, url, ctx, e, s),
                    lambda e: self._error(kind, url, ctx, e), lambda e, s: self._timeout(kind, url, ctx, e, s),
                    timeout, retry, delay)

    def onManifestLoading(self, event: str, data: Any) -> None:
        self._load("manifest", data["url"], {})

    def onLevelLoading(self, event: str, data: Any) -> None:
        self._load("level", data["url"], {"level": data["level"], "id": data.get("id", 0)})

    def _success(self, kind: str, url: str, ctx: dict, event: Any, stats: Any) -> None:
        self.loaders.pop(kind, None)
        text = event.currentTarget.response
        if isinstance(text, (bytes, bytearray)):
            text = text.decode()
        hls = self.hls
        stats.tparsed = hls.loop.now()
        try:
            if kind == "manifest":
                if is_master(text):
                    levels = parse_master(text, url)
                    hls.trigger(Events.MANIFEST_LOADED, {"levels": levels, "url": url, "stats": stats})
                else:  # a media playlist given directly: one level
                    details = parse_media(text, url, 0)
                    lvl = Level(url=[url], bitrate=0)
                    hls.trigger(Events.MANIFEST_LOADED, {"levels": [lvl], "url": url, "stats": stats})
                    hls.trigger(Events.LEVEL_LOADED, {"details": details, "level": 0, "id": 0, "stats": stats})
            else:
                details = parse_media(text, url, ctx["level"])
                details.tload = stats.tload or hls.loop.now()
                hls.trigger(Events.LEVEL_LOADED, {"details": details, "level": ctx["level"], "id": ctx["id"],
                                                  "stats": stats})
        except PlaylistError as e:
            det = ErrorDetails.MANIFEST_PARSING_ERROR if kind == "manifest" else ErrorDetails.LEVEL_LOAD_ERROR
            hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR, "details": det, "fatal": True,
                                       "url": url, "reason": str(e)})

    def _error(self, kind: str, url: str, ctx: dict, event: Any) -> None:
        self.loaders.pop(kind, None)
        if kind == "manifest":
            self.hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR,
                                            "details": ErrorDetails.MANIFEST_LOAD_ERROR, "fatal": True, "url": url,
                                            "response": event})
        else:
            self.hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR,
                                            "details": ErrorDetails.LEVEL_LOAD_ERROR, "fatal": False, "url": url,
                                            "level": ctx["level"], "response": event})

    def _timeout(self, kind: str, url: str, ctx: dict, event: Any, stats: Any) -> None:
        loader = self.loaders.pop(kind, None)
        if loader is not None:
            loader.abort()
        det = ErrorDetails.MANIFEST_LOAD_TIMEOUT if kind == "manifest" else ErrorDetails.LEVEL_LOAD_TIMEOUT
        self.hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR, "details": det,
                                        "fatal": kind == "manifest", "url": url, "level": ctx.get("level")})


# ---------------------------------------------------------------------------- levels
def _sn_delta(ref: List[Fragment], frags: List[Fragment], targetduration: Optional[float]) -> float:
    """Shift that puts ``frags`` on the timeline of ``ref`` (playlists of one live stream):
    through the first sn both hold, else by the sn distance from ``ref``'s last fragment."""
    by_sn = {f.sn: f for f in ref}
    for f in frags:
        o = by_sn.get(f.sn)
        if o is not None:
            return o.start - f.start
    gap = frags[0].sn - ref[-1].sn - 1
    return ref[-1].end + gap * (targetduration or 0) - frags[0].start


class LevelController:
    def __init__(self, hls) -> None:
        self.hls = hls
        self._levels: Optional[List[Level]] = None
        self._level = -1
        self._manualLevel = -1
        self.firstLevel = 0
        self._reload_timer = None
        hls.on(Events.MANIFEST_LOADED, self.onManifestLoaded)
        hls.on(Events.LEVEL_LOADED, self.onLevelLoaded)
        hls.on(Events.ERROR, self.onError)

    def destroy(self) -> None:
        if self._reload_timer is not None:
            self._reload_timer.cancel()
            self._reload_timer = None

    @property
    def levels(self) -> Optional[List[Level]]:
        return self._levels

    def onManifestLoaded(self, event: str, data: Any) -> None:
        self._levels = list(data["levels"])
        start = self.hls.config.get("startLevel")
        self.firstLevel = start if isinstance(start, int) and 0 <= start < len(self._levels) else 0
        self.hls.trigger(Events.MANIFEST_PARSED, {"levels": self._levels, "firstLevel": self.firstLevel,
                                                  "stats": data.get("stats")})

    @property
    def level(self) -> int:
        return self._level

    @level.setter
    def level(self, new: int) -> None:
        levels = self._levels
        if not levels or not (0 <= new < len(levels)):
            self.hls.trigger(Events.ERROR, {"type": ErrorTypes.OTHER_ERROR,
                                            "details": ErrorDetails.LEVEL_SWITCH_ERROR, "level": new,
                                            "fatal": False, "reason": "invalid level idx"})
            return
        if self._level != new or levels[new].details is None:
            self._set_level(new)

    def _set_level(self, new: int) -> None:
        if self._reload_timer is not None:
            self._reload_timer.cancel()
            self._reload_timer = None
        switched = self._level != new
        self._level = new
        lvl = self._levels[new]  # type: ignore[index]
        if switched:
            self.hls.trigger(Events.LEVEL_SWITCH, {"level": new})
        if lvl.details is None or lvl.details.live:
            self._request(new)

    def _request(self, idx: int) -> None:
        lvl = self._levels[idx]  # type: ignore[index]
        url_id = lvl.urlId if 0 <= lvl.urlId < len(lvl.url) else 0
        self.hls.trigger(Events.LEVEL_LOADING, {"url": lvl.url[url_id], "level": idx, "id": url_id})

    @property
    def manualLevel(self) -> int:
        return self._manualLevel

    @manualLevel.setter
    def manualLevel(self, v: int) -> None:
        self._manualLevel = v
        if v != -1:
            self.level = v

    def onLevelLoaded(self, event: str, data: Any) -> None:
        idx = data["level"]
        levels = self._levels
        if not levels or idx >= len(levels):
            return
        lvl = levels[idx]
        details: LevelDetails = data["details"]
        old = lvl.details
        if (old is None or not old.fragments) and details.live and details.fragments:
            # a live level's first playlist starts its own timeline at 0: put it on the timeline
            # playback is on, through the sn the levels share (hls.js alignStream / adjustSliding),
            # or a switch lands the playhead segments away from the fragments it needs
            ref = self._timeline_ref(idx)
            if ref is not None:
                delta = _sn_delta(ref.fragments, details.fragments, details.targetduration)
                if delta:
                    for f in details.fragments:
                        f.start += delta
                    details.totalduration = details.fragments[-1].end
        if old is not None and old.fragments and details.fragments:
            # live reload: a refreshed playlist restarts its timeline at 0; align it on the
            # previous one through a common sn (hls.js mergeDetails) and keep Fragment
            # identity for sn present in both (in-flight loads refer to them)
            by_sn = {f.sn: f for f in old.fragments}
            delta = _sn_delta(old.fragments, details.fragments, details.targetduration)
            merged = []
            for f in details.fragments:
                o = by_sn.get(f.sn)
                if o is not None:
                    o.duration, o.url = f.duration, f.url
                    merged.append(o)
                else:
                    f.start += delta
                    merged.append(f)
            details.fragments = merged
            details.totalduration = merged[-1].end
        lvl.details = details
        self.hls.trigger(Events.LEVEL_UPDATED, {"details": details, "level": idx})
        if details.live and idx == self._level:
            interval = 1000.0 * (details.averagetargetduration or details.targetduration or 1.0)
            self._reload_timer = self.hls.loop.set_timeout(self._reload, interval, idx)

    def _timeline_ref(self, idx: int) -> Optional["LevelDetails"]:
        """Details of another level already on the playback timeline (the current one first)."""
        order = [self._level] + [i for i in range(len(self._levels or ())) if i != self._level]
        for i in order:
            if i != idx and 0 <= i < len(self._levels or ()):
                d = self._levels[i].details  # type: ignore[index]
                if d is not None and d.fragments:
                    return d
        return None

    def _reload(self, idx: int) -> None:
        self._reload_timer = None
        if idx == self._level and self._levels:
            self._request(idx)

    def onError(self, event: str, data: Any) -> None:
        det = data.get("details")
        if det in (ErrorDetails.LEVEL_LOAD_ERROR, ErrorDetails.LEVEL_LOAD_TIMEOUT, ErrorDetails.FRAG_LOAD_ERROR,
                   ErrorDetails.FRAG_LOAD_TIMEOUT):
            idx = data.get("level")
            if idx is None and data.get("frag") is not None:
                idx = data["frag"].level
            if idx is None or not self._levels or idx >= len(self._levels):
                return
            lvl = self._levels[idx]
            if len(lvl.url) > 1:  # redundant stream failover: next urlId is a different track
                lvl.urlId = (lvl.urlId + 1) % len(lvl.url)
                data["fatal"] = False
                if det in (ErrorDetails.LEVEL_LOAD_ERROR, ErrorDetails.LEVEL_LOAD_TIMEOUT):
                    self._request(idx)


# ---------------------------------------------------------------------------- keys
class KeyLoader:
    def __init__(self, hls) -> None:
        self.hls = hls
        self.keys: Dict[str, bytes] = {}
        self._pending: Dict[str, List[Fragment]] = {}
        self.loaders: Dict[str, Any] = {}
        hls.on(Events.KEY_LOADING, self.onKeyLoading)

    def destroy(self) -> None:
        for l in self.loaders.values():
            l.destroy()
        self.loaders.clear()

    def onKeyLoading(self, event: str, data: Any) -> None:
        frag: Fragment = data["frag"]
        dd = frag.decryptdata
        uri = dd.uri
        if uri in self.keys:
            dd.key = self.keys[uri]
            self.hls.trigger(Events.KEY_LOADED, {"frag": frag})
            return
        waiting = self._pending.setdefault(uri, [])
        waiting.append(frag)
        if len(waiting) > 1:
            return
        cfg = self.hls.config
        loader = cfg.loader(cfg)  # the default loader: keys never go through the P2P fLoader
        self.loaders[uri] = loader
        loader.load(uri, "arraybuffer", lambda e, s: self._ok(uri, e), lambda e: self._fail(uri, e, False),
                    lambda e, s: self._fail(uri, e, True), cfg.fragLoadingTimeOut, cfg.fragLoadingMaxRetry,
                    cfg.fragLoadingRetryDelay)

    def _ok(self, uri: str, event: Any) -> None:
        self.loaders.pop(uri, None)
        key = event.currentTarget.response
        if not isinstance(key, (bytes, bytearray)):
            key = bytes(memoryview(key.numpy() if hasattr(key, "numpy") else key))
        key = bytes(key)
        self.keys[uri] = key
        for frag in self._pending.pop(uri, []):
            frag.decryptdata.key = key
            self.hls.trigger(Events.KEY_LOADED, {"frag": frag})

    def _fail(self, uri: str, event: Any, timeout: bool) -> None:
        loader = self.loaders.pop(uri, None)
        if loader is not None:
            loader.abort()
        for frag in self._pending.pop(uri, []):
            self.hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR,
                                            "details": ErrorDetails.KEY_LOAD_TIMEOUT if timeout else
                                            ErrorDetails.KEY_LOAD_ERROR, "fatal": False, "frag": frag,
                                            "response": event})


# ---------------------------------------------------------------------------- fragments
class FragmentLoader:
    """Creates one ``config.fLoader`` (or ``config.loader``) per fragment and calls it with
    the hls.js 10-argument signature."""

    def __init__(self, hls) -> None:
        self.hls = hls
        self.loaders: Dict[int, Any] = {}
        hls.on(Events.FRAG_LOADING, self.onFragLoading)

    def destroy(self) -> None:
        for l in list(self.loaders.values()):
            l.destroy()
        self.loaders.clear()

    def abort(self, frag: Fragment) -> None:
        loader = self.loaders.pop(id(frag), None)
        if loader is not None:
            loader.abort()
        frag.loader = None

    def onFragLoading(self, event: str, data: Any) -> None:
        frag: Fragment = data["frag"]
        frag.loaded = 0
        cfg = self.hls.config
        cls = _loader_class(cfg, "fLoader")
        loader = cls(cfg)
        frag.loader = loader
        self.loaders[id(frag)] = loader
        loader.load(frag.url, "arraybuffer", lambda e, s: self._success(frag, e, s), lambda e: self._error(frag, e),
                    lambda e, s: self._timeout(frag, e, s), cfg.fragLoadingTimeOut, cfg.fragLoadingMaxRetry,
                    cfg.fragLoadingRetryDelay, lambda e, s: self._progress(frag, e, s), frag)

    def _success(self, frag: Fragment, event: Any, stats: Any) -> None:
        if isinstance(event, dict):  # JsObject / plain dict event
            ct = event["currentTarget"]
            payload = ct["response"] if isinstance(ct, dict) else ct.response
        else:
            payload = event.currentTarget.response
        length = _byte_length(payload)
        if isinstance(stats, dict):
            stats["length"] = length
        else:
            stats.length = length
        self.loaders.pop(id(frag), None)
        frag.loader = None
        self.hls.trigger(Events.FRAG_LOADED, {"payload": payload, "frag": frag, "stats": stats})

    def _error(self, frag: Fragment, event: Any) -> None:
        loader = self.loaders.pop(id(frag), None)
        if loader is not None:
            loader.abort()
        self.hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR, "details": ErrorDetails.FRAG_LOAD_ERROR,
                                        "fatal": False, "frag": frag, "response": event})

    def _timeout(self, frag: Fragment, event: Any, stats: Any) -> None:
        loader = self.loaders.pop(id(frag), None)
        if loader is not None:
            loader.abort()
        self.hls.trigger(Events.ERROR, {"type": ErrorTypes.NETWORK_ERROR, "details": ErrorDetails.FRAG_LOAD_TIMEOUT,
                                        "fatal": False, "frag": frag})

    def _progress(self, frag: Fragment, event: Any, stats: Any) -> None:
        frag.loaded = stats["loaded"] if isinstance(stats, dict) else stats.loaded
        if self.hls.listening(Events.FRAG_LOAD_PROGRESS):
            self.hls.trigger(Events.FRAG_LOAD_PROGRESS, {"frag": frag, "stats": stats})


def _byte_length(payload: Any) -> int:
    if payload is None:
        return 0
    if hasattr(payload, "numel"):
        return int(payload.numel())
    if hasattr(payload, "nbytes"):
        return int(payload.nbytes)
    return len(payload)


# ---------------------------------------------------------------------------- stream
class _Inflight(dict):
    """The fragments in flight, keyed by ``(level, sn)``, in load order -- and whether they
    form one chain in that order (each starts within 0.5 s of the previous one's end and ends
    after it), kept up to date as fragments are added and removed.  ``tick`` needs the end of
    the in-flight run that continues the buffer; for a chain that is the last fragment's end
    (O(1)), where the scan over every fragment in flight (256 per player at the bench's depth)
    cost ~5 µs of each fragment's player CPU."""

    __slots__ = ("chain_ok", "tail")

    def __init__(self) -> None:
        super().__init__()
        self.chain_ok = True
        self.tail: Optional[Fragment] = None

    def __setitem__(self, key, frag) -> None:
        t = self.tail
        if not self:
            ok = True
        elif key in self or t is None or not self.chain_ok:
            ok = False  # a re-inserted key keeps its old position in the order
        else:
            te = t._start + t.duration
            ok = frag._start <= te + 0.5 and frag._start + frag.duration > te
        dict.__setitem__(self, key, frag)
        self.tail = frag
        self.chain_ok = ok

    def pop(self, key, *default):
        if self.chain_ok and key in self and key != next(iter(self)):
            self.chain_ok = False  # removing a fragment other than the oldest may open a gap
        return dict.pop(self, key, *default)

    def __delitem__(self, key) -> None:
        self.pop(key)

    def clear(self) -> None:
        dict.clear(self)
        self.chain_ok = True
        self.tail = None


class StreamController:
    STOPPED, IDLE, ERROR, ENDED = "STOPPED", "IDLE", "ERROR", "ENDED"

    def __init__(self, hls) -> None:
        self.hls = hls
        self.loop = hls.loop
        self.state = self.STOPPED
        self.inflight: Dict[Tuple[int, int], Fragment] = _Inflight()
        self._chain_gen = -1  # fragment_generation() when the chain flag was last checked by a scan
        self.run_scans = 0  # _run_end calls that scanned every fragment in flight
        self.fragPrevious: Optional[Fragment] = None
        self.fragLastKbps = 0
        self.stats = None
        self.startPosition = -1.0
        self._start_pending = False
        self._timer = None
        self._tick_pending = False
        self._retry: Dict[Tuple[int, int], int] = {}
        self._retry_until = 0.0
        self._eos = False
        self._init_levels: set = set()
        self._starts_cache: Tuple[int, int, List[float]] = (0, 0, [])
        self.fragments_buffered = 0
        self.bytes_buffered = 0
        on = hls.on
        on(Events.MEDIA_ATTACHED, self.onMediaAttached)
        on(Events.MEDIA_DETACHING, self.onMediaDetaching)
        on(Events.MANIFEST_PARSED, self.onManifestParsed)
        on(Events.LEVEL_LOADED, lambda e, d: self._kick())
        on(Events.KEY_LOADED, self.onKeyLoaded)
        on(Events.FRAG_LOADED, self.onFragLoaded)
        on(Events.ERROR, self.onError)

    # ------------------------------------------------------------ lifecycle
    def destroy(self) -> None:
        self.stopLoad()

    def startLoad(self, startPosition: float = -1) -> None:
        self.startPosition = float(startPosition if startPosition is not None else -1)
        self._start_pending = True
        self.state = self.IDLE
        self._eos = False
        if self._timer is None:
            self._timer = self.loop.set_interval(self.tick, self.hls.config.get("tickInterval", 100))
        self._kick()

    def stopLoad(self) -> None:
        for frag in list(self.inflight.values()):
            self.hls.fragmentLoader.abort(frag)
        self.inflight.clear()
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        self.state = self.STOPPED

    def _kick(self) -> None:
        # hls.js's tick() is re-entrant and cheap per call; here one pending tick per loop
        # iteration serves every state change of that iteration (a swarm round completes
        # dozens of fragments at once)
        if self.state not in (self.STOPPED, self.ERROR) and not self._tick_pending:
            self._tick_pending = True
            self.loop.call_soon(self._kicked_tick)

    def _kicked_tick(self) -> None:
        self._tick_pending = False
        self.tick()

    def onMediaAttached(self, event: str, data: Any) -> None:
        media = data["media"]
        media.on("seeking", self._on_seeking)
        media.on("ended", self._on_ended)
        self._kick()

    def onMediaDetaching(self, event: str, data: Any) -> None:
        media = self.hls.media
        if media is not None:
            media.remove_listener("seeking", self._on_seeking)
            media.remove_listener("ended", self._on_ended)

    def onManifestParsed(self, event: str, data: Any) -> None:
        self.hls.levelController.level = data["firstLevel"]
        if self.hls.config.autoStartLoad:
            self.startLoad(self.hls.config.startPosition)

    def _on_seeking(self) -> None:
        media = self.hls.media
        pos = media.currentTime
        for key, frag in list(self.inflight.items()):
            if not (frag.start - 0.5 <= pos < frag.end + 0.5) and frag.end <= pos or frag.start > pos + 60:
                self.hls.fragmentLoader.abort(frag)
                self.inflight.pop(key, None)
        self._eos = False
        if self.state == self.ENDED:
            self.state = self.IDLE
        self._kick()

    def _on_ended(self) -> None:
        self.state = self.ENDED

    # ------------------------------------------------------------ buffering loop
    def _frag_at(self, details: LevelDetails, t: float) -> Optional[Fragment]:
        frags = details.fragments
        if not frags:
            return None
        key = (id(frags), len(frags))
        if self._starts_cache[:2] != key:
            self._starts_cache = (key[0], key[1], [f.start for f in frags])
        starts = self._starts_cache[2]
        tol = self.hls.config.get("maxFragLookUpTolerance", 0.2)
        i = bisect.bisect_right(starts, t + tol) - 1
        if i < 0:
            return frags[0] if details.live else frags[0]
        f = frags[i]
        if t >= f.end - 1e-6:
            return frags[i + 1] if i + 1 < len(frags) else None
        return f

    def _live_start(self, details: LevelDetails) -> float:
        cfg = self.hls.config
        if cfg.get("liveSyncDuration") is not None:
            back = float(cfg.liveSyncDuration)
        else:
            back = float(cfg.get("liveSyncDurationCount", 3)) * (details.targetduration or 1.0)
        start = details.fragments[0].start if details.fragments else 0.0
        return max(start, details.totalduration - back)

    def _ensure_in_live_window(self, media: Any, cfg: Any, details: LevelDetails) -> None:
        """A live playhead whose buffer ends before the sliding window's first fragment (a
        seek back past the DVR window, a long pause) can never be fed: reset it to the live
        sync position (hls.js stream-controller ``_ensureFragmentAtLivePoint``)."""
        first = details.fragments[0].start - float(cfg.get("maxFragLookUpTolerance", 0.2))
        pos = media.currentTime
        if pos >= first:
            return
        hole = cfg.maxBufferHole
        for s, e in media.buffered:
            if s - hole <= pos < e:
                pos = e
                break
        if pos < first:
            media.currentTime = self._live_start(details)

    def tick(self) -> None:
        hls = self.hls
        if self.state in (self.STOPPED, self.ERROR):
            return
        media = hls.media
        levels = hls.levels
        if media is None or not levels:
            return
        if self.loop.now() < self._retry_until:
            return
        lvl_idx = hls.nextLoadLevel
        lc = hls.levelController
        if lvl_idx != lc.level:
            lc.level = lvl_idx
        level = levels[lvl_idx]
        details = level.details
        if details is None:
            return
        if self._start_pending:
            self._start_pending = False
            if self.startPosition >= 0:
                pos0 = self.startPosition
            elif details.live:
                pos0 = self._live_start(details)
            else:
                pos0 = 0.0
            if abs(media.currentTime - pos0) > 1e-9:
                media.currentTime = pos0
        cfg = hls.config
        if details.live and details.fragments:
            self._ensure_in_live_window(media, cfg, details)
        ranges = list(media.buffered)  # one walk of the buffered ranges per tick
        if ranges and (media.seeking or not media.paused):
            self._seek_over_hole(media, cfg, ranges)
        pos = media.currentTime
        hole = cfg.maxBufferHole
        buf_end = pos
        later = None  # buffered ranges past the one the playhead is in
        for i, (s, e) in enumerate(ranges):
            if s - hole <= pos < e:
                buf_end = e
                later = ranges[i + 1:]
                break
            if s > pos:
                later = ranges[i:]
                break
        bitrate = level.bitrate or 1
        max_buf = max(8.0 * (cfg.maxBufferSize or 0) / bitrate, float(cfg.maxBufferLength))
        max_buf = min(max_buf, float(cfg.maxMaxBufferLength))
        max_inflight = max(1, int(cfg.get("maxFragLoadsInFlight", 1) or 1))
        nxt = self._run_end(buf_end)
        while len(self.inflight) < max_inflight and nxt - pos < max_buf:
            frag = self._frag_at(details, nxt)
            if frag is None:
                if not details.live and nxt >= details.totalduration - 0.05 and not self.inflight and not self._eos:
                    self._eos = True
                    media.duration = details.totalduration
                    hls.trigger(Events.BUFFER_EOS, {})
                break
            key = (frag.level, frag.sn)
            if key in self.inflight:
                nxt = frag.end
                continue
            if later:
                # a fragment already in a later buffered range (after a seek to just before
                # it, with fragments in flight) is skipped, not loaded again: reloading it from
                # the cache would complete at once and re-kick this loop forever.  Covered: one
                # range from the fragment's start (a range evicted up to just past it leaves a
                # hole to fill) to within a hole of its end (ranges end at the media end)
                fs = frag._start
                fe = fs + frag.duration
                if any(s <= fs + 1e-3 and e >= fe - hole for s, e in later):
                    nxt = fe
                    continue
            self._load(frag)
            nxt = frag.end

    def _seek_over_hole(self, media: Any, cfg: Any, ranges: List[Tuple[float, float]]) -> None:
        """hls.js ``_checkBuffer``: no media at the playhead but a buffered range starts less
        than ``maxSeekHole`` ahead (a seek that landed just before a range, a range evicted up
        to just past a fragment's start, a gap between appends) -> jump to that range's start +
        ``seekHoleNudgeDuration`` and report ``BUFFER_SEEK_OVER_HOLE`` (non-fatal).  The stream
        loop counts the playhead as inside a range that starts within ``maxBufferHole``, so it
        never loads that hole; without the jump the playhead waits there forever."""
        pos = media.currentTime
        nxt = None
        for s, e in ranges:
            if s <= pos < e:
                return  # media at the playhead
            if s > pos:
                nxt = s
                break
        if nxt is None or nxt - pos >= float(cfg.get("maxSeekHole", 2) or 0):
            return
        target = nxt + float(cfg.get("seekHoleNudgeDuration", 0.01) or 0)
        media.currentTime = target
        self.hls.trigger(Events.ERROR, {"type": ErrorTypes.MEDIA_ERROR, "details": ErrorDetails.BUFFER_SEEK_OVER_HOLE,
                                        "fatal": False, "hole": target - pos})

    def _run_end(self, nxt: float) -> float:
        """The end of the in-flight run that continues the buffer (which ends at ``nxt``): one
        pass in load order, each fragment starting within 0.5 s of the covered end extends
        it.  For a chain (:class:`_Inflight`) whose oldest fragment extends the buffer that is
        the newest fragment's end."""
        inflight = self.inflight
        if not inflight:
            return nxt
        gen = _START_GENERATION[0]
        first = next(iter(inflight.values()))
        fs = first._start
        fe = fs + first.duration
        if inflight.chain_ok and self._chain_gen == gen and fe > nxt and fs <= nxt + 0.5:
            t = inflight.tail
            return t._start + t.duration
        self.run_scans += 1
        ok, prev = True, None
        for f in inflight.values():
            fs = f._start
            fe = fs + f.duration
            if prev is not None and not (fs <= prev + 0.5 and fe > prev):
                ok = False
            prev = fe
            if fe > nxt and fs <= nxt + 0.5:
                nxt = fe
        inflight.chain_ok = ok
        inflight.tail = f
        self._chain_gen = gen
        return nxt

    def _load(self, frag: Fragment) -> None:
        frag.loadCounter += 1
        frag.autoLevel = self.hls.autoLevelEnabled
        self.inflight[(frag.level, frag.sn)] = frag
        dd = frag.decryptdata
        if dd is not None and dd.needs_key:
            key = self._cached_key(dd)
            if key is None:
                self.hls.trigger(Events.KEY_LOADING, {"frag": frag})
                return
            dd.key = key  # what KeyLoader.onKeyLoading -> KEY_LOADED -> onKeyLoaded would do
        self.hls.trigger(Events.FRAG_LOADING, {"frag": frag})

    def _cached_key(self, dd) -> Optional[bytes]:
        """The already-loaded key of ``dd`` when the KEY_LOADING / KEY_LOADED round trip would
        only reach the engine's own handlers (the key loader and this controller): then the
        result is the same without the two events (once per fragment of an encrypted
        stream).  With any other listener, the events are sent as usual."""
        obs = self.hls._observer._listeners
        kl = obs.get(Events.KEY_LOADING)
        kd = obs.get(Events.KEY_LOADED)
        if kl is None or kd is None or len(kl) != 1 or len(kd) != 1:
            return None
        key_loader = self.hls.keyLoader
        if kl[0] != key_loader.onKeyLoading or kd[0] != self.onKeyLoaded:
            return None
        return key_loader.keys.get(dd.uri)

    def onKeyLoaded(self, event: str, data: Any) -> None:
        frag = data["frag"]
        if self.inflight.get((frag.level, frag.sn)) is frag:
            self.hls.trigger(Events.FRAG_LOADING, {"frag": frag})

    def onFragLoaded(self, event: str, data: Any) -> None:
        frag: Fragment = data["frag"]
        if self.inflight.get((frag.level, frag.sn)) is not frag:
            return  # aborted / stale
        self.stats = data["stats"]
        dd = frag.decryptdata
        key = dd.key if (dd is not None and dd.method == "AES-128") else None
        iv = frag.iv_for_decrypt() if key is not None else None
        stats = data["stats"]
        payload = data["payload"]
        if type(payload) is RemoteSegment:  # fleet player: the node process already transmuxed it
            self.loop.call_soon(self._on_parsed, frag, stats, payload.transmux_result)
            return
        dev = self.hls.transmux_device(payload)
        # a segment a peer sent, delivered before its CRC check (gpuSwarm.deferVerify): the
        # transmux batch verifies it on the way through the decrypt
        ticket = getattr(payload, "swarm_verify", None)
        pipeline_for(dev, self.loop).submit(
            TransmuxJob(payload, key, iv, lambda r: self._on_parsed(frag, stats, r), frag, ticket))

    def _on_parsed(self, frag: Fragment, stats: Any, r: Any) -> None:  # r: dict-like transmux result
        hls = self.hls
        key = (frag.level, frag.sn)
        if self.inflight.get(key) is not frag:
            return
        if r.get("verify_failed"):
            # the peer's copy was corrupted: nothing was buffered, the node detached the copy and
            # this fragment's next load goes to the CDN -- a transport retry, not a media error
            self.inflight.pop(key, None)
            log.warning("fragment sn=%s level=%s: peer copy failed its CRC check; reloading", frag.sn, frag.level)
            self._kick()
            return
        if r.get("error") is not None or r.get("status", 0) & 0b111111:
            self.inflight.pop(key, None)
            details = (ErrorDetails.FRAG_DECRYPT_ERROR if r.get("plain_bytes", 0) < 0
                       else ErrorDetails.FRAG_PARSING_ERROR)
            # retried like a load error: back-off, up to fragLoadingMaxRetry, then fatal.  An
            # immediate reload of bytes that fail the same way (a cached copy) would spin this
            # loop without time advancing; the wrapper drops the cached copy on this event
            cfg = hls.config
            n = self._retry.get(key, 0) + 1
            data = {"type": ErrorTypes.MEDIA_ERROR, "details": details, "fatal": n > cfg.fragLoadingMaxRetry,
                    "frag": frag, "reason": str(r.get("error") or r.get("status"))}
            hls.trigger(Events.ERROR, data)
            if data["fatal"]:
                log.error("fragment sn=%s level=%s failed: %s", frag.sn, frag.level, details)
                self.state = self.ERROR
                return
            self._retry[key] = n
            delay = min(2 ** (n - 1) * cfg.fragLoadingRetryDelay, 64000)
            self._retry_until = self.loop.now() + delay
            self.loop.set_timeout(self._kick, delay)
            return
        info = r["info"]
        if frag.level not in self._init_levels:
            self._init_levels.add(frag.level)
            hls.trigger(Events.FRAG_PARSING_INIT_SEGMENT, {"frag": frag, "tracks": {
                "video": {"pid": info["video_pid"], "type": info["video_type"]},
                "audio": {"pid": info["audio_pid"], "type": info["audio_type"]}}})
        # events nobody listens to are not built (no observable difference: hls.trigger with
        # no listener does nothing); this runs once per buffered fragment
        listening = hls.listening
        if listening(Events.FRAG_PARSING_METADATA) and r["id3"].numel():
            hls.trigger(Events.FRAG_PARSING_METADATA, {"frag": frag, "samples": r["id3"]})
        vfirst, vlast, nv = info["video_first_pts"], info["video_last_pts"], info["n_video_pes"]
        if vfirst >= 0 and vlast >= vfirst and nv > 1:
            frame = (vlast - vfirst) / (nv - 1)
            dur = (vlast - vfirst + frame) / 90000.0
        else:
            dur = frag.duration
        start = frag.start
        end = start + dur
        if listening(Events.FRAG_PARSING_DATA):
            hls.trigger(Events.FRAG_PARSING_DATA, {"frag": frag, "type": "video", "startPTS": start, "endPTS": end,
                                                   "data1": r["video"], "nb": nv, "pts": (vfirst, vlast)})
            hls.trigger(Events.FRAG_PARSING_DATA, {"frag": frag, "type": "audio", "startPTS": start, "endPTS": end,
                                                   "data1": r["audio"], "nb": info["n_audio_pes"],
                                                   "pts": (info["audio_first_pts"], info["audio_last_pts"])})
        if listening(Events.FRAG_PARSED):
            hls.trigger(Events.FRAG_PARSED, {"frag": frag})
        media = hls.media
        vb, ab = info.get("video_bytes"), info.get("audio_bytes")  # the ES views stay unbuilt
        nbytes = int(vb + ab) if vb is not None and ab is not None else int(r["video"].numel() + r["audio"].numel())
        if listening(Events.BUFFER_APPENDING):
            hls.trigger(Events.BUFFER_APPENDING, {"type": "video", "parent": "main", "bytes": nbytes})
        if media is not None:
            retain = (r["video"], r["audio"]) if hls.config.get("retainMediaData") else None
            if retain is not None:
                media.retain = True
            media.append(start, end, nbytes, retain)
        now = self.loop.now()
        if isinstance(stats, dict):  # JsObject stats (every built-in loader): plain item access
            stats["tbuffered"] = now
            tfirst = stats.get("tfirst")
            if tfirst is None:
                tfirst = stats.get("trequest")
            length = stats.get("length") or 0
        else:
            stats.tbuffered = now
            tfirst = stats.tfirst if stats.tfirst is not None else stats.trequest
            length = stats.length or 0
        dt = max(now - tfirst, 1e-3)
        self.fragLastKbps = round(8 * length / dt)
        self.inflight.pop(key, None)
        if self._retry:
            self._retry.pop(key, None)  # loaded, decrypted and demuxed: its retry count starts over
        self.fragPrevious = frag
        self.fragments_buffered += 1
        self.bytes_buffered += int(length)
        if listening(Events.BUFFER_APPENDED):
            hls.trigger(Events.BUFFER_APPENDED, {"parent": "main", "pending": 0})
        hls.trigger(Events.FRAG_BUFFERED, {"stats": stats, "frag": frag})
        self._kick()

    def onError(self, event: str, data: Any) -> None:
        det = data.get("details")
        frag = data.get("frag")
        if det in (ErrorDetails.FRAG_LOAD_ERROR, ErrorDetails.FRAG_LOAD_TIMEOUT, ErrorDetails.KEY_LOAD_ERROR,
                   ErrorDetails.KEY_LOAD_TIMEOUT) and frag is not None:
            key = (frag.level, frag.sn)
            self.inflight.pop(key, None)
            n = self._retry.get(key, 0) + 1
            cfg = self.hls.config
            if det == ErrorDetails.FRAG_LOAD_ERROR and not data.get("fatal") and len(
                    self.hls.levels[frag.level].url) <= 1:
                # the loader already retried maxRetry times with back-off: give up
                data["fatal"] = True
            elif n <= cfg.fragLoadingMaxRetry:
                self._retry[key] = n
                delay = min(2 ** (n - 1) * cfg.fragLoadingRetryDelay, 64000)
                self._retry_until = self.loop.now() + delay
                self.loop.set_timeout(self._kick, delay)
                return
            else:
                data["fatal"] = True
            if data.get("fatal"):
                # escalate in place (listeners registered after the controllers — i.e. the
                # application — observe fatal=True on this same ERROR event)
                log.error("fragment sn=%s level=%s failed: %s", frag.sn, frag.level, det)
                self.state = self.ERROR
            else:
                self._kick()
        elif data.get("fatal") and det in (ErrorDetails.MANIFEST_LOAD_ERROR, ErrorDetails.MANIFEST_LOAD_TIMEOUT,
                                           ErrorDetails.MANIFEST_PARSING_ERROR):
            self.state = self.ERROR
