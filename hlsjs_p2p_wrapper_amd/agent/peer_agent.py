"""PeerAgent — the ``streamroot-p2p`` module contract, backed by a :class:`SwarmNode`.

Contract as seen from the reference:

* ``PeerAgent(playerInterface, contentUrl, mediaMap, p2pConfig, SegmentView,
  PeerAgent.StreamTypes.HLS, 'v2')`` (``lib/hlsjs-p2p-wrapper-private.js:201-224``);
* ``getSegment(reqInfo{url, headers, withCredentials}, callbacks{onSuccess, onError,
  onProgress}, segmentView)`` → handle with ``abort()`` (``p2p-loader-generator.js:164``);
* ``dispose()``, ``setMediaElement(el)`` (``private.js:111,176``);
* ``stats`` = ``{cdn, p2p, upload, peers}`` (``README.md:232-237``),
  ``p2pDownloadOn`` / ``p2pUploadOn`` read/write (``hlsjs-p2p-wrapper.js:20-36``).

The swarm is keyed by ``p2pConfig.contentId`` (default: ``contentUrl``,
``MIGRATION.md:43``).  ``p2pConfig.gpuSwarm`` selects the node backend / device / cache
size (namespaced so it never collides with the reference's keys).
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional

import numpy as np

from ..utils.events import JsObject
from .node import SwarmNode, node_for_config, swarm_id_for

log = logging.getLogger("hlsjs_p2p_wrapper_amd.agent")


class PeerAgent:
    """Per-session P2P agent: serves the loader's fragment requests from the swarm node
    (HBM cache, peers, CDN), follows the playhead for prefetch and live-window eviction, and
    keeps the session's ``stats``."""
    StreamTypes = JsObject(HLS="hls", DASH="dash", SMOOTH="smooth")

    def __init__(self, playerInterface: Any, contentUrl: str, mediaMap: Any, p2pConfig: Dict[str, Any],
                 SegmentViewClass: Any = None, streamType: str = "hls", integrationVersion: str = "v2",
                 node: Optional[SwarmNode] = None) -> None:
        self.player = playerInterface
        self.contentUrl = contentUrl
        self.mediaMap = mediaMap
        self.p2pConfig = p2pConfig if p2pConfig is not None else {}
        self.SegmentView = SegmentViewClass
        self.streamType = streamType
        self.integrationVersion = integrationVersion
        if isinstance(self.p2pConfig, dict) and self.p2pConfig.get("debug"):
            from ..utils.log import configure

            configure(debug=True)
        content_id = self.p2pConfig.get("contentId") if isinstance(self.p2pConfig, dict) else None
        self.contentId = content_id or contentUrl
        self.swarm_id = swarm_id_for(str(self.contentId))
        self.node = node or node_for_config(self.p2pConfig)
        self.node.attach(self)
        self.media = None
        self.currentTrack = None
        self._stats = {"cdn": 0, "p2p": 0, "upload_base": self.node.stats["upload"], "cache": 0}
        gs = (self.p2pConfig.get("gpuSwarm") or {}) if isinstance(self.p2pConfig, dict) else {}
        # prefetch planning (the agent plans ahead of the player with
        # MediaMap.getSegmentList / getSegmentTime and the playhead from setMediaElement)
        self.prefetch_seconds = float(gs.get("prefetchSeconds", 0.0) or 0.0)
        self.prefetch_max = int(gs.get("prefetchMaxSegments", 8))
        self._prefetch_mark = None
        # live streams: segments that slid out of the playlist window can no longer be
        # requested -> evict them ("evict by sn < head - window")
        self.live_evict = bool(gs.get("liveWindowEvict", True))
        self._evicted_below = -1
        self.evicted = 0
        # live buffer negotiation: the reference moved ``liveMinBufferMargin`` into the agent
        # (``CHANGELOG.md:13-15``), and the bridge exposes ``isLive`` / ``getBufferLevelMax`` /
        # ``setBufferMarginLive`` for it (``lib/integration/player-interface.js:31-66``).  On a
        # live stream the agent keeps the player's buffer target ``liveMinBufferMargin``
        # seconds below the live sync point, the room the swarm has to exchange the newest
        # segments before the player needs them; a VOD stream is left alone.
        margin = gs.get("liveMinBufferMargin", self.p2pConfig.get("liveMinBufferMargin", 4.0)
                        if isinstance(self.p2pConfig, dict) else 4.0)
        self.live_margin = float(margin or 0.0)
        self.is_live: Optional[bool] = None  # unknown until a level playlist is parsed
        self.live_buffer_level: Optional[float] = None
        self.disposed = False
        self._requests = []
        if playerInterface is not None and hasattr(playerInterface, "addEventListener"):
            playerInterface.addEventListener("onTrackChange", self._on_track_change)

    # ------------------------------------------------------------------ contract
    def getSegment(self, reqInfo: Any, callbacks: Any, segmentView: Any):
        """Queue a fragment request on the node; ``callbacks`` get ``onProgress`` then
        ``onSuccess(data)`` / ``onError(err)``.  Returns the request handle (``abort()``)."""
        if self.disposed:
            raise RuntimeError("PeerAgent is disposed")
        if self.is_live is None:
            self.negotiate_live_buffer()
        url = _get(reqInfo, "url")
        headers = _get(reqInfo, "headers") or {}
        tv = segmentView.trackView
        key = (self.swarm_id, int(tv.level or 0), int(tv.urlId or 0), int(segmentView.sn or 0))
        req = self.node.request(key, url, headers, callbacks, agent=self, view=segmentView)
        return req

    get_segment = getSegment

    def invalidateSegment(self, segmentView: Any) -> None:
        """The player could not decrypt or demux the bytes it got for ``segmentView``: the
        node drops its cached copy and fetches the segment from the CDN when it is asked
        again (an extension of the reference's agent contract; the wrapper calls it on
        ``FRAG_DECRYPT_ERROR`` / ``FRAG_PARSING_ERROR``)."""
        if self.disposed:
            return
        tv = segmentView.trackView
        key = (self.swarm_id, int(tv.level or 0), int(tv.urlId or 0), int(segmentView.sn or 0))
        invalidate = getattr(self.node, "invalidate", None)
        if invalidate is not None:
            invalidate(np.array([key], dtype=np.int64))

    def setMediaElement(self, media: Any) -> None:
        """The media element whose playhead drives prefetch and eviction."""
        self.media = media

    def negotiate_live_buffer(self) -> Optional[bool]:
        """Once a level playlist is parsed: on a live stream, set the player's buffer target
        to ``getBufferLevelMax() - liveMinBufferMargin`` through ``setBufferMarginLive``.
        Returns whether the stream is live (None: not known yet, asked again later)."""
        if self.is_live is not None or self.disposed or self.player is None or not hasattr(self.player, "isLive"):
            return self.is_live
        try:
            live = bool(self.player.isLive())
        except Exception:  # noqa: BLE001 - playlists not parsed yet
            return None
        self.is_live = live
        if not live:
            return False
        try:
            level_max = float(self.player.getBufferLevelMax())
        except Exception as e:  # noqa: BLE001 - a negative buffer target in the player config
            log.error("%s", e)
            return True
        level = level_max - self.live_margin
        if level <= 0:
            log.error("Invalid configuration: hlsjsConfig buffer target (%.1f s) must be greater than "
                      "p2pConfig.liveMinBufferMargin (%.1f s)", level_max, self.live_margin)
            return True
        self.player.setBufferMarginLive(level)
        self.live_buffer_level = level
        return True

    def before_round(self) -> None:
        """Node hook, run right before each round's wants are sent."""
        if self.is_live is None:
            self.negotiate_live_buffer()
        if self.live_evict:
            self.evict_live_window()
        self.plan_prefetch()

    def evict_live_window(self) -> int:
        """Drop this content's cached segments older than every parsed level's live window."""
        if self.disposed or self.player is None:
            return 0
        hls = getattr(self.player, "hls", None)
        levels = getattr(hls, "levels", None) if hls is not None else None
        if not levels:
            return 0
        first = []
        for lv in levels:
            d = getattr(lv, "details", None)
            if d is None or not getattr(d, "live", False) or not d.fragments:
                continue
            first.append(int(d.fragments[0].sn))
        if not first:
            return 0
        min_sn = min(first)
        if min_sn <= self._evicted_below:
            return 0
        self._evicted_below = min_sn
        n = int(self.node.store.evict_below(self.swarm_id, min_sn))
        self.evicted += n
        return n

    def plan_prefetch(self) -> None:
        """Called by the node right before each round's wants are sent: request the
        current track's segments in ``[currentTime, currentTime + prefetchSeconds]`` that
        are neither cached nor in flight.  The player's own later request for one of them
        is then a local cache hit (or joins the in-flight want)."""
        if self.prefetch_seconds <= 0 or self.disposed or self.media is None or not self.p2pDownloadOn:
            return
        track = self.currentTrack
        if track is None:
            return
        t = float(getattr(self.media, "currentTime", 0.0) or 0.0)
        mark = (round(t, 1), track.level, track.urlId)
        if mark == self._prefetch_mark:
            return
        try:
            svs = self.mediaMap.getSegmentLists([(track, t, self.prefetch_seconds)])[0]
        except Exception:  # noqa: BLE001  (level gone: nothing to plan)
            return
        if not svs:
            return  # not parsed yet: retry next round
        self._prefetch_mark = mark
        for sv in svs[:self.prefetch_max]:
            frag = self.mediaMap.fragment(sv)
            url = getattr(frag, "url", None) if frag is not None else None
            if not url:
                continue
            headers = {}
            s, e = getattr(frag, "byteRangeStartOffset", None), getattr(frag, "byteRangeEndOffset", None)
            if isinstance(s, int) and isinstance(e, int):
                headers["Range"] = f"bytes={s}-{e - 1}"
            self.node.prefetch((self.swarm_id, int(track.level or 0), int(track.urlId or 0), int(sv.sn)), url,
                               headers)

    def dispose(self) -> None:
        """End the session: detach from the node and the player bridge (idempotent)."""
        if self.disposed:
            return
        self.disposed = True
        if self.player is not None and hasattr(self.player, "removeEventListener"):
            self.player.removeEventListener("onTrackChange", self._on_track_change)
        self.node.detach(self)

    @property
    def stats(self) -> JsObject:
        """``{cdn, p2p, upload, peers}``: bytes by source for this session, peers online."""
        node = self.node
        peers = int(node.peer_online.sum()) - 1 if node.online else 0
        return JsObject(cdn=self._stats["cdn"], p2p=self._stats["p2p"],
                        upload=node.stats["upload"] - self._stats["upload_base"], peers=max(0, peers))

    # The toggles belong to this session, as in the reference (``lib/hlsjs-p2p-wrapper.js:20-36``
    # sets them on the session's own agent): several sessions share one GPU node, and turning
    # one player's download off must not touch the others.  The node serves this session's
    # fragments from the CDN only while its download is off, and uploads to peers while any
    # of its sessions allows it.
    @property
    def p2pDownloadOn(self) -> bool:
        """Read / write: fetch this session's fragments from peers."""
        return self.node.session_flags(self)[0]

    @p2pDownloadOn.setter
    def p2pDownloadOn(self, on: bool) -> None:
        self.node.set_session_flags(self, bool(on), self.node.session_flags(self)[1])

    @property
    def p2pUploadOn(self) -> bool:
        """Read / write: let peers be served from the cache (the node uploads while any of its
        sessions has this on)."""
        return self.node.session_flags(self)[1]

    @p2pUploadOn.setter
    def p2pUploadOn(self, on: bool) -> None:
        self.node.set_session_flags(self, self.node.session_flags(self)[0], bool(on))

    # ------------------------------------------------------------------ internals
    def _account(self, source: str, nbytes: int) -> None:
        if source == "cdn":
            self._stats["cdn"] += nbytes
        elif source == "p2p":
            self._stats["p2p"] += nbytes
        else:
            self._stats["cache"] += nbytes

    def _on_track_change(self, data: Any) -> None:
        self.currentTrack = _get(data, "video")


def _get(obj: Any, name: str) -> Any:
    if isinstance(obj, dict):
        return obj.get(name)
    return getattr(obj, name, None)
