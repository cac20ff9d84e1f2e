"""HlsjsP2PWrapperPrivate — session orchestration (component C4).

Parity: ``lib/hlsjs-p2p-wrapper-private.js:12-240`` — one media engine and one peer agent
per wrapper at a time; both constructors are dependency-injected.

Documented decisions on the reference quirks:

* ``startSession`` in the reference passes the possibly-null ``hlsjs`` to
  ``createPeerAgent`` (``:134``) and would crash when asked to create the engine itself;
  we pass the engine it actually created (the only behaviour that can work) — fixed.
* ``createSRModule`` overwrites ``p2pConfig.contentId`` with its (default ``None``)
  argument (``:64``) — kept: legacy callers rely on it.
* ``newMediaEngine`` mutates the user's config dict with the defaults (lodash
  ``defaults``, ``:157``) — kept.
* Each ``P2PLoader`` access returns a fresh class (``:72-74``) — kept.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Optional

from ..agent.node import apply_network_config
from ..integration.p2p_loader import p2p_loader_generator
from ..integration.player_interface import PlayerInterface
from ..models.media_map import MediaMap
from ..models.segment_view import SegmentView
from ..models.track_view import TrackView
from ..utils.js import truthy

log = logging.getLogger("hlsjs_p2p_wrapper_amd.wrapper")


def _defaults(target: Dict[str, Any], source: Dict[str, Any]) -> Dict[str, Any]:
    """lodash ``defaults``: fill keys that are undefined in ``target`` (mutates it)."""
    for k, v in source.items():
        if target.get(k) is None:
            target[k] = v
    return target


class HlsjsP2PWrapperPrivate:
    """Session orchestrator: one media engine and one peer agent at a time, both constructors
    injected."""

    def __init__(self, hlsjsConstructor: Any = None, peerAgentModuleConstructor: Any = None) -> None:
        if not peerAgentModuleConstructor:
            raise Exception("Constructor needs DI of PeerAgent")
        self.Hlsjs = hlsjsConstructor
        self.StreamrootPeerAgentModule = peerAgentModuleConstructor
        self.hls = None
        self.peerAgentModule = None

    # ------------------------------------------------------------------ engines
    def createMediaEngine(self, hlsjsConfig: Optional[Dict[str, Any]] = None, p2pConfig: Any = None):
        """New engine (P2P loader config merged in); the session starts on its ``MANIFEST_LOADING``."""
        Hlsjs = self.Hlsjs
        apply_network_config(p2pConfig)  # the manifest may come from the real CDN: before loadSource
        mediaEngine = self.newMediaEngine(hlsjsConfig if hlsjsConfig is not None else {})

        def on_manifest_loading(event: str, data: Any) -> None:
            # once the manifest is loading the engine's url is defined
            self.startSession(mediaEngine, hlsjsConfig, p2pConfig, mediaEngine.url)

        mediaEngine.on(Hlsjs.Events.MANIFEST_LOADING, on_manifest_loading)
        return mediaEngine

    def createPlayer(self, hlsjsConfig: Optional[Dict[str, Any]] = None, p2pConfig: Any = None):
        """Public name of ``createMediaEngine``."""
        return self.createMediaEngine(hlsjsConfig, p2pConfig)

    def createSRModule(self, p2pConfig: Dict[str, Any], mediaEngine: Any, hlsEventsEnum: Any,
                       contentId: Optional[str] = None) -> None:
        """Legacy v2 API (deprecated): keeps overwriting ``contentId`` like the reference."""
        p2pConfig["contentId"] = contentId
        self.createPeerAgent(p2pConfig, mediaEngine, hlsEventsEnum, None)

    @property
    def P2PLoader(self) -> type:
        """A fresh fragment-loader class bound to this wrapper (new class on every access)."""
        return p2p_loader_generator(self)

    def getConfig(self) -> Dict[str, Any]:
        """Engine defaults the wrapper needs: ``fLoader`` (P2P), no byte cap, 30 s buffer / live sync."""
        # fLoader, never `loader`: playlists and keys must not go through the P2P loader
        return {
            "fLoader": p2p_loader_generator(self),
            "maxBufferSize": 0,
            "maxBufferLength": 30,
            "liveSyncDuration": 30,
        }

    # ------------------------------------------------------------------ session
    def onDispose(self) -> None:
        """Engine destroyed: end the session."""
        self.stopSession()

    def stopSession(self) -> None:
        """Dispose the peer agent, if any (idempotent)."""
        if not self.peerAgentModule:
            return
        self.peerAgentModule.dispose()
        self.peerAgentModule = None

    def startSession(self, hlsjs: Any, hlsjsConfig: Optional[Dict[str, Any]], p2pConfig: Any,
                     contentUrl: Optional[str]):
        """Attach a peer agent to ``hlsjs`` (or to a new engine); ``p2pConfig`` must be a dict."""
        Hlsjs = self.Hlsjs
        if not truthy(p2pConfig) or not isinstance(p2pConfig, dict):  # JS: {} is a valid object
            raise Exception("p2pConfig must be a valid config object")
        mediaEngine = hlsjs or self.newMediaEngine(hlsjsConfig if hlsjsConfig is not None else {})
        self.createPeerAgent(p2pConfig, mediaEngine, Hlsjs.Events, contentUrl)
        return mediaEngine

    def newMediaEngine(self, hlsjsConfig: Optional[Dict[str, Any]] = None):
        """Engine built with ``getConfig()`` defaults filled into ``hlsjsConfig`` (a user ``fLoader`` is
        an error; ``liveSyncDurationCount`` suppresses the ``liveSyncDuration`` default)."""
        if hlsjsConfig is None:
            hlsjsConfig = {}
        Hlsjs = self.Hlsjs
        if not Hlsjs:
            raise Exception("Can not create Hls.js instance: dependency was not injected")
        if hlsjsConfig.get("fLoader"):
            raise Exception("`fLoader` in Hls.js config must not be defined")
        newDefaultConf = self.getConfig()
        if hlsjsConfig.get("liveSyncDurationCount") is not None:
            # don't override liveSyncDuration when the user chose liveSyncDurationCount
            del newDefaultConf["liveSyncDuration"]
        return Hlsjs(_defaults(hlsjsConfig, newDefaultConf))

    def hasSession(self) -> bool:
        """A peer agent is attached."""
        return bool(self.peerAgentModule)

    def _setMediaElement(self, hlsjs: Any, hlsEventsEnum: Any) -> None:
        if hlsjs.media:
            self.peerAgentModule.setMediaElement(hlsjs.media)
        else:
            def on_attaching(event: str, data: Any) -> None:
                if self.peerAgentModule:
                    self.peerAgentModule.setMediaElement(hlsjs.media)

            hlsjs.on(hlsEventsEnum.MEDIA_ATTACHING, on_attaching)

    def createPeerAgent(self, p2pConfig: Dict[str, Any], hlsjs: Any, hlsEventsEnum: Any,
                        url: Optional[str] = None) -> None:
        """Build player bridge + media map + peer agent for ``hlsjs`` (one session at a time; the
        content URL is ``url`` or the engine's ``url``)."""
        self.hls = hlsjs
        StreamrootPeerAgentModule = self.StreamrootPeerAgentModule
        streamType = StreamrootPeerAgentModule.StreamTypes.HLS
        integrationVersion = "v2"
        if self.hasSession():
            raise Exception("Streamroot session already started")
        contentUrl = url or hlsjs.url
        if not contentUrl:
            raise Exception("Hls.js instance must have valid `url` property or `contentUrl` must be passed")
        if not truthy(hlsEventsEnum):
            raise Exception("Need valid Hls.js Events enumeration")
        hlsjs.on(hlsEventsEnum.ERROR, self.onMediaEngineError)
        hlsjs.on(hlsEventsEnum.ERROR, self._invalidateUnusableFragment)
        playerBridge = PlayerInterface(hlsjs, hlsEventsEnum, self.onDispose)
        mediaMap = MediaMap(hlsjs)
        self.peerAgentModule = StreamrootPeerAgentModule(playerBridge, contentUrl, mediaMap, p2pConfig, SegmentView,
                                                         streamType, integrationVersion)
        self._setMediaElement(hlsjs, hlsEventsEnum)

    def _invalidateUnusableFragment(self, event: str, data: Any) -> None:
        """A fragment the engine could not decrypt or demux: the agent drops the cached copy
        it served, so the engine's retry fetches the segment from the CDN instead of getting
        the same bytes again (extension; the reference's agent contract has no such call)."""
        details = data.get("details") if isinstance(data, dict) else getattr(data, "details", None)
        if details not in ("fragDecryptError", "fragParsingError"):
            return
        frag = data.get("frag") if isinstance(data, dict) else getattr(data, "frag", None)
        invalidate = getattr(self.peerAgentModule, "invalidateSegment", None)
        if frag is None or invalidate is None or self.hls is None:
            return
        levels = self.hls.levels or []
        lvl = levels[frag.level] if 0 <= frag.level < len(levels) else None
        invalidate(SegmentView._owning(frag.sn, TrackView(level=frag.level, urlId=getattr(lvl, "urlId", 0)),
                                       frag.start))

    @staticmethod
    def onMediaEngineError(event: str, data: Any) -> None:
        """Log engine errors (fatal -> error, otherwise warning)."""
        fatal = data.get("fatal") if isinstance(data, dict) else getattr(data, "fatal", False)
        typ = data.get("type") if isinstance(data, dict) else getattr(data, "type", None)
        details = data.get("details") if isinstance(data, dict) else getattr(data, "details", None)
        if fatal:
            log.error("Hls.js fatal error: %s - %s", typ, details)
        else:
            log.warning("Hls.js non-fatal error: %s - %s", typ, details)


class _VersionDescriptor:
    def __get__(self, obj, owner):
        from .. import version as _v

        return _v.VERSION


HlsjsP2PWrapperPrivate.version = _VersionDescriptor()  # static getter, like `static get version`
