"""``Hls`` — the media engine the wrapper bootstraps (hls.js API surface).

Statics: ``Hls.Events``, ``Hls.ErrorTypes``, ``Hls.ErrorDetails``, ``Hls.DefaultConfig``,
``Hls.isSupported()``, ``Hls.version``.  Instance: ``config``, ``on/off/once/trigger``,
``url``, ``media``, ``levels``, ``loadSource``, ``attachMedia``, ``detachMedia``,
``startLoad``, ``stopLoad``, ``destroy``, ``recoverMediaError``, ``swapAudioCodec``,
``currentLevel``, ``loadLevel``, ``nextLoadLevel``, ``nextLevel``, ``firstLevel``,
``startLevel``, ``autoLevelCapping``, ``autoLevelEnabled``, ``manualLevel``,
``levelController._levels``, ``abrController.bwEstimator.getEstimate()``.
"""
from __future__ import annotations

import logging
from typing import Any, Callable, Mapping, Optional

import torch

from ..net.event_loop import get_event_loop
from ..utils.events import Observer
from .abr import AbrController
from .config import HlsConfig, default_config, merge_config
from .controllers import FragmentLoader, KeyLoader, LevelController, PlaylistLoader, StreamController
from .events import ErrorDetails, ErrorTypes, Events
from .transmux import default_transmux_device

log = logging.getLogger("hlsjs_p2p_wrapper_amd.hls")

HLS_ENGINE_VERSION = "0.6.1-mi355x"


class _DefaultConfigDescriptor:
    def __get__(self, obj, owner):
        return default_config()


class Hls:
    """hls.js-compatible media engine: playlist / key / fragment loaders, level and ABR
    controllers, transmux to the media element; events through ``on`` / ``trigger``."""
    Events = Events
    ErrorTypes = ErrorTypes
    ErrorDetails = ErrorDetails
    DefaultConfig = _DefaultConfigDescriptor()
    version = HLS_ENGINE_VERSION

    @staticmethod
    def isSupported() -> bool:
        """MSE analog available: the engine needs PyTorch (always) — GPU optional."""
        try:
            import torch  # noqa: F401
            return True
        except Exception:  # pragma: no cover
            return False

    def __init__(self, config: Optional[Mapping[str, Any]] = None) -> None:
        self.config: HlsConfig = merge_config(config)
        if self.config.get("debug"):  # hlsjsConfig.debug -> engine debug logging
            from ..utils.log import configure

            configure(debug=True)
        self.loop = get_event_loop()
        self._observer = Observer()
        self.url: Optional[str] = None
        self.media = None
        self._destroyed = False
        self.autoLevelCapping = -1
        self.levelController = LevelController(self)
        self.playlistLoader = PlaylistLoader(self)
        self.keyLoader = KeyLoader(self)
        self.fragmentLoader = FragmentLoader(self)
        abr_cls = self.config.abrController or AbrController
        self.abrController = abr_cls(self)
        stream_cls = self.config.streamController or StreamController
        self.streamController = stream_cls(self)
        self._transmux_device: Optional[torch.device] = None
        self.on(Events.ERROR, self._log_error)

    # ------------------------------------------------------------------ events
    def on(self, event: str, listener: Callable[[str, Any], Any]) -> None:
        """Subscribe ``listener(event, data)``."""
        self._observer.on(event, listener)

    def once(self, event: str, listener: Callable[[str, Any], Any]) -> None:
        """Subscribe for one delivery."""
        self._observer.once(event, listener)

    def off(self, event: str, listener: Callable[[str, Any], Any]) -> None:
        """Unsubscribe."""
        self._observer.off(event, listener)

    def trigger(self, event: str, data: Any = None) -> None:
        """Emit ``event`` with ``data`` (``{}`` when omitted)."""
        if data is None:
            data = {}
        self._observer.trigger(event, data)

    def listening(self, event: str) -> bool:
        """True when ``event`` has a listener (hot paths skip building unheard payloads)."""
        return bool(self._observer._listeners.get(event))

    emit = trigger

    def _log_error(self, event: str, data: Any) -> None:
        if self.config.debug:
            log.warning("hls error: %s", data)

    # ------------------------------------------------------------------ lifecycle
    def loadSource(self, url: str) -> None:
        """Set ``url`` and start loading the master playlist (``MANIFEST_LOADING``)."""
        self.url = url
        self.trigger(Events.MANIFEST_LOADING, {"url": url})

    def attachMedia(self, media: Any) -> None:
        """Bind a media element (``MEDIA_ATTACHING`` / ``MEDIA_ATTACHED``)."""
        self.media = media
        self.trigger(Events.MEDIA_ATTACHING, {"media": media})
        self.trigger(Events.MEDIA_ATTACHED, {"media": media})

    def detachMedia(self) -> None:
        """Unbind the media element (``MEDIA_DETACHING`` / ``MEDIA_DETACHED``)."""
        if self.media is None:
            return
        self.trigger(Events.MEDIA_DETACHING, {})
        media = self.media
        self.media = None
        if hasattr(media, "stop"):
            media.stop()
        self.trigger(Events.MEDIA_DETACHED, {})

    def startLoad(self, startPosition: float = -1) -> None:
        """Start fragment loading at ``startPosition`` (-1: default position)."""
        self.streamController.startLoad(startPosition)

    def stopLoad(self) -> None:
        """Stop fragment loading."""
        self.streamController.stopLoad()

    def destroy(self) -> None:
        """``DESTROYING``, then stop every loader and drop listeners (idempotent)."""
        if self._destroyed:
            return
        self.trigger(Events.DESTROYING, {})
        self._destroyed = True
        self.detachMedia()
        self.streamController.destroy()
        self.fragmentLoader.destroy()
        self.keyLoader.destroy()
        self.playlistLoader.destroy()
        self.levelController.destroy()
        self.abrController.destroy()
        self.url = None
        self._observer.remove_all_listeners()

    # ------------------------------------------------------------------ levels
    @property
    def levels(self):
        """Parsed variant levels (``None`` before the master playlist)."""
        return self.levelController.levels

    @property
    def currentLevel(self) -> int:
        """Level of the last loaded fragment; setting it switches immediately."""
        frag = self.streamController.fragPrevious
        return frag.level if frag is not None else self.levelController.level

    @currentLevel.setter
    def currentLevel(self, v: int) -> None:
        self.loadLevel = v

    @property
    def loadLevel(self) -> int:
        """Level being loaded; setting it forces a manual level."""
        return self.levelController.level

    @loadLevel.setter
    def loadLevel(self, v: int) -> None:
        self.levelController.manualLevel = v

    @property
    def nextLevel(self) -> int:
        """Level of the next fragment; setting it switches at the next fragment."""
        return self.nextLoadLevel

    @nextLevel.setter
    def nextLevel(self, v: int) -> None:
        self.loadLevel = v

    @property
    def manualLevel(self) -> int:
        """Forced level, -1 in auto mode."""
        return self.levelController.manualLevel

    @property
    def autoLevelEnabled(self) -> bool:
        """ABR chooses the level."""
        return self.levelController.manualLevel == -1

    @property
    def nextLoadLevel(self) -> int:
        """Level the next fragment load will use (manual, else the ABR choice)."""
        if self.levelController.manualLevel != -1:
            return self.levelController.manualLevel
        return self.abrController.nextAutoLevel

    @nextLoadLevel.setter
    def nextLoadLevel(self, v: int) -> None:
        self.levelController.manualLevel = v

    @property
    def startLevel(self) -> int:
        """First level loaded."""
        return self.levelController.firstLevel

    @startLevel.setter
    def startLevel(self, v: int) -> None:
        # hls.js: the level the next manifest starts on (config.startLevel); -1 = automatic
        self.config.startLevel = v

    @property
    def firstLevel(self) -> int:
        """First level of the manifest (``startLevel`` when it names a level, else 0)."""
        return self.levelController.firstLevel

    @firstLevel.setter
    def firstLevel(self, v: int) -> None:
        self.levelController.firstLevel = v

    def recoverMediaError(self) -> None:
        """hls.js's recovery for a fatal media error: detach the media element and attach it
        again, which restarts buffering at its current position."""
        media = self.media
        if media is None:
            return
        self.detachMedia()
        self.attachMedia(media)
        restart = getattr(media, "restart", None)
        if restart is not None:
            restart()

    def swapAudioCodec(self) -> None:
        """hls.js toggles the audio codec string (``mp4a.40.2`` / ``mp4a.40.5``) it hands to
        MSE on the next init segment, to recover from a decoder that rejects one.  The
        elementary streams here go to :class:`MediaElement`, which takes no codec string,
        so the flag is kept (``audioCodecSwap``) for callers that read it and changes no
        output."""
        self.audioCodecSwap = not getattr(self, "audioCodecSwap", False)

    @property
    def bandwidthEstimate(self) -> float:
        """ABR bandwidth estimate, bits/s."""
        return self.abrController.bwEstimator.getEstimate()

    # ------------------------------------------------------------------ transmux placement
    def transmux_device(self, payload: Any = None) -> torch.device:
        """Device for decrypt/demux: the payload's device if it already lives on a GPU
        (P2P path: a view of the node's HBM arena), else the configured/default one."""
        if isinstance(payload, torch.Tensor) and payload.device.type == "cuda":
            return payload.device
        if self._transmux_device is None:
            td = self.config.get("transmuxDevice", "auto")
            self._transmux_device = default_transmux_device() if td in (None, "auto") else torch.device(td)
        return self._transmux_device
