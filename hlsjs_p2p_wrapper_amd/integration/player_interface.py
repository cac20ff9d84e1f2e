"""PlayerInterface — the player bridge handed to the peer agent.

Parity: ``lib/integration/player-interface.js:4-84`` (component C10):

* re-emits ``LEVEL_SWITCH`` as ``'onTrackChange' {video: TrackView{level, urlId}}``
  (``:15-20``) and calls ``onDispose`` on ``DESTROYING`` (``:22-24``);
* ``isLive()`` from the first parsed level's ``details.live``; throws before the master
  playlist or before any level playlist is parsed (``:31-43``);
* ``getBufferLevelMax()`` → ``liveSyncDuration`` if set, else ``maxBufferLength``; throws
  on a negative value (``:45-61``);
* ``setBufferMarginLive(level)`` sets ``maxBufferSize = 0``, ``maxBufferLength = level``
  (``:63-66``);
* ``addEventListener``/``removeEventListener`` only accept ``'onTrackChange'`` and
  silently ignore anything else (``:68-82``).
"""
from __future__ import annotations

from typing import Any, Callable

from ..models.track_view import TrackView
from ..utils.events import EventEmitter


class PlayerInterface(EventEmitter):
    """Player bridge given to the peer agent: live / buffer queries on the engine, and
    ``onTrackChange`` events re-emitted from the engine's level switches."""

    __slots__ = ("hls", "onDispose")

    def __init__(self, hls: Any, Events: Any, onDispose: Callable[[], Any], *_legacy: Any) -> None:
        super().__init__()
        self.hls = hls
        self.onDispose = onDispose
        level_switch = _attr(Events, "LEVEL_SWITCH")
        destroying = _attr(Events, "DESTROYING")

        def on_level_switch(event: str, data: Any) -> None:
            idx = data["level"] if isinstance(data, dict) else data.level
            level = self.hls.levels[idx]
            self.emit("onTrackChange", {"video": TrackView(level=idx, urlId=_attr(level, "urlId"))})

        def on_destroying(event: str, data: Any) -> None:
            self.onDispose()

        self.hls.on(level_switch, on_level_switch)
        self.hls.on(destroying, on_destroying)

    def isLive(self) -> bool:
        """``details.live`` of the first parsed level; raises before any playlist is parsed."""
        levels = self.hls.levels
        if levels is None:  # (an empty JS array is truthy: only "undefined" means unparsed)
            raise Exception("Called isLive before the master playlist was parsed")
        for level in levels:
            details = _attr(level, "details")
            if details:
                return bool(_attr(details, "live"))
        raise Exception("Called isLive before any levelplaylist was parsed")

    def getBufferLevelMax(self) -> float:
        """Target buffer in seconds: ``liveSyncDuration`` if set, else ``maxBufferLength``."""
        cfg = self.hls.config
        if _attr(cfg, "liveSyncDuration"):
            conf_param = "liveSyncDuration"
            max_level = _attr(cfg, "liveSyncDuration")
        else:
            conf_param = "maxBufferLength"
            max_level = _attr(cfg, "maxBufferLength")
        if max_level < 0:
            raise Exception(f"Invalid configuration: hlsjsConfig.{conf_param} must be greater than "
                            f"p2pConfig.liveMinBufferMargin")
        return max_level

    def setBufferMarginLive(self, bufferLevel: float) -> None:
        """Set the engine's buffer target to ``bufferLevel`` seconds (and lift the byte cap)."""
        cfg = self.hls.config
        _set(cfg, "maxBufferSize", 0)
        _set(cfg, "maxBufferLength", bufferLevel)

    def addEventListener(self, eventName: str, listener: Callable) -> None:
        """Subscribe to ``'onTrackChange'``; other names are ignored."""
        if eventName == "onTrackChange":
            self.on(eventName, listener)

    def removeEventListener(self, eventName: str, listener: Callable) -> None:
        """Unsubscribe from ``'onTrackChange'``; other names are ignored."""
        if eventName == "onTrackChange":
            self.remove_listener(eventName, listener)

    is_live = isLive
    get_buffer_level_max = getBufferLevelMax
    set_buffer_margin_live = setBufferMarginLive


def _attr(obj: Any, name: str) -> Any:
    if isinstance(obj, dict):
        return obj.get(name)
    return getattr(obj, name, None)


def _set(obj: Any, name: str, value: Any) -> None:
    if isinstance(obj, dict):
        obj[name] = value
    else:
        setattr(obj, name, value)
