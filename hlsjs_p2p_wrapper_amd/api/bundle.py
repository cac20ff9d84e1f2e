"""``Hls`` bundle: drop-in replacement of the media-engine constructor (components C1/C2).

Parity: ``lib/hlsjs-p2p-bundle.js:1-72``.  ``Hls(hlsjsConfig, p2pConfig)`` returns a real
media-engine instance bootstrapped with the P2P agent, produced by
``HlsjsP2PWrapper(engine).createPlayer(...)``; construction returns that *different*
object, so the engine's constructor runs exactly once (no zombie context, ``:15-16``).
All engine statics (``Hls.Events``, ``Hls.DefaultConfig`` …) are mirrored read-only
(``:36-39``); ``isSupported`` and ``getBrowserName`` are overridden *after* the mirroring
(``:41-70``): supported = engine supported and not Safari and not mobile/tablet/console
(Android/iOS count as mobile).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

from ..player.hls import Hls as _Engine
from ..utils import ua as _ua
from ..utils.statics import StaticMirrorMeta, inheritStaticPropertiesReadOnly
from .wrapper import HlsjsP2PWrapper

_UA = _ua.current_user_agent()  # parsed once at import, like the reference's module load


class Hls(_Engine, metaclass=StaticMirrorMeta):
    """Media-engine constructor with P2P built in: ``Hls(hlsjsConfig, p2pConfig)`` returns an engine
    whose fragment loader is the P2P loader; engine statics are mirrored read-only."""

    def __new__(cls, hlsjsConfig: Optional[Dict[str, Any]] = None, p2pConfig: Optional[Dict[str, Any]] = None):
        return HlsjsP2PWrapper(_Engine).createPlayer(hlsjsConfig, p2pConfig)

    def __init__(self, *args: Any, **kwargs: Any) -> None:  # pragma: no cover - never reached
        pass


inheritStaticPropertiesReadOnly(Hls, _Engine)


def _is_supported() -> bool:
    """Engine supported, and the user agent is neither Safari nor a mobile / tablet / console."""
    res = _UA if _ua._override is None else _ua.current_user_agent()
    return _Engine.isSupported() and not _ua.is_safari(res) and not _ua.is_mobile(res)


def _get_browser_name() -> Optional[str]:
    """Browser name parsed from the user agent (``None`` when unknown)."""
    res = _UA if _ua._override is None else _ua.current_user_agent()
    return res.browser.get("name")


type.__setattr__(Hls, "isSupported", staticmethod(_is_supported))
type.__setattr__(Hls, "getBrowserName", staticmethod(_get_browser_name))

StreamrootHlsjsBundle = Hls
