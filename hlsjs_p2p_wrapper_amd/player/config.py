"""hls.js-style configuration object.

A plain mapping with attribute access, so both ``hls.config.maxBufferLength`` (hls.js
style, mutated by the player bridge at ``lib/integration/player-interface.js:63-66``) and
``config["fLoader"]`` work.  ``None`` plays the role of JavaScript ``undefined``.

Defaults follow hls.js 0.5/0.6 (the versions the reference supports, ``README.md:6-9``)
for every key the engine implements, plus the MI355X-engine extensions at the bottom.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Mapping, Optional


class HlsConfig(dict):
    def __getattr__(self, name: str) -> Any:
        try:
            return self[name]
        except KeyError:
            if name.startswith("__"):
                raise AttributeError(name)
            return None

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value

    def __delattr__(self, name: str) -> None:
        self.pop(name, None)

    def copy(self) -> "HlsConfig":
        return HlsConfig(self)


def _default_config() -> Dict[str, Any]:
    from .abr import AbrController
    from .loader import XhrLoader
    from .controllers import StreamController

    return {
        "autoStartLoad": True,
        "startPosition": -1,
        "debug": False,
        "capLevelToPlayerSize": False,
        "maxBufferLength": 30,
        "maxBufferSize": 60 * 1000 * 1000,
        "maxBufferHole": 0.5,
        "maxSeekHole": 2,
        "seekHoleNudgeDuration": 0.01,
        "maxFragLookUpTolerance": 0.2,
        "liveSyncDurationCount": 3,
        "liveMaxLatencyDurationCount": math.inf,
        "liveSyncDuration": None,
        "liveMaxLatencyDuration": None,
        "maxMaxBufferLength": 600,
        "enableWorker": True,
        "enableSoftwareAES": True,
        "manifestLoadingTimeOut": 10000,
        "manifestLoadingMaxRetry": 1,
        "manifestLoadingRetryDelay": 1000,
        "levelLoadingTimeOut": 10000,
        "levelLoadingMaxRetry": 4,
        "levelLoadingRetryDelay": 1000,
        "fragLoadingTimeOut": 20000,
        "fragLoadingMaxRetry": 6,
        "fragLoadingRetryDelay": 1000,
        "fragLoadingLoopThreshold": 3,
        "startFragPrefetch": False,
        "appendErrorMaxRetry": 3,
        "loader": XhrLoader,
        "fLoader": None,
        "pLoader": None,
        "xhrSetup": None,
        "abrController": AbrController,
        "streamController": StreamController,
        "abrEwmaFastLive": 5.0,
        "abrEwmaSlowLive": 9.0,
        "abrEwmaFastVoD": 4.0,
        "abrEwmaSlowVoD": 15.0,
        "abrEwmaDefaultEstimate": 5e5,
        "abrBandWidthFactor": 0.8,
        "abrBandWidthUpFactor": 0.7,
        "minAutoBitrate": 0,
        # --- MI355X engine extensions ------------------------------------------------
        # fragments loaded concurrently (hls.js loads one at a time: 1 keeps parity;
        # serving/throughput deployments raise it so one exchange round moves many)
        "maxFragLoadsInFlight": 1,
        # where decrypt/demux run: "auto" (the media pipeline's device), "cpu", "cuda:N"
        "transmuxDevice": "auto",
        # stream-controller tick period (hls.js uses 100 ms)
        "tickInterval": 100,
        # keep demuxed ES tensors referenced by the media element (False: account only)
        "retainMediaData": False,
    }


_DEFAULTS: Optional[Dict[str, Any]] = None


def default_config() -> HlsConfig:
    global _DEFAULTS
    if _DEFAULTS is None:
        _DEFAULTS = _default_config()
    return HlsConfig(_DEFAULTS)


def merge_config(user: Optional[Mapping[str, Any]]) -> HlsConfig:
    """hls.js constructor semantics: user keys override defaults (``undefined`` skipped)."""
    cfg = default_config()
    if user:
        for k, v in user.items():
            if v is not None:
                cfg[k] = v
    return cfg
