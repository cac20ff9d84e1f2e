"""Bandwidth estimation and automatic level selection (hls.js ``AbrController`` semantics).

The P2P loader's whole timing logic exists to feed this estimator realistic numbers
(``lib/integration/p2p-loader-generator.js:167-204``); the reference pins the contract
with ``test/hls-controllers.js:11-33``: 128,000 B loaded with ``trequest = now - 1000``
must estimate 1,024,000 bit/s (± 4,000).

Estimator: two exponentially-weighted moving averages (fast / slow half-lives in seconds
of transfer time), each sample weighted by its duration, zero-bias corrected, the
estimate being the min of the two — hls.js's ``EwmaBandWidthEstimator``.
"""
from __future__ import annotations

import math
from typing import Any

from ..net.event_loop import get_event_loop
from .events import Events


class Ewma:
    def __init__(self, half_life: float) -> None:
        self.alpha = math.exp(math.log(0.5) / half_life) if half_life > 0 else 0.0
        self.estimate = 0.0
        self.total_weight = 0.0

    def sample(self, weight: float, value: float) -> None:
        adj = self.alpha ** weight
        self.estimate = value * (1.0 - adj) + adj * self.estimate
        self.total_weight += weight

    def get_total_weight(self) -> float:
        return self.total_weight

    def get_estimate(self) -> float:
        if self.alpha:
            zero_factor = 1.0 - self.alpha ** self.total_weight
            if zero_factor > 0:
                return self.estimate / zero_factor
        return self.estimate

    getEstimate = get_estimate


class EwmaBandWidthEstimator:
    MIN_WEIGHT = 0.001
    MIN_DELAY_MS = 50.0

    def __init__(self, hls: Any, slow: float, fast: float, default_estimate: float) -> None:
        self.hls = hls
        self.default_estimate = default_estimate
        self.slow = Ewma(slow)
        self.fast = Ewma(fast)

    def sample(self, duration_ms: float, num_bytes: float) -> None:
        duration_ms = max(float(duration_ms), self.MIN_DELAY_MS)
        bandwidth = 8000.0 * num_bytes / duration_ms  # bit/s
        weight = duration_ms / 1000.0
        self.fast.sample(weight, bandwidth)
        self.slow.sample(weight, bandwidth)

    def can_estimate(self) -> bool:
        return self.fast.get_total_weight() >= self.MIN_WEIGHT

    def get_estimate(self) -> float:
        if self.can_estimate():
            return min(self.fast.get_estimate(), self.slow.get_estimate())
        return self.default_estimate

    getEstimate = get_estimate
    canEstimate = can_estimate


class AbrController:
    def __init__(self, hls: Any) -> None:
        self.hls = hls
        self.loop = getattr(hls, "loop", None) or get_event_loop()
        cfg = hls.config
        live = False
        self.bwEstimator = EwmaBandWidthEstimator(
            hls, cfg.get("abrEwmaSlowVoD", 15.0) if not live else cfg.get("abrEwmaSlowLive", 9.0),
            cfg.get("abrEwmaFastVoD", 4.0) if not live else cfg.get("abrEwmaFastLive", 5.0),
            cfg.get("abrEwmaDefaultEstimate", 5e5))
        self.lastLoadedFragLevel = 0
        self._nextAutoLevel = -1
        self.fragCurrent = None
        self.lastfetchduration = 0.0
        self.lastbw = 0.0
        if hasattr(hls, "on"):
            hls.on(Events.FRAG_LOADING, lambda e, d: self.onFragLoading(d))
            hls.on(Events.FRAG_LOADED, lambda e, d: self.onFragLoaded(d))

    def destroy(self) -> None:
        self.fragCurrent = None

    def onFragLoading(self, data: Any) -> None:
        self.fragCurrent = data["frag"] if type(data) is dict else _get(data, "frag")

    def onFragLoaded(self, data: Any) -> None:
        if type(data) is dict:  # what Hls.trigger passes: skip the generic accessor
            stats, frag = data.get("stats"), data.get("frag")
        else:
            stats, frag = _get(data, "stats"), _get(data, "frag")
        sget = stats.get if isinstance(stats, dict) else (lambda k, d=None: _get(stats, k, d))
        # only the first load of a fragment is a fair bandwidth sample (a reload may be
        # served from a cache and look infinitely fast)
        if sget("aborted") is None and _get(frag, "loadCounter", 1) == 1:
            ms = self.loop.now() - sget("trequest")
            loaded = sget("loaded") or 0
            self.lastfetchduration = ms / 1000.0
            self.lastbw = (loaded * 8) / max(self.lastfetchduration, 1e-9)
            self.bwEstimator.sample(ms, loaded)
            self.lastLoadedFragLevel = _get(frag, "level", 0)

    @property
    def autoLevelCapping(self) -> int:
        return getattr(self.hls, "autoLevelCapping", -1)

    @property
    def nextAutoLevel(self) -> int:
        if self._nextAutoLevel != -1:
            return self._nextAutoLevel
        levels = getattr(self.hls, "levels", None) or []
        if not levels:
            return 0
        cfg = self.hls.config
        bw = self.bwEstimator.get_estimate()
        cap = self.autoLevelCapping
        max_level = len(levels) - 1 if cap is None or cap < 0 else min(cap, len(levels) - 1)
        for i in range(max_level, -1, -1):
            factor = cfg.get("abrBandWidthFactor", 0.8) if i <= self.lastLoadedFragLevel else \
                cfg.get("abrBandWidthUpFactor", 0.7)
            if levels[i].bitrate < bw * factor:
                return i
        return 0

    @nextAutoLevel.setter
    def nextAutoLevel(self, v: int) -> None:
        self._nextAutoLevel = v


def _get(obj: Any, name: str, default: Any = None) -> Any:
    if obj is None:
        return default
    if isinstance(obj, dict):
        v = obj.get(name, default)
        return default if v is None and default is not None else v
    return getattr(obj, name, default)
