"""P2PLoader — the hls.js fragment loader that routes media fragments to the peer agent.

Parity: ``lib/integration/p2p-loader-generator.js:11-211`` (component C6).
``p2p_loader_generator(wrapper)`` returns a NEW loader class bound to ``wrapper`` on every
call (``private.js:72-74``: each ``wrapper.P2PLoader`` access yields a fresh class).

Behaviour kept line-for-line:

* ``load`` guards: progress callback required, ``frag`` required, agent must exist;
  ``byteRange`` set only when both offsets are numbers and it persists on the instance;
  ``stats = {trequest: now, retry: 0}``.
* ``loadInternal``: throws if a previous agent request is unfinalized; runs the user's
  ``xhrSetup`` in the sandbox; ``Range: bytes=s-(e-1)``; builds
  ``TrackView{level, urlId: hls.levels[frag.level].urlId}`` and
  ``SegmentView{sn, trackView, time: frag.start}``; resets ``tfirst``/``loaded``; arms the
  per-attempt timeout; calls ``agent.getSegment(reqInfo, callbacks, segmentView)``.
* ``loadProgress``: ``loaded = cdnDownloaded + p2pDownloaded``; on the first progress of
  an attempt with P2P bytes and a positive duration, rewrite
  ``trequest = now - srTime`` and ``tfirst = trequest + min(round(srTime/2), 10)`` so ABR
  sees the peer transfer rate instead of an instantaneous hit.
* ``loadSuccess``/``loadError`` ignored once aborted; errors retry with exponential
  back-off (×2, capped at 64 s) up to ``maxRetry``, then ``onError({target:{status}})``.
* ``reset(cancelRetry=True)`` keeps the retry timer alive during a retry (the race fix of
  ``CHANGELOG.md:76``).
"""
from __future__ import annotations

import logging
import math
from typing import Any, Callable, Optional

from ..models.segment_view import SegmentView
from ..models.track_view import TrackView
from ..net.event_loop import get_event_loop
from ..utils.events import JsObject
from ..utils.xhr import extractInfoFromXhrSetup

log = logging.getLogger("hlsjs_p2p_wrapper_amd.p2p_loader")


def _js_round(x: float) -> int:
    return int(math.floor(x + 0.5))


def _is_number(v: Any) -> bool:
    return isinstance(v, (int, float)) and not isinstance(v, bool) and not (isinstance(v, float) and math.isnan(v))


def p2p_loader_generator(hlsjsWrapper: Any) -> type:
    class P2PLoader:
        def __init__(self, config: Any = None) -> None:
            self.loop = get_event_loop()
            self.xhrSetup = None
            if config:
                self.xhrSetup = (config.get("xhrSetup") if isinstance(config, dict)
                                 else getattr(config, "xhrSetup", None))
            self.stats = JsObject()
            self.byteRange = None
            self.requestTimeout = None
            self.retryTimeout = None
            self.peerAgentLoader = None
            self.reset()

        def destroy(self) -> None:
            self.abort()

        def abort(self) -> None:
            if self.peerAgentLoader:
                self.stats.aborted = True
                self.peerAgentLoader.abort()
            self.reset()

        def reset(self, cancelRetry: bool = True) -> None:
            self.loop.clear_timeout(self.requestTimeout)
            self.requestTimeout = None
            # only a full reset cancels the retry; during a retry routine it must survive
            if cancelRetry:
                self.loop.clear_timeout(self.retryTimeout)
                self.retryTimeout = None
            self.peerAgentLoader = None

        def load(self, url: str, responseType: str, onSuccess: Callable, onError: Callable, onTimeout: Callable,
                 timeout: float, maxRetry: int, retryDelay: float, onProgress: Optional[Callable] = None,
                 frag: Any = None) -> None:
            if not onProgress:
                raise Exception("P2P loader expects progress-callback to be passed for ABR stats "
                                "(use only as `fLoader` in config)")
            if not frag:
                raise Exception("P2P loader can only be used for media fragments (use only as `fLoader` in config)")
            if not getattr(hlsjsWrapper, "peerAgentModule", None):
                raise Exception("Peer agent is not existing yet")
            if _is_number(_attr(frag, "byteRangeStartOffset")) and _is_number(_attr(frag, "byteRangeEndOffset")):
                self.byteRange = f"{frag.byteRangeStartOffset}-{frag.byteRangeEndOffset}"
            self.frag = frag
            self.url = url
            self.responseType = responseType
            self.onSuccess = onSuccess
            self.onProgress = onProgress
            self.onTimeout = onTimeout
            self.onError = onError
            self.stats = JsObject(trequest=self.loop.now(), retry=0)
            self.timeout = timeout
            self.maxRetry = maxRetry
            self.retryDelay = retryDelay
            self.loadInternal()

        def loadSuccess(self, segmentData: Any) -> None:
            stats = self.stats  # a JsObject: item access here skips its __getattr__ hook
            if stats.get("aborted"):  # late callback after abort
                return
            event = JsObject(currentTarget=JsObject(response=segmentData))
            stats["tload"] = self.loop.now()
            self.onSuccess(event, stats)
            self.reset()

        # errors from the peer agent are always HTTP-like: it ultimately falls through to the CDN
        def loadError(self, httpError: Any) -> None:
            if self.stats.aborted:
                return
            status = _attr(httpError, "status")
            if self.stats.retry < self.maxRetry:
                log.warning("%s while loading %s, retrying in %s...", status, self.url, self.retryDelay)
                self.retryTimeout = self.loop.set_timeout(self.loadInternal, self.retryDelay)
                self.retryDelay = min(2 * self.retryDelay, 64000)  # exponential back-off
                self.stats.retry += 1
                self.reset(False)
            else:
                log.error("%s while loading %s", status, self.url)
                self.onError(JsObject(target=JsObject(status=status)))
                self.reset()

        def loadInternal(self) -> None:
            if self.peerAgentLoader:
                raise Exception("P2P loader was not reset correctly, internal state indicates unfinalized request")
            info = extractInfoFromXhrSetup(self.xhrSetup, self.url)
            headers, withCredentials = info["headers"], info["withCredentials"]
            if self.byteRange:
                headers["Range"] = f"bytes={self.frag.byteRangeStartOffset}-{self.frag.byteRangeEndOffset - 1}"
            level = hlsjsWrapper.hls.levels[self.frag.level]
            frag = self.frag
            # a fresh TrackView handed over: the view need not deep-copy it (segment-view.js:24)
            segmentView = SegmentView._owning(frag.sn, TrackView(level=frag.level, urlId=_attr(level, "urlId")),
                                              frag.start)
            reqInfo = JsObject(url=self.url, headers=headers, withCredentials=withCredentials)
            callbacks = JsObject(onSuccess=self.loadSuccess, onError=self.loadError, onProgress=self.loadProgress)
            stats = self.stats
            stats["tfirst"] = None
            stats["loaded"] = 0
            self.requestTimeout = self.loop.set_timeout(self.loadTimeout, self.timeout)
            self.peerAgentLoader = hlsjsWrapper.peerAgentModule.getSegment(reqInfo, callbacks, segmentView)

        def loadProgress(self, event: Any) -> None:
            get = event.get if isinstance(event, dict) else (lambda k: getattr(event, k, None))
            loaded = 0
            cdn = get("cdnDownloaded")
            p2p = get("p2pDownloaded")
            if cdn:
                loaded += cdn
            if p2p:
                loaded += p2p
            stats = self.stats
            stats["loaded"] = loaded
            if stats.get("tfirst") is None:
                now = self.loop.now()
                p2p_d = get("p2pDuration")
                cdn_d = get("cdnDuration")
                # a P2P hit reports once, immediately: move trequest back by the transfer time
                # so the ABR estimate reflects the peer rate, with a synthetic RTT of at most 10 ms
                if _is_number(p2p_d) and _is_number(cdn_d) and (p2p_d + cdn_d > 0) and (p2p or 0) > 0:
                    srTime = p2p_d + cdn_d
                    stats["trequest"] = now - srTime
                    stats["tfirst"] = stats["trequest"] + min(_js_round(srTime / 2), 10)
                else:
                    stats["tfirst"] = now
            self.onProgress(event, stats)

        def loadTimeout(self) -> None:
            self.onTimeout(None, self.stats)

    P2PLoader.__qualname__ = "P2PLoader"
    return P2PLoader


def _attr(obj: Any, name: str) -> Any:
    if isinstance(obj, dict):
        return obj.get(name)
    return getattr(obj, name, None)


P2PLoaderGenerator = p2p_loader_generator
