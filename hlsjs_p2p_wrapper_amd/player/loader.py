"""Default (non-P2P) loader — the hls.js ``XhrLoader`` contract over the in-process CDN.

Used for playlists and keys always, and for fragments when no ``fLoader`` is configured.
Keys and playlists must never go through the P2P loader (``private.js:82-85``,
``CHANGELOG.md:121-123``), which is why the wrapper sets ``fLoader`` and not ``loader``.

Contract (hls.js ≤ 0.6):
``load(url, responseType, onSuccess, onError, onTimeout, timeout, maxRetry, retryDelay,
onProgress=None, frag=None)``; ``onSuccess(event{currentTarget{response}}, stats)``,
``onError(event{target{status}})``, ``onTimeout(event, stats)``,
``onProgress(event{loaded, total}, stats)``; stats = ``{trequest, tfirst, tload, loaded,
total, retry, aborted}``.  Transfer time follows :class:`~..net.http.Shaper`
(``maxBandwidth`` kbit/s, ``minLatency`` ms) on the event-loop clock, with a progress
event per ~50 ms of transfer, like a browser XHR.
"""
from __future__ import annotations

import logging
import math
from typing import Any, Callable, Optional

from ..net.event_loop import get_event_loop
from ..net.http import HttpError, Shaper, fetch_async
from ..utils.events import JsObject

log = logging.getLogger("hlsjs_p2p_wrapper_amd.loader")


class _XhrShim:
    """What ``xhrSetup(xhr, url)`` sees from the default loader: a permissive XHR."""

    def __init__(self, headers: dict) -> None:
        self._headers = headers
        self.withCredentials = False

    def setRequestHeader(self, k: str, v: Any) -> None:
        self._headers[k] = v

    def open(self, *args: Any) -> None:  # tolerated, like a real XHR
        pass


class XhrLoader:
    PROGRESS_MS = 50.0

    def __init__(self, config: Any = None) -> None:
        self.xhrSetup = getattr(config, "xhrSetup", None) if config is not None else None
        self.loop = get_event_loop()
        self.stats = JsObject()
        self._timers: list = []
        self._request_timeout = None
        self._retry_timeout = None
        self._inflight = False
        self._attempt = 0
        self.byteRange: Optional[str] = None

    # ------------------------------------------------------------------ API
    def destroy(self) -> None:
        self.abort()

    def abort(self) -> None:
        if self._inflight:
            self.stats.aborted = True
        self._cancel_all()

    def load(self, url: str, responseType: str, onSuccess: Callable, onError: Callable, onTimeout: Callable,
             timeout: float, maxRetry: int, retryDelay: float, onProgress: Optional[Callable] = None,
             frag: Any = None) -> None:
        self.url = url
        self.responseType = responseType
        self.onSuccess, self.onError, self.onTimeout, self.onProgress = onSuccess, onError, onTimeout, onProgress
        self.frag = frag
        if frag is not None and isinstance(getattr(frag, "byteRangeStartOffset", None), (int, float)) and \
                isinstance(getattr(frag, "byteRangeEndOffset", None), (int, float)):
            self.byteRange = f"{frag.byteRangeStartOffset}-{frag.byteRangeEndOffset}"
        self.stats = JsObject(trequest=self.loop.now(), retry=0)
        self.timeout = timeout
        self.maxRetry = maxRetry
        self.retryDelay = retryDelay
        self._load_internal()

    # ------------------------------------------------------------------ internals
    def _cancel_all(self) -> None:
        for t in self._timers:
            t.cancel()
        self._timers.clear()
        if self._request_timeout is not None:
            self._request_timeout.cancel()
            self._request_timeout = None
        if self._retry_timeout is not None:
            self._retry_timeout.cancel()
            self._retry_timeout = None
        self._inflight = False

    def _load_internal(self) -> None:
        self._retry_timeout = None
        headers: dict = {}
        shim = _XhrShim(headers)
        if self.xhrSetup:
            self.xhrSetup(shim, self.url)
        if self.byteRange is not None and self.frag is not None:
            headers["Range"] = f"bytes={self.frag.byteRangeStartOffset}-{self.frag.byteRangeEndOffset - 1}"
        self.stats.tfirst = None
        self.stats.loaded = 0
        self._inflight = True
        self._request_timeout = self.loop.set_timeout(self._on_timeout, self.timeout)
        self._attempt += 1
        attempt = self._attempt
        # in-process origins answer before fetch_async returns; a network origin answers on
        # this loop later (a stale answer of an aborted / retried attempt is dropped)
        fetch_async(self.url, headers, shim.withCredentials, self.loop,
                    lambda resp: self._on_response(attempt, resp), lambda e: self._on_fetch_error(attempt, e))

    def _on_fetch_error(self, attempt: int, e: HttpError) -> None:
        if attempt != self._attempt or not self._inflight:
            return
        delay = Shaper.minLatency
        self._timers.append(self.loop.set_timeout(self._on_error, delay, e.status))

    def _on_response(self, attempt: int, resp) -> None:
        if attempt != self._attempt or not self._inflight:
            return
        total = resp.length
        duration = Shaper.transfer_ms(total)
        self.stats.total = total
        if duration <= 0:
            self.loop.call_soon(self._deliver, resp, total, True)
            return
        # progress every PROGRESS_MS of transfer, completion at `duration`
        latency = Shaper.minLatency
        body_ms = max(0.0, duration - latency)
        n = max(1, int(math.ceil(body_ms / self.PROGRESS_MS)))
        for i in range(1, n + 1):
            t = latency + body_ms * i / n
            loaded = total if i == n else int(total * i / n)
            self._timers.append(self.loop.set_timeout(self._deliver, t, resp, loaded, i == n))

    def _deliver(self, resp, loaded: int, done: bool) -> None:
        if not self._inflight or self.stats.aborted:
            return
        now = self.loop.now()
        if self.stats.tfirst is None:
            self.stats.tfirst = now
        self.stats.loaded = loaded
        if self.onProgress is not None:
            self.onProgress(JsObject(loaded=loaded, total=resp.length, lengthComputable=True), self.stats)
        if done:
            self.stats.tload = max(now, self.stats.tfirst)
            self._cancel_all()
            body = resp.body
            if self.responseType != "text" and isinstance(body, str):
                body = body.encode()
            event = JsObject(currentTarget=JsObject(response=body, status=resp.status, responseURL=resp.url))
            self.onSuccess(event, self.stats)

    def _on_error(self, status: int) -> None:
        if not self._inflight:
            return
        if self._request_timeout is not None:
            self._request_timeout.cancel()
            self._request_timeout = None
        if self.stats.retry < self.maxRetry:
            log.warning("%s while loading %s, retrying in %s...", status, self.url, self.retryDelay)
            self._inflight = False
            self._retry_timeout = self.loop.set_timeout(self._load_internal, self.retryDelay)
            self.retryDelay = min(2 * self.retryDelay, 64000)
            self.stats.retry += 1
        else:
            log.error("%s while loading %s", status, self.url)
            self._cancel_all()
            self.onError(JsObject(target=JsObject(status=status)))

    def _on_timeout(self) -> None:
        self._request_timeout = None
        log.warning("timeout while loading %s", self.url)
        self.onTimeout(JsObject(target=JsObject(status=0)), self.stats)
