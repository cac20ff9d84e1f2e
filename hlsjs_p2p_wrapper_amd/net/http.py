"""The "HTTP" layer: URL -> origin resolution, responses, errors, bandwidth shaping.

There is no network on an MI355X node's data path: the CDN is modelled by in-process
*origins* (:mod:`.origin`) registered under URL prefixes, holding playlists as text and
segments in pinned host memory.  :func:`fetch` resolves a URL (with an optional
``Range: bytes=s-e`` header, inclusive end as in HTTP — the P2P loader converts hls.js's
exclusive ``byteRangeEndOffset``, ``lib/integration/p2p-loader-generator.js:142-144``).

:class:`Shaper` reproduces the xhr-shaper global the reference's browser tests use to
throttle and inject latency (``test/html/tests.js:6``, ``p2p-loader-generator.js:37``):
``Shaper.maxBandwidth`` is in kbit/s (``inf`` = unshaped) and ``Shaper.minLatency`` in ms.
"""
from __future__ import annotations

import math
import re
import threading
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple


class HttpError(Exception):
    """Error delivered to loaders; the reference expects an object with ``status``
    (``CHANGELOG.md:17-18`` "Expect HttpError instance passed in loadError callback")."""

    def __init__(self, status: int, url: str = "", message: str = "") -> None:
        super().__init__(message or f"HTTP {status} for {url}")
        self.status = status
        self.url = url


@dataclass
class Response:
    status: int
    body: Any              # str (text) or a uint8 view (numpy / torch CPU tensor)
    url: str
    length: int
    source: Any = None     # (origin, resource) for zero-copy device fetches
    offset: int = 0        # byte offset inside the resource for range requests


class Shaper:
    """Process-wide request shaping (xhr-shaper analog)."""

    maxBandwidth: float = math.inf  # kbit/s
    minLatency: float = 0.0         # ms

    @classmethod
    def reset(cls) -> None:
        cls.maxBandwidth = math.inf
        cls.minLatency = 0.0

    @classmethod
    def transfer_ms(cls, nbytes: int) -> float:
        """Wall time a transfer of ``nbytes`` takes under the current shaping."""
        t = float(cls.minLatency)
        if math.isfinite(cls.maxBandwidth) and cls.maxBandwidth > 0:
            t += nbytes * 8.0 / cls.maxBandwidth  # kbit/s == bit/ms
        return t


_registry: Dict[str, Any] = {}
_reg_lock = threading.Lock()
# url -> (origin, path): every fragment URL is resolved at request (size) and again at
# fetch time; the longest-prefix scan is done once per URL.  Cleared on any registry change.
# URL directory (everything up to the last "/") -> (origin, length of its base URL).  Base
# URLs end with "/", so a base is a prefix of a URL iff it is a prefix of the URL's directory:
# every URL of one directory resolves to the same origin, and the cache holds one entry per
# playlist directory instead of one per segment URL.
_resolved: Dict[str, Tuple[Any, int]] = {}
_RESOLVED_MAX = 1 << 12
# bumped on every registry change: callers that cache what a URL resolved to (the swarm
# node's source locators) drop their cache when it moves
_generation = 0


def generation() -> int:
    """Registry generation (changes whenever an origin is (un)registered or cleared)."""
    return _generation


def _bump() -> None:
    global _generation
    _generation += 1


def register_origin(base_url: str, origin: Any) -> None:
    if not base_url.endswith("/"):
        base_url += "/"
    with _reg_lock:
        _registry[base_url] = origin
        _resolved.clear()
        _bump()


def unregister_origin(base_url: str) -> None:
    if not base_url.endswith("/"):
        base_url += "/"
    with _reg_lock:
        _registry.pop(base_url, None)
        _resolved.clear()
        _bump()


def clear_origins() -> None:
    with _reg_lock:
        origins = list(_registry.values())
        _registry.clear()
        _resolved.clear()
        _bump()
    for o in origins:  # network origins own worker threads and staged host buffers
        if getattr(o, "staged_fetch", False):
            o.close()


_network: Optional[Dict[str, Any]] = None  # enable_network() options; None = in-process origins only


def enable_network(on: bool = True, **options: Any) -> None:
    """Let ``http(s)://`` URLs that no registered origin claims resolve to a real CDN: one
    :class:`~.network.HttpOrigin` per scheme://host, created on first use with ``options``
    (``workers``, ``timeout_s``, ``pin_memory`` ...).  ``enable_network(False)`` turns it off
    (origins already created stay registered until :func:`clear_origins`)."""
    global _network
    with _reg_lock:
        _network = dict(options) if on else None
        _resolved.clear()
        _bump()


def network_enabled() -> bool:
    return _network is not None


def _network_origin(url: str) -> Optional[Tuple[str, Any]]:
    if _network is None or not (url.startswith("http://") or url.startswith("https://")):
        return None
    from urllib.parse import urlsplit

    from .network import HttpOrigin

    u = urlsplit(url)
    base = f"{u.scheme}://{u.netloc}/"
    with _reg_lock:
        origin = _registry.get(base)
        if origin is None:
            origin = HttpOrigin(base, register=False, **_network)
            _registry[base] = origin
    return base, origin


def resolve(url: str) -> Tuple[Any, str]:
    """``(origin, path)`` for ``url``: the registered origin with the longest base-URL prefix
    (or, with :func:`enable_network`, the host's :class:`~.network.HttpOrigin`)."""
    d = url[:url.rfind("/") + 1]
    hit = _resolved.get(d)
    if hit is not None:
        return hit[0], url[hit[1]:]
    best = None
    for base, origin in list(_registry.items()):
        if d.startswith(base) and (best is None or len(base) > len(best[0])):
            best = (base, origin)
    if best is None:
        best = _network_origin(url)
    if best is None:
        raise HttpError(0, url, f"no origin serves {url}")  # status 0 = network error
    if len(_resolved) >= _RESOLVED_MAX:
        _resolved.clear()
    _resolved[d] = (best[1], len(best[0]))
    return best[1], url[len(best[0]):]


_RANGE = re.compile(r"bytes=(\d+)-(\d*)")


def parse_range(headers: Optional[Dict[str, str]]) -> Optional[Tuple[int, Optional[int]]]:
    if not headers:
        return None
    v = headers.get("Range") or headers.get("range")
    if not v:
        return None
    m = _RANGE.fullmatch(v.strip())
    if not m:
        raise HttpError(416, "", f"bad range {v!r}")
    start = int(m.group(1))
    end = int(m.group(2)) if m.group(2) else None
    return start, end


def fetch(url: str, headers: Optional[Dict[str, str]] = None, with_credentials: bool = False) -> Response:
    """Synchronous origin fetch (the transfer time is modelled by the caller)."""
    origin, path = resolve(url)
    rng = parse_range(headers)
    return origin.serve(path, url, rng, headers or {}, with_credentials)


def fetch_async(url: str, headers: Optional[Dict[str, str]], with_credentials: bool, loop: Any,
                on_response: Callable[[Response], Any], on_error: Callable[[HttpError], Any]) -> None:
    """:func:`fetch` that never blocks ``loop``: an origin with ``serve_async`` (a network
    origin) runs on its worker pool and the callback is posted back to ``loop``; in-process
    origins answer synchronously (the callback runs before this returns, as before)."""
    try:
        origin, path = resolve(url)
        rng = parse_range(headers)
    except HttpError as e:
        on_error(e)
        return
    serve_async = getattr(origin, "serve_async", None)
    if serve_async is None:
        try:
            resp = origin.serve(path, url, rng, headers or {}, with_credentials)
        except HttpError as e:
            on_error(e)
            return
        on_response(resp)
        return
    loop.hold()

    def done(resp: Optional[Response], err: Optional[HttpError]) -> None:
        try:
            if err is not None:
                loop.call_soon_threadsafe(on_error, err)
            else:
                loop.call_soon_threadsafe(on_response, resp)
        finally:
            loop.release()

    serve_async(path, url, rng, headers or {}, with_credentials, done)


def head(url: str, headers: Optional[Dict[str, str]] = None) -> int:
    """Size of a resource (or of the requested range) without transferring it."""
    origin, path = resolve(url)
    rng = parse_range(headers)
    return origin.size(path, url, rng)


def request_log() -> List[Tuple[str, str]]:
    out = []
    for base, origin in list(_registry.items()):
        out.extend((base, p) for p in getattr(origin, "requests", []))
    return out
