"""Network origins: a real HTTP(S) CDN behind the swarm.

The reference's agent falls through to XHRs against the CDN for everything the swarm
cannot serve (``lib/integration/p2p-loader-generator.js:103-104``); the hls.js loaders fetch
playlists and keys over XHR.  The in-process origins (:mod:`.origin`) model that CDN as
pinned host memory for benches and tests; :class:`HttpOrigin` is the production path: the
same origin interface over a real ``http://`` / ``https://`` base URL.

Design for the swarm (the host side of the CDN path, not a browser's):

* **Staged fetches.**  A media segment is never fetched on the event-loop thread.  The
  swarm node asks the origin to *stage* it (:meth:`HttpOrigin.stage`): a worker thread runs
  the GET (keep-alive connection per thread and host, ``Range`` honoured) and reads the body
  straight into a pinned host buffer (``readinto``, no intermediate copy).  The completion
  comes back to the node's loop (``call_soon_threadsafe``); from then on the segment is a
  pinned-host resource like an in-process one, and the round's CDN phase moves it into HBM
  with the same merged ``hipMemcpyAsync``.  The staged copy is released once that DMA has
  completed.
* **One download per segment per swarm.**  The node only stages what the round planner
  assigns it (``plan_round``'s stage rows): with CDN de-duplication one wanting rank
  downloads and forwards to the others over RCCL, so the network carries each segment once.
* Playlists and keys (small, text or 16 bytes) go through :meth:`HttpOrigin.serve_async` on
  the same pool; the default loader delivers them on its loop.

``http.enable_network()`` (or ``p2pConfig.gpuSwarm.network``) makes every ``http(s)://``
URL that no in-process origin claims resolve to a per-host :class:`HttpOrigin`.
"""
from __future__ import annotations

import concurrent.futures as cf
import http.client
import logging
import re
import ssl
import threading
import urllib.parse
from typing import Any, Callable, Dict, Optional, Tuple

import torch

from .http import HttpError, Response, register_origin

log = logging.getLogger("hlsjs_p2p_wrapper_amd.network")

_TEXT_SUFFIXES = (".m3u8", ".m3u", ".txt", ".xml", ".json")
Range = Optional[Tuple[int, Optional[int]]]
_CONTENT_RANGE = re.compile(r"bytes\s+(\d+)-(\d+)/(\d+|\*)$")


def _check_content_range(value: Optional[str], rng: Tuple[int, Optional[int]], url: str) -> None:
    """A 206 must carry the range that was asked for (``Content-Range: bytes s-e/total``)."""
    if not value:
        return  # some servers omit it; Content-Length still bounds the body
    m = _CONTENT_RANGE.match(value.strip())
    if m is None:
        raise HttpError(502, url, f"malformed Content-Range {value!r}")
    s, e = int(m.group(1)), int(m.group(2))
    want_s, want_e = rng
    if s != want_s or (want_e is not None and e > want_e):
        raise HttpError(502, url, f"Content-Range {value!r} does not match the requested bytes={want_s}-"
                                  + ("" if want_e is None else str(want_e)))


def _slice_range(body: Any, n: int, rng: Tuple[int, Optional[int]], pin: bool, url: str) -> Tuple[Any, int]:
    """Cut the requested inclusive range out of a full-resource (200) body."""
    s, e = rng
    e = n - 1 if e is None else min(e, n - 1)
    if s >= n:
        raise HttpError(416, url, f"range start {s} beyond the {n}-byte resource")
    k = max(0, e - s + 1)
    if isinstance(body, str):
        return body.encode()[s:s + k].decode("utf-8", errors="replace"), k
    out = torch.empty(max(k, 1), dtype=torch.uint8, pin_memory=pin)
    out[:k] = body[s:s + k]
    return out, k


class HttpOrigin:
    """An HTTP(S) CDN under ``base_url`` (origin interface of :mod:`.origin`, plus staging)."""

    staged_fetch = True  # SwarmNode: media segments must be staged before a round's DMA

    def __init__(self, base_url: str, workers: int = 8, timeout_s: float = 20.0, max_redirects: int = 5,
                 pin_memory: Optional[bool] = None, register: bool = True,
                 ssl_context: Optional[ssl.SSLContext] = None) -> None:
        self.base_url = base_url if base_url.endswith("/") else base_url + "/"
        u = urllib.parse.urlsplit(self.base_url)
        if u.scheme not in ("http", "https") or not u.netloc:
            raise ValueError(f"HttpOrigin needs an http(s):// base URL, got {base_url!r}")
        self.timeout_s = float(timeout_s)
        self.max_redirects = int(max_redirects)
        self.pin_memory = torch.cuda.is_available() if pin_memory is None else bool(pin_memory)
        self._ssl = ssl_context
        self._pool = cf.ThreadPoolExecutor(max_workers=max(1, int(workers)), thread_name_prefix="hlsp2p-http")
        self._tls = threading.local()  # per worker thread: {(scheme, netloc): connection}
        self._lock = threading.Lock()
        self._staged: Dict[Tuple[str, Range], Tuple[torch.Tensor, int]] = {}
        self._inflight: Dict[Tuple[str, Range], cf.Future] = {}
        self.requests = 0
        self.bytes_in = 0
        self.errors = 0
        self.closed = False
        if register:
            register_origin(self.base_url, self)

    # ------------------------------------------------------------------ transport
    def _conn(self, scheme: str, netloc: str, fresh: bool = False) -> http.client.HTTPConnection:
        conns = getattr(self._tls, "conns", None)
        if conns is None:
            conns = self._tls.conns = {}
        key = (scheme, netloc)
        c = conns.get(key)
        if c is None or fresh:
            if c is not None:
                c.close()
            if scheme == "https":
                c = http.client.HTTPSConnection(netloc, timeout=self.timeout_s,
                                                context=self._ssl or ssl.create_default_context())
            else:
                c = http.client.HTTPConnection(netloc, timeout=self.timeout_s)
            conns[key] = c
        return c

    def _get(self, url: str, headers: Dict[str, str], rng: Range, head: bool = False):
        """GET (or HEAD) with redirects; returns ``(response, url)`` with the body unread."""
        hdrs = {k: v for k, v in (headers or {}).items() if k.lower() != "range"}
        if rng is not None:
            s, e = rng
            hdrs["Range"] = f"bytes={s}-" + ("" if e is None else str(e))
        for _ in range(self.max_redirects + 1):
            u = urllib.parse.urlsplit(url)
            target = u.path or "/"
            if u.query:
                target += "?" + u.query
            for attempt in (0, 1):  # a keep-alive connection the server closed: reconnect once
                c = self._conn(u.scheme, u.netloc, fresh=attempt > 0)
                try:
                    c.request("HEAD" if head else "GET", target, headers=hdrs)
                    resp = c.getresponse()
                    break
                except (http.client.HTTPException, ConnectionError, OSError):
                    if attempt:
                        raise
            if resp.status in (301, 302, 303, 307, 308):
                loc = resp.getheader("Location")
                resp.read()
                if not loc:
                    raise HttpError(resp.status, url, "redirect without Location")
                url = urllib.parse.urljoin(url, loc)
                continue
            return resp, url
        raise HttpError(310, url, "too many redirects")

    def _fetch(self, url: str, headers: Dict[str, str], rng: Range, binary: bool) -> Tuple[int, Any, int]:
        """``(status, body, length)``: body is a (pinned when ``pin_memory``) uint8 CPU tensor
        for binary resources, ``str`` for text ones.  HTTP errors raise :class:`HttpError`."""
        try:
            resp, url = self._get(url, headers, rng)
        except HttpError:
            with self._lock:
                self.errors += 1
            raise
        except (http.client.HTTPException, OSError) as e:
            with self._lock:
                self.errors += 1
            raise HttpError(0, url, f"network error: {e}") from e  # status 0, as XHR reports it
        status = resp.status
        if status >= 400:
            resp.read()
            with self._lock:
                self.errors += 1
            raise HttpError(status, url)
        n = resp.getheader("Content-Length")
        if rng is not None:
            if status == 206:
                _check_content_range(resp.getheader("Content-Range"), rng, url)
            elif status != 200:  # a range request answered 204 / 2xx without the body part
                resp.read()
                with self._lock:
                    self.errors += 1
                raise HttpError(status, url, "unexpected status for a Range request")
        if binary and n is not None:
            n = int(n)
            body = torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=self.pin_memory)
            mv = memoryview(body.numpy())[:n]
            got = 0
            while got < n:
                k = resp.readinto(mv[got:])
                if not k:
                    raise HttpError(0, url, f"connection closed after {got} of {n} bytes")
                got += k
        else:
            raw = resp.read()
            n = len(raw)
            if binary:
                body = torch.empty(max(n, 1), dtype=torch.uint8, pin_memory=self.pin_memory)
                if n:
                    body[:n] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
            else:
                body = raw.decode("utf-8", errors="replace")
        if rng is not None and status == 200:
            # the CDN ignored the Range header and sent the whole resource: keep only the
            # requested part (the node must stage, DMA and deliver exactly that range)
            body, n = _slice_range(body, n, rng, self.pin_memory, url)
        with self._lock:
            self.requests += 1
            self.bytes_in += n
        return status, body, n

    @staticmethod
    def _is_text(path: str) -> bool:
        return path.split("?", 1)[0].lower().endswith(_TEXT_SUFFIXES)

    # ------------------------------------------------------------------ staging (media)
    def stage(self, path: str, url: str, rng: Range, headers: Dict[str, str],
              on_done: Callable[[Optional[int], Optional[HttpError]], None]) -> None:
        """Fetch ``url`` (``rng``: inclusive byte range) into pinned host memory on a worker
        thread; ``on_done(length, None)`` or ``on_done(None, error)`` runs ON THAT THREAD (the
        caller hops to its loop).  Concurrent stages of one resource share the download."""
        key = (path, rng)
        with self._lock:
            hit = self._staged.get(key)
            fut = self._inflight.get(key)
            if hit is None and fut is None:
                try:
                    fut = self._pool.submit(self._stage_job, key, url, dict(headers or {}))
                except RuntimeError:  # submit after close(): fail the stage instead of dropping it
                    fut = None
                else:
                    self._inflight[key] = fut
        if hit is None and fut is None:
            on_done(None, HttpError(0, url, "cancelled: origin closed"))
            return
        if hit is not None:
            on_done(hit[1], None)
            return

        def _cb(f: cf.Future) -> None:
            if f.cancelled():  # the pool shut down first: still complete the caller's hold
                on_done(None, HttpError(0, url, "cancelled: origin closed"))
                return
            err = f.exception()
            if err is None:
                on_done(f.result(), None)
            else:
                on_done(None, err if isinstance(err, HttpError) else HttpError(0, url, str(err)))

        fut.add_done_callback(_cb)

    def _stage_job(self, key, url: str, headers: Dict[str, str]) -> int:
        try:
            status, body, n = self._fetch(url, headers, key[1], binary=True)
            with self._lock:
                self._staged[key] = (body, n)
            return n
        finally:
            with self._lock:
                self._inflight.pop(key, None)

    def staged_size(self, path: str, rng: Range = None) -> Optional[int]:
        """Length of a staged resource, ``None`` when it is not staged."""
        with self._lock:
            hit = self._staged.get((path, rng))
        return None if hit is None else hit[1]

    def resource_range(self, path: str, rng: Range = None):
        """``(pinned tensor, offset, length, crc)`` of a staged resource (crc unused: 0)."""
        with self._lock:
            hit = self._staged.get((path, rng))
        if hit is None:
            raise HttpError(503, path, "resource is not staged")
        return hit[0], 0, hit[1], 0

    def release(self, path: str, rng: Range = None) -> None:
        """Drop a staged copy (after its DMA into HBM has completed)."""
        with self._lock:
            self._staged.pop((path, rng), None)

    @property
    def staged_bytes(self) -> int:
        """Host bytes held by staged resources."""
        with self._lock:
            return sum(n for _, n in self._staged.values())

    # ------------------------------------------------------------------ origin interface
    def resource(self, path: str):
        """The staged full resource (origin interface of the in-process origins)."""
        return self.resource_range(path, None)

    def size(self, path: str, url: str = "", rng: Range = None) -> int:
        """Length of a resource: the staged copy's, else a ``HEAD`` request (blocking)."""
        n = self.staged_size(path, rng)
        if n is not None:
            return n
        resp, _ = self._get(url or self.base_url + path, {}, rng, head=True)
        resp.read()
        if resp.status >= 400:
            raise HttpError(resp.status, url)
        return int(resp.getheader("Content-Length") or 0)

    def should_corrupt(self, path: str) -> bool:
        """Fault-injection hook of the in-process origins: never for a real CDN."""
        return False

    def serve(self, path: str, url: str, rng: Range, headers: Dict[str, str], with_credentials: bool) -> Response:
        """Blocking fetch (playlists, keys; the loaders prefer :meth:`serve_async`)."""
        status, body, n = self._fetch(url, headers, rng, binary=not self._is_text(path))
        return Response(status, body, url, n)

    def serve_async(self, path: str, url: str, rng: Range, headers: Dict[str, str], with_credentials: bool,
                    on_done: Callable[[Optional[Response], Optional[HttpError]], None]) -> None:
        """:meth:`serve` on a worker thread; ``on_done(response, error)`` runs on that thread."""
        def job():
            try:
                on_done(self.serve(path, url, rng, headers, with_credentials), None)
            except HttpError as e:
                on_done(None, e)
            except Exception as e:  # noqa: BLE001 - surfaced to the loader as a network error
                on_done(None, HttpError(0, url, str(e)))

        try:
            fut = self._pool.submit(job)
        except RuntimeError:  # submit after close()
            on_done(None, HttpError(0, url, "cancelled: origin closed"))
            return
        # a job cancelled by close() never runs: answer it here so the caller's hold is released
        fut.add_done_callback(lambda f: on_done(None, HttpError(0, url, "cancelled: origin closed"))
                              if f.cancelled() else None)

    def close(self) -> None:
        """Stop the worker pool and drop every staged copy."""
        self.closed = True
        self._pool.shutdown(wait=False, cancel_futures=True)
        with self._lock:
            self._staged.clear()

    def __repr__(self) -> str:
        return f"HttpOrigin({self.base_url!r}, requests={self.requests}, bytes_in={self.bytes_in})"
