"""Fleet: player processes in front of one GPU's swarm node.

One MI355X is one swarm peer (one process, one ``SwarmNode``, the RCCL rank).  The players
it serves need not share that process: the per-fragment host path of the hls.js-compatible
engine (stream controller, loaders, ABR, events, ~13 us of Python per fragment) is what
bounds a node's segment rate once P2P takes the CDN load off PCIe (``profiles/r2_cyprof``).
With a fleet, ``W`` player processes run that path in parallel; the GPU process keeps only
the node side (rounds, CDN DMA, RCCL, CRC) and the transmux, which it runs in batches.
The player processes never touch the GPU (``HIP_VISIBLE_DEVICES`` is empty for them).

The rank side is columnar end to end: requests arrive as arrays, join the node's native
want table as 64-bit tokens (``player << 40 | rid``) through ``SwarmNode.request_batch``,
come back from the round as delivery columns (token, source, bytes, timings, arena
offset), feed the batched GPU transmux as columns, and leave as answer columns.  No
per-fragment Python object exists on the rank: the ``getSegment(reqInfo, callbacks,
segmentView)`` hop of ``lib/integration/p2p-loader-generator.js:133-165`` is one row.

Protocol (one ``multiprocessing`` pipe per player process, batched per loop iteration):

* player -> node: ``("req", cols, handled)`` with ``cols`` = ``(rid int64[n], key int64[n, 4],
  urls, headers or None, key_id int32[n] (-1: clear), iv uint8[n, 16], new_keys {id: 16 B})``
  -- the fragment requests as ``PeerAgent.getSegment`` issues them plus the AES-128 key id /
  IV the GPU transmux needs (each distinct key crosses the pipe once);
  ``("abort", [rid, ...])``; ``("evict", swarm, sn)``; ``("flags", down, up)`` (this
  player's ``p2pDownloadOn`` / ``p2pUploadOn``); ``("mark", tag, counters)`` (bench window
  markers); ``("payload", on)``; ``("fetch", id, keys int64[n, 4])`` (an answer chunk's
  bytes on demand, answered by ``("bytes", id, [array or None per key])``); ``("bye",)``.
* node -> player: ``("done", chunks, errors, swarm_state)``.  Each chunk holds the fragments
  of one transmux batch as columns: ``rid``, ``source`` code (:data:`SOURCES`), ``nbytes``,
  ``cdn_ms``, ``p2p_ms``, ``plain`` bytes, ``has_row``, the transmux info ``rows`` ``[n,
  INFO_WORDS]``, and, for a player that asked for payloads, ``(shm name, offsets, lengths)``
  of the fragments' bytes.  ``errors``: ``[(rid, status), ...]``.

Player side, :class:`RemoteNode` stands in for the ``SwarmNode`` behind the unchanged
``PeerAgent`` (``gpuSwarm.backend = "remote"``): the loader's ``onSuccess`` gets a
:class:`RemoteSegment` whose ``transmux_result`` the stream controller uses instead of
transmuxing itself (it holds the info row: durations, PTS, ES byte counts).  Its bytes (the
reference ``onSuccess`` contract ``{currentTarget: {response: ArrayBuffer}}``,
``lib/integration/p2p-loader-generator.js:92-99``) are ``RemoteSegment.data()``: fetched from
the rank's HBM cache on demand by default (nothing moves for a player that does not read
them), or, with ``gpuSwarm.fleetPayload``, copied device-to-host for every fragment into a
shared-memory ring the player maps (one batched D2H per transmux batch).
"""
from __future__ import annotations

import collections
import logging
import os
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..net.http import HttpError

log = logging.getLogger("hlsjs_p2p_wrapper_amd.fleet")

SOURCES = ("cdn", "p2p", "cache")  # source codes of the answer columns (agent/node.py SRC_*)
_SOURCE_CODE = {s: i for i, s in enumerate(SOURCES)}
TOKEN_SHIFT = 40  # token = player << TOKEN_SHIFT | rid
_RID_MASK = (1 << TOKEN_SHIFT) - 1
_RING = 1 << 16  # per-player request slots (rid % _RING): far above the fragments in flight


# ============================================================================ player side
class RemoteSegment:
    """``onSuccess`` payload of a remotely served fragment: its size, its transmux result and
    its bytes (:meth:`data`) -- the reference hands the player the response bytes
    (``lib/integration/p2p-loader-generator.js:92-99``)."""

    __slots__ = ("nbytes", "transmux_result", "_bytes", "_src")

    def __init__(self, nbytes: int, transmux_result: Any, data: Any = None, src: Any = None) -> None:
        self.nbytes = nbytes
        self.transmux_result = transmux_result
        self._bytes = data
        self._src = src  # (_BatchFetch, index): where data() fetches the bytes on demand

    def numel(self) -> int:
        return self.nbytes

    def __len__(self) -> int:
        return self.nbytes

    def data(self) -> Optional[np.ndarray]:
        """The fragment's bytes as a read-only ``uint8`` array.

        With ``gpuSwarm.fleetPayload`` they arrived with the answer batch: a zero-copy view into
        the rank's shared payload ring, valid while the player handles the batch (the
        ``onSuccess`` callbacks) -- ``.copy()`` what must outlive it.  Otherwise they are
        fetched on demand, the first time this is called: the rank copies the segment out of
        its HBM cache (one D2H) and sends it over the player's pipe, so a player that never
        reads bytes pays nothing and one that reads some pays per segment read.  None when
        the rank no longer holds the segment (evicted from its cache)."""
        if self._bytes is None and self._src is not None:
            batch, i = self._src
            self._src = None
            self._bytes = batch.get(i)
        return self._bytes


class _BatchFetch:
    """The keys of one answer chunk whose bytes were not shipped with it: the first
    ``RemoteSegment.data()`` of the chunk fetches every one of them in ONE request (one
    gather + D2H on the rank, one pipe message), so a player that reads all bytes pays a
    round trip per batch, not per fragment; one that reads none pays nothing."""

    __slots__ = ("node", "keys", "data")

    def __init__(self, node: "RemoteNode") -> None:
        self.node = node
        self.keys: List[Tuple[int, int, int, int]] = []
        self.data: Optional[list] = None

    def get(self, i: int) -> Optional[np.ndarray]:
        if self.data is None:
            self.data = self.node.fetch_bytes_many(self.keys)
        return self.data[i]


class RemoteResult(dict):
    """Transmux result of a remote fragment (``status``, ``info``, ``plain_bytes``, ``error``);
    the elementary-stream bytes stay in the GPU process, so ``video`` / ``audio`` / ``id3``
    are empty."""

    __slots__ = ()

    def __missing__(self, key):
        if key in ("video", "audio", "id3"):
            import torch

            v = torch.empty(0, dtype=torch.uint8)
            self[key] = v
            return v
        raise KeyError(key)


class _RemoteRequest:
    __slots__ = ("node", "rid", "key", "callbacks", "agent", "aborted", "done")

    def __init__(self, node, rid, key, callbacks, agent) -> None:
        self.node = node
        self.rid = rid
        self.key = key
        self.callbacks = callbacks
        self.agent = agent
        self.aborted = False
        self.done = False

    def abort(self) -> None:
        if not self.aborted and not self.done:
            self.aborted = True
            node = self.node
            node._aborts.append(self.rid)
            # the node never answers an aborted request: forget it here (a late answer that
            # crossed the abort finds no pending entry and is dropped)
            if node._pending.pop(self.rid, None) is not None:
                node.inflight -= 1


class _RemoteStore:
    def __init__(self, node: "RemoteNode") -> None:
        self._node = node

    def evict_below(self, swarm: int, sn: int) -> int:
        self._node._out.append(("evict", int(swarm), int(sn)))
        return 0


class _ShmRing:
    """Player side of the payload ring: the rank's shared-memory segment, mapped once."""

    def __init__(self) -> None:
        self.name = None
        self.shm = None
        self.buf: Optional[np.ndarray] = None

    def view(self, name: str) -> np.ndarray:
        if name != self.name:
            from multiprocessing import shared_memory

            self.close()
            self.shm = shared_memory.SharedMemory(name=name, create=False)
            self.buf = np.ndarray((self.shm.size,), dtype=np.uint8, buffer=self.shm.buf)
            self.name = name
        return self.buf

    def close(self) -> None:
        if self.shm is not None:
            self.buf = None
            try:
                self.shm.close()
            except BufferError:  # a payload view is still referenced: the OS unmaps at exit
                pass
            self.shm = None
            self.name = None


class RemoteNode:
    """The ``SwarmNode`` surface ``PeerAgent`` uses, served by a node in another process."""

    def __init__(self, conn: Any, world: int = 1, rank: int = 0, payload: bool = False) -> None:
        self.conn = conn
        self.world = world
        self.rank = rank
        self.closed = False
        self.online = True
        self.peer_online = np.ones(world, dtype=bool)
        self._down, self._up = True, True
        self.stats: Dict[str, int] = {"cdn": 0, "p2p": 0, "upload": 0, "cache": 0, "segments": 0}
        self.swarm_stats = {"cdn": 0, "p2p": 0, "upload": 0}
        self.store = _RemoteStore(self)
        self._agents: List[Any] = []
        self._pending: Dict[int, _RemoteRequest] = {}
        # request columns accumulated until the next flush
        self._rid: List[int] = []
        self._key: List[Tuple[int, int, int, int]] = []
        self._url: List[str] = []
        self._hdr: List[Optional[Dict[str, str]]] = []
        self._kid: List[int] = []
        self._iv: List[bytes] = []
        self._key_ids: Dict[bytes, int] = {}
        self._new_keys: Dict[int, bytes] = {}
        self._aborts: List[int] = []
        self._out: List[tuple] = []
        self._next = 0
        self.inflight = 0
        self.control: List[tuple] = []
        self.batches = 0  # answer batches handled (reported to the node, which paces on it)
        self._reported = 0
        self._ring = _ShmRing()
        self.payload_revoked = False
        self._stash: List[tuple] = []  # messages read while waiting for fetched bytes
        self._fetch_id = 0
        self.bytes_fetched = 0
        if payload:
            self._out.append(("payload", True))

    # -------------------------------------------------------------- SwarmNode surface
    def attach(self, agent: Any) -> None:
        """Register the player's PeerAgent (as on a SwarmNode)."""
        self._agents.append(agent)

    def detach(self, agent: Any) -> None:
        """Unregister an agent."""
        if agent in self._agents:
            self._agents.remove(agent)

    def session_flags(self, session: Any) -> Tuple[bool, bool]:
        """``(download, upload)`` of this player's session."""
        return self._down, self._up

    def set_session_flags(self, session: Any, download: bool, upload: bool) -> None:
        """This player's ``p2pDownloadOn`` / ``p2pUploadOn``, forwarded to the node (which
        applies them to this player's requests only)."""
        self._down, self._up = bool(download), bool(upload)
        self._out.append(("flags", self._down, self._up))

    @property
    def download_on(self) -> bool:
        """Read / write: P2P download of this player's session."""
        return self._down

    @download_on.setter
    def download_on(self, on: bool) -> None:
        self.set_session_flags(None, on, self._up)

    @property
    def upload_on(self) -> bool:
        """Read / write: P2P upload of this player's session."""
        return self._up

    @upload_on.setter
    def upload_on(self, on: bool) -> None:
        self.set_session_flags(None, self._down, on)

    def request(self, key, url: str, headers, callbacks: Any, agent: Any = None, view: Any = None):
        """Queue a fragment request for the node (sent at the next flush); ``view`` finds the
        fragment's AES key / IV for the GPU transmux.  Returns the handle (``abort()``)."""
        rid = self._next
        self._next += 1
        req = _RemoteRequest(self, rid, key, callbacks, agent)
        kid, iv = -1, b"\0" * 16
        if agent is not None and view is not None:  # the GPU transmux needs the AES key / IV
            frag = agent.mediaMap.fragment(view)
            if frag is not None:
                dd = frag.decryptdata
                if dd is not None and dd.method == "AES-128" and dd.key is not None:
                    kb = bytes(dd.key)
                    kid = self._key_ids.get(kb)
                    if kid is None:
                        kid = self._key_ids[kb] = len(self._key_ids)
                        self._new_keys[kid] = kb
                    iv = bytes(frag.iv_for_decrypt())
        self._pending[rid] = req
        self._rid.append(rid)
        self._key.append(tuple(int(k) for k in key))
        self._url.append(url)
        self._hdr.append(dict(headers) if headers else None)
        self._kid.append(kid)
        self._iv.append(iv)
        self.inflight += 1
        return req

    def prefetch(self, key, url: str, headers=None) -> bool:
        """Agent-driven prefetch is a single-process feature: nothing is issued."""
        return False

    def swarm_offload_ratio(self) -> float:
        """P2P / (P2P + CDN) bytes over the whole swarm, as last reported by the node."""
        c, p = self.swarm_stats["cdn"], self.swarm_stats["p2p"]
        return p / (p + c) if (p + c) else 0.0

    # -------------------------------------------------------------- transport
    def _columns(self) -> tuple:
        n = len(self._rid)
        hdr = self._hdr if any(h is not None for h in self._hdr) else None
        cols = (np.asarray(self._rid, dtype=np.int64), np.asarray(self._key, dtype=np.int64).reshape(n, 4),
                self._url, hdr, np.asarray(self._kid, dtype=np.int32),
                np.frombuffer(b"".join(self._iv), dtype=np.uint8).reshape(n, 16), self._new_keys)
        self._rid, self._key, self._url, self._hdr, self._kid, self._iv = [], [], [], [], [], []
        self._new_keys = {}
        return cols

    def flush(self) -> None:
        """Send everything queued since the last flush (one message per kind), with the count
        of answer batches handled so far (the node paces its rounds on it).  The agents'
        per-round planning (live buffer negotiation, live-window eviction) runs first, as it
        does before a local node's round."""
        for agent in self._agents:
            hook = getattr(agent, "before_round", None)
            if hook is not None:
                hook()
        for m in self._out:  # flags / payload mode first: they apply to the requests below
            self.conn.send(m)
        self._out = []
        if self._rid:
            self.conn.send(("req", self._columns(), self.batches))
            self._reported = self.batches
        elif self.batches != self._reported:
            self.conn.send(("ack", self.batches))
            self._reported = self.batches
        if self._aborts:
            self.conn.send(("abort", self._aborts))
            self._aborts = []

    def invalidate(self, keys) -> int:
        """Ask the rank to drop its cached copies of ``keys`` (int64[n, 4]) and take them from
        the CDN next time (:meth:`SwarmNode.invalidate`); sent before the next requests."""
        self._out.append(("invalidate", np.asarray(keys, dtype=np.int64).reshape(-1, 4)))
        return 0

    def fetch_bytes_many(self, keys) -> list:
        """Segments' bytes from the node (:meth:`RemoteSegment.data` on demand): a ``("fetch",
        id, keys)`` request, answered by ``("bytes", id, [array or None per key])``.  Other
        messages that arrive meanwhile are kept for :meth:`poll` (this runs inside an
        ``onSuccess`` callback, i.e. inside the delivery of an earlier message)."""
        self._fetch_id += 1
        fid = self._fetch_id
        self.conn.send(("fetch", fid, np.asarray(keys, dtype=np.int64).reshape(-1, 4)))
        while True:
            msg = self.conn.recv()
            if msg[0] == "bytes" and msg[1] == fid:
                out = msg[2]
                for d in out:
                    if d is not None:
                        d.flags.writeable = False
                        self.bytes_fetched += len(d)
                return out
            self._stash.append(msg)

    def poll(self, timeout: float = 0.0) -> int:
        """Deliver every answer that has arrived (waiting up to ``timeout`` s for the first)."""
        n = 0
        conn = self.conn
        stash = self._stash
        if not stash and not conn.poll(timeout):
            return 0
        while True:
            msg = stash.pop(0) if stash else conn.recv()
            if msg[0] == "done":
                for chunk in msg[1]:
                    n += self._deliver(chunk)
                if msg[2]:
                    self._fail(msg[2])
                self.batches += 1
                st = msg[3]
                if st is not None:
                    self.stats["upload"] = st["upload"]
                    self.swarm_stats = st["swarm"]
                    self.peer_online = np.asarray(st["online"], dtype=bool)
            elif msg[0] == "revoke":  # the node stopped this player's payloads (it stalled on its acks)
                log.warning("fleet player (rank %d): the node stopped sending fragment bytes to this player; "
                            "onSuccess payloads arrive without data from now on", self.rank)
                self.payload_revoked = True
            else:  # a control message ("mark", "stop"): the player acts on it before reading on
                self.control.append(msg)
                return n
            if not stash and not conn.poll(0):
                return n

    def _fail(self, errors: List[Tuple[int, int]]) -> None:
        pending = self._pending
        for rid, status in errors:
            req = pending.pop(rid, None)
            if req is None:
                continue
            self.inflight -= 1
            if req.aborted:
                continue
            req.done = True
            cb = req.callbacks
            on_error = cb.get("onError") if isinstance(cb, dict) else getattr(cb, "onError", None)
            if on_error is not None:
                on_error(HttpError(status, ""))

    def _deliver(self, chunk: tuple) -> int:
        from ..player.transmux import InfoRow

        rid_a, src_a, nbytes_a, cdn_a, p2p_a, plain_a, has_a, rows_a = chunk[:8]
        payload = chunk[8] if len(chunk) > 8 else None
        buf = poff = None
        lazy = None
        if payload is not None:
            buf = self._ring.view(payload[0])
            poff = payload[1].tolist()
        pending = self._pending
        if payload is None:  # this chunk's bytes, fetched together on the first data()
            lazy = _BatchFetch(self)
            gone = (0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF)  # an answer nobody waits for
            lazy.keys = [pending[r].key if r in pending else gone for r in rid_a.tolist()]
        stats = self.stats
        n = 0
        for i, (rid, code, nbytes, cdn_ms, p2p_ms, plain, has, info) in enumerate(zip(
                rid_a.tolist(), src_a.tolist(), nbytes_a.tolist(), cdn_a.tolist(), p2p_a.tolist(),
                plain_a.tolist(), has_a.tolist(), rows_a.tolist())):
            req = pending.pop(rid, None)
            if req is None:
                continue
            self.inflight -= 1
            if req.aborted:
                continue
            req.done = True
            cb = req.callbacks
            source = SOURCES[code]
            stats[source] = stats.get(source, 0) + nbytes
            stats["segments"] += 1
            if req.agent is not None:
                req.agent._account(source, nbytes)
            if isinstance(cb, dict):
                on_progress, on_success = cb.get("onProgress"), cb.get("onSuccess")
            else:
                on_progress, on_success = getattr(cb, "onProgress", None), getattr(cb, "onSuccess", None)
            p2p = code != 0
            if on_progress is not None:
                on_progress({"cdnDownloaded": 0 if p2p else nbytes, "p2pDownloaded": nbytes if p2p else 0,
                             "cdnDuration": 0.0 if p2p else cdn_ms, "p2pDuration": p2p_ms if p2p else 0.0})
            if req.aborted or on_success is None:
                continue
            if not has:
                info = None
            r = RemoteResult(status=int(info[0]) if info else -1, info=InfoRow(info), plain_bytes=plain)
            if plain < 0:
                r["error"] = ValueError("decryption failed (bad PKCS#7 padding)")
            data = None
            if buf is not None:  # zero-copy: valid while this batch is handled (see RemoteSegment.data)
                data = buf[poff[i]:poff[i] + nbytes]
                data.flags.writeable = False
            on_success(RemoteSegment(nbytes, r, data, None if lazy is None else (lazy, i)))
            n += 1
        return n

    def close(self) -> None:
        """Flush and tell the node this player is leaving."""
        if not self.closed:
            self.closed = True
            try:
                self.flush()
                self.conn.send(("bye",))
            except (OSError, EOFError, BrokenPipeError):
                pass
            self._ring.close()


# ============================================================================ node side
class _Queue:
    """One player's admitted-later requests: column chunks consumed front to back."""

    __slots__ = ("chunks", "pos", "n")

    def __init__(self) -> None:
        self.chunks: List[tuple] = []  # (rid, key, urls, headers, force)
        self.pos = 0  # rows of chunks[0] already taken
        self.n = 0

    def push(self, rid, key, urls, headers, force) -> None:
        self.chunks.append((rid, key, urls, headers, force))
        self.n += len(rid)

    def take(self, k: int):
        """Up to ``k`` rows as ``(rid, key, urls, headers, force)`` (None when empty)."""
        if not self.n or k <= 0:
            return None
        parts = []
        while k > 0 and self.chunks:
            rid, key, urls, hdr, force = self.chunks[0]
            a = self.pos
            b = min(len(rid), a + k)
            parts.append((rid[a:b], key[a:b], urls[a:b], None if hdr is None else hdr[a:b], force[a:b]))
            k -= b - a
            self.n -= b - a
            if b == len(rid):
                self.chunks.pop(0)
                self.pos = 0
            else:
                self.pos = b
        if len(parts) == 1:
            return parts[0]
        hdr = None
        if any(p[3] is not None for p in parts):
            hdr = [h for p in parts for h in (p[3] if p[3] is not None else [None] * len(p[0]))]
        return (np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]),
                [u for p in parts for u in p[2]], hdr, np.concatenate([p[4] for p in parts]))

    def drop(self, rids: set) -> None:
        """Remove not-yet-admitted requests (aborted by their player)."""
        out = []
        for i, (rid, key, urls, hdr, force) in enumerate(self.chunks):
            a = self.pos if i == 0 else 0
            keep = ~np.isin(rid[a:], np.fromiter(rids, dtype=np.int64, count=len(rids)))
            idx = np.flatnonzero(keep) + a
            if len(idx):
                out.append((rid[idx], key[idx], [urls[j] for j in idx.tolist()],
                            None if hdr is None else [hdr[j] for j in idx.tolist()], force[idx]))
        self.chunks = out
        self.pos = 0
        self.n = sum(len(c[0]) for c in out)


class _PayloadRing:
    """Rank side of the payload ring: a shared-memory segment the fragments' bytes go to for
    players that asked for them.  On a GPU node the segment is registered with HIP (pinned),
    so one asynchronous D2H per transmux batch lands the bytes where the players read them --
    no host copy.  Regions are handed out in FIFO order; a region is reused only after every
    player it was sent to has acknowledged that answer batch (players read their fragments as
    zero-copy views while they handle the batch).

    The segment's pages are reserved up front (``posix_fallocate``: a /dev/shm too small for
    it fails here with a clear error instead of a SIGBUS on first touch), and a failed HIP
    registration leaves the ring unpinned: the rank then stages each batch through a pinned
    bounce buffer and copies it in on the host (``pinned`` False)."""

    def __init__(self, nbytes: int, pin: bool = False) -> None:
        from multiprocessing import shared_memory

        self.shm = shared_memory.SharedMemory(create=True, size=nbytes)
        try:
            fd = getattr(self.shm, "_fd", -1)
            if fd >= 0:
                os.posix_fallocate(fd, 0, nbytes)
        except OSError as e:
            self.shm.close()
            self.shm.unlink()
            raise RuntimeError(f"cannot reserve a {nbytes}-byte payload ring in /dev/shm ({e}); lower "
                               "HLSP2P_FLEET_PAYLOAD_BYTES or the fragments in flight") from e
        self.cap = nbytes
        self.buf = np.ndarray((nbytes,), dtype=np.uint8, buffer=self.shm.buf)
        self.head = 0
        self.wraps = 0
        self.live: "collections.deque" = collections.deque()  # [start, end, {player: batch no} | None]
        self.tensor = None
        self.pinned = False
        if pin and os.environ.get("HLSP2P_FLEET_RING_PIN", "1") == "0":  # test hook: the fallback path
            pin = False
        if pin:
            import torch

            err = torch._C._cudart.cudaHostRegister(self.buf.ctypes.data, nbytes, 0)
            if int(err) == 0:
                self.pinned = True
                self.tensor = torch.from_numpy(self.buf)
            else:
                log.warning("hipHostRegister of the %d-byte payload ring failed (%s): staging payloads through a "
                            "pinned bounce buffer instead", nbytes, err)

    def release_done(self, acked) -> None:
        """Drop the oldest regions whose players have all acknowledged them (no waiting)."""
        while self.live and self.live[0][2] is not None and acked(self.live[0][2]):
            self.live.popleft()

    def try_place(self, total: int) -> Optional[Tuple[int, list]]:
        """``(start, region)`` of a free ``total``-byte region after the head (wrapping), or
        None while it would overlap a live region; ``region[2]`` takes the players' batch
        numbers once the batch is sent."""
        if total > self.cap:
            return None
        start = self.head
        wrapped = start + total > self.cap
        if wrapped:
            start = 0
        if any(s < start + total and start < e for s, e, _ in self.live):
            return None
        if wrapped:
            self.wraps += 1
        region = [start, start + total, None]
        self.live.append(region)
        self.head = start + total
        return start, region

    def close(self) -> None:
        if self.pinned:
            import torch

            torch.cuda.synchronize()
            torch._C._cudart.cudaHostUnregister(self.buf.ctypes.data)
            self.pinned = False
        self.tensor = None
        self.buf = None
        try:
            self.shm.close()
            self.shm.unlink()
        except (BufferError, FileNotFoundError):
            pass


def _shm_free_bytes() -> Optional[int]:
    try:
        st = os.statvfs("/dev/shm")
    except OSError:
        return None
    return st.f_bavail * st.f_frsize


class FleetServer:
    """Node-process side of a fleet: request columns in, transmuxed answer columns out."""

    def __init__(self, node: Any, pipeline: Any, conns: List[Any]) -> None:
        self.node = node
        self.pipe = pipeline
        self.conns = list(conns)
        W = len(self.conns)
        self.open = [True] * W
        self._q = [_Queue() for _ in range(W)]
        # per player request slots (rid % _RING): AES key index (global, -1 = clear) and IV
        self._gkey = [np.full(_RING, -1, dtype=np.int32) for _ in range(W)]
        self._iv = [np.zeros((_RING, 16), dtype=np.uint8) for _ in range(W)]
        self._skey = [np.zeros((_RING, 4), dtype=np.int64) for _ in range(W)]  # segment key (32-bit fields)
        self._kmap: List[Dict[int, int]] = [{} for _ in range(W)]  # player key id -> global key index
        self._gk: Dict[bytes, int] = {}
        self._drk = np.zeros((0, 44), dtype=np.uint32)  # round keys per global key index
        self._rawkeys = np.zeros((0, 16), dtype=np.uint8)  # the keys themselves (CPU transmux)
        self._down = [True] * W
        self._payload = [False] * W
        self._ring: Optional[_PayloadRing] = None
        self._retired: List[_PayloadRing] = []  # replaced rings, closed once their regions are released
        # pinned staging of an unpinned ring's batches: one buffer per batch in flight (batch
        # N+1's D2H is queued before batch N's host copy runs), back to the pool after that copy
        self._bounce_free: List[Any] = []
        self.bounce_buffers = 0  # allocated so far (a pool the size of the batches in flight)
        self._pstream = None  # side stream of the payload gathers + D2H
        self.ring_ack_timeout_s = float(os.environ.get("HLSP2P_FLEET_ACK_TIMEOUT", "10"))
        self.revoked: set = set()  # players whose payloads were stopped (stalled on their acks)
        self.payload_bytes = 0  # copied into the payload ring
        self.payload_wait_s = 0.0  # host time blocked on a batch's payload D2H
        self._delivered: List[tuple] = []  # delivery columns from the node, not transmuxed yet
        self._chunks: List[List[tuple]] = [[] for _ in range(W)]  # answer columns per player
        self._errors: List[List[Tuple[int, int]]] = [[] for _ in range(W)]
        self.marks: Dict[Any, Dict[int, Any]] = {}
        self.ready: set = set()
        self.requests = [0] * W
        self.sent = 0
        self.evicted = 0  # cache entries dropped by the players' live-window eviction
        self.batches_sent = [0] * W  # answer batches sent to each player ...
        self.batches_done = [0] * W  # ... and handled by it (reported back)
        # entries answered to an on-demand player stay pinned until it handled their answer
        # batch, so RemoteSegment.data() in its onSuccess finds them cached: per player
        # (answer batch number, time sent, entry ids, their keys)
        self._holds: List["collections.deque"] = [collections.deque() for _ in range(W)]
        # transmux batches launched and not completed: their delivered entries (deliver's pin)
        # and those delivered with an expected CRC (the node's audit balances both)
        self._tx_inflight: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
        node.set_bulk_sink(self)
        if hasattr(node, "pin_holders"):
            node.pin_holders.append(self._pinned_entries)
            node.expect_holders.append(self._expect_entries)
        # segments received from peers are CRC-checked by the transmux that decrypts them (the
        # CRC fused into the AES kernel), not by a separate read in the node's round: results
        # of a copy that fails go to no player, the node asks the CDN again (verify_done)
        if hasattr(node, "verify_deferred") and os.environ.get("HLSP2P_DEFER_VERIFY", "1") != "0":
            node.verify_deferred = True
        self.verify_failures = 0
        self.bytes_fetched = 0  # segment bytes sent to players on demand (RemoteSegment.data)
        self._fetches: List[tuple] = []  # on-demand copies in flight, answered in order

    # -------------------------------------------------------------- audit ledgers
    def _pinned_entries(self) -> np.ndarray:
        """Entry ids this server holds one pin on each (agent/audit.py): delivered and not
        transmuxed yet, in a transmux batch in flight, answered to an on-demand player that has
        not handled the batch yet, or being copied for an on-demand fetch."""
        parts = [it[6] for it in self._delivered]
        parts += [p for p, _ in self._tx_inflight.values()]
        parts += [h[2] for q in self._holds for h in q]
        parts += [f[4] for f in self._fetches]
        return np.concatenate([np.asarray(p, dtype=np.int64).reshape(-1) for p in parts]) if parts else \
            np.zeros(0, dtype=np.int64)

    def _expect_entries(self) -> np.ndarray:
        """Entries delivered with an expected CRC whose check has not been reported yet."""
        parts = [it[6][np.asarray(it[7]) >= 0] for it in self._delivered]
        parts += [e for _, e in self._tx_inflight.values()]
        return np.concatenate([np.asarray(p, dtype=np.int64).reshape(-1) for p in parts]) if parts else \
            np.zeros(0, dtype=np.int64)

    # -------------------------------------------------------------- node sink
    def deliver(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect=None) -> None:
        """Delivery columns of the node's round (``SwarmNode.set_bulk_sink``); ``expect``: the
        CRC each fragment's bytes must have (-1: verified by the node already)."""
        if expect is None:
            expect = np.full(len(tok), -1, dtype=np.int64)
        # pinned from here until the answer is out: through the transmux that reads them, and
        # for an on-demand player until it handled the answer (see complete_transmux)
        he = eids[eids >= 0]
        if len(he):
            self.node.store.pin(he)
        self._delivered.append((tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect))

    def fail(self, tok, status) -> None:
        """Requests the node could not serve (HTTP-like status per token)."""
        w = (tok >> TOKEN_SHIFT).tolist()
        rid = (tok & _RID_MASK).tolist()
        for p, r, s in zip(w, rid, np.asarray(status).tolist()):
            if 0 <= p < len(self._errors):
                self._errors[p].append((r, int(s) or 500))

    # -------------------------------------------------------------- inbound
    def _take_requests(self, w: int, cols: tuple) -> int:
        rid, key, urls, hdr, kid, iv, new_keys = cols
        if new_keys:
            from ..ops import aes as _aes

            for k_id, kb in new_keys.items():
                g = self._gk.get(kb)
                if g is None:
                    g = self._gk[kb] = len(self._gk)
                    self._drk = np.concatenate([self._drk, np.asarray(_aes.round_keys_le(kb),
                                                                      dtype=np.uint32).reshape(1, 44)])
                    self._rawkeys = np.concatenate([self._rawkeys, np.frombuffer(kb, dtype=np.uint8).reshape(1, 16)])
                self._kmap[w][int(k_id)] = g
        slot = rid % _RING
        if (kid >= 0).any():
            km = self._kmap[w]
            lut = np.full(max(km) + 2 if km else 1, -1, dtype=np.int32)
            for k_id, g in km.items():
                lut[k_id] = g
            self._gkey[w][slot] = np.where(kid >= 0, lut[np.maximum(kid, 0)], -1)
        else:
            self._gkey[w][slot] = -1
        self._iv[w][slot] = iv
        self._skey[w][slot] = np.asarray(key, dtype=np.int64).reshape(-1, 4) & 0xFFFFFFFF
        force = np.full(len(rid), not self._down[w], dtype=bool)
        self._q[w].push(rid, key, urls, hdr, force)
        self.requests[w] += len(rid)
        return len(rid)

    def poll(self) -> int:
        """Take every queued player message; returns the number of new requests."""
        n = 0
        node = self.node
        if self._fetches:
            self._finish_fetches()
        for w, conn in enumerate(self.conns):
            if not self.open[w]:
                if self._holds[w]:
                    self._release_holds(w)
                continue
            try:
                while conn.poll(0):
                    msg = conn.recv()
                    kind = msg[0]
                    if kind == "req":
                        n += self._take_requests(w, msg[1])
                        self.batches_done[w] = msg[2]
                    elif kind == "ack":
                        self.batches_done[w] = msg[1]
                    elif kind == "abort":
                        rids = set(int(r) for r in msg[1])
                        self._q[w].drop(rids)  # not handed to the node yet
                        tok = (np.fromiter(rids, dtype=np.int64, count=len(rids)) | (w << TOKEN_SHIFT))
                        node.abort_tokens(tok)
                    elif kind == "evict":  # a live window slid: its old segments cannot be asked for
                        self.evicted += int(node.store.evict_below(msg[1], msg[2]))
                    elif kind == "flags":  # this player's session toggles only
                        self._down[w] = bool(msg[1])
                        node.set_session_flags(("fleet", w), bool(msg[1]), bool(msg[2]))
                    elif kind == "payload":
                        self._payload[w] = bool(msg[1])
                    elif kind == "invalidate":  # the player could not decrypt / demux these copies
                        node.invalidate(msg[1])
                    elif kind == "fetch":  # RemoteSegment.data() on demand (one answer chunk's keys)
                        self._start_fetch(w, msg[1], msg[2])
                    elif kind == "mark":
                        self.marks.setdefault(msg[1], {})[w] = msg[2]
                    elif kind == "ready":
                        self.ready.add(w)
                    elif kind == "bye":
                        self.open[w] = False
                        break
            except (EOFError, OSError):
                self.open[w] = False
            if self._holds[w]:
                self._release_holds(w)
        return n

    def _release_holds(self, w: int) -> None:
        """Unpin the entries of answer batches player ``w`` has handled -- or that it did not
        acknowledge within ``ring_ack_timeout_s``, or all of them once it left."""
        q = self._holds[w]
        done, stale, gone = self.batches_done[w], time.monotonic() - self.ring_ack_timeout_s, not self.open[w]
        store = self.node.store
        while q and (gone or q[0][0] <= done or q[0][1] < stale):
            store.unpin(q.popleft()[2])

    def _start_fetch(self, w: int, fid: int, keys) -> None:
        """Start copying an answer chunk's cached segments to the host for player ``w``
        (``RemoteSegment.data()`` on demand): on a GPU node one gather kernel into a packed
        block and ONE asynchronous D2H into pinned memory on the payload side stream; the
        answer goes out from a later :meth:`poll` once the copy has landed, so the rank never
        blocks on it.  A key the cache no longer holds answers None.  Entries the host
        delivered are resident (their round was waited on); they stay pinned until the copy
        is done."""
        store = self.node.store
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64).reshape(-1, 4) & 0xFFFFFFFF)
        eids = store.lookup(keys, False)
        if self._holds[w]:
            # the copies this player was answered with, while its batches hold them: the cache's
            # index may name another copy by now (a second request for a segment whose peer copy
            # awaited its check fetched it again) or none (detached), the held bytes stay put
            held = {}
            for _, _, he, hk in self._holds[w]:
                held.update(zip(map(tuple, hk.tolist()), he.tolist()))
            for i, k in enumerate(map(tuple, keys.tolist())):
                e = held.get(k)
                if e is not None:
                    eids[i] = e
        hit = np.flatnonzero(eids >= 0)
        ids = np.ascontiguousarray(eids[hit])
        lens = np.zeros(0, dtype=np.int64)
        pack = lens
        host = ev = None
        if len(hit):
            store.pin(ids)
            ent = store.entries(ids)
            offs, lens = ent[:, 0].copy(), ent[:, 1].copy()
            pack = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            total = int(lens.sum())
            arena = self.node.arena
            if arena.is_cuda:
                import torch

                from ..ops import segment as _seg

                if self._pstream is None:
                    self._pstream = torch.cuda.Stream(device=arena.device)
                ps = self._pstream
                ps.wait_stream(torch.cuda.current_stream(arena.device))
                with torch.cuda.stream(ps):  # staging allocated, used and freed in ps's stream order
                    staged = torch.empty(max(total, 1), dtype=torch.uint8, device=arena.device)
                    _seg.copy_segments(arena, staged, offs, pack, lens)
                    host = torch.empty(max(total, 1), dtype=torch.uint8, pin_memory=True)
                    host.copy_(staged, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(ps)
            else:
                a = arena.numpy()
                host = np.concatenate([a[o:o + n] for o, n in zip(offs.tolist(), lens.tolist())]) if total else \
                    np.zeros(0, dtype=np.uint8)
        self._fetches.append((w, fid, len(keys), hit, ids, pack, lens, host, ev))
        self._finish_fetches()

    def _finish_fetches(self) -> None:
        """Answer every on-demand fetch whose copy has landed (in request order)."""
        while self._fetches:
            w, fid, n, hit, ids, pack, lens, host, ev = self._fetches[0]
            if ev is not None and not ev.query():
                return
            self._fetches.pop(0)
            if len(ids):
                self.node.store.unpin(ids)
            out: list = [None] * n
            if host is not None:
                h = host.numpy() if not isinstance(host, np.ndarray) else host
                for j, p, k in zip(hit.tolist(), pack.tolist(), lens.tolist()):
                    out[j] = h[p:p + k]
                self.bytes_fetched += int(lens.sum())
            if self.open[w]:
                try:
                    self.conns[w].send(("bytes", fid, out))
                except (OSError, BrokenPipeError):
                    self.open[w] = False

    def admit(self, per_player: int) -> int:
        """Hand up to ``per_player`` queued requests of every player to the node (call right
        before the node's round): one ``request_batch`` per player."""
        node = self.node
        n = 0
        for w, q in enumerate(self._q):
            got = q.take(per_player)
            if got is None:
                continue
            rid, key, urls, hdr, force = got
            node.request_batch(key, urls, hdr, rid | (w << TOKEN_SHIFT), force if force.any() else None)
            n += len(rid)
        return n

    # -------------------------------------------------------------- outbound
    def launch_transmux(self):
        """Enqueue the GPU transmux of everything the node delivered since the last call:
        decrypt keys and IVs looked up by token, one columnar launch."""
        items, self._delivered = self._delivered, []
        if not items:
            return None
        if len(items) == 1:
            tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect = items[0]
        else:
            tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect = (np.concatenate(c) for c in zip(*items))
        w = tok >> TOKEN_SHIFT
        slot = (tok & _RID_MASK) % _RING
        gk = np.empty(len(tok), dtype=np.int32)
        iv = np.empty((len(tok), 16), dtype=np.uint8)
        for p in np.unique(w).tolist():
            sel = w == p
            gk[sel] = self._gkey[p][slot[sel]]
            iv[sel] = self._iv[p][slot[sel]]
        enc = gk >= 0
        if len(self._drk):
            drk, keys = self._drk[np.maximum(gk, 0)], self._rawkeys[np.maximum(gk, 0)]
        else:
            drk, keys = np.zeros((len(tok), 44), dtype=np.uint32), None
        verify = expect >= 0
        pay = self._payload_stage(w, offs, nbytes) if any(self._payload) else None
        tag = (tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect if verify.any() else None, pay)
        batch = self.pipe.launch_columns(self.node.arena, offs, nbytes, enc, drk, iv, tag, keys=keys,
                                         expect=expect if verify.any() else None)
        if batch is None:  # (every delivered row goes into a batch: a lost one would keep its pins)
            raise RuntimeError("transmux pipeline returned no batch for delivered fragments")
        self._tx_inflight[id(batch)] = (eids[eids >= 0], eids[(expect >= 0) & (eids >= 0)])
        return batch

    def complete_transmux(self, batch) -> None:
        """Wait for a launched transmux batch; its info rows go to the players as columns."""
        if batch is None:
            return
        self._tx_inflight.pop(id(batch), None)
        tag, rows, plain, has, verified = self.pipe.complete_columns(batch)
        tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect, pay = tag
        ring_off = None
        if pay is not None:
            ring_off, region, ev, post = pay
            if ev is not None:
                t0 = time.perf_counter()
                ev.synchronize()  # the batch's D2H into the ring (queued at launch)
                if post is not None:  # unpinned ring: the bounce buffer's bytes go in on the host
                    post()
                self.payload_wait_s += time.perf_counter() - t0
        if expect is not None:  # deferred receive checks: the node commits or re-fetches
            chk = expect >= 0
            self.verify_failures += self.node.verify_done(eids[chk], verified[chk], tok[chk])
            if not verified.all():  # no answer for a corrupted copy: the CDN retry answers
                keep = verified
                dropped = eids[~keep]
                dropped = dropped[dropped >= 0]
                if len(dropped):
                    self.node.store.unpin(dropped)  # (deliver's pin)
                tok, src, nbytes, cdn_ms, p2p_ms, offs, eids = (tok[keep], src[keep], nbytes[keep], cdn_ms[keep],
                                                                p2p_ms[keep], offs[keep], eids[keep])
                rows, plain, has = rows[keep], plain[keep], has[keep]
                if ring_off is not None:
                    ring_off = ring_off[keep]
        w = tok >> TOKEN_SHIFT
        rid = tok & _RID_MASK
        need = {}
        for p in np.unique(w).tolist():
            sel = np.flatnonzero(w == p)
            chunk = (rid[sel], src[sel].astype(np.int8), nbytes[sel], cdn_ms[sel], p2p_ms[sel], plain[sel],
                     has[sel], rows[sel])
            if ring_off is not None and self._payload[p]:
                chunk = chunk + ((self._ring.shm.name, ring_off[sel], nbytes[sel]),)
                need[p] = self.batches_sent[p] + 1  # the answer batch the next send() carries
            he = eids[sel]
            cached = he >= 0
            he = he[cached]
            if len(he):  # deliver's pin: kept for an on-demand player until it handled this batch
                if self.open[p] and not (ring_off is not None and self._payload[p]):
                    hk = self._skey[p][rid[sel][cached] % _RING]
                    self._holds[p].append((self.batches_sent[p] + 1, time.monotonic(), he, hk))
                else:
                    self.node.store.unpin(he)
            self._chunks[p].append(chunk)
        if pay is not None:
            region[2] = need

    def _payload_stage(self, w: np.ndarray, offs: np.ndarray, lens: np.ndarray):
        """Queue the copy of the payload players' fragments from the HBM arena into the shared
        ring: one gather kernel into a packed staging block and one asynchronous D2H into the
        pinned ring, on a side stream (they overlap the transmux).  Returns ``(ring offset per
        fragment or -1, ring region, done event)``."""
        want = np.fromiter((self._payload[p] for p in w.tolist()), dtype=bool, count=len(w))
        if not want.any():
            return None
        arena = self.node.arena
        idx = np.flatnonzero(want)
        n = lens[idx]
        al = (n + 63) // 64 * 64
        pack = np.concatenate([[0], np.cumsum(al)[:-1]]).astype(np.int64)
        total = int(al.sum())
        self._reap_retired()
        ring, (start, region) = self._place(total)
        self.payload_bytes += total
        ring_off = np.full(len(w), -1, dtype=np.int64)
        ring_off[idx] = start + pack
        ev = post = None
        if arena.is_cuda:
            import torch

            from ..ops import segment as _seg

            if self._pstream is None:
                self._pstream = torch.cuda.Stream(device=arena.device)
            ps = self._pstream
            ps.wait_stream(torch.cuda.current_stream(arena.device))
            with torch.cuda.stream(ps):  # staging allocated, used and freed in ps's stream order
                staged = torch.empty(max(total, 1), dtype=torch.uint8, device=arena.device)
                _seg.copy_segments(arena, staged, offs[idx], pack, n)
                if ring.pinned:
                    ring.tensor[start:start + total].copy_(staged[:total], non_blocking=True)
                else:  # registration failed: D2H into a pinned bounce buffer, host copy at completion
                    bounce = self._take_bounce(total)
                    bounce[:total].copy_(staged[:total], non_blocking=True)

                    def post(buf=ring.buf, bounce=bounce, start=start, total=total):
                        buf[start:start + total] = bounce[:total].numpy()
                        self._bounce_free.append(bounce)  # this batch's D2H has landed: reusable
                ev = torch.cuda.Event()
                ev.record(ps)
        else:
            host, buf = arena.numpy(), ring.buf
            for o, p, k in zip(offs[idx].tolist(), (start + pack).tolist(), n.tolist()):
                buf[p:p + k] = host[o:o + k]
        return ring_off, region, ev, post

    def _take_bounce(self, total: int):
        """A pinned bounce buffer of at least ``total`` bytes that no batch in flight uses."""
        import torch

        for i, b in enumerate(self._bounce_free):
            if b.numel() >= total:
                return self._bounce_free.pop(i)
        self.bounce_buffers += 1
        return torch.empty(max(total, 64 << 20), dtype=torch.uint8, pin_memory=True)

    # -------------------------------------------------------------- payload ring
    def _acked(self, need) -> bool:
        return all(not self.open[p] or self.batches_done[p] >= k for p, k in need.items())

    RING_MIN = 256 << 20  # smallest automatic payload ring

    def _new_ring(self, total: int) -> _PayloadRing:
        """A (bigger) payload ring; the current one is retired, kept until every region on it
        is acknowledged.  Size: ``HLSP2P_FLEET_PAYLOAD_BYTES`` for the first ring (at least this
        batch), else room
        for 4 batches of this size (>= 256 MiB, doubling on growth), capped to half of the
        free /dev/shm, and never below 2 batches."""
        old = self._ring
        env = os.environ.get("HLSP2P_FLEET_PAYLOAD_BYTES")
        if old is None and env:
            size = max(int(env), total)  # (never below the batch asking for it)
        else:
            size = max(self.RING_MIN, 4 * total, 2 * old.cap if old is not None else 0)
            size = (size + (1 << 20) - 1) // (1 << 20) * (1 << 20)
            free = _shm_free_bytes()
            if free is not None:
                size = min(size, free // 2)
            if size < 2 * total:
                raise RuntimeError(f"/dev/shm has {free} bytes free: too little for a payload ring of two "
                                   f"{total}-byte batches (lower the fragments in flight)")
        ring = _PayloadRing(size, pin=self.node.arena.is_cuda)
        if old is not None:
            if old.live:
                self._retired.append(old)
            else:
                old.close()
        self._ring = ring
        return ring

    def _reap_retired(self) -> None:
        for ring in list(self._retired):
            ring.release_done(self._acked)
            if not ring.live:
                ring.close()
                self._retired.remove(ring)

    def _place(self, total: int):
        """A ring region for a ``total``-byte batch.  Regions free in FIFO order once their
        players acknowledged them; when the next region is still held by a batch in flight
        (the ring is too small for the batches in flight) or by players that do not
        acknowledge within ``HLSP2P_FLEET_ACK_TIMEOUT`` s, the rank moves to a bigger ring
        instead of failing -- and stops sending payloads to the stalled players (their
        regions stay valid on the retired ring until they acknowledge or leave)."""
        ring = self._ring
        if ring is None or total > ring.cap:
            ring = self._new_ring(total)
        while True:
            ring.release_done(self._acked)
            got = ring.try_place(total)
            if got is not None:
                return ring, got
            if not ring.live:  # empty and still too small for this batch
                ring = self._new_ring(total)
                continue
            need = ring.live[0][2]
            if need is None or not self._wait_acks(need):
                if need is not None:
                    self._revoke([p for p, k in need.items() if self.open[p] and self.batches_done[p] < k])
                ring = self._new_ring(total)

    def _wait_acks(self, need) -> bool:
        """Wait up to ``ring_ack_timeout_s`` for the players of a region to acknowledge it."""
        from multiprocessing.connection import wait

        end = time.monotonic() + self.ring_ack_timeout_s
        while not self._acked(need):
            if time.monotonic() > end:
                return False
            conns = [c for p, c in enumerate(self.conns) if self.open[p]]
            if conns:
                wait(conns, timeout=0.005)
            self.poll()
        return True

    def _revoke(self, players: List[int]) -> None:
        """Stop sending payloads to players that stopped acknowledging their answer batches:
        one stalled player must not stall (or fail) the rank's other players.  The player is
        told (``("revoke",)``): its later fragments arrive without bytes."""
        for p in players:
            if p in self.revoked:
                continue
            self.revoked.add(p)
            self._payload[p] = False
            log.warning("fleet player %d did not acknowledge its payload batches in %.0f s: no more payloads for "
                        "it", p, self.ring_ack_timeout_s)
            try:
                self.conns[p].send(("revoke",))
            except (OSError, BrokenPipeError):
                self.open[p] = False

    def send(self) -> int:
        """One answer batch per player (plus the swarm state the agents' stats read)."""
        node = self.node
        st = {"upload": node.stats["upload"], "swarm": dict(getattr(node, "swarm_stats", {}) or
                                                             {"cdn": 0, "p2p": 0, "upload": 0}),
              "online": np.asarray(node.peer_online, dtype=bool).tolist()}
        n = 0
        for w in range(len(self.conns)):
            chunks, errs = self._chunks[w], self._errors[w]
            if not (chunks or errs) or not self.open[w]:
                continue
            try:
                self.conns[w].send(("done", chunks, errs, st))
                n += sum(len(c[0]) for c in chunks) + len(errs)
                self.batches_sent[w] += 1
            except (OSError, BrokenPipeError):
                self.open[w] = False
            self._chunks[w] = []
            self._errors[w] = []
        self.sent += n
        return n

    def await_players(self, depth: int = 1, timeout_s: float = 0.02) -> None:
        """Pace the node by its players: wait until every player has handled all but at most
        ``depth`` of the answer batches sent to it (a player sends its next requests right
        after handling a batch).  ``depth`` 1 overlaps one batch of player work with one node
        step; at most ``timeout_s`` (a player with nothing left to ask must not stall)."""
        from multiprocessing.connection import wait

        end = time.monotonic() + timeout_s
        while True:
            behind = [self.conns[w] for w in range(len(self.conns))
                      if self.open[w] and self.batches_sent[w] - self.batches_done[w] > depth]
            if not behind:
                return
            left = end - time.monotonic()
            if left <= 0:
                return
            wait(behind, left)
            self.poll()

    def wait_marks(self, tag: Any, timeout_s: float = 120.0) -> Dict[int, Any]:
        """Block until every open player has sent ``("mark", tag, ...)``."""
        end = time.monotonic() + timeout_s
        while True:
            got = self.marks.get(tag, {})
            if all(not self.open[w] or w in got for w in range(len(self.conns))):
                return got
            if time.monotonic() > end:
                raise TimeoutError(f"fleet players did not reach mark {tag!r}")
            for c, o in zip(self.conns, self.open):
                if o:
                    c.poll(0.01)
            self.poll()

    def close(self) -> None:
        """Release the payload rings (after the players stopped)."""
        for ring in self._retired:
            ring.close()
        self._retired = []
        if self._ring is not None:
            self._ring.close()
            self._ring = None


# ============================================================================ player process
def _script_action(hls: Any, media: Any, loop: Any, action: str, arg: Any) -> None:
    """One scripted player action (``player_main`` ``spec["script"]``)."""
    if action == "seek":
        media.currentTime = float(arg)
    elif action == "seek_rel":  # (live: back into the DVR window)
        media.currentTime = max(0.0, media.currentTime + float(arg))
    elif action == "pause":
        media.pause()
        loop.set_timeout(media.play, float(arg))
    elif action == "level":
        if hls.levels:
            hls.nextLevel = int(arg) % len(hls.levels)
    elif action == "restart":
        hls.stopLoad()
        loop.set_timeout(lambda: hls.startLoad(media.currentTime), float(arg))
    else:
        raise ValueError(f"unknown scripted action {action!r}")


def player_main(conn: Any, spec: Dict[str, Any]) -> None:
    """A fleet player process: the bundle ``Hls`` over a :class:`RemoteNode`, drained as fast
    as the node answers (the throughput bench's player).  ``spec``: ``origin`` (keyword
    arguments of ``SyntheticHlsOrigin``: the player reads playlists and keys from it, the
    node process serves the segments), ``hls_config``, ``p2p_config``, ``world``, ``rank``;
    for tests, ``script`` (scheduled seeks, pauses, level switches, load restarts) and
    ``read_bytes`` (read every fragment's bytes back through ``RemoteSegment.data()``) and
    ``in_process`` (a thread in the node's process: leave its torch threads, GPU and GC alone).
    Control from the node: ``("mark", tag)`` -> reply ``("mark", tag, counters)`` once every
    answer sent before it is buffered; ``("stop",)`` -> close and exit."""
    import copy

    from .. import Hls
    from ..agent.node import node_for_config, set_current_node
    from ..net import new_event_loop
    from ..net.origin import SyntheticHlsOrigin
    from ..player import MediaElement
    from ..utils.runtime import cpu_calibration_us, tune_gc

    import torch

    in_process = bool(spec.get("in_process"))  # a thread beside the node (tests/fleet_chaos.py)
    if not in_process:
        torch.set_num_threads(1)  # a player does no tensor math: no intra-op pool competing for cores
    if torch.cuda.device_count() and not in_process:
        log.warning("fleet player sees %d GPU(s); it should not (HIP_VISIBLE_DEVICES)", torch.cuda.device_count())
    set_current_node(None)
    speed = float(spec.get("clock_speed", 1.0))
    loop = new_event_loop("real", speed=speed)  # a live bench's channel runs on a compressed clock
    origin = SyntheticHlsOrigin(**spec["origin"])
    p2p = copy.deepcopy(spec["p2p_config"])
    gs = dict(p2p.get("gpuSwarm") or {})
    p2p["gpuSwarm"] = {"backend": "remote", "conn": conn, "world": spec.get("world", 1), "rank": spec.get("rank", 0),
                       "fleetPayload": bool(gs.get("fleetPayload", False))}
    node = node_for_config(p2p)
    hls = Hls(dict(spec["hls_config"]), p2p)
    media = MediaElement(mode=spec.get("media_mode", "drain"), loop=loop)
    counters = {"buffered": 0, "errors": 0, "level_switches": 0, "bytes": 0}
    live_lat: List[float] = []  # media seconds from a live segment's publication to its buffering

    def on_buffered(e, d):
        counters["buffered"] += 1
        if origin.live and origin.live_epoch is not None:
            sn = d["frag"].sn
            published = origin.live_epoch + (sn - (origin.start_sn + origin.window - 1)) * \
                origin.segment_duration / origin.live_speed
            live_lat.append((time.time() - published) * origin.live_speed)

    hls.on(Hls.Events.FRAG_BUFFERED, on_buffered)
    hls.on(Hls.Events.ERROR, lambda e, d: counters.__setitem__("errors", counters["errors"] + 1))
    hls.on(Hls.Events.ERROR,
           lambda e, d: counters.__setitem__("fatal", counters.get("fatal", 0) + bool(d.get("fatal"))))
    if spec.get("read_bytes"):  # every fragment's bytes read back through RemoteSegment.data()

        def read_back(e, d):
            seg = d.get("payload")
            data = seg.data() if isinstance(seg, RemoteSegment) else None
            if data is None or len(data) != seg.nbytes:
                counters["byte_errors"] = counters.get("byte_errors", 0) + 1
            else:
                counters["bytes_read"] = counters.get("bytes_read", 0) + len(data)
        hls.on(Hls.Events.FRAG_LOADED, read_back)
    hls.on(Hls.Events.LEVEL_SWITCH, lambda e, d: counters.__setitem__("level_switches",
                                                                     counters["level_switches"] + 1))
    # start together: a player that started early would run ahead into the next one's slice
    conn.send(("ready",))
    while True:
        msg = conn.recv()
        if msg[0] == "go":
            opts = msg[1] if len(msg) > 1 else {}
            if opts.get("live_epoch") is not None:  # the channel's clock, shared with the node
                origin.live_epoch = float(opts["live_epoch"])
            break
        if msg[0] == "stop":
            node.close()
            return
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    sc = hls.streamController
    # tests / diagnostics: scripted player actions, (ms after start, action, argument)
    for t_ms, action, arg in spec.get("script") or ():
        loop.set_timeout(_script_action, float(t_ms), hls, media, loop, action, arg)

    def drain():
        loop.run_once(block=False)  # due timers too (live playlist reloads, the playback clock)
        for _ in range(1000):
            if not loop._ready and not loop._threadsafe:
                return
            loop.run_once(block=False)

    gc_tuned = False
    prof = None
    if os.environ.get("HLSP2P_PLAYER_PROFILE"):  # cProfile this player from its first request to stop
        import cProfile

        prof = cProfile.Profile()
    debug = os.environ.get("HLSP2P_FLEET_DEBUG")
    t_dbg = time.monotonic()
    try:
        while True:
            if debug and time.monotonic() - t_dbg > 1.0:
                t_dbg = time.monotonic()
                log.warning("player %s: state %s inflight %d node-inflight %d t %.1f ranges %s counters %s "
                            "retry_until %.1f now %.1f", spec.get("rank"), sc.state, len(sc.inflight), node.inflight,
                            media.currentTime, media.buffered, counters, sc._retry_until, loop.now())
            node.poll(0.0005)
            drain()
            sc.tick()
            drain()
            node.flush()
            if not gc_tuned and node.inflight:  # started: freeze the start-up heap
                if not in_process:  # (the process's GC is its owner's to tune)
                    tune_gc()
                gc_tuned = True
                if prof is not None:
                    prof.enable()
            while node.control:
                msg = node.control.pop(0)
                if msg[0] == "mark":
                    counters["bytes"] = node.stats.get("cdn", 0) + node.stats.get("p2p", 0)
                    out = dict(counters)
                    out["cpu_s"] = time.process_time()
                    out["t"] = media.currentTime
                    if len(msg) > 2 and msg[2].get("calib"):  # soak analysis: core speed at the mark
                        out["calib_us"] = cpu_calibration_us()
                    if len(msg) > 2 and msg[2].get("state"):  # a stalled player says what it waits on
                        sc = hls.streamController
                        out["state"] = {"buffered": [tuple(r) for r in media.buffered], "paused": media.paused,
                                        "seeking": media.seeking, "stream": sc.state, "level": hls.currentLevel,
                                        "inflight": sorted(sc.inflight), "pending": len(node._pending),
                                        "node_inflight": node.inflight}
                        fl = hls.fragmentLoader.loaders
                        out["state"]["loaders"] = [
                            (k, id(f) in fl, getattr(fl.get(id(f)), "requestTimeout", None) is not None,
                             getattr(fl.get(id(f)), "peerAgentLoader", None) is not None)
                            for k, f in sc.inflight.items()]
                        out["state"]["n_loaders"] = len(fl)
                        out["state"]["remote_pending"] = [(rid, q.key[3], q.aborted, q.done)
                                                          for rid, q in node._pending.items()]
                        lc = hls.levelController
                        lv = hls.levels[lc.level] if hls.levels and 0 <= lc.level < len(hls.levels) else None
                        det = lv.details if lv is not None else None
                        if det is not None and det.fragments:
                            out["state"].update(last_sn=det.fragments[-1].sn, last_end=det.fragments[-1].end,
                                                reload_timer=lc._reload_timer is not None,
                                                playlist_loaders=sorted(hls.playlistLoader.loaders))
                            if origin.live:
                                out["state"]["edge_sn"] = origin.live_edge()
                    if live_lat:  # live latency behind the edge since the previous mark
                        out["live_latency_s"] = live_lat[:]
                        live_lat.clear()
                    conn.send(("mark", msg[1], out))
                elif msg[0] == "stop":
                    return
    finally:
        if prof is not None:
            import io
            import pstats

            prof.disable()
            out = io.StringIO()
            pstats.Stats(prof, stream=out).sort_stats("tottime").print_stats(40)
            stem = f"{os.environ['HLSP2P_PLAYER_PROFILE']}.player{spec.get('rank', 0)}_{os.getpid()}"
            with open(stem + ".txt", "w") as f:
                f.write(f"buffered {counters['buffered']}\n" + out.getvalue())
            prof.dump_stats(stem + ".prof")  # for pstats' callers / callees views
        try:
            hls.destroy()
        finally:
            node.close()
