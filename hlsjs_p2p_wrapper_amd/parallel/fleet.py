"""Fleet: player processes in front of one GPU's swarm node.

One MI355X is one swarm peer (one process, one ``SwarmNode``, the RCCL rank).  The players
it serves need not share that process: the per-fragment host path of the hls.js-compatible
engine (stream controller, loaders, ABR, events, ~13 us of Python per fragment) is what
bounds a node's segment rate once P2P takes the CDN load off PCIe (``profiles/r2_cyprof``).
With a fleet, ``W`` player processes run that path in parallel; the GPU process keeps only
the node side (rounds, CDN DMA, RCCL, CRC) and the transmux, which it runs in batches.
The player processes never touch the GPU (``HIP_VISIBLE_DEVICES`` is empty for them).

Protocol (one ``multiprocessing`` pipe per player process, batched per loop iteration):

* player -> node: ``("req", [(rid, key4, url, headers, aes_key, iv), ...])`` — a fragment
  request as ``PeerAgent.getSegment`` issues it, plus the AES key / IV the GPU transmux
  needs; ``("abort", [rid, ...])``; ``("evict", swarm, sn)``; ``("flags", down, up)``;
  ``("mark", tag, counters)`` (bench window markers); ``("bye",)``.
* node -> player: ``("done", chunks, errors, swarm_state)``.  Each chunk holds the fragments of
  one transmux batch as columns (numpy arrays, pickled as flat buffers): ``rid``, ``source``
  code (:data:`SOURCES`), ``nbytes``, ``cdn_ms``, ``p2p_ms``, ``plain`` bytes, ``has_row`` and
  the transmux info ``rows`` ``[n, INFO_WORDS]``.  ``errors``: ``[(rid, status), ...]`` with
  the HTTP-like error status of requests the node could not serve.

Player side, :class:`RemoteNode` stands in for the ``SwarmNode`` behind the unchanged
``PeerAgent`` (``gpuSwarm.backend = "remote"``): the loader's ``onSuccess`` gets a
:class:`RemoteSegment` whose ``transmux_result`` the stream controller uses instead of
transmuxing itself (it holds the info row: durations, PTS, ES byte counts; the ES bytes stay
on the GPU).  Node side, :class:`FleetServer` feeds requests to the node, and per node round
transmuxes what was delivered and answers each player with one batch.
"""
from __future__ import annotations

import collections
import logging
import os
import time
from typing import Any, Dict, List, Tuple

import numpy as np

from ..net.http import HttpError

log = logging.getLogger("hlsjs_p2p_wrapper_amd.fleet")

SOURCES = ("cdn", "p2p", "cache")  # source codes of the answer columns
_SOURCE_CODE = {s: i for i, s in enumerate(SOURCES)}


# ============================================================================ player side
class RemoteSegment:
    """``onSuccess`` payload of a remotely served fragment: its size and transmux result."""

    __slots__ = ("nbytes", "transmux_result")

    def __init__(self, nbytes: int, transmux_result: Any) -> None:
        self.nbytes = nbytes
        self.transmux_result = transmux_result

    def numel(self) -> int:
        return self.nbytes

    def __len__(self) -> int:
        return self.nbytes


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


class RemoteNode:
    """The ``SwarmNode`` surface ``PeerAgent`` uses, served by a node in another process."""

    def __init__(self, conn: Any, world: int = 1, rank: int = 0) -> None:
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
        self._reqs: List[tuple] = []
        self._aborts: List[int] = []
        self._out: List[tuple] = []
        self._next = 0
        self.inflight = 0
        self.control: List[tuple] = []
        self.batches = 0  # answer batches handled (reported to the node, which paces on it)
        self._reported = 0

    # -------------------------------------------------------------- SwarmNode surface
    def attach(self, agent: Any) -> None:
        """Register the player's PeerAgent (as on a SwarmNode)."""
        self._agents.append(agent)

    def detach(self, agent: Any) -> None:
        """Unregister an agent."""
        if agent in self._agents:
            self._agents.remove(agent)

    @property
    def download_on(self) -> bool:
        """Read / write: P2P download, forwarded to the node."""
        return self._down

    @download_on.setter
    def download_on(self, on: bool) -> None:
        self._down = bool(on)
        self._out.append(("flags", self._down, self._up))

    @property
    def upload_on(self) -> bool:
        """Read / write: P2P upload, forwarded to the node."""
        return self._up

    @upload_on.setter
    def upload_on(self, on: bool) -> None:
        self._up = bool(on)
        self._out.append(("flags", self._down, self._up))

    def request(self, key, url: str, headers, callbacks: Any, agent: Any = None, view: Any = None):
        """Queue a fragment request for the node (sent at the next flush); ``view`` finds the
        fragment's AES key / IV for the GPU transmux.  Returns the handle (``abort()``)."""
        rid = self._next
        self._next += 1
        req = _RemoteRequest(self, rid, key, callbacks, agent)
        aes_key = iv = None
        if agent is not None and view is not None:  # the GPU transmux needs the AES key / IV
            frag = agent.mediaMap.fragment(view)
            if frag is not None:
                dd = frag.decryptdata
                if dd is not None and dd.method == "AES-128" and dd.key is not None:
                    aes_key, iv = bytes(dd.key), frag.iv_for_decrypt()
        self._pending[rid] = req
        self._reqs.append((rid, tuple(key), url, dict(headers) if headers else None, aes_key, iv))
        self.inflight += 1
        return req

    def prefetch(self, key, url: str, headers=None) -> bool:
        """Agent-driven prefetch is a single-process feature: nothing is issued."""
        return False  # agent-driven prefetch stays a single-process feature

    def swarm_offload_ratio(self) -> float:
        """P2P / (P2P + CDN) bytes over the whole swarm, as last reported by the node."""
        c, p = self.swarm_stats["cdn"], self.swarm_stats["p2p"]
        return p / (p + c) if (p + c) else 0.0

    # -------------------------------------------------------------- transport
    def flush(self) -> None:
        """Send everything queued since the last flush (one message per kind), with the count
        of answer batches handled so far (the node paces its rounds on it)."""
        if self._reqs:
            self.conn.send(("req", self._reqs, self.batches))
            self._reqs = []
            self._reported = self.batches
        elif self.batches != self._reported:
            self.conn.send(("ack", self.batches))
            self._reported = self.batches
        if self._aborts:
            self.conn.send(("abort", self._aborts))
            self._aborts = []
        for m in self._out:
            self.conn.send(m)
        self._out = []

    def poll(self, timeout: float = 0.0) -> int:
        """Deliver every answer that has arrived (waiting up to ``timeout`` s for the first)."""
        n = 0
        conn = self.conn
        if not conn.poll(timeout):
            return 0
        while True:
            msg = conn.recv()
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
            else:  # a control message ("mark", "stop"): the player acts on it before reading on
                self.control.append(msg)
                return n
            if not conn.poll(0):
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

        rid_a, src_a, nbytes_a, cdn_a, p2p_a, plain_a, has_a, rows_a = chunk
        pending = self._pending
        stats = self.stats
        n = 0
        for rid, code, nbytes, cdn_ms, p2p_ms, plain, has, info in zip(
                rid_a.tolist(), src_a.tolist(), nbytes_a.tolist(), cdn_a.tolist(), p2p_a.tolist(),
                plain_a.tolist(), has_a.tolist(), rows_a.tolist()):
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
            on_success(RemoteSegment(nbytes, r))
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


# ============================================================================ node side
class _Pending:
    """One remote request on the node side; also its ``getSegment`` callbacks object."""

    __slots__ = ("server", "w", "rid", "aes_key", "iv", "req", "source", "nbytes", "cdn_ms", "p2p_ms")

    def __init__(self, server: "FleetServer", w: int, rid: int, aes_key, iv) -> None:
        self.server = server
        self.w = w
        self.rid = rid
        self.aes_key = aes_key
        self.iv = iv
        self.req = None
        self.source = "cdn"
        self.nbytes = 0
        self.cdn_ms = 0.0
        self.p2p_ms = 0.0

    def onProgress(self, ev: dict) -> None:  # noqa: N802 - loader callback contract
        if ev["p2pDownloaded"]:
            self.source, self.nbytes, self.p2p_ms = "p2p", ev["p2pDownloaded"], ev["p2pDuration"]
        else:
            self.source, self.nbytes, self.cdn_ms = "cdn", ev["cdnDownloaded"], ev["cdnDuration"]

    def onSuccess(self, data: Any) -> None:  # noqa: N802
        self.server._delivered.append((self, data))

    def onDelivered(self, source: str, nbytes: int, cdn_ms: float, p2p_ms: float, data: Any) -> None:  # noqa: N802
        """The node's one-call delivery (progress + success): cache hits count as P2P, as
        the progress event reports them."""
        if source == "cdn":
            self.source, self.nbytes, self.cdn_ms = "cdn", nbytes, cdn_ms
        else:
            self.source, self.nbytes, self.p2p_ms = "p2p", nbytes, p2p_ms
        self.server._delivered.append((self, data))

    def onError(self, err: Any) -> None:  # noqa: N802
        self.server._errors[self.w].append((self.rid, int(getattr(err, "status", 0) or 0) or 500))


class FleetServer:
    """Node-process side of a fleet: requests in, transmuxed deliveries out."""

    def __init__(self, node: Any, pipeline: Any, conns: List[Any]) -> None:
        self.node = node
        self.pipe = pipeline
        self.conns = list(conns)
        self.open = [True] * len(self.conns)
        self._by_rid: List[Dict[int, _Pending]] = [{} for _ in self.conns]
        self._delivered: List[Tuple[_Pending, Any]] = []
        self._chunks: List[List[tuple]] = [[] for _ in self.conns]  # answer columns per player
        self._errors: List[List[Tuple[int, int]]] = [[] for _ in self.conns]
        self.marks: Dict[Any, Dict[int, Any]] = {}
        self.ready: set = set()
        self.requests = [0] * len(self.conns)
        self.sent = 0
        # requests wait here until admitted: at most `per_player` per player and round, so
        # each player advances at the same pace on every rank and the swarm shares its slice
        self._queued: List[collections.deque] = [collections.deque() for _ in self.conns]
        self.batches_sent = [0] * len(self.conns)  # answer batches sent to each player ...
        self.batches_done = [0] * len(self.conns)  # ... and handled by it (reported back)

    # -------------------------------------------------------------- inbound
    def poll(self) -> int:
        """Take every queued player message; returns the number of new requests."""
        n = 0
        node = self.node
        for w, conn in enumerate(self.conns):
            if not self.open[w]:
                continue
            try:
                while conn.poll(0):
                    msg = conn.recv()
                    kind = msg[0]
                    if kind == "req":
                        self._queued[w].extend(msg[1])
                        n += len(msg[1])
                        self.requests[w] += len(msg[1])
                        self.batches_done[w] = msg[2]
                    elif kind == "ack":
                        self.batches_done[w] = msg[1]
                    elif kind == "abort":
                        by_rid = self._by_rid[w]
                        aborted = set()
                        for rid in msg[1]:
                            p = by_rid.pop(rid, None)
                            if p is not None and p.req is not None:
                                p.req.abort()
                            elif p is None:
                                aborted.add(rid)
                        if aborted:  # not handed to the node yet
                            q = self._queued[w]
                            self._queued[w] = collections.deque(r for r in q if r[0] not in aborted)
                    elif kind == "evict":
                        node.store.evict_below(msg[1], msg[2])
                    elif kind == "flags":
                        node.download_on, node.upload_on = bool(msg[1]), bool(msg[2])
                    elif kind == "mark":
                        self.marks.setdefault(msg[1], {})[w] = msg[2]
                    elif kind == "ready":
                        self.ready.add(w)
                    elif kind == "bye":
                        self.open[w] = False
                        break
            except (EOFError, OSError):
                self.open[w] = False
        return n

    def admit(self, per_player: int) -> int:
        """Hand up to ``per_player`` queued requests of every player to the node (call right
        before the node's round)."""
        node = self.node
        n = 0
        for w, q in enumerate(self._queued):
            if not q:
                continue
            by_rid = self._by_rid[w]
            for _ in range(min(per_player, len(q))):
                rid, key, url, headers, aes_key, iv = q.popleft()
                p = _Pending(self, w, rid, aes_key, iv)
                by_rid[rid] = p
                p.req = node.request(key, url, headers, p)
                n += 1
        return n

    # -------------------------------------------------------------- outbound
    def launch_transmux(self):
        """Enqueue the GPU transmux of everything the node delivered since the last call."""
        from ..player.transmux import TransmuxJob

        items, self._delivered = self._delivered, []
        if not items:
            return None
        pipe = self.pipe
        for p, data in items:
            pipe.submit(TransmuxJob(data, p.aes_key, p.iv, None, p))  # the pending rides as the job's frag
        return pipe.launch()

    def complete_transmux(self, batch) -> None:
        """Wait for a launched transmux batch; its info rows go to the players as columns."""
        jobs, rows, plain, has = self.pipe.complete_arrays(batch)
        if not jobs:
            return
        by_rid = self._by_rid
        per: Dict[int, List[Tuple[int, _Pending]]] = {}
        for i, job in enumerate(jobs):
            p = job.frag
            by_rid[p.w].pop(p.rid, None)
            p.req = None  # Request.callbacks is p: drop the cycle so refcounting frees both now
            c = per.get(p.w)
            if c is None:
                c = per[p.w] = []
            c.append((i, p))
        code = _SOURCE_CODE
        for w, c in per.items():
            idx = np.fromiter([i for i, _ in c], dtype=np.int64, count=len(c))
            self._chunks[w].append((
                np.fromiter([p.rid for _, p in c], dtype=np.int64, count=len(c)),
                np.fromiter([code[p.source] for _, p in c], dtype=np.int8, count=len(c)),
                np.fromiter([p.nbytes for _, p in c], dtype=np.int64, count=len(c)),
                np.fromiter([p.cdn_ms for _, p in c], dtype=np.float64, count=len(c)),
                np.fromiter([p.p2p_ms for _, p in c], dtype=np.float64, count=len(c)),
                plain[idx], has[idx], rows[idx]))

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



# ============================================================================ player process
def player_main(conn: Any, spec: Dict[str, Any]) -> None:
    """A fleet player process: the bundle ``Hls`` over a :class:`RemoteNode`, drained as fast
    as the node answers (the throughput bench's player).  ``spec``: ``origin`` (keyword
    arguments of ``SyntheticHlsOrigin``: the player reads playlists and keys from it, the
    node process serves the segments), ``hls_config``, ``p2p_config``, ``world``, ``rank``.
    Control from the node: ``("mark", tag)`` -> reply ``("mark", tag, counters)`` once every
    answer sent before it is buffered; ``("stop",)`` -> close and exit."""
    import copy

    from .. import Hls
    from ..agent.node import node_for_config, set_current_node
    from ..net import new_event_loop
    from ..net.origin import SyntheticHlsOrigin
    from ..player import MediaElement
    from ..utils.runtime import tune_gc

    import torch

    torch.set_num_threads(1)  # a player does no tensor math: no intra-op pool competing for cores
    if torch.cuda.device_count():
        log.warning("fleet player sees %d GPU(s); it should not (HIP_VISIBLE_DEVICES)", torch.cuda.device_count())
    set_current_node(None)
    loop = new_event_loop("real")
    origin = SyntheticHlsOrigin(**spec["origin"])
    p2p = copy.deepcopy(spec["p2p_config"])
    p2p["gpuSwarm"] = {"backend": "remote", "conn": conn, "world": spec.get("world", 1), "rank": spec.get("rank", 0)}
    node = node_for_config(p2p)
    hls = Hls(dict(spec["hls_config"]), p2p)
    media = MediaElement(mode="drain", loop=loop)
    counters = {"buffered": 0, "errors": 0, "level_switches": 0, "bytes": 0}

    def on_buffered(e, d):
        counters["buffered"] += 1

    hls.on(Hls.Events.FRAG_BUFFERED, on_buffered)
    hls.on(Hls.Events.ERROR, lambda e, d: counters.__setitem__("errors", counters["errors"] + 1))
    hls.on(Hls.Events.LEVEL_SWITCH, lambda e, d: counters.__setitem__("level_switches",
                                                                     counters["level_switches"] + 1))
    # start together: a player that started early would run ahead into the next one's slice
    conn.send(("ready",))
    while True:
        msg = conn.recv()
        if msg[0] == "go":
            break
        if msg[0] == "stop":
            node.close()
            return
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    sc = hls.streamController

    def drain():
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
                tune_gc()
                gc_tuned = True
                if prof is not None:
                    prof.enable()
            while node.control:
                msg = node.control.pop(0)
                if msg[0] == "mark":
                    counters["bytes"] = node.stats.get("cdn", 0) + node.stats.get("p2p", 0)
                    conn.send(("mark", msg[1], dict(counters)))
                elif msg[0] == "stop":
                    return
    finally:
        if prof is not None:
            import io
            import pstats

            prof.disable()
            out = io.StringIO()
            pstats.Stats(prof, stream=out).sort_stats("tottime").print_stats(40)
            with open(f"{os.environ['HLSP2P_PLAYER_PROFILE']}.player{spec.get('rank', 0)}_{os.getpid()}.txt", "w") as f:
                f.write(f"buffered {counters['buffered']}\n" + out.getvalue())
        try:
            hls.destroy()
        finally:
            node.close()
