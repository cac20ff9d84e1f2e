"""SwarmNode — one MI355X (or CPU) peer of the swarm: HBM segment cache + exchange rounds.

This is the engine behind the peer agent's ``getSegment`` (the closed-source
``streamroot-p2p`` module in the reference), designed for the hardware:

* **Cache**: one ``uint8`` arena tensor in HBM (sized for the 288 GB part) whose layout
  is managed by the native ``SegmentStore`` ring allocator; segments received in a round
  land contiguously.
* **Rounds** (SURVEY §5.8): requests accumulate; every rank then runs one collective
  round — all-gather of a small control message (wants, cache delta, flags, counters) on
  the control plane, identical deterministic planning everywhere (native
  ``plan_round``), a CDN phase (pinned-host -> HBM ``hipMemcpyAsync`` batch on a side
  stream, the DMA engines) with ingest CRC on the MFMA CRC kernel, and a P2P phase: ONE
  contiguous buffer per peer pair over RCCL (one native ncclGroupStart/Send/Recv group on the
  node's stream, ``kernels/rccl_comm.cpp``), the sender's CRCs as
  a trailer, verified on device by the receiver.
* **Asynchronous rounds**: :meth:`launch_round` (collective) only *enqueues* device work
  and records an event; :meth:`complete_round` (local) waits for it, commits/drops and
  delivers.  A throughput deployment keeps round ``t+1`` in flight on the device while the
  host completes round ``t`` (``tick()`` = launch + complete for event-loop players).
* **Faults**: a peer copy failing its CRC is dropped and re-requested from the CDN next
  round; churn is modelled by ranks announcing ``online=False`` (they still join the
  collectives, as an RCCL communicator cannot shrink).

Completion semantics match the reference loader contract: ``onProgress({cdnDownloaded,
p2pDownloaded, cdnDuration, p2pDuration})`` then ``onSuccess(data)`` where ``data`` is a
zero-copy ``uint8`` view of the arena, or ``onError(HttpError)``
(``lib/integration/p2p-loader-generator.js:164-208``).
"""
from __future__ import annotations

import contextlib
import itertools
import logging
import os
import threading
import time
import zlib
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..net import http
from ..net.event_loop import get_event_loop
from ..ops import crc as _crc
from ..ops import segment as _seg
from ..ops._native import runtime as _rt
from ..parallel.comm import LocalComm, SwarmComm
from ..utils.trace import PhaseTimer, RequestTrace, TraceLog

log = logging.getLogger("hlsjs_p2p_wrapper_amd.node")

MAGIC = 0x48505032  # "HPP2"
HDR = 16
ALIGN = 256
SLACK = 4096
PIN_DELAY_ROUNDS = 2  # delivered segments stay pinned this many launches (consumers run async)


def swarm_id_for(content_id: str) -> int:
    return zlib.crc32(content_id.encode()) & 0x7FFFFFFF


_M32 = 0xFFFFFFFF


class Request:
    """One ``getSegment`` request: the loader handle (``abort()``) and its delivery state."""

    __slots__ = ("node", "key", "url", "headers", "callbacks", "agent", "aborted", "done", "t_submit")

    def __init__(self, node: "SwarmNode", key: Tuple[int, int, int, int], url: str, headers: Dict[str, str],
                 callbacks: Any, agent: Any = None, aborted: bool = False, done: bool = False,
                 t_submit: float = 0.0) -> None:
        self.node = node
        self.key = key
        self.url = url
        self.headers = headers
        self.callbacks = callbacks
        self.agent = agent
        self.aborted = aborted
        self.done = done
        self.t_submit = t_submit

    def abort(self) -> None:
        self.aborted = True

    def __repr__(self) -> str:
        return f"Request(key={self.key}, url={self.url!r}, aborted={self.aborted}, done={self.done})"


class _Want:
    """One wanted segment of this rank (all requests for one key share it).  Slotted plain
    class: one per request, and a dataclass ``__init__`` is interpreted code even here."""

    __slots__ = ("key", "url", "headers", "size", "want_id", "waiters", "force_cdn", "attempts", "round",
                 "prefetch", "row", "net", "staged", "staging", "src", "loc")

    def __init__(self, key: Tuple[int, int, int, int], url: str, headers: Dict[str, str], size: int,
                 want_id: int, waiters: Optional[List[Request]] = None, force_cdn: bool = False,
                 attempts: int = 0, round: int = -1, prefetch: bool = False) -> None:
        self.key = key
        self.url = url
        self.headers = headers
        self.size = size
        self.want_id = want_id
        self.waiters = [] if waiters is None else waiters
        self.force_cdn = force_cdn
        self.attempts = attempts
        self.round = round  # round it is in flight in (-1: waiting)
        self.prefetch = prefetch  # issued by an agent's prefetch planner (may have no waiters)
        self.row = ()  # control-message encoding (key x4, size, want_id | force_cdn << 62 | ...)
        # network origin (net/network.py): (origin, path, range); the body must be staged in
        # host memory (staged) before a round may fetch it; staging: download in progress
        self.net = None
        self.staged = True
        self.staging = False
        self.src = None  # (origin, path, range) resolved at creation: the CDN phase reuses it
        self.loc = None  # (host tensor, offset, length) when the origin's bytes never move (VOD)

    def __repr__(self) -> str:
        return f"_Want(key={self.key}, size={self.size}, want_id={self.want_id}, round={self.round})"

    def encode(self) -> None:
        self.row = (*self.key, self.size,
                    self.want_id | ((1 if self.force_cdn else 0) << 62) | ((0 if self.staged else 1) << 61)
                    | ((1 if self.staging else 0) << 60))


class _Completion:
    __slots__ = ("req", "data", "source", "nbytes", "cdn_ms", "p2p_ms", "entry", "delay", "peer")

    def __init__(self, req, data, source, nbytes, cdn_ms, p2p_ms, entry=-1, delay=0.0, peer=-1):
        self.peer = peer
        self.req = req
        self.data = data
        self.source = source
        self.nbytes = nbytes
        self.cdn_ms = cdn_ms
        self.p2p_ms = p2p_ms
        self.entry = entry
        self.delay = delay


@dataclass(eq=False)
class RoundHandle:
    round: int
    all_leaving: bool
    empty: bool = True
    wants: List[_Want] = field(default_factory=list)
    by_id: Dict[int, _Want] = field(default_factory=dict)
    cdn_entries: List[Tuple[_Want, int, int, int]] = field(default_factory=list)
    # received segments, plain ints: (want_id, src rank, entry id, arena offset, length)
    recv_entries: List[Tuple[int, int, int, int, int]] = field(default_factory=list)
    send_pins: Optional[np.ndarray] = None
    hold: List[np.ndarray] = field(default_factory=list)  # in-flight entries pinned until delivered
    release: List[Any] = field(default_factory=list)  # network-origin wants whose staged copy this round DMAs
    sent_bytes: int = 0
    ev_cdn: Any = None
    dmas: int = 0
    ev_p2p: Any = None
    cdn_ms: float = 0.0
    p2p_ms: float = 0.0
    shaped_ms: float = 0.0
    ok_dev: Any = None
    ok_host: Any = None
    done: Any = None
    n_wants: int = 0
    n_send: int = 0
    t0: float = 0.0
    completed: bool = False


class _EventPool:
    """Recycled HIP events (a fresh torch.cuda.Event costs ~5 us of host time; a round uses
    five).  An event goes back to the pool only after the host has waited on its round."""

    def __init__(self) -> None:
        self._free: Dict[bool, List[Any]] = {True: [], False: []}

    def get(self, timing: bool = False):
        free = self._free[timing]
        return free.pop() if free else torch.cuda.Event(enable_timing=timing)

    def put(self, timing: bool, *events) -> None:
        self._free[timing].extend(e for e in events if e is not None)


class SwarmNode:
    """One swarm peer (one GPU per process): HBM segment cache, collective exchange rounds,
    the request queue the peer agents feed."""
    def __init__(self, comm: Optional[SwarmComm] = None, device: Any = "auto", cache_bytes: int = 1 << 30,
                 loop=None, cdn_dedup: bool = True, round_interval_ms: Optional[float] = None,
                 auto_tick: bool = True, max_wants_per_round: Optional[int] = None) -> None:
        self.comm = comm or LocalComm()
        self.rank = self.comm.rank
        self.world = self.comm.world_size
        if device in (None, "auto"):
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.is_cuda = self.device.type == "cuda"
        self.loop = loop or get_event_loop()
        self.rt = _rt()
        self.cache_bytes = int(cache_bytes)
        self.store = self.rt.SegmentStore(self.cache_bytes, ALIGN)
        self.directory = self.rt.Directory()
        self.arena = torch.empty(self.cache_bytes + SLACK, dtype=torch.uint8, device=self.device)
        self.crc_dev = torch.zeros(1024, dtype=torch.int32, device=self.device)  # CRC per entry id
        # all node device work (ingest CRC, RCCL, verify CRC) runs on its own stream: consumers
        # (decrypt/demux of the previous round) on the default stream overlap it.  The CDN
        # H2D DMAs get a copy stream of their own, so round t+1's DMA queues directly behind
        # round t's instead of behind round t's ingest CRC: the PCIe link never idles between
        # rounds (the node stream waits for each round's DMA with an event).  Reuse of arena
        # space is ordered by the store's pins, not by stream order: reserved and in-flight
        # entries stay pinned until complete_round, delivered ones PIN_DELAY_ROUNDS launches.
        self.stream = torch.cuda.Stream(self.device) if self.is_cuda else None
        self.copy_stream = (torch.cuda.Stream(self.device) if self.is_cuda and
                            os.environ.get("HLSP2P_COPY_STREAM", "1") != "0" else None)
        self._events = _EventPool()
        self.online = True
        self.upload_on = True
        self.download_on = True
        self.cdn_dedup = cdn_dedup
        self.round = 0
        self.round_interval_ms = round_interval_ms
        self.auto_tick = auto_tick
        self.max_wants_per_round = max_wants_per_round
        self.leaving = False
        self.closed = False
        self._wants: Dict[Tuple[int, int, int, int], _Want] = {}
        self._next_want_id = 1
        self._tick_scheduled = False
        self._timer = None
        self._pins: List[Tuple[int, np.ndarray]] = []  # (release at launch #, entry ids)
        self._agents: List[Any] = []
        self._prefetched: Dict[Tuple[int, int, int, int], str] = {}  # key -> "cdn" | "p2p"
        self._net_wants = False  # some want came from a network origin (plans may carry STAGE rows)
        self.peer_online = np.ones(self.world, dtype=bool)
        self.stats = {"cdn": 0, "p2p": 0, "upload": 0, "cache": 0, "rounds": 0, "crc_failures": 0,
                      "segments": 0, "cdn_segments": 0, "p2p_segments": 0, "prefetched": 0}
        self.swarm_stats = {"cdn": 0, "p2p": 0, "upload": 0}
        self.last_round: Dict[str, Any] = {}
        self.corrupt_next_recv = 0  # fault injection: flip a byte in the next N received rounds
        self.link_kbps: Dict[int, float] = {}  # fault injection: slow link from peer -> kbit/s
        self.timer = PhaseTimer()
        # per-request trace records {key, trequest, tfirst, tload, source, bytes, peer, round}
        # (SURVEY §5.1); None = off (p2pConfig["gpuSwarm"]["trace"] or enable_trace())
        self.trace: Optional[TraceLog] = None
        self.metrics_server: Any = None  # utils.metrics.MetricsServer (gpuSwarm.metricsPort)
        self._lock = threading.RLock()
        if self.world > 1 and auto_tick:
            self._timer = self.loop.set_interval(self._timer_tick, round_interval_ms or 10.0)

    # ------------------------------------------------------------------ agents
    def attach(self, agent: Any) -> None:
        """Register a peer agent (its requests, stats and metrics)."""
        self._agents.append(agent)

    def detach(self, agent: Any) -> None:
        """Unregister an agent and fail its pending requests."""
        if agent in self._agents:
            self._agents.remove(agent)
        for w in list(self._wants.values()):
            w.waiters = [r for r in w.waiters if r.agent is not agent]

    @property
    def flags(self) -> int:
        """Control-message flag bits: online / download / upload state."""
        f = 0
        if self.online:
            f |= self.rt.FLAG_ONLINE
        if self.upload_on:
            f |= self.rt.FLAG_UPLOAD
        if self.download_on:
            f |= self.rt.FLAG_DOWNLOAD
        if self.cdn_dedup:
            f |= self.rt.FLAG_CDN_DEDUP
        return f

    # ------------------------------------------------------------------ requests
    def request(self, key: Tuple[int, int, int, int], url: str, headers: Optional[Dict[str, str]],
                callbacks: Any, agent: Any = None, view: Any = None) -> Request:
        """Queue a fragment request for key ``(swarm, level, urlId, sn)``; served from the cache,
        a peer or the CDN in the next round.  (``view``: the agent's SegmentView, which a
        fleet's remote node uses to find the fragment's AES key; unused here.)"""
        k0, k1, k2, k3 = key
        req = Request(self, (int(k0) & _M32, int(k1) & _M32, int(k2) & _M32, int(k3) & _M32), url,
                      dict(headers) if headers else {}, callbacks, agent, False, False, self.loop.now())
        eid = self.store.lookup1(*req.key)
        if eid >= 0:  # local cache hit
            self.store.pin(np.array([eid], dtype=np.int64))
            self.loop.call_soon(self._serve_local, req, eid)
            return req
        self._prefetched.pop(req.key, None)  # evicted before use
        w = self._wants.get(req.key)
        if w is None:
            try:
                w = self._new_want(req.key, url, req.headers)
            except http.HttpError as e:
                self.loop.call_soon(self._fail, req, e)
                return req
            self._wants[req.key] = w
        w.waiters.append(req)
        self._schedule()
        return req

    def _new_want(self, key, url: str, headers: Dict[str, str], prefetch: bool = False) -> _Want:
        """A want for ``url``: its size from the origin, or, for a network origin whose body is
        not staged yet, size 0 and ``staged=False`` (the planner then has it staged first)."""
        origin, path = http.resolve(url)
        rng = http.parse_range(headers) if headers else None
        net = loc = None
        if getattr(origin, "staged_fetch", False):
            size = origin.staged_size(path, rng)
            net = (origin, path, rng)
        else:
            locate = getattr(origin, "locate", None)
            loc = locate(path, url, rng) if locate is not None else None
            size = loc[2] if loc is not None else origin.size(path, url, rng)
        wid = self._next_want_id
        self._next_want_id = wid + 1
        w = _Want(key, url, headers, int(size or 0), wid, prefetch=prefetch)
        if net is not None:
            w.net = net
            w.staged = size is not None
            self._net_wants = True
            w.encode()
        else:
            w.src = (origin, path, rng)
            w.loc = loc
            w.row = key + (w.size, wid)  # encode() of a fresh, staged, not forced want
        return w

    def _stage(self, w: _Want) -> None:
        """Plan said: download ``w``'s body from its network origin into host memory.  The
        completion comes back to this loop; the want is planned again once staged."""
        if w.staging or w.staged or w.net is None:
            return
        origin, path, rng = w.net
        w.staging = True
        w.encode()  # published as downloading: the planner stages it nowhere else meanwhile
        loop = self.loop
        loop.hold()

        def done(n, err):  # worker thread
            try:
                loop.call_soon_threadsafe(self._on_staged, w, n, err)
            finally:
                loop.release()

        origin.stage(path, w.url, rng, w.headers, done)

    def _on_staged(self, w: _Want, n, err) -> None:
        w.staging = False
        w.encode()
        if err is not None:
            if self._wants.get(w.key) is w:
                del self._wants[w.key]
            for req in w.waiters:
                self._fail(req, err)
            return
        w.size = int(n)
        w.staged = True
        w.encode()
        if self._wants.get(w.key) is w:
            self._schedule()
        else:  # nobody waits any more (aborted / served meanwhile): drop the host copy
            origin, path, rng = w.net
            origin.release(path, rng)

    def prefetch(self, key: Tuple[int, int, int, int], url: str, headers: Optional[Dict[str, str]] = None) -> bool:
        """Fill the cache with a segment no player asked for yet (agent prefetch planning,
        SURVEY §2.3).  It travels in the next round like any want (P2P from a holder, or
        the CDN); a player request arriving meanwhile simply joins it.  True if issued."""
        key = tuple(int(k) & 0xFFFFFFFF for k in key)
        if key in self._wants or self.store.lookup1(*key) >= 0:
            return False
        try:
            w = self._new_want(key, url, dict(headers or {}), prefetch=True)
        except http.HttpError:
            return False
        self._wants[key] = w
        self.stats["prefetched"] += 1
        self._schedule()
        return True

    def _schedule(self) -> None:
        if self.world == 1 and self.auto_tick and not self._tick_scheduled:
            self._tick_scheduled = True
            self.loop.call_soon(self._local_tick)

    def _local_tick(self) -> None:
        self._tick_scheduled = False
        if self._wants:
            self.tick()

    def _timer_tick(self) -> None:
        if not self.closed:
            self.tick()

    def _serve_local(self, req: Request, eid: int) -> None:
        try:
            if req.aborted:
                return
            off, n = (int(x) for x in self.store.entries(np.array([eid], dtype=np.int64))[0][:2])
            # first delivery of a prefetched segment is accounted where its bytes came from
            src = self._prefetched.pop(req.key, None)
            if src is None:
                self.stats["cache"] += n
            self._deliver_now([_Completion(req, self.arena[off:off + n], src or "cache", n, 0.0, 0.0)])
        finally:
            self.store.unpin(np.array([eid], dtype=np.int64))

    def _fail(self, req: Request, err: Exception) -> None:
        if req.aborted or req.done:
            return
        req.done = True
        cb = req.callbacks
        on_error = cb.get("onError") if isinstance(cb, dict) else getattr(cb, "onError", None)
        if on_error is not None:
            on_error(err)

    # ------------------------------------------------------------------ control messages
    def _encode(self, wants: List[_Want], adds: np.ndarray, rms: np.ndarray) -> np.ndarray:
        hdr = np.zeros(HDR, dtype=np.int64)
        hdr[0] = MAGIC
        hdr[1] = self.flags
        hdr[2] = len(wants)
        hdr[3] = len(adds)
        hdr[4] = len(rms)
        hdr[5] = 1 if self.leaving else 0
        hdr[6] = self.round
        hdr[7] = self.stats["cdn"]
        hdr[8] = self.stats["p2p"]
        hdr[9] = self.stats["upload"]
        if wants:
            # rows pre-encoded at want creation: one flat fromiter (~3x faster than np.array of tuples)
            w = np.fromiter(itertools.chain.from_iterable([x.row for x in wants]), dtype=np.int64,
                            count=6 * len(wants))
        else:
            w = np.zeros((0, 6), dtype=np.int64)
        return np.concatenate([hdr, w.reshape(-1), adds.reshape(-1).astype(np.int64),
                               rms.reshape(-1).astype(np.int64)])

    def _grow_crc(self, n: int) -> None:
        if n > self.crc_dev.numel():
            new = torch.zeros(max(n, 2 * self.crc_dev.numel()), dtype=torch.int32, device=self.device)
            new[:self.crc_dev.numel()] = self.crc_dev
            self.crc_dev = new

    # ------------------------------------------------------------------ rounds
    def tick(self) -> bool:
        """One synchronous collective round (launch + complete).  True when every rank
        is leaving."""
        with self._lock:
            h = self.launch_round()
            self.complete_round(h)
            return h.all_leaving

    def launch_round(self) -> RoundHandle:
        """Collective: exchange control messages, plan, and ENQUEUE this round's device
        work (CDN copies, ingest CRC, RCCL transfers, verify CRC).  Host does not wait."""
        rt = self.rt
        t0 = time.perf_counter()
        self.round += 1
        self.stats["rounds"] += 1
        keep = []
        for rel, ids in self._pins:
            if rel <= self.round:
                self.store.unpin(ids)
            else:
                keep.append((rel, ids))
        self._pins = keep
        # ---------------- 1. control plane
        for agent in self._agents:  # agents plan (prefetch, live-window eviction) before wants go out
            hook = getattr(agent, "before_round", None)
            if hook is not None:
                hook()
        wants, spec = [], []  # player requests first, then speculative (prefetch-only) wants
        cap = self.max_wants_per_round
        for k in list(self._wants):
            w = self._wants[k]
            if w.round >= 0:
                continue
            if not w.waiters and w.prefetch:
                spec.append(w)
                continue
            if not any(not r.aborted for r in w.waiters):
                del self._wants[k]
                if w.net is not None and w.staged:  # nobody wants it any more: drop the host copy
                    w.net[0].release(w.net[1], w.net[2])
                continue
            wants.append(w)
            if cap is not None and len(wants) >= cap:
                break
        if spec and (cap is None or len(wants) < cap):
            wants.extend(spec if cap is None else spec[:cap - len(wants)])
        wants = self._admit(wants)
        adds, rms = self.store.take_delta()
        parts = self.comm.allgather_control(self._encode(wants, adds, rms))
        # every rank's deltas into the directory + the round's want rows, in one native call
        all_wants, flags, all_leaving, swarm_tot = rt.ingest_control(self.directory, parts, MAGIC, HDR)
        self.peer_online = (flags & rt.FLAG_ONLINE) != 0
        self.swarm_stats = {"cdn": int(swarm_tot[0]), "p2p": int(swarm_tot[1]), "upload": int(swarm_tot[2])}
        h = RoundHandle(self.round, all_leaving, t0=t0)
        t_ctrl = time.perf_counter()
        self.timer.add("control", t_ctrl - t0)
        if not len(all_wants):
            return h
        h.empty = False
        plan = rt.plan_round(self.directory, all_wants, flags, self.world)
        me = self.rank
        h.wants = wants
        h.by_id = {w.want_id: w for w in wants}
        for w in wants:
            w.round = self.round
        h.n_wants = len(all_wants)
        cdn_rows = plan[(plan[:, 5] == -1) & (plan[:, 6] == me)]
        if self._net_wants:  # network-origin wants this rank must download first (STAGE rows)
            for wid in plan[(plan[:, 5] == -2) & (plan[:, 6] == me), 7].tolist():
                w = h.by_id.get(wid)
                if w is not None:
                    self._stage(w)
        send_rows = plan[plan[:, 5] == me]
        recv_rows = plan[(plan[:, 6] == me) & (plan[:, 5] >= 0)]
        h.n_send = len(send_rows)
        # ---------------- 2. pin what we send from cache (seeded rows come from the CDN phase)
        # send_eids[i]: store entry of send row i (-1: missing), aligned with send_rows
        send_eids = np.full(len(send_rows), -1, dtype=np.int64)
        cached = send_rows[:, 8] == 0
        if cached.any():
            ids = self.store.lookup(np.ascontiguousarray(send_rows[cached, :4]), False)
            send_eids[cached] = ids
            valid = ids[ids >= 0]
            if len(valid):
                self.store.pin(valid)
                h.send_pins = valid
        t_cdn0 = time.perf_counter()
        self.timer.add("plan", t_cdn0 - t_ctrl)
        with (torch.cuda.stream(self.stream) if self.is_cuda else contextlib.nullcontext()):
            # ---------------- 3. CDN phase (pinned host -> HBM, DMA engines)
            if len(cdn_rows):
                self._cdn_phase(h, cdn_rows)
                seeded = np.flatnonzero(~cached)
                if len(seeded) and h.cdn_entries:  # forwarded in this same round
                    fetched = {w.key: eid for w, eid, _, _ in h.cdn_entries}
                    send_eids[seeded] = [fetched.get(k, -1) for k in map(tuple, send_rows[seeded, :4].tolist())]
            t_p2p0 = time.perf_counter()
            self.timer.add("cdn_enqueue", t_p2p0 - t_cdn0)
            # ---------------- 4. P2P phase: entered by EVERY rank when the (identical) plan
            # has any transfer, so a collective transport (the in-process hub) stays in step;
            # RCCL point-to-point with no local ops posts nothing
            if bool((plan[:, 5] >= 0).any()):
                self._p2p_phase(h, send_rows, recv_rows, send_eids)
            h.sent_bytes = int(send_rows[:, 4].sum()) if len(send_rows) else 0
            if self.is_cuda:
                h.done = self._events.get()
                h.done.record(self.stream)  # explicit stream: skips torch's current_stream() lookup
        self.timer.add("p2p_enqueue", time.perf_counter() - t_p2p0)
        return h

    def complete_round(self, h: RoundHandle) -> None:
        """Local: wait for the round's device work, verify, commit and deliver."""
        if h.completed:
            return
        h.completed = True
        if h.empty:
            self.last_round = {"wants": 0, "ms": (time.perf_counter() - h.t0) * 1e3}
            return
        t0 = time.perf_counter()
        if h.done is not None and not h.done.query():
            self._wait_round(h)
        t1 = time.perf_counter()
        self.timer.add("wait_device", t1 - t0)
        if h.ev_cdn is not None:
            h.cdn_ms = h.ev_cdn[0].elapsed_time(h.ev_cdn[1])
            self._events.put(True, *h.ev_cdn)
        if h.ev_p2p is not None:
            h.p2p_ms = h.ev_p2p[0].elapsed_time(h.ev_p2p[1])
            self._events.put(True, *h.ev_p2p)
        if h.done is not None:
            self._events.put(False, h.done)
            h.done = None
        okl = h.ok_host.numpy().tolist() if h.ok_host is not None else None
        if okl is None or all(okl):
            good, bad = h.recv_entries, []
        else:
            good = [e for e, k in zip(h.recv_entries, okl) if k]
            bad = [e for e, k in zip(h.recv_entries, okl) if not k]
        if good:
            self.store.commit(np.asarray([e[2] for e in good], dtype=np.int64))
        if bad:
            self.store.drop(np.asarray([e[2] for e in bad], dtype=np.int64))
            self.stats["crc_failures"] += len(bad)
        if h.send_pins is not None:
            self.store.unpin(h.send_pins)
        for w in h.release:  # the round's DMAs are done: drop the staged host copies
            origin, path, rng = w.net
            origin.release(path, rng)
        self.stats["upload"] += h.sent_bytes
        completions: List[_Completion] = []
        cdn_views = self._views([e[2] for e in h.cdn_entries], [e[3] for e in h.cdn_entries])
        cdn_ms = max(h.cdn_ms, h.shaped_ms)
        for (w, eid, off, n), view in zip(h.cdn_entries, cdn_views):
            if self._wants.get(w.key) is w:
                del self._wants[w.key]
            if w.prefetch and not w.waiters:
                self._prefetched[w.key] = "cdn"
            for req in w.waiters:
                completions.append(_Completion(req, view, "cdn", n, cdn_ms, 0.0, eid, h.shaped_ms))
        link_q: Dict[int, int] = {}  # slow-link fault injection: bytes queued per source link
        link_kbps = self.link_kbps
        wants_map = self._wants
        p2p_views = self._views([e[3] for e in good], [e[4] for e in good])
        for (want_id, src, eid, off, n), view in zip(good, p2p_views):
            w = h.by_id.get(want_id)
            if w is None:
                continue
            if wants_map.get(w.key) is w:
                del wants_map[w.key]
            if w.net is not None and w.staged:  # staged here, but a peer's copy came first
                w.net[0].release(w.net[1], w.net[2])
            if w.prefetch and not w.waiters:
                self._prefetched[w.key] = "p2p"
            p2p_ms, delay = h.p2p_ms, 0.0
            kbps = link_kbps.get(src) if link_kbps else None
            if kbps:
                link_q[src] = link_q.get(src, 0) + n
                delay = link_q[src] * 8.0 / kbps  # kbit/s == bit/ms
                p2p_ms = max(p2p_ms, delay)
            for req in w.waiters:
                completions.append(_Completion(req, view, "p2p", n, 0.0, p2p_ms, eid, delay, peer=src))
        for e in bad:
            w = h.by_id.get(e[0])
            if w is not None:
                w.force_cdn = True  # corrupted peer copy: go to the CDN next round
                w.encode()
                w.attempts += 1
                w.round = -1
        served = None
        for w in h.wants:  # planned but not served (e.g. a CDN error already reported)
            if w.round == h.round and wants_map.get(w.key) is w:
                if served is None:
                    served = {id(e[0]) for e in h.cdn_entries}
                    served.update(id(h.by_id.get(e[0])) for e in h.recv_entries)
                if id(w) not in served:
                    w.round = -1
        t2 = time.perf_counter()
        self.timer.add("commit", t2 - t1)
        self._deliver(completions)  # delivered entries stay pinned PIN_DELAY_ROUNDS launches
        for ids in h.hold:  # in-flight pins from reservation (dropped entries: no-op)
            self.store.unpin(ids)
        h.hold = []
        self.timer.add("deliver", time.perf_counter() - t2)
        self.timer.add("dev_cdn_ms", h.cdn_ms / 1e3)
        self.timer.add("dev_p2p_ms", h.p2p_ms / 1e3)
        self.last_round = {"wants": h.n_wants, "cdn": len(h.cdn_entries), "send": h.n_send,
                           "recv": len(h.recv_entries), "cdn_ms": h.cdn_ms, "dmas": h.dmas, "p2p_ms": h.p2p_ms,
                           "ms": (time.perf_counter() - h.t0) * 1e3}
        if any(w.round < 0 and not w.staging for w in self._wants.values()):
            self._schedule()  # (a want being downloaded is rescheduled when it lands)

    ROUND_SPIN_S = 0.02  # busy-poll a round's completion this long before checking for peer failures

    def _wait_round(self, h: RoundHandle) -> None:
        """Wait for a round's device work without hanging on a dead peer.

        A round whose RCCL transfers wait for a peer that crashed never completes, and
        ``hipEventSynchronize`` would block forever.  Instead: poll the round's event (the
        common case finishes within the first ``ROUND_SPIN_S``), then poll it every
        millisecond while asking the communicator for an asynchronous error
        (``ncclCommGetAsyncError``) and watching the ``HLSP2P_ROUND_TIMEOUT`` deadline
        (default 600 s); either one raises instead of hanging the rank."""
        ev = h.done
        spin_end = time.perf_counter() + self.ROUND_SPIN_S
        while time.perf_counter() < spin_end:
            if ev.query():
                return
        check = getattr(self.comm, "async_error", None)
        deadline = time.perf_counter() + float(os.environ.get("HLSP2P_ROUND_TIMEOUT", "600"))
        while not ev.query():
            err = check() if check is not None else ""
            if err:
                raise RuntimeError(f"rank {self.rank}: swarm round {h.round} failed in the data plane: {err}")
            if time.perf_counter() > deadline:
                raise TimeoutError(f"rank {self.rank}: swarm round {h.round} did not complete on the device "
                                   "(HLSP2P_ROUND_TIMEOUT); a peer may have stopped")
            time.sleep(1e-3)

    def _views(self, offs: List[int], lens: List[int]) -> List[torch.Tensor]:
        """Zero-copy uint8 views of the arena for a round's deliveries (one native call on
        the GPU; a Python slice costs ~1.5 us per view)."""
        if not offs:
            return []
        if self.is_cuda:
            from ..ops._native import device as _dev

            return _dev().arena_views(self.arena, np.asarray(offs, dtype=np.int64), np.asarray(lens, dtype=np.int64))
        arena = self.arena
        return [arena[o:o + n] for o, n in zip(offs, lens)]

    # ------------------------------------------------------------------ phases
    def _admit(self, wants: List[_Want]) -> List[_Want]:
        """Backpressure: a rank only ever receives what it asked for, so cap this round's
        wants to what the ring can place now without evicting pinned (in-flight or
        being-consumed) entries; the rest wait for the next round."""
        if not wants:
            return wants
        st = self.store
        sizes = [st.aligned(w.size) for w in wants]
        total = sum(sizes)
        if st.fits(total):
            return wants
        lo, hi = 0, len(wants)  # largest prefix that fits
        while lo < hi:
            mid = (lo + hi + 1) // 2
            if st.fits(sum(sizes[:mid])):
                lo = mid
            else:
                hi = mid - 1
        kept = wants[:lo]
        for w, a in zip(wants[lo:], sizes[lo:]):
            if a > self.cache_bytes:  # can never fit: fail it
                if self._wants.get(w.key) is w:
                    del self._wants[w.key]
                if w.net is not None and w.staged:
                    w.net[0].release(w.net[1], w.net[2])
                err = http.HttpError(507, f"segment of {w.size} bytes exceeds the {self.cache_bytes}-byte cache")
                for req in w.waiters:
                    self.loop.call_soon(self._fail, req, err)
        self.stats["deferred"] = self.stats.get("deferred", 0) + len(wants) - lo
        return kept

    def _cdn_phase(self, h: RoundHandle, cdn_rows: np.ndarray) -> None:
        wants, sources = [], []
        for wid in cdn_rows[:, 7].tolist():
            w = h.by_id.get(wid)
            if w is None:
                continue
            try:
                if w.net is not None:  # network origin: the staged (already ranged) host copy
                    origin, path, rng = w.net
                    data, off, n, _ = origin.resource_range(path, rng)
                    corrupt = False
                    h.release.append(w)
                elif w.loc is not None:  # VOD origin: located when the want was created
                    data, off, n = w.loc
                    corrupt = w.src[0].should_corrupt(w.src[1])
                else:
                    if w.src is not None:
                        origin, path, rng = w.src
                    else:
                        origin, path = http.resolve(w.url)
                        rng = http.parse_range(w.headers) if w.headers else None
                    data, off, n, _ = origin.resource(path)
                    if rng is not None:
                        s, e = rng
                        e = n - 1 if e is None else min(e, n - 1)
                        off, n = off + s, max(0, e - s + 1)
                    corrupt = origin.should_corrupt(path)
            except http.HttpError as e:
                if self._wants.get(w.key) is w:
                    del self._wants[w.key]
                for req in w.waiters:
                    self.loop.call_soon(self._fail, req, e)
                continue
            wants.append(w)
            sources.append((data, off, n, corrupt))
        if not wants:
            return
        keys = np.asarray([w.key for w in wants], dtype=np.int64)
        lens = np.asarray([s[2] for s in sources], dtype=np.int64)
        res = self.store.reserve_run(keys, lens, self.round)
        if res is None:  # _admit guarantees room; reaching this is a bookkeeping bug
            raise RuntimeError("segment cache cannot make room (pinned entries block eviction)")
        _, ids, offs = res
        self.store.pin(ids)  # in flight until delivered (complete_round unpins)
        h.hold.append(ids)
        self._grow_crc(int(ids.max()) + 1)
        if self.is_cuda:
            start = self._events.get(True)
            end = self._events.get(True)
            cs = self.copy_stream
            with (torch.cuda.stream(cs) if cs is not None else contextlib.nullcontext()):
                start.record(cs if cs is not None else self.stream)
                h.dmas = _h2d_batch(self.arena, offs, sources)
                end.record(cs if cs is not None else self.stream)
            if cs is not None:
                self.stream.wait_event(end)  # ingest CRC / forwarding sends read the DMA'd bytes
            h.ev_cdn = (start, end)
        else:
            t = time.perf_counter()
            arena = self.arena.numpy()  # numpy slices: a small torch copy_ costs ~0.1 ms on CPU
            for (data, off, n, _), doff in zip(sources, offs.tolist()):
                arena[doff:doff + n] = data.numpy()[off:off + n]
            h.cdn_ms = (time.perf_counter() - t) * 1e3
        for (_, _, n, corrupt), doff in zip(sources, offs.tolist()):
            if corrupt and n:
                self.arena[doff + n // 2] ^= 0xFF
        _crc.crc32_batch(self.arena, offs, lens, scatter_to=self.crc_dev, scatter_idx=ids)  # ingest CRCs
        self.store.commit(ids)  # announced next round; peers' reads are stream-ordered after the H2D
        # CDN bandwidth shaping (xhr-shaper analog): completions are deferred by the modelled
        # transfer time of this round's CDN bytes
        h.shaped_ms = http.Shaper.transfer_ms(int(lens.sum()))
        self.stats["cdn"] += int(lens.sum())
        self.stats["cdn_segments"] += len(wants)
        h.cdn_entries = [(w, eid, o, n) for w, eid, o, n in zip(wants, ids.tolist(), offs.tolist(), lens.tolist())]

    def _p2p_phase(self, h: RoundHandle, send_rows: np.ndarray, recv_rows: np.ndarray,
                   send_eids: np.ndarray) -> None:
        """Post this round's transfers.  Plan rows arrive sorted by (src, dst, key), so each
        peer's rows are one contiguous run.  Bookkeeping is batched over ALL peers: the
        per-peer layout and ring reservations in one native call, one gather of the send CRC
        trailers, one trailer buffer for every receive, the arena views in one call, and the
        received entry ids riding the verify CRC's descriptor block (per-peer Python and
        tensor ops cost ~50 us of host time per peer per round)."""
        sends: List[Tuple[int, torch.Tensor]] = []
        recvs: List[Tuple[int, torch.Tensor]] = []
        dev = self.device
        t_prep = time.perf_counter()
        # per-peer layout in ONE native call: contiguous send spans (or gather lists),
        # one pinned ring reservation per source (SegmentStore.p2p_layout)
        srun, gath, rrun, rid_a, roff_a = self.store.p2p_layout(
            np.ascontiguousarray(send_rows), np.ascontiguousarray(send_eids, dtype=np.int64),
            np.ascontiguousarray(recv_rows), self.round)
        # --- sends: one buffer (+ CRC trailer slice) per destination
        if len(send_rows):
            present_all = send_eids >= 0
            idx = _dev_index(np.where(present_all, send_eids, 0), dev)
            trailer_all = torch.index_select(self.crc_dev, 0, idx)
            if not present_all.all():  # missing entry: a bad CRC, the receiver re-fetches from the CDN
                trailer_all[torch.from_numpy(np.flatnonzero(~present_all)).to(dev)] = -1
            spans = self._views(srun[:, 4].tolist(), srun[:, 5].tolist()) if len(srun) and (srun[:, 3] == 0).all() \
                else None
            for k, (dst, a, b, mode, off, total) in enumerate(srun.tolist()):
                if mode == 0:
                    buf = spans[k] if spans is not None else self.arena[off:off + total]
                else:  # entries not back to back in the arena: gather into a staging buffer
                    buf = torch.zeros(total, dtype=torch.uint8, device=dev)
                    g = gath[gath[:, 0] == k]
                    if len(g):
                        _seg.copy_segments(self.arena, buf, g[:, 1], g[:, 2], g[:, 3])
                sends.append((dst, buf))
                sends.append((dst, trailer_all[a:b]))
        # --- recvs: the reserved runs; one trailer buffer for all of them
        if len(rrun):
            trailers = torch.empty(len(recv_rows), dtype=torch.int32, device=dev)
            views = self._views(rrun[:, 3].tolist(), rrun[:, 4].tolist())
            for (src, a, b, _, _), view in zip(rrun.tolist(), views):
                recvs.append((src, view))
                recvs.append((src, trailers[a:b]))
            h.hold.append(rid_a)  # pinned by p2p_layout until complete_round
            self._grow_crc(int(rid_a.max()) + 1)
            rlen = recv_rows[:, 4]
            rsrc = recv_rows[:, 5]
            h.recv_entries = list(zip(recv_rows[:, 7].tolist(), rsrc.tolist(), rid_a.tolist(), roff_a.tolist(),
                                      rlen.tolist()))
        self.timer.add("p2p_prep", time.perf_counter() - t_prep)
        t = time.perf_counter()
        if self.is_cuda:
            start = self._events.get(True)
            end = self._events.get(True)
            start.record(self.stream)  # launch_round runs this phase on the node stream
        self.comm.exchange(sends, recvs)
        if self.is_cuda:
            end.record(self.stream)
            h.ev_p2p = (start, end)
        else:
            h.p2p_ms = (time.perf_counter() - t) * 1e3
        if not h.recv_entries:
            return
        if self.corrupt_next_recv > 0:  # fault injection: transport corruption
            self.corrupt_next_recv -= 1
            o, n = h.recv_entries[0][3:5]
            if n:
                self.arena[o + n // 2] ^= 0x5A
        # verify against the senders' trailers; the combine kernel also scatters the computed
        # CRCs into the per-entry table (ids ride the descriptor H2D): a mismatching entry is
        # dropped in complete_round, so the table only ever serves verified values
        _, ok = _crc.crc32_batch(self.arena, roff_a, recv_rows[:, 4], expect_dev=trailers,
                                 scatter_to=self.crc_dev, scatter_idx=rid_a)
        if self.is_cuda:
            h.ok_host = torch.empty(ok.numel(), dtype=torch.uint8, pin_memory=True)
            h.ok_host.copy_(ok, non_blocking=True)
        else:
            h.ok_host = ok
        self.stats["p2p"] += int(recv_rows[:, 4].sum())
        self.stats["p2p_segments"] += len(recv_rows)

    # ------------------------------------------------------------------ delivery
    def _deliver(self, completions: List[_Completion]) -> None:
        now_list = [c for c in completions if c.delay <= 0]
        later = [c for c in completions if c.delay > 0]
        if later:  # shaped CDN / slowed-link transfers complete after their modelled duration
            ids = np.asarray([c.entry for c in later if c.entry is not None and c.entry >= 0], dtype=np.int64)
            if len(ids):
                self.store.pin(ids)
            delay = max(c.delay for c in later)
            for c in later:
                c.delay = 0.0
            self.loop.set_timeout(self._deliver_deferred, delay, later, ids)
        self._deliver_now(now_list)

    def _deliver_deferred(self, completions: List[_Completion], ids: np.ndarray) -> None:
        try:
            self._deliver_now(completions)
        finally:
            if len(ids):
                self.store.unpin(ids)

    def _deliver_now(self, completions: List[_Completion]) -> None:
        pin = [c.entry for c in completions if c.entry is not None and c.entry >= 0]
        if pin:
            arr = np.asarray(pin, dtype=np.int64)
            self.store.pin(arr)
            self._pins.append((self.round + PIN_DELAY_ROUNDS, arr))
        trace = self.trace
        now = self.loop.now() if trace is not None else 0.0
        for c in completions:
            req = c.req
            if req.aborted or req.done:
                continue
            req.done = True
            self.stats["segments"] += 1
            if trace is not None:
                xfer = c.p2p_ms if c.source == "p2p" else c.cdn_ms
                trace.add(RequestTrace(req.key, req.t_submit, max(req.t_submit, now - xfer), now, c.source,
                                       c.nbytes, c.peer if c.source == "p2p" else self.rank, self.round))
            if req.agent is not None:
                req.agent._account(c.source, c.nbytes)
            cb = req.callbacks
            if isinstance(cb, dict):
                on_progress, on_success = cb.get("onProgress"), cb.get("onSuccess")
            else:
                delivered = getattr(cb, "onDelivered", None)
                if delivered is not None:  # one call instead of a progress event + onSuccess (fleet)
                    delivered(c.source, c.nbytes, c.cdn_ms, c.p2p_ms, c.data)
                    continue
                on_progress, on_success = getattr(cb, "onProgress", None), getattr(cb, "onSuccess", None)
            if on_progress is not None:
                p2p = c.source in ("p2p", "cache")
                on_progress({"cdnDownloaded": 0 if p2p else c.nbytes, "p2pDownloaded": c.nbytes if p2p else 0,
                             "cdnDuration": 0.0 if p2p else c.cdn_ms, "p2pDuration": c.p2p_ms if p2p else 0.0})
            if req.aborted:
                continue
            if on_success is not None:
                on_success(c.data)

    # ------------------------------------------------------------------ lifecycle
    def enable_trace(self, maxlen: int = 100_000) -> TraceLog:
        """Start (or return) the round / request trace log."""
        if self.trace is None:
            self.trace = TraceLog(maxlen)
        return self.trace

    def save_cache(self, path: str) -> Dict[str, int]:
        """Checkpoint the resident segments (SURVEY §5.4 warm restart; see checkpoint.py)."""
        from .checkpoint import save_cache

        return save_cache(self, path)

    def load_cache(self, path: str) -> Dict[str, int]:
        """Restore a checkpoint; restored segments are announced in the next round."""
        from .checkpoint import load_cache

        return load_cache(self, path)

    def set_link_bandwidth(self, peer: int, kbps: Optional[float]) -> None:
        """Fault injection (SURVEY §5.3 "slow link"): model the link from ``peer`` to this
        node at ``kbps`` kbit/s — segments received from it complete after their modelled
        transfer time (None / 0 restores the real xGMI link)."""
        if kbps:
            self.link_kbps[int(peer)] = float(kbps)
        else:
            self.link_kbps.pop(int(peer), None)

    def set_online(self, online: bool) -> None:
        """Announce online / offline to the swarm from the next round (churn)."""
        self.online = bool(online)

    def close(self, timeout_rounds: int = 100000) -> None:
        """Collective shutdown: keep running rounds until every rank is leaving."""
        self.leaving = True
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        try:
            if self.world > 1:
                for _ in range(timeout_rounds):
                    if self.tick():
                        break
        finally:
            self.closed = True
            if self.metrics_server is not None:
                srv, self.metrics_server = self.metrics_server, None
                srv.close()

    def swarm_offload_ratio(self) -> float:
        """P2P bytes / (P2P + CDN bytes) over the whole swarm."""
        c, p = self.swarm_stats["cdn"], self.swarm_stats["p2p"]
        return p / (p + c) if (p + c) else 0.0


def _runs(col: np.ndarray) -> List[Tuple[int, int, int]]:
    """(value, start, end) of each run of equal values in a sorted column."""
    n = len(col)
    if n == 0:
        return []
    cuts = np.flatnonzero(col[1:] != col[:-1]) + 1
    starts = [0] + cuts.tolist()
    ends = cuts.tolist() + [n]
    return list(zip(col[starts].tolist(), starts, ends))


def _dev_index(idx: np.ndarray, dev: torch.device) -> torch.Tensor:
    """int64 index array on ``dev`` (pinned staging + one async H2D on GPUs)."""
    if dev.type == "cuda":
        from ..ops.desc import pack_to_device

        return pack_to_device({"i": np.ascontiguousarray(idx, dtype=np.int64)}, dev)["i"]
    return torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64))


def _h2d_batch(arena: torch.Tensor, dst_offs: np.ndarray, sources: List[Tuple[torch.Tensor, int, int, bool]]) -> None:
    """Enqueue the pinned-host -> HBM copies of a round on the current stream in a single
    native call; copies contiguous in both the origin pool and the arena are merged into
    one DMA (see ``h2d_batch`` in ``kernels/bindings.cpp``)."""
    from ..ops._native import device as _dev

    bases = []
    on_dev = sources[0][0].is_cuda
    for d, _, _, _ in sources:
        if d.is_cuda != on_dev:
            raise RuntimeError("CDN origin buffers of one round must all be pinned host or all HBM")
        p = d.data_ptr()
        if not on_dev and p not in _PINNED_OK:
            if not d.is_pinned():
                raise RuntimeError("CDN origin buffers must be pinned host memory for the async H2D path")
            _PINNED_OK.add(p)
        bases.append(p)
    src_alloc = np.asarray(bases, dtype=np.int64)
    src_ptrs = src_alloc + np.asarray([o for _, o, _, _ in sources], dtype=np.int64)
    lens = np.asarray([n for _, _, n, _ in sources], dtype=np.int64)
    return _dev().h2d_batch(arena, np.ascontiguousarray(dst_offs, dtype=np.int64), src_ptrs, lens, src_alloc, ALIGN,
                            on_dev)


_PINNED_OK: set = set()  # base pointers of origin tensors already checked to be pinned


# ---------------------------------------------------------------------- registry
_local = threading.local()


def current_node() -> Optional[SwarmNode]:
    return getattr(_local, "node", None)


def set_current_node(node: Optional[SwarmNode]) -> None:
    _local.node = node


def node_for_config(p2p_config: Any) -> SwarmNode:
    """The calling thread's node, created from ``p2pConfig["gpuSwarm"]`` on first use.

    ``gpuSwarm`` keys: ``backend`` ("auto" | "local" | "dist" | "thread"), ``hub`` and
    ``rank`` (thread backend), ``device``, ``cacheBytes``, ``cdnDedup``,
    ``roundIntervalMs``, ``autoTick``, ``maxWantsPerRound``, ``trace``, ``linkKbps``
    (``{peer: kbit/s}`` slow-link fault injection), ``metricsPort`` (serve Prometheus
    ``GET /metrics`` on port + rank, 0 = ephemeral; ``metricsHost`` defaults to
    127.0.0.1), ``network`` (``True`` or ``HttpOrigin`` options: fetch ``http(s)://`` URLs
    no in-process origin serves from the real CDN, :mod:`..net.network`); the agent reads
    ``prefetchSeconds`` / ``prefetchMaxSegments``.  ``numaBind``: run this process on the CPUs
    local to the node's GPU (``utils.runtime.bind_to_gpu_numa``; ``bench.py --numa auto``).
    """
    apply_network_config(p2p_config)
    node = current_node()
    if node is not None and not node.closed:
        return node
    cfg = {}
    if isinstance(p2p_config, dict):
        cfg = dict(p2p_config.get("gpuSwarm") or {})
    backend = cfg.get("backend", "auto")
    comm: SwarmComm
    if backend == "auto":
        import torch.distributed as dist

        backend = "dist" if (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1) else "local"
    if backend == "local":
        comm = LocalComm()
    elif backend == "thread":
        comm = cfg["hub"].comm(int(cfg["rank"]))
    elif backend == "dist":
        from ..parallel.comm import DistComm

        comm = DistComm()
    elif backend == "remote":  # fleet player process: the node lives in the GPU process
        from ..parallel.fleet import RemoteNode

        node = RemoteNode(cfg["conn"], world=int(cfg.get("world", 1)), rank=int(cfg.get("rank", 0)))
        set_current_node(node)
        return node
    else:
        raise ValueError(f"unknown gpuSwarm backend {backend!r}")
    node = SwarmNode(comm, device=cfg.get("device", "auto"), cache_bytes=int(cfg.get("cacheBytes", 1 << 30)),
                     cdn_dedup=bool(cfg.get("cdnDedup", True)), round_interval_ms=cfg.get("roundIntervalMs"),
                     auto_tick=bool(cfg.get("autoTick", True)), max_wants_per_round=cfg.get("maxWantsPerRound"))
    if cfg.get("numaBind") and node.is_cuda:
        from ..utils.runtime import bind_to_gpu_numa

        bind_to_gpu_numa(node.device.index if node.device.index is not None else torch.cuda.current_device())
    if cfg.get("trace"):
        node.enable_trace()
    for peer, kbps in (cfg.get("linkKbps") or {}).items():
        node.set_link_bandwidth(int(peer), kbps)
    if cfg.get("metricsPort") is not None:
        node.metrics_server = _start_metrics(node, cfg, backend)
    set_current_node(node)
    return node


def apply_network_config(p2p_config: Any) -> None:
    """``p2pConfig.gpuSwarm.network``: ``True`` / a dict of :class:`~..net.network.HttpOrigin`
    options turns on real-CDN resolution for ``http(s)://`` URLs (``http.enable_network``)."""
    gs = p2p_config.get("gpuSwarm") if isinstance(p2p_config, dict) else None
    net = gs.get("network") if isinstance(gs, dict) else None
    if net and not http.network_enabled():
        http.enable_network(True, **(net if isinstance(net, dict) else {}))


def _start_metrics(node: SwarmNode, cfg: dict, backend: str) -> Any:
    """Serve ``GET /metrics`` for ``node`` on ``metricsPort`` + the node-local rank.

    The endpoint is optional observability: a bind failure (port taken, two jobs on one
    host) logs a warning and the rank keeps serving without it — it must never take a
    rank out of the collective rounds its peers are already waiting in.  The offset is
    ``LOCAL_RANK`` under torchrun (ports stay within [port, port + ranks per host) on
    every host of a multi-host job), the in-process rank otherwise."""
    from ..utils.metrics import MetricsServer

    port = int(cfg["metricsPort"])
    if port:
        local = os.environ.get("LOCAL_RANK") if backend == "dist" else None
        port += int(local) if local is not None else node.rank
    try:
        return MetricsServer(node, port=port, host=str(cfg.get("metricsHost", "127.0.0.1")))
    except OSError as e:
        log.warning("metrics endpoint disabled on rank %d: cannot bind port %d (%s)", node.rank, port, e)
        return None
