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
CHECK_WORD = 10  # header words 10..12: directory digest, previous plan digest, its round (ingest_control)
# a rank whose CDN copies keep its ingest link busy for more than this share of its rounds
# reports FLAG_CDN_BOUND (the planner's CDN balance relieves only such ranks): a PCIe-origin
# leader measures ~0.96, the HBM-origin rehearsal's leader ~0.2 (profiles/r4_balance)
CDN_BOUND_BUSY = 0.6
ALIGN = 256
SLACK = 4096
PIN_DELAY_ROUNDS = 2  # delivered segments stay pinned this many launches (consumers run async)


def swarm_id_for(content_id: str) -> int:
    return zlib.crc32(content_id.encode()) & 0x7FFFFFFF


_M32 = 0xFFFFFFFF


W_FORCE_CDN, W_NOT_STAGED, W_STAGING, W_PREFETCH, W_PY, W_CORRUPT = 1, 2, 4, 8, 16, 32
# the origin bytes live in device memory (diagnostic HBM origin): D2D copies.  (Was 64, the
# want table's own "held" bit: a requeued want -- a corrupted peer copy -- then looked
# device-resident to the CDN phase.)
W_ON_DEV = 128
SRC_CDN, SRC_P2P, SRC_CACHE = 0, 1, 2  # source codes of delivery columns (parallel/fleet.SOURCES)
SOURCE_NAMES = ("cdn", "p2p", "cache")


class SwarmPeerLost(TimeoutError):
    """A swarm collective did not complete: a peer died, or stopped answering within the
    round / control deadline (``gpuSwarm.roundTimeoutMs`` / ``controlTimeoutMs``).  The
    message carries this rank's plan of the last round it posted."""


class Request:
    """One in-process ``getSegment`` request: the loader handle (``abort()``) and its
    delivery state.  Its want-table token is negative (fleet tokens are >= 0)."""

    __slots__ = ("node", "key", "url", "headers", "callbacks", "agent", "aborted", "done", "t_submit", "token")

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
        self.token = None

    def abort(self) -> None:
        if not self.aborted:
            self.aborted = True
            if self.token is not None:
                self.node._abort_token(self.token)

    def __repr__(self) -> str:
        return f"Request(key={self.key}, url={self.url!r}, aborted={self.aborted}, done={self.done})"


class _WantX:
    """Python-side state of a want whose bytes the CDN phase cannot take from a fixed
    address: a network origin (staged into host memory first) or a live origin (resolved at
    fetch time).  Every other want is a row of the native want table only."""

    __slots__ = ("url", "headers", "net", "src", "staged", "staging")

    def __init__(self, url: str, headers: Dict[str, str], net=None, src=None, staged: bool = True) -> None:
        self.url = url
        self.headers = headers
        self.net = net  # (origin, path, range) of a network origin
        self.src = src  # (origin, path, range) resolved again at fetch time
        self.staged = staged
        self.staging = False


@dataclass(eq=False)
class RoundHandle:
    round: int
    all_leaving: bool
    empty: bool = True
    ids: Any = None  # want ids admitted into this round (int64[k])
    # CDN fetches of this rank: want ids, store entry ids, arena offsets, lengths, keys [n, 4]
    cdn: Any = None
    # received segments: want ids, source ranks, entry ids, arena offsets, lengths, keys [n, 4]
    recv: Any = None
    failed: Any = None  # want ids failed in the CDN phase (origin error)
    send_pins: Optional[np.ndarray] = None
    hold: List[np.ndarray] = field(default_factory=list)  # in-flight entries pinned until delivered
    keep: List[Any] = field(default_factory=list)  # origin buffers this round's DMAs read
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
    defer: Any = None  # bool per received row: its CRC is checked by the consumer's decrypt (fleet)
    expect_host: Any = None  # the senders' CRC trailers of the received rows (host copy)
    plan: Any = None  # (send rows, recv rows) of this rank's plan
    t_post: float = 0.0  # host time the exchange was posted
    done: Any = None
    n_wants: int = 0
    n_send: int = 0
    t0: float = 0.0
    completed: bool = False


class VerifyTicket:
    """A received segment delivered before its CRC check (``SwarmNode.defer_inproc``): its
    consumer -- the player's transmux batch, which computes the CRC inside the decrypt --
    passes ``expect`` to the check and calls :meth:`report` with the outcome.  Until then the
    node keeps the entry pinned and does not announce it to peers; a failed check detaches it
    and the player's next request for the key goes to the CDN.

    A report that comes after the node swept the entry (``VERIFY_STALE_ROUNDS``) is ignored:
    the ticket remembers the round its entry went pending, and by then the entry id may hold
    another segment that is pending on its own check."""

    __slots__ = ("node", "eid", "expect", "token", "stamp", "done")

    def __init__(self, node: "SwarmNode", eid: int, expect: int, token: int) -> None:
        self.node = node
        self.eid = eid
        self.expect = expect
        self.token = token
        self.stamp = int(node._vround[eid])
        self.done = False

    def report(self, ok: bool) -> None:
        if not self.done:
            self.done = True
            node, e = self.node, self.eid
            if node._vflag[e] and node._vround[e] == self.stamp:
                node.verify_done(np.array([e], dtype=np.int64), np.array([bool(ok)]),
                                 np.array([self.token], dtype=np.int64))

    def __repr__(self) -> str:
        return f"VerifyTicket(eid={self.eid}, expect={self.expect:#010x}, done={self.done})"


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
    and the want table every request of the rank joins.

    Two request paths feed the same table: :meth:`request` (one ``getSegment`` of an
    in-process agent: a :class:`Request` handle and loader callbacks) and
    :meth:`request_batch` (columns of requests, e.g. a fleet's player processes: tokens in,
    delivery columns out through :meth:`set_bulk_sink`, no per-request Python object)."""

    def __init__(self, comm: Optional[SwarmComm] = None, device: Any = "auto", cache_bytes: int = 1 << 30,
                 loop=None, cdn_dedup: bool = True, round_interval_ms: Optional[float] = None,
                 auto_tick: bool = True, max_wants_per_round: Optional[int] = None) -> None:
        self.comm = comm or LocalComm()
        self.rank = self.comm.rank
        self.world = self.comm.world_size
        # The ingest CRC of a CDN fetch only produces the trailer a peer's receive check compares
        # against (the CDN sends none).  A one-rank swarm never sends, so it skips that pass
        # (HLSP2P_INGEST_CRC=1 forces it; agent/checkpoint.py computes the CRCs it saves then).
        self.ingest_crc = self.world > 1 or os.environ.get("HLSP2P_INGEST_CRC", "0") == "1"
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
        # all node device work (ingest CRC, RCCL, verify CRC) runs on its own stream: consumers
        # (decrypt/demux of the previous round) on the default stream overlap it.  The CDN
        # H2D DMAs get a copy stream of their own, so round t+1's DMA queues directly behind
        # round t's instead of behind round t's ingest CRC: the PCIe link never idles between
        # rounds (the node stream waits for each round's DMA with an event).  Reuse of arena
        # space is ordered by the store's pins, not by stream order: reserved and in-flight
        # entries stay pinned until complete_round, delivered ones PIN_DELAY_ROUNDS launches.
        #
        # Ownership rule for every other device tensor (the caching allocator hands a freed
        # block straight back to the pool of the stream it was ALLOCATED on, without waiting
        # for work queued on other streams):
        #   * a tensor the node stream writes or reads is allocated on the node stream (inside
        #     `torch.cuda.stream(self.stream)`: launch_round's phases, _grow_crc, the per-round
        #     trailers / staging / verify outputs), so its free is ordered behind that work;
        #   * the arena is allocated once and never freed while the node lives;
        #   * a tensor that must outlive a stream switch is `record_stream`-ed on the consuming
        #     stream before its last Python reference drops (_grow_crc's old table);
        #   * the copy stream only writes the arena (h2d_batch allocates nothing on it);
        #   * consumers on other streams (transmux, fleet payload copies, checkpoints) read the
        #     arena only after the host waited on the round's event (complete_round).
        # Round 3's 2-rank fault at 128 in flight was this rule broken: the CRC table, allocated
        # on the default stream, was replaced from the node stream while that stream's verify
        # CRC (stalled behind a peer's IPC event) still had to scatter into it; the transmux
        # descriptor block took the freed block and was overwritten (profiles/r4_uaf).
        self.stream = torch.cuda.Stream(self.device) if self.is_cuda else None
        self.copy_stream = (torch.cuda.Stream(self.device) if self.is_cuda and
                            os.environ.get("HLSP2P_COPY_STREAM", "1") != "0" else None)
        # CRC per store entry id.  Entry ids are bounded by the live entries; the table starts
        # big enough for any realistic segment size (>= 8 KiB average) so it never grows on
        # the hot path, and a grow is stream-safe anyway (_grow_crc)
        with self._on_node_stream():
            self.crc_dev = torch.zeros(self._crc_capacity(), dtype=torch.int32, device=self.device)
        self._events = _EventPool()
        self._clk = None  # (timing event, host time it completed): node-stream clock -> host clock
        self.online = True
        self._upload_default = True
        self._download_default = True
        # per-session P2P toggles (p2pDownloadOn / p2pUploadOn of each attached agent or fleet
        # player): a session with download off gets its fragments from the CDN only; the node
        # serves peers while any session (or the node default, without sessions) has upload on
        self._sessions: Dict[Any, Tuple[bool, bool]] = {}
        self.cdn_dedup = cdn_dedup
        self.round = 0
        self.round_interval_ms = round_interval_ms
        # fail-fast deadlines (gpuSwarm.roundTimeoutMs; the control all-gather's is the comm's
        # control_timeout_s, gpuSwarm.controlTimeoutMs): None = HLSP2P_ROUND_TIMEOUT or 60 s
        self.round_timeout_s: Optional[float] = None
        self._last_posted: Optional[RoundHandle] = None  # for the diagnostic of a lost peer
        # fault injection (SURVEY 5.3 "drop peer"): HLSP2P_FAULT_EXIT=<rank>:<round> makes that
        # rank's process die abruptly (os._exit) when it starts that round, as a crashed peer
        self._exit_at = None
        fe = os.environ.get("HLSP2P_FAULT_EXIT")
        if fe:
            fr, _, fk = fe.partition(":")
            if int(fr) == self.rank:
                self._exit_at = int(fk)
        self.auto_tick = auto_tick
        self.max_wants_per_round = max_wants_per_round
        self.leaving = False
        self.closed = False
        # health (utils/metrics.py GET /healthz): the first replicated-state or collective failure
        # this rank saw (divergence, a lost peer), and when its last round completed
        self.failed: Optional[str] = None
        self.last_complete: Optional[float] = None
        # the want table: every wanted segment and the tokens waiting for it (native rows)
        self._wt = self.rt.WantTable()
        self._wx: Dict[int, _WantX] = {}  # want id -> Python-side state (network / live origins)
        self._tok_req: Dict[int, Request] = {}  # in-process request tokens (< -1) -> handle
        self._next_tok = -2
        self._bulk: Any = None  # delivery sink of request_batch (deliver / fail columns)
        self._bulk_hits: List[Tuple[np.ndarray, np.ndarray]] = []  # cache hits to answer next
        self._bulk_hits_scheduled = False
        # (url, Range header) -> (size, address, allocation base, want flags) of VOD origin bytes
        self._locs: Dict[Tuple[str, Optional[str]], Tuple[int, int, int, int]] = {}
        self._locs_gen = -1
        self._loc_keep: Dict[int, torch.Tensor] = {}  # origin allocations the table points into
        # native batch locator of fixed-address origins (runtime/locator.cpp): the directories
        # of every origin registered this registry generation; `_locator_origins` are checked
        # for injected faults before each batch (faults take the per-request Python path)
        self._locator = self.rt.SegmentLocator()
        self._locator_gen = -1
        self._locator_origins: Dict[int, Any] = {}
        self._locator_skip: set = set()  # origins that can never use the locator (see _register_locator)
        self._tick_scheduled = False
        self._timer = None
        self._pins: List[Tuple[int, np.ndarray]] = []  # (release at launch #, entry ids)
        # pin / token ledgers the audit (agent/audit.py) balances against the store's pins:
        # rounds launched and not completed, cache hits waiting for _serve_local, delayed
        # deliveries (entry ids, tokens), and outside holders (a fleet's batches) as callables
        self._inflight: Dict[int, RoundHandle] = {}
        self._local_hits: Dict[int, int] = {}
        self._delayed: Dict[int, Tuple[np.ndarray, np.ndarray]] = {}
        self._delayed_seq = 0
        self.pin_holders: List[Any] = []  # callables -> entry ids they hold one pin on each
        self.expect_holders: List[Any] = []  # callables -> entry ids delivered with an expected CRC
        # HLSP2P_AUDIT=1 / gpuSwarm.audit: check the replicated-state invariants after every
        # launch_round and complete_round (agent/audit.py); on in the whole test suite
        self.audit_on = os.environ.get("HLSP2P_AUDIT", "0") == "1"
        self._agents: List[Any] = []
        self._prefetched: Dict[Tuple[int, int, int, int], str] = {}  # key -> "cdn" | "p2p"
        self._net_wants = False  # some want came from a network origin (plans may carry STAGE rows)
        self.peer_online = np.ones(self.world, dtype=bool)
        # "p2p" / "p2p_segments": peer copies delivered whose CRC check passed, counted when
        # they are delivered (complete_round: the node's own check, or -- for a check deferred
        # to the consumer's decrypt -- provisionally, moved to "p2p_rejected" by verify_done
        # if it fails).  A copy that fails is never counted as delivered P2P: it counts in
        # "p2p_rejected" and its CDN re-fetch in "cdn", so cdn + p2p is what the players were
        # served and offload = p2p / (cdn + p2p) is exact under corruption (counting at
        # delivery keeps P2P and CDN bytes on the same clock for a timed window).  Wire-level:
        # "p2p_wire" (every byte received) and "p2p_links" ((round, source peer) pairs): link rates
        self.stats = {"cdn": 0, "p2p": 0, "upload": 0, "cache": 0, "rounds": 0, "crc_failures": 0,
                      "segments": 0, "cdn_segments": 0, "p2p_segments": 0, "prefetched": 0,
                      "p2p_links": 0, "p2p_wire": 0, "p2p_rejected": 0, "p2p_rejected_segments": 0,
                      "cache_segments": 0}
        self.swarm_stats = {"cdn": 0, "p2p": 0, "upload": 0}
        self.last_round: Dict[str, Any] = {}
        self.corrupt_next_recv = 0  # fault injection: flip a byte in the next N received rounds
        # fault injection: the next N rounds with sends each send one segment from ANOTHER
        # resident entry of the same length (a sender's bookkeeping bug: its bytes and its table
        # CRC agree with each other, not with the key the receiver asked for)
        self.misroute_next_send = 0
        # cross-rank consistency (SURVEY 5.2 state-machine assertions): every rank replays the
        # same control messages into its own directory and plans every round independently; a
        # two-sided data plane (RCCL send / recv) then needs the plans to match exactly.  The
        # directory digest and the previous plan's digest ride every control message and are
        # compared before anything is applied (HLSP2P_DIVERGENCE_CHECK=0 turns it off)
        self.divergence_check = self.world > 1 and os.environ.get("HLSP2P_DIVERGENCE_CHECK", "1") != "0"
        self._plan_digest = 0
        self._plan_round = 0
        # bytes received from each source peer (the fan-in over the point-to-point links)
        self.p2p_from = np.zeros(self.world, dtype=np.int64)
        # Deferred receive verification (set by a fleet server, parallel/fleet.py): a segment a
        # peer sent is not CRC-read by the node; its trailer travels with the delivery and the
        # batch that decrypts it computes the CRC on the way (kernels/aes_cbc.hip AesCrc).  The
        # entry stays pending -- pinned, not announced, not served -- until verify_done.
        self.verify_deferred = False
        # planner CDN balance (plan_round_into), opt-in (HLSP2P_CDN_BALANCE=1; measured in
        # profiles/r4_balance): this rank reports FLAG_CDN_BOUND while its CDN copies keep its
        # ingest link busy (`_cdn_busy`, an average over rounds of the copy time per round
        # interval), and the plan then holds its lone wants back once when another rank is about
        # to want them
        self.cdn_balance = os.environ.get("HLSP2P_CDN_BALANCE", "0") == "1"
        self._cdn_busy = 0.0
        self._cdn_num = self._cdn_den = 0.0
        self._cdn_t = None
        # entries waiting for a deferred check, by entry id: flag + want info row (a CDN retry's source)
        self._vflag = np.zeros(0, dtype=bool)
        self._vinfo = np.zeros((0, 10), dtype=np.int64)
        self._vround = np.zeros(0, dtype=np.int64)  # round each pending entry was delivered in
        self._vexp = np.zeros(0, dtype=np.int64)  # its expected CRC (the sender's trailer)
        # bulk tokens asking for a segment whose received copy awaits its check: answered from
        # that copy once it passes (another fetch of the segment would replace the copy in the
        # index while its first consumers still read it), or from the CDN if it fails
        self._vwait: Dict[int, List[np.ndarray]] = {}
        # in-process requests join the deferred check too (gpuSwarm.deferVerify): their bytes
        # reach the loader with a VerifyTicket, the player's transmux batch verifies them (the
        # CRC fused into its decrypt) and reports back; a copy that fails is detached and the
        # player's re-request goes to the CDN (_force_cdn_keys).  Entries whose ticket never comes
        # back (a fragment dropped before its transmux) are checked by the node after
        # VERIFY_STALE_ROUNDS rounds
        self.defer_inproc = False
        self._force_cdn_keys: set = set()
        self.link_kbps: Dict[int, float] = {}  # fault injection: slow link from peer -> kbit/s
        self.timer = PhaseTimer()
        # per-request trace records {key, trequest, tfirst, tload, source, bytes, peer, round}
        # (SURVEY §5.1); None = off (p2pConfig["gpuSwarm"]["trace"] or enable_trace())
        self.trace: Optional[TraceLog] = None
        self.metrics_server: Any = None  # utils.metrics.MetricsServer (gpuSwarm.metricsPort)
        self._lock = threading.RLock()
        if self.world > 1 and auto_tick:
            self._timer = self.loop.set_interval(self._timer_tick, round_interval_ms or 10.0)

    # ------------------------------------------------------------------ agents / sessions
    def attach(self, agent: Any) -> None:
        """Register a peer agent (its requests, stats and metrics)."""
        self._agents.append(agent)

    def detach(self, agent: Any) -> None:
        """Unregister an agent: its pending requests are withdrawn (no callback runs)."""
        if agent in self._agents:
            self._agents.remove(agent)
        self._sessions.pop(agent, None)
        gone = [t for t, r in self._tok_req.items() if r.agent is agent]
        for t in gone:
            self._tok_req.pop(t, None)
            self._wt.abort1(t)

    def set_session_flags(self, session: Any, download: bool, upload: bool) -> None:
        """Per-session ``p2pDownloadOn`` / ``p2pUploadOn`` (``lib/hlsjs-p2p-wrapper.js:20-36``)."""
        self._sessions[session] = (bool(download), bool(upload))

    def session_flags(self, session: Any) -> Tuple[bool, bool]:
        """``(download, upload)`` of a session (the node defaults until it set its own)."""
        return self._sessions.get(session, (self._download_default, self._upload_default))

    @property
    def download_on(self) -> bool:
        """Node-wide P2P download: on while any session (or, without sessions, the node
        default) downloads from peers.  The setter sets the node default."""
        if self._sessions:
            return any(d for d, _ in self._sessions.values())
        return self._download_default

    @download_on.setter
    def download_on(self, on: bool) -> None:
        self._download_default = bool(on)

    @property
    def upload_on(self) -> bool:
        """Node-wide P2P upload (serving peers): on while any session has it on."""
        if self._sessions:
            return any(u for _, u in self._sessions.values())
        return self._upload_default

    @upload_on.setter
    def upload_on(self, on: bool) -> None:
        self._upload_default = bool(on)

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
        if self.cdn_balance and self._cdn_busy > CDN_BOUND_BUSY:
            f |= self.rt.FLAG_CDN_BOUND
        return f

    def pending(self) -> int:
        """Wanted segments not delivered yet."""
        return len(self._wt)

    # ------------------------------------------------------------------ sources
    def _resolve(self, url: str, headers: Optional[Dict[str, str]]) -> Tuple[int, int, int, int, Optional[_WantX]]:
        """Where a want's bytes come from: ``(size, address, allocation base, want flags,
        Python state)``.  A VOD origin's bytes never move: their pinned-host (or HBM) address
        is taken once and the CDN phase DMAs from it with no Python per want; a network
        origin's body is staged first (size 0 and ``W_NOT_STAGED`` until then); a live
        origin is resolved again at fetch time (its window moves)."""
        rng_hdr = (headers.get("Range") or headers.get("range")) if headers else None
        gen = http.generation()
        if gen != self._locs_gen:
            self._locs.clear()
            self._locs_gen = gen
        ck = (url, rng_hdr)
        hit = self._locs.get(ck)
        if hit is not None:
            return hit[0], hit[1], hit[2], hit[3], None
        origin, path = http.resolve(url)
        if id(origin) not in self._locator_origins or self._locator_gen != http.generation():
            self._register_locator(origin)
        rng = http.parse_range(headers) if headers else None
        if getattr(origin, "staged_fetch", False):
            size = origin.staged_size(path, rng)
            self._net_wants = True
            x = _WantX(url, dict(headers or {}), net=(origin, path, rng), staged=size is not None)
            return int(size or 0), 0, 0, W_PY | (0 if size is not None else W_NOT_STAGED), x
        locate = getattr(origin, "locate", None)
        loc = locate(path, url, rng) if locate is not None else None
        if loc is None:
            size = origin.size(path, url, rng)
            return int(size or 0), 0, 0, W_PY, _WantX(url, dict(headers or {}), src=(origin, path, rng))
        data, off, n = loc
        base = data.data_ptr()
        flags = 0
        if data.is_cuda:
            flags |= W_ON_DEV
        elif base not in self._loc_keep and self.is_cuda and not data.is_pinned():
            raise RuntimeError("CDN origin buffers must be pinned host memory for the async H2D path")
        self._loc_keep.setdefault(base, data)
        corrupt = bool(getattr(origin, "_corrupt", None)) and origin.should_corrupt(path)
        if corrupt:
            flags |= W_CORRUPT
        res = (int(n), base + int(off), base, flags)
        if not corrupt and not getattr(origin, "_failures", None):
            if len(self._locs) > 1 << 16:
                self._locs.clear()
            self._locs[ck] = res
        return res[0], res[1], res[2], res[3], None

    def _register_locator(self, origin: Any) -> None:
        """Hand a fixed-address origin's segment directories to the native locator (once per
        origin and registry generation).  Origins without them, or whose host bytes are not
        pinned (the async H2D path needs pinned memory: the Python path raises for them),
        stay on the per-request path for good; an origin whose directories are unavailable
        right now (faults injected) is asked again on a later miss.  An origin is recorded
        only once ALL its directories are registered, so a partial registration never
        happens and a fault-time refusal does not lock it out of the fast path."""
        if http.generation() != self._locator_gen:
            self._locator.clear()
            self._locator_origins.clear()
            self._locator_skip.clear()
            self._locator_gen = http.generation()
        if id(origin) in self._locator_skip:
            return
        dirs_fn = getattr(origin, "segment_dirs", None)
        if dirs_fn is None:
            self._locator_skip.add(id(origin))
            return
        dirs = dirs_fn()
        if not dirs:
            return  # e.g. faults configured now: retried on a later miss
        if any(not d[5].is_cuda and self.is_cuda and not d[5].is_pinned() for d in dirs):
            self._locator_skip.add(id(origin))
            return
        for d, prefix, suffix, lo, hi, data, offs, lens in dirs:
            base = data.data_ptr()
            self._loc_keep.setdefault(base, data)
            self._locator.add_dir(d, prefix, suffix, int(lo), int(hi), base, W_ON_DEV if data.is_cuda else 0,
                                  np.asarray(offs, dtype=np.int64), np.asarray(lens, dtype=np.int64))
        self._locator_origins[id(origin)] = origin

    def _locator_usable(self) -> bool:
        """The native locator may answer this batch: it holds directories of the current
        registry generation and none of their origins has faults injected since."""
        if not len(self._locator) or self._locator_gen != http.generation():
            return False
        for o in self._locator_origins.values():
            if getattr(o, "_failures", None) or getattr(o, "_corrupt", None):
                self._locator.clear()
                self._locator_origins.clear()
                return False
        return True

    # ------------------------------------------------------------------ requests
    def request(self, key: Tuple[int, int, int, int], url: str, headers: Optional[Dict[str, str]],
                callbacks: Any, agent: Any = None, view: Any = None) -> Request:
        """Queue a fragment request for key ``(swarm, level, urlId, sn)``; served from the cache,
        a peer or the CDN in the next round.  (``view``: the agent's SegmentView, which a
        fleet's remote node uses to find the fragment's AES key; unused here.)"""
        k0, k1, k2, k3 = key
        k = (int(k0) & _M32, int(k1) & _M32, int(k2) & _M32, int(k3) & _M32)
        req = Request(self, k, url, dict(headers) if headers else {}, callbacks, agent, False, False,
                      self.loop.now())
        eid = self.store.lookup1(*k)
        if eid >= 0:  # local cache hit
            self.store.pin(np.array([eid], dtype=np.int64))
            self._local_hits[eid] = self._local_hits.get(eid, 0) + 1
            self.loop.call_soon(self._serve_local, req, eid)
            return req
        if self._prefetched:
            self._prefetched.pop(k, None)  # evicted before use
        wt = self._wt
        flags = 0
        if agent is not None and self._sessions and not self.session_flags(agent)[0]:
            flags = W_FORCE_CDN  # this session does not download from peers
        if self._force_cdn_keys and k in self._force_cdn_keys:
            self._force_cdn_keys.discard(k)
            flags |= W_FORCE_CDN  # its peer copy failed the player's check: from the CDN
        size = ptr = base = 0
        x = None
        if wt.lookup1(*k) < 0:
            try:
                size, ptr, base, wf, x = self._resolve(url, req.headers)
            except http.HttpError as e:
                self.loop.call_soon(self._fail, req, e)
                return req
            flags |= wf
        tok = self._next_tok
        self._next_tok = tok - 1
        req.token = tok
        self._tok_req[tok] = req
        r = wt.add1(k[0], k[1], k[2], k[3], size, ptr, base, flags, tok)
        if r < 0 and x is not None:
            self._wx[-r - 1] = x
        self._schedule()
        return req

    def set_bulk_sink(self, sink: Any) -> None:
        """Where :meth:`request_batch` deliveries go: ``sink.deliver(tokens, source, nbytes,
        cdn_ms, p2p_ms, arena_off, entry)`` (columns; ``source`` codes ``SRC_*``; the bytes are
        ``arena[arena_off : arena_off + nbytes]``, pinned for ``PIN_DELAY_ROUNDS`` launches)
        and ``sink.fail(tokens, status)``."""
        self._bulk = sink

    def request_batch(self, keys: np.ndarray, urls: List[str], headers: Optional[List[Optional[Dict[str, str]]]],
                      tokens: np.ndarray, force_cdn: Optional[np.ndarray] = None) -> None:
        """Columns of fragment requests (``keys`` int64[n, 4] = ``(swarm, level, urlId, sn)``,
        one URL and optional header dict each, caller ``tokens`` >= 0 int64[n]); the answers
        go to the bulk sink.  ``force_cdn[i]``: request ``i`` may not be served by a peer (its
        session has P2P download off).  One native lookup for the cache, one native insert
        into the want table; per request only a dict lookup of its URL's source."""
        n = len(tokens)
        if n == 0:
            return
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64).reshape(n, 4) & _M32)
        tokens = np.ascontiguousarray(tokens, dtype=np.int64)
        eids = self.store.lookup(keys, False)
        hit = eids >= 0
        if hit.any():
            he = eids[hit]
            self.store.pin(he)
            self._bulk_hits.append((tokens[hit], he))
            if not self._bulk_hits_scheduled:
                self._bulk_hits_scheduled = True
                self.loop.call_soon(self._serve_bulk_hits)
            miss = np.flatnonzero(~hit)
            if not len(miss):
                return
        else:
            miss = None
        if self._vflag.any():  # (a flag per entry id: small)
            miss = self._park_on_pending(keys, tokens, miss)
            if miss is not None and not len(miss):
                return
        idx = range(n) if miss is None else miss.tolist()
        m = n if miss is None else len(miss)
        sizes = np.zeros(m, dtype=np.int64)
        ptrs = np.zeros(m, dtype=np.int64)
        bases = np.zeros(m, dtype=np.int64)
        flags = np.zeros(m, dtype=np.int64)
        if force_cdn is not None:
            fc = np.asarray(force_cdn, dtype=bool)
            flags[:] = np.where(fc if miss is None else fc[miss], W_FORCE_CDN, 0)
        if self._force_cdn_keys:  # keys whose copy a consumer rejected (invalidate / verify): from the CDN
            fk = self._force_cdn_keys
            for j, row in enumerate((keys if miss is None else keys[miss]).tolist()):
                t = tuple(row)
                if t in fk:
                    fk.discard(t)
                    flags[j] |= W_FORCE_CDN
        xs: Dict[int, _WantX] = {}
        bad: List[Tuple[int, int]] = []
        resolve = self._resolve
        done = None
        if self._locator_usable():  # one native call for the fixed-address origins' URLs
            sel_urls = urls if miss is None else [urls[i] for i in idx]
            s_, p_, b_, f_, done, found = self._locator.resolve(sel_urls if isinstance(sel_urls, list)
                                                                else list(sel_urls))
            if headers is not None:  # byte ranges take the general path
                done &= np.fromiter((not h or ("Range" not in h and "range" not in h)
                                     for h in (headers if miss is None else [headers[i] for i in idx])),
                                    dtype=bool, count=m)
            sizes[done] = s_[done]
            ptrs[done] = p_[done]
            bases[done] = b_[done]
            flags[done] |= f_[done]
            if done.all():
                idx = ()
        for j, i in enumerate(idx):
            if done is not None and done[j]:
                continue
            try:
                sizes[j], ptrs[j], bases[j], wf, x = resolve(urls[i], headers[i] if headers is not None else None)
            except http.HttpError as e:
                bad.append((j, int(e.status or 0) or 500))
                continue
            flags[j] |= wf
            if x is not None:
                xs[j] = x
        sel_keys = keys if miss is None else keys[miss]
        sel_tok = tokens if miss is None else tokens[miss]
        if bad:
            bj = np.asarray([j for j, _ in bad], dtype=np.int64)
            self._fail_bulk(sel_tok[bj], np.asarray([s for _, s in bad], dtype=np.int64))
            keep = np.ones(m, dtype=bool)
            keep[bj] = False
            remap = np.cumsum(keep) - 1
            xs = {int(remap[j]): x for j, x in xs.items()}
            sel_keys, sel_tok = sel_keys[keep], sel_tok[keep]
            sizes, ptrs, bases, flags = sizes[keep], ptrs[keep], bases[keep], flags[keep]
        if self._prefetched:
            for kk in map(tuple, sel_keys.tolist()):
                self._prefetched.pop(kk, None)
        ids, created = self._wt.add(sel_keys, sizes, ptrs, bases, flags, sel_tok)
        for j, x in xs.items():
            if created[j]:
                self._wx[int(ids[j])] = x
        self._schedule()

    def abort_tokens(self, tokens: np.ndarray) -> int:
        """Withdraw bulk requests (no answer is sent for them)."""
        return int(self._wt.abort(np.ascontiguousarray(tokens, dtype=np.int64)))

    def _abort_token(self, token: int) -> None:
        self._tok_req.pop(token, None)
        self._wt.abort1(token)

    def _stage(self, wid: int, x: _WantX) -> None:
        """Plan said: download want ``wid``'s body from its network origin into host memory.
        The completion comes back to this loop; the want is planned again once staged."""
        if x.staging or x.staged or x.net is None:
            return
        origin, path, rng = x.net
        x.staging = True
        self._wt.set(wid, -1, W_STAGING, 0)  # announced as downloading: staged nowhere else meanwhile
        loop = self.loop
        loop.hold()

        def done(n, err):  # worker thread
            try:
                loop.call_soon_threadsafe(self._on_staged, wid, x, n, err)
            finally:
                loop.release()

        origin.stage(path, x.url, rng, x.headers, done)

    def _on_staged(self, wid: int, x: _WantX, n, err) -> None:
        x.staging = False
        alive = self._wx.get(wid) is x
        if err is not None:
            if alive:
                self._finish_failed(np.array([wid], dtype=np.int64), err)
            return
        x.staged = True
        if alive and self._wt.set(wid, int(n), 0, W_STAGING | W_NOT_STAGED):
            self._schedule()
        else:  # nobody waits any more (aborted / served meanwhile): drop the host copy
            origin, path, rng = x.net
            origin.release(path, rng)

    def prefetch(self, key: Tuple[int, int, int, int], url: str, headers: Optional[Dict[str, str]] = None) -> bool:
        """Fill the cache with a segment no player asked for yet (agent prefetch planning,
        SURVEY §2.3).  It travels in the next round like any want (P2P from a holder, or
        the CDN); a player request arriving meanwhile simply joins it.  True if issued."""
        k = tuple(int(v) & _M32 for v in key)
        if self._wt.lookup1(*k) >= 0 or self.store.lookup1(*k) >= 0:
            return False
        try:
            size, ptr, base, wf, x = self._resolve(url, dict(headers or {}))
        except http.HttpError:
            return False
        r = self._wt.add1(k[0], k[1], k[2], k[3], size, ptr, base, wf | W_PREFETCH, self.rt.NO_TOKEN)
        if r < 0 and x is not None:
            self._wx[-r - 1] = x
        self.stats["prefetched"] += 1
        self._schedule()
        return True

    def _schedule(self) -> None:
        if self.world == 1 and self.auto_tick and not self._tick_scheduled:
            self._tick_scheduled = True
            self.loop.call_soon(self._local_tick)

    def _local_tick(self) -> None:
        self._tick_scheduled = False
        if len(self._wt):
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
                self.stats["cache_segments"] += 1
            self._deliver_req(req, src or "cache", n, 0.0, 0.0, self.arena[off:off + n], -1, eid)
        finally:
            self.store.unpin(np.array([eid], dtype=np.int64))
            n = self._local_hits.get(eid, 0) - 1
            if n > 0:
                self._local_hits[eid] = n
            else:
                self._local_hits.pop(eid, None)

    def _park_on_pending(self, keys: np.ndarray, tokens: np.ndarray, miss: Optional[np.ndarray]) -> np.ndarray:
        """Requests (rows ``miss`` of ``keys``; all when None) for segments whose received copy
        is delivered and awaits its deferred check wait for that check (:meth:`verify_done`)
        instead of fetching the segment again.  Returns the rows still to fetch."""
        rows = np.arange(len(tokens)) if miss is None else miss
        pe = self.store.lookup(np.ascontiguousarray(keys[rows]), True)
        park = pe >= 0
        park[park] = pe[park] < len(self._vflag)
        park[park] = self._vflag[pe[park]]
        if not park.any():
            return rows if miss is not None else None
        for e, t in zip(pe[park].tolist(), tokens[rows[park]].tolist()):
            self._vwait.setdefault(e, []).append(t)
        self.stats["parked"] = self.stats.get("parked", 0) + int(park.sum())
        return rows[~park]

    def _release_parked(self, e: int, ok: bool) -> None:
        toks = np.asarray(self._vwait.pop(e), dtype=np.int64)
        if ok:  # the copy is committed: a cache hit
            arr = np.array([e], dtype=np.int64)
            ids = np.repeat(arr, len(toks))
            self.store.pin(ids)
            self._bulk_hits.append((toks, ids))
            if not self._bulk_hits_scheduled:
                self._bulk_hits_scheduled = True
                self.loop.call_soon(self._serve_bulk_hits)
        else:
            self._retry_cdn(self._vinfo[e], toks)

    def _serve_bulk_hits(self) -> None:
        """Answer the bulk requests that hit the cache (pinned at request time)."""
        self._bulk_hits_scheduled = False
        hits, self._bulk_hits = self._bulk_hits, []
        for tok, eids in hits:
            try:
                ent = self.store.entries(eids)
                offs, lens = ent[:, 0].copy(), ent[:, 1].copy()
                self.stats["cache"] += int(lens.sum())
                self.stats["cache_segments"] += len(tok)
                z = np.zeros(len(tok), dtype=np.float64)
                self._deliver_cols(tok, np.full(len(tok), SRC_CACHE, dtype=np.int8), lens, z, z, offs, eids)
            finally:
                self.store.unpin(eids)

    def _fail(self, req: Request, err: Exception) -> None:
        if req.aborted or req.done:
            return
        req.done = True
        cb = req.callbacks
        on_error = cb.get("onError") if isinstance(cb, dict) else getattr(cb, "onError", None)
        if on_error is not None:
            on_error(err)

    def _fail_bulk(self, tokens: np.ndarray, status: np.ndarray) -> None:
        if self._bulk is not None and len(tokens):
            self._bulk.fail(tokens, status)

    def _finish_failed(self, wids: np.ndarray, err: http.HttpError) -> None:
        """Remove wants whose fetch failed and report ``err`` to every waiter (the loader
        falls through to its retry logic, as after a failed XHR)."""
        tok, _, _ = self._wt.finish(np.ascontiguousarray(wids, dtype=np.int64))
        for w in wids.tolist():
            x = self._wx.pop(w, None)
            if x is not None and x.net is not None and x.staged:
                x.net[0].release(x.net[1], x.net[2])
        if not len(tok):
            return
        bulk = tok >= 0
        if bulk.any():
            self._fail_bulk(tok[bulk], np.full(int(bulk.sum()), int(err.status or 0) or 500, dtype=np.int64))
        for t in tok[~bulk].tolist():
            req = self._tok_req.pop(t, None)
            if req is not None:
                self.loop.call_soon(self._fail, req, err)

    # ------------------------------------------------------------------ control messages
    def _encode(self, rows: np.ndarray, adds: np.ndarray, rms: np.ndarray) -> np.ndarray:
        hdr = np.zeros(HDR, dtype=np.int64)
        hdr[0] = MAGIC
        hdr[1] = self.flags
        hdr[2] = len(rows)
        hdr[3] = len(adds)
        hdr[4] = len(rms)
        hdr[5] = 1 if self.leaving else 0
        hdr[6] = self.round
        hdr[7] = self.stats["cdn"]
        hdr[8] = self.stats["p2p"]
        hdr[9] = self.stats["upload"]
        # consistency words (checked by every rank in ingest_control): this replica's directory
        # digest before the round's deltas, and the digest of the previous round's full plan
        hdr[CHECK_WORD] = self.directory.digest
        hdr[CHECK_WORD + 1] = self._plan_digest
        hdr[CHECK_WORD + 2] = self._plan_round
        return np.concatenate([hdr, rows.reshape(-1), adds.reshape(-1).astype(np.int64),
                               rms.reshape(-1).astype(np.int64)])

    CRC_TABLE_MAX = 1 << 20  # initial CRC-table entries at most (4 MiB)

    def _crc_capacity(self) -> int:
        return int(min(max(1024, self.cache_bytes // (8 << 10) + 1), self.CRC_TABLE_MAX))

    def _on_node_stream(self):
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _grow_crc(self, n: int) -> None:
        """Make the CRC table hold entry ids ``< n``.  The new table is allocated and filled on
        the node stream, and the old one is recorded on it, so node-stream kernels still
        queued against the old table (ingest / verify scatters, trailer gathers) finish
        before the allocator can hand its block to anyone (see the ownership rule above)."""
        old = self.crc_dev
        if n <= old.numel():
            return
        with self._on_node_stream():
            new = torch.zeros(max(n, 2 * old.numel()), dtype=torch.int32, device=self.device)
            new[:old.numel()] = old
        if old.is_cuda:
            old.record_stream(self.stream)
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
        h = self._launch_round()
        if self.audit_on:
            from .audit import audit_node

            audit_node(self, "launch_round")
        return h

    def complete_round(self, h: RoundHandle) -> None:
        """Local: wait for the round's device work, verify, commit and deliver."""
        self._complete_round(h)
        if self.audit_on:
            from .audit import audit_node

            audit_node(self, "complete_round")

    def _launch_round(self) -> RoundHandle:
        rt = self.rt
        t0 = time.perf_counter()
        self.round += 1
        self.stats["rounds"] += 1
        if self._exit_at is not None and self.round >= self._exit_at:
            log.error("rank %d: injected crash at round %d (HLSP2P_FAULT_EXIT)", self.rank, self.round)
            os._exit(17)
        if self.verify_deferred and self.round % 8 == 0 and len(self._vflag):
            self._sweep_pending()
        if self._pins:
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
        # the round's wants, in one native pass: FIFO, requests before prefetch, capped,
        # admitted only as far as the HBM ring can place them now (backpressure)
        cap = self.max_wants_per_round
        ids, rows, dropped, too_big, deferred = self._wt.select(self.store, self.directory,
                                                               -1 if cap is None else int(cap), self.round)
        if len(dropped) and self._wx:  # every waiter aborted: drop staged host copies
            for w in dropped.tolist():
                x = self._wx.pop(w, None)
                if x is not None and x.net is not None and x.staged:
                    x.net[0].release(x.net[1], x.net[2])
        if len(too_big):
            self._finish_failed(too_big, http.HttpError(507, "", f"segment exceeds the {self.cache_bytes}-byte cache"))
        if deferred:
            self.stats["deferred"] = self.stats.get("deferred", 0) + int(deferred)
        if len(rows):
            # the entries this round's reservations overwrite leave the directory in this
            # round's control message, so no peer plans a transfer from them: a send would pin
            # them after admission and the reservation would find them pinned.  Sizes are the
            # admitted ones (the planner never sends a copy larger than a want announced); a
            # want the planner then holds back (at most once, kWHeld) retired its share too --
            # the hold is decided from every rank's wants, after this message must go out
            need = int(np.maximum((rows[:, 4] + (ALIGN - 1)) // ALIGN * ALIGN, ALIGN).sum())
            self.store.retire_region(need)
            # the round's runs (CDN + one per source peer) all land in the region admission
            # checked: if they would cross the ring's end, the ring wraps before the first
            if not self.store.wrap_for(need):
                raise RuntimeError("segment cache cannot wrap for the round (pinned entries block eviction)")
            if self.audit_on:
                from .audit import check_region

                check_region(self, need)
        adds, rms = self.store.take_delta()
        try:
            parts = self.comm.allgather_control(self._encode(rows, adds, rms))
        except Exception as e:  # noqa: BLE001 - a dead or stalled peer (deadline: comm.control_timeout_s)
            raise self._peer_lost("control all-gather", e) from e
        # every rank's deltas into the directory + the round's want rows, in one native call
        # (after checking that every replica and the last plans agree)
        try:
            all_wants, flags, all_leaving, swarm_tot = rt.ingest_control(
                self.directory, parts, MAGIC, HDR, CHECK_WORD if self.divergence_check else -1)
        except rt.SwarmDivergence as e:
            self._diverged(str(e))
            raise
        self.peer_online = (flags & rt.FLAG_ONLINE) != 0
        self.swarm_stats = {"cdn": int(swarm_tot[0]), "p2p": int(swarm_tot[1]), "upload": int(swarm_tot[2])}
        h = RoundHandle(self.round, all_leaving, t0=t0)
        h.ids = ids
        self._inflight[h.round] = h
        t_ctrl = time.perf_counter()
        self.timer.add("control", t_ctrl - t0)
        if not len(all_wants):  # (every rank sees the same want rows: all skip planning alike)
            self._plan_digest, self._plan_round = 0, self.round
            return h
        h.empty = False
        # only the rows this rank sends, receives or fetches (the full plan is identical on
        # every rank; any_p2p says whether the round has transfers at all)
        me = self.rank
        # each rank's cumulative CDN bytes (header word 7): the planner's CDN balance holds a
        # lone want of a rank over its share back once when another rank is about to want it
        cdn_bytes = np.fromiter((int(p[7]) for p in parts), dtype=np.int64, count=len(parts)) \
            if self.cdn_balance and self.world > 1 else None
        plan, any_p2p, self._plan_digest = rt.plan_round_for(self.directory, all_wants, flags, self.world, me,
                                                             cdn_bytes)
        self._plan_round = self.round
        h.n_wants = len(all_wants)
        cdn_rows = plan[(plan[:, 5] == -1) & (plan[:, 6] == me)]
        if self._net_wants and self._wx:  # network-origin wants this rank must download first (STAGE rows)
            for wid in plan[(plan[:, 5] == -2) & (plan[:, 6] == me), 7].tolist():
                x = self._wx.get(wid)
                if x is not None:
                    self._stage(wid, x)
        send_rows = plan[plan[:, 5] == me]
        recv_rows = plan[(plan[:, 6] == me) & (plan[:, 5] >= 0)]
        h.n_send = len(send_rows)
        h.plan = (send_rows, recv_rows)  # kept for the diagnostic of a round that never completes
        self._last_posted = h
        # ---------------- 2. pin what we send from cache (seeded rows come from the CDN phase)
        # send_eids[i]: store entry of send row i (-1: missing), aligned with send_rows
        send_eids = np.full(len(send_rows), -1, dtype=np.int64)
        cached = send_rows[:, 8] == 0
        if cached.any():
            eids = self.store.lookup(np.ascontiguousarray(send_rows[cached, :4]), False)
            send_eids[cached] = eids
            valid = eids[eids >= 0]
            if len(valid):
                self.store.pin(valid)
                h.send_pins = valid
            if self.misroute_next_send > 0:
                self._misroute(send_rows, send_eids)
        t_cdn0 = time.perf_counter()
        self.timer.add("plan", t_cdn0 - t_ctrl)
        with (torch.cuda.stream(self.stream) if self.is_cuda else contextlib.nullcontext()):
            # ---------------- 3. CDN phase (pinned host -> HBM, DMA engines)
            if len(cdn_rows):
                self._cdn_phase(h, cdn_rows)
                seeded = np.flatnonzero(~cached)
                if len(seeded) and h.cdn is not None:  # forwarded in this same round: the CDN
                    # phase committed (and pinned) them, so the store finds them by key
                    send_eids[seeded] = self.store.lookup(np.ascontiguousarray(send_rows[seeded, :4]), False)
            t_p2p0 = time.perf_counter()
            self.timer.add("cdn_enqueue", t_p2p0 - t_cdn0)
            # ---------------- 4. P2P phase: entered by EVERY rank when the (identical) plan
            # has any transfer, so a collective transport (the in-process hub) stays in step;
            # RCCL point-to-point with no local ops posts nothing
            if any_p2p:
                self._p2p_phase(h, send_rows, recv_rows, send_eids)
            h.sent_bytes = int(send_rows[:, 4].sum()) if len(send_rows) else 0
            if self.is_cuda:
                h.done = self._events.get(True)  # timing: it also calibrates the device clock (_clock_sync)
                h.done.record(self.stream)  # explicit stream: skips torch's current_stream() lookup
        self.timer.add("p2p_enqueue", time.perf_counter() - t_p2p0)
        return h

    def _complete_round(self, h: RoundHandle) -> None:
        if h.completed:
            return
        h.completed = True
        self._inflight.pop(h.round, None)
        if h.empty:
            self.last_complete = time.monotonic()
            self.last_round = {"wants": 0, "ms": (time.perf_counter() - h.t0) * 1e3}
            if h.ids is not None and len(h.ids):  # (a lone rank's wants always plan: defensive)
                self._wt.requeue(h.ids, False)
            return
        t0 = time.perf_counter()
        if h.done is not None and not h.done.query():
            self._wait_round(h)
            # the host saw the round's last event complete just now: a (device, host) time pair
            self._clock_sync(h.done, time.perf_counter())
            h.done = None
        t1 = time.perf_counter()
        self.timer.add("wait_device", t1 - t0)
        if h.ev_cdn is not None:
            h.cdn_ms = h.ev_cdn[0].elapsed_time(h.ev_cdn[1])
            self._events.put(True, *h.ev_cdn)
        if h.ev_p2p is not None:
            h.p2p_ms = h.ev_p2p[0].elapsed_time(h.ev_p2p[1])
            if self._clk is not None:
                # host time the node stream reached the exchange minus the host time it was
                # posted: how long the round's transfers waited behind earlier node-stream work
                ev, t_host = self._clk
                q = t_host + ev.elapsed_time(h.ev_p2p[0]) / 1e3 - h.t_post
                self.timer.add("exchange_queued", max(0.0, q))
                self.timer.add("exchange_queued_n", 1.0)
            self._events.put(True, *h.ev_p2p)
        if h.done is not None:
            self._events.put(True, h.done)
            h.done = None
        wt = self._wt
        recv = h.recv
        good = bad = None
        dgood = exp_good = None  # deferred verification (verify_deferred): rows of `good`, their CRCs
        if recv is not None:
            ok = (h.ok_host.numpy() if isinstance(h.ok_host, torch.Tensor) else np.asarray(h.ok_host)).astype(bool)
            if ok.all():
                good = recv
            else:
                good = tuple(c[ok] for c in recv)
                bad = tuple(c[~ok] for c in recv)
            if h.defer is not None:
                dgood = h.defer[ok]
                eh = h.expect_host.numpy() if isinstance(h.expect_host, torch.Tensor) else np.asarray(h.expect_host)
                # the trailers are keyed CRCs: unbind them with the keys this rank asked for, so
                # the consumer (the CRC fused into its decrypt) compares plain CRC-32s -- a copy
                # sent under another key then fails there
                eh = eh.astype(np.int32) ^ _crc.key_digest(recv[5])
                exp_good = eh.astype(np.int64)[ok]
                if not dgood.any():
                    dgood = None
            commit = good[2] if dgood is None else good[2][~dgood]
            if len(commit):
                self.store.commit(commit)
            # delivered now: checked by the node's verify CRC, or deferred to the consumer
            # (a deferred copy that fails later is moved to p2p_rejected: _settle_deferred /
            # verify_done)
            self._count_p2p(good[4], True)
            if bad is not None:
                self.store.drop(bad[2])
                self.stats["crc_failures"] += len(bad[0])
                self._count_p2p(bad[4], False)  # never delivered
        if h.send_pins is not None:
            self.store.unpin(h.send_pins)
        for x in h.release:  # the round's DMAs are done: drop the staged host copies
            origin, path, rng = x.net
            origin.release(path, rng)
        self.stats["upload"] += h.sent_bytes
        t2 = time.perf_counter()
        # ---- deliveries: served wants leave the table, their tokens come back as columns
        if h.cdn is not None and len(h.cdn[0]):
            wids, eids, offs, lens = h.cdn[0], h.cdn[1], h.cdn[2], h.cdn[3]
            # CDN and P2P bytes both count when the round delivers them (one clock for a timed
            # window's offload ratio)
            self.stats["cdn"] += int(lens.sum())
            self.stats["cdn_segments"] += len(wids)
            tok, idx, pf = wt.finish(wids)
            self._after_finish(wids, pf, h.cdn[4], "cdn")
            cdn_ms = max(h.cdn_ms, h.shaped_ms)
            k = len(tok)
            if k:
                self._deliver_cols(tok, np.zeros(k, dtype=np.int8), lens[idx], np.full(k, cdn_ms),
                                   np.zeros(k), offs[idx], eids[idx], delay=h.shaped_ms)
        if good is not None and len(good[0]):
            wids, srcs, eids, offs, lens, keys = good
            winfo = wt.info(np.ascontiguousarray(wids[dgood])) if dgood is not None else None
            tok, idx, pf = wt.finish(wids)
            exp_tok = None
            if dgood is not None:
                tok, idx, exp_tok = self._settle_deferred(h, good, dgood, exp_good, tok, idx, winfo)
            self._after_finish(wids, pf, keys, "p2p")
            k = len(tok)
            if k:
                p2p_ms = np.full(len(wids), h.p2p_ms)
                delay = None
                if self.link_kbps:  # slow-link fault injection: bytes queued per source link
                    delay = np.zeros(len(wids))
                    link_q: Dict[int, int] = {}
                    for i, (src, n) in enumerate(zip(srcs.tolist(), lens.tolist())):
                        kbps = self.link_kbps.get(src)
                        if kbps:
                            link_q[src] = link_q.get(src, 0) + n
                            delay[i] = link_q[src] * 8.0 / kbps  # kbit/s == bit/ms
                            p2p_ms[i] = max(p2p_ms[i], delay[i])
                    delay = delay[idx]
                self._deliver_cols(tok, np.ones(k, dtype=np.int8), lens[idx], np.zeros(k), p2p_ms[idx], offs[idx],
                                   eids[idx], peers=srcs[idx], delay=delay, expect=exp_tok)
        if bad is not None and len(bad[0]):
            wt.requeue(bad[0], True)  # corrupted peer copy: from the CDN next round
        # planned but not served (a STAGE row, a CDN error already reported): waiting again
        if h.ids is not None and len(h.ids):
            served = [a for a in (h.cdn[0] if h.cdn is not None else None,
                                  h.recv[0] if h.recv is not None else None, h.failed) if a is not None and len(a)]
            rest = np.setdiff1d(h.ids, np.concatenate(served), assume_unique=False) if served else h.ids
            if len(rest):
                wt.requeue(rest, False)
        for ids in h.hold:  # in-flight pins from reservation (dropped entries: no-op)
            self.store.unpin(ids)
        h.hold = []
        self.timer.add("commit", t2 - t1)
        self.timer.add("deliver", time.perf_counter() - t2)
        self.timer.add("dev_cdn_ms", h.cdn_ms / 1e3)
        now = time.perf_counter()
        if self._cdn_t is not None:  # busy share of the ingest link: copy time over wall time, both
            # averaged over rounds (rounds in flight can complete back to back: a per-round ratio
            # would read a burst as a saturated link)
            self._cdn_num += 0.2 * (h.cdn_ms / 1e3 - self._cdn_num)
            self._cdn_den += 0.2 * ((now - self._cdn_t) - self._cdn_den)
            self._cdn_busy = min(1.0, self._cdn_num / self._cdn_den) if self._cdn_den > 0 else 0.0
        self._cdn_t = now
        self.timer.add("dev_p2p_ms", h.p2p_ms / 1e3)
        self.last_complete = time.monotonic()
        self.last_round = {"wants": h.n_wants, "cdn": 0 if h.cdn is None else len(h.cdn[0]), "send": h.n_send,
                           "recv": 0 if h.recv is None else len(h.recv[0]), "cdn_ms": h.cdn_ms, "dmas": h.dmas,
                           "p2p_ms": h.p2p_ms, "ms": (time.perf_counter() - h.t0) * 1e3}
        if wt.waiting:
            self._schedule()  # (a want being downloaded is rescheduled when it lands)

    def _after_finish(self, wids: np.ndarray, prefetch_only: np.ndarray, keys: np.ndarray, source: str) -> None:
        """Bookkeeping of wants that just left the table: Python-side state, and where a
        prefetched segment nobody asked for yet came from (its first cache hit is accounted
        as that source)."""
        if self._wx:
            for w in wids.tolist():
                x = self._wx.pop(w, None)
                if x is not None and x.net is not None and x.staged and source == "p2p":
                    x.net[0].release(x.net[1], x.net[2])  # staged here, but a peer's copy came first
        if prefetch_only.any():
            for i in np.flatnonzero(prefetch_only).tolist():
                self._prefetched[tuple(int(v) for v in keys[i])] = source

    def _clock_sync(self, ev, t_host: float) -> None:
        """Keep ``ev`` (a timing event the host just saw complete at ``t_host``) as the
        reference that maps node-stream event times to host time (the previous reference goes
        back to the pool).  Error: one event query (~µs); refreshed at every waited round, so
        device / host clock drift never accumulates."""
        old = self._clk
        self._clk = (ev, t_host)
        if old is not None:
            self._events.put(True, old[0])

    ROUND_SPIN_S = 0.02  # busy-poll a round's completion this long before checking for peer failures

    def _wait_round(self, h: RoundHandle) -> None:
        """Wait for a round's device work without hanging on a dead peer.

        A round whose RCCL transfers wait for a peer that crashed never completes, and
        ``hipEventSynchronize`` would block forever.  Instead: poll the round's event (the
        common case finishes within the first ``ROUND_SPIN_S``), then poll it every
        millisecond while asking the communicator for an asynchronous error
        (``ncclCommGetAsyncError``) and watching the round deadline (``gpuSwarm.roundTimeoutMs``,
        else ``HLSP2P_ROUND_TIMEOUT`` seconds, else 60 s: :meth:`round_deadline_s`); either one
        raises instead of hanging the rank."""
        ev = h.done
        spin_end = time.perf_counter() + self.ROUND_SPIN_S
        while time.perf_counter() < spin_end:
            if ev.query():
                return
        check = getattr(self.comm, "async_error", None)
        deadline = time.perf_counter() + self.round_deadline_s()
        while not ev.query():
            err = check() if check is not None else ""
            if err:
                self.failed = self.failed or f"round {h.round}: data plane error: {err}"
                raise RuntimeError(f"rank {self.rank}: swarm round {h.round} failed in the data plane: {err}")
            if time.perf_counter() > deadline:
                summary = self.plan_summary(h)
                log.error("rank %d: swarm round %d did not complete; this rank's plan: %s", self.rank, h.round,
                          summary)
                self._dump_plan(h)
                self.failed = self.failed or f"round {h.round} did not complete within {self.round_deadline_s():g} s"
                raise SwarmPeerLost(f"rank {self.rank}: swarm round {h.round} did not complete on the device "
                                    f"within {self.round_deadline_s():g} s (gpuSwarm.roundTimeoutMs); a peer may have "
                                    f"stopped.  Plan: {summary}")
            time.sleep(1e-3)

    ROUND_TIMEOUT_S = 60.0  # library default of the round deadline (was 600 s outside bench.py)

    def round_deadline_s(self) -> float:
        """Seconds a round may wait for its transfers: ``gpuSwarm.roundTimeoutMs`` when set,
        else ``HLSP2P_ROUND_TIMEOUT`` (read at each wait), else :attr:`ROUND_TIMEOUT_S`."""
        if self.round_timeout_s is not None:
            return float(self.round_timeout_s)
        return float(os.environ.get("HLSP2P_ROUND_TIMEOUT", str(self.ROUND_TIMEOUT_S)))

    def _peer_lost(self, where: str, err: BaseException) -> "SwarmPeerLost":
        """A collective of the swarm failed (a peer died or stopped answering within the
        deadline): stop the data plane without waiting on peers, and build the error with this
        rank's plan of the last round it posted (what its peers were to send / receive)."""
        summary = self.plan_summary(self._last_posted) if self._last_posted is not None else {}
        log.error("rank %d: swarm %s failed in round %d: %s; last posted plan: %s", self.rank, where, self.round,
                  err, summary)
        self._diverged(f"{where} failed: {err}")
        return SwarmPeerLost(f"rank {self.rank}: swarm {where} failed in round {self.round} ({type(err).__name__}: "
                             f"{err}); a peer may have stopped.  Plan of round "
                             f"{summary.get('round', '-')}: {summary}")

    @staticmethod
    def plan_summary(h: RoundHandle) -> Dict[str, Any]:
        """Per peer: the rows and bytes this rank was to send / receive in round ``h`` (what its
        data-plane group posted), for the diagnostic of a round that does not complete."""
        out: Dict[str, Any] = {"round": h.round, "send": {}, "recv": {}}
        if h.plan is None:
            return out
        for name, rows, col in (("send", h.plan[0], 6), ("recv", h.plan[1], 5)):
            if len(rows):
                peers, inv = np.unique(rows[:, col], return_inverse=True)
                nbytes = np.bincount(inv, weights=rows[:, 4])
                count = np.bincount(inv)
                out[name] = {int(p): [int(c), int(b)] for p, c, b in zip(peers, count, nbytes)}
        return out

    def _dump_plan(self, h: RoundHandle) -> None:
        """Write this rank's plan rows of round ``h`` under ``HLSP2P_PLAN_DUMP`` (a directory;
        one ``plan.r<round>.rank<rank>.npz`` per rank), so the ranks' views can be compared."""
        d = os.environ.get("HLSP2P_PLAN_DUMP")
        if not d or h.plan is None:
            return
        try:
            os.makedirs(d, exist_ok=True)
            np.savez(os.path.join(d, f"plan.r{h.round}.rank{self.rank}.npz"), send=h.plan[0], recv=h.plan[1],
                     directory_digest=np.int64(self.directory.digest))
        except OSError as e:  # a diagnostic must not mask the timeout itself
            log.warning("rank %d: plan dump failed: %s", self.rank, e)

    def _diverged(self, what: str) -> None:
        """Replicated state differs across ranks: no rank may post another data-plane group.
        Abort the communicator (transfers already posted would never be matched) and log."""
        if self.failed is None:
            self.failed = what
        log.error("rank %d: %s", self.rank, what)
        abort = getattr(self.comm, "abort", None)
        if abort is not None:
            try:
                abort()
            except Exception as e:  # noqa: BLE001 - the divergence is the error to report
                log.warning("rank %d: communicator abort failed: %s", self.rank, e)

    def _views(self, offs: List[int], lens: List[int]) -> List[torch.Tensor]:
        """Zero-copy uint8 views of the arena for a round's deliveries (one native call on
        the GPU; a Python slice costs ~1.5 us per view)."""
        if not len(offs):
            return []
        if self.is_cuda:
            from ..ops._native import device as _dev

            return _dev().arena_views(self.arena, np.asarray(offs, dtype=np.int64), np.asarray(lens, dtype=np.int64))
        arena = self.arena
        return [arena[o:o + n] for o, n in zip(offs, lens)]

    # ------------------------------------------------------------------ phases
    def _cdn_phase(self, h: RoundHandle, cdn_rows: np.ndarray) -> None:
        wids = np.ascontiguousarray(cdn_rows[:, 7])
        info = self._wt.info(wids)  # [n, 10]: key x4, size, src_ptr, src_base, flags, round, attempts
        ptrs = info[:, 5].copy()
        bases = info[:, 6].copy()
        lens = info[:, 4].copy()
        wflags = info[:, 7]
        keep = info[:, 0] >= 0
        failed: List[int] = []
        slow = np.flatnonzero(keep & ((wflags & W_PY) != 0))
        for i in slow.tolist():  # network / live origins: Python resolves the bytes now
            wid = int(wids[i])
            x = self._wx.get(wid)
            try:
                if x is None:
                    raise http.HttpError(500, "", "want lost its origin state")
                if x.net is not None:  # network origin: the staged (already ranged) host copy
                    origin, path, rng = x.net
                    data, off, n, _ = origin.resource_range(path, rng)
                    h.release.append(x)
                    self._wx.pop(wid, None)
                    x.staged = False  # released by this round
                else:
                    origin, path, rng = x.src
                    data, off, n, _ = origin.resource(path)
                    if rng is not None:
                        s, e = rng
                        e = n - 1 if e is None else min(e, n - 1)
                        off, n = off + s, max(0, e - s + 1)
                    if origin.should_corrupt(path):
                        wflags[i] |= W_CORRUPT
            except http.HttpError as e:
                self._finish_failed(np.array([wid], dtype=np.int64), e)
                failed.append(wid)
                keep[i] = False
                continue
            base = data.data_ptr()
            if not data.is_cuda and self.is_cuda and base not in self._loc_keep and not data.is_pinned():
                raise RuntimeError("CDN origin buffers must be pinned host memory for the async H2D path")
            if data.is_cuda:
                wflags[i] |= W_ON_DEV
            h.keep.append(data)  # the source stays alive until the round completes
            ptrs[i], bases[i], lens[i] = base + int(off), base, int(n)
        if failed:
            h.failed = np.asarray(failed, dtype=np.int64)
        if not keep.all():
            wids, ptrs, bases, lens, wflags = wids[keep], ptrs[keep], bases[keep], lens[keep], wflags[keep]
            keys = np.ascontiguousarray(info[keep, :4])
        else:
            keys = np.ascontiguousarray(info[:, :4])
        if not len(wids):
            return
        res = self.store.reserve_run(keys, lens, self.round)
        if res is None:  # admission guarantees room; reaching this is a bookkeeping bug
            raise RuntimeError("segment cache cannot make room (pinned entries block eviction)")
        _, eids, offs = res
        self.store.pin(eids)  # in flight until delivered (complete_round unpins)
        h.hold.append(eids)
        self._grow_crc(int(eids.max()) + 1)
        if self.is_cuda:
            on_dev = (wflags & W_ON_DEV) != 0
            if on_dev.any() and not on_dev.all():
                raise RuntimeError("CDN origin buffers of one round must all be pinned host or all HBM")
            start = self._events.get(True)
            end = self._events.get(True)
            cs = self.copy_stream
            with (torch.cuda.stream(cs) if cs is not None else contextlib.nullcontext()):
                start.record(cs if cs is not None else self.stream)
                from ..ops._native import device as _dev

                h.dmas = _dev().h2d_batch(self.arena, offs, ptrs, lens, bases, ALIGN, bool(on_dev[0]))
                end.record(cs if cs is not None else self.stream)
            if cs is not None:
                self.stream.wait_event(end)  # ingest CRC / forwarding sends read the DMA'd bytes
            h.ev_cdn = (start, end)
        else:
            t = time.perf_counter()
            self.rt.host_copy_batch(self.arena.data_ptr(), self.arena.numel(), offs, ptrs, lens)
            h.cdn_ms = (time.perf_counter() - t) * 1e3
        corrupt = np.flatnonzero((wflags & W_CORRUPT) != 0)
        for i in corrupt.tolist():
            if lens[i]:
                self.arena[int(offs[i]) + int(lens[i]) // 2] ^= 0xFF
        if self.ingest_crc:  # the trailers this rank's sends carry: each CRC bound to its key
            _crc.crc32_batch(self.arena, offs, lens, scatter_to=self.crc_dev, scatter_idx=eids, keys=keys)
        self.store.commit(eids)  # announced next round; peers' reads are stream-ordered after the H2D
        # CDN bandwidth shaping (xhr-shaper analog): completions are deferred by the modelled
        # transfer time of this round's CDN bytes
        total = int(lens.sum())
        h.shaped_ms = http.Shaper.transfer_ms(total)
        h.cdn = (wids, eids, offs, lens, keys)  # counted in stats["cdn"] at delivery (complete_round)

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
        # the native RCCL plane takes the round as pointer columns: with every send run a
        # contiguous arena span, no tensor view or Python object is built per peer
        spans_plane = getattr(self.comm, "exchange_spans", None) if self.is_cuda else None
        if spans_plane is not None and len(srun) and not (srun[:, 3] == 0).all():
            spans_plane = None  # a gathered run needs its staging tensor: the general path
        trailer_all = trailers = None
        # --- sends: one buffer (+ CRC trailer slice) per destination
        if len(send_rows):
            present_all = send_eids >= 0
            idx = _dev_index(np.where(present_all, send_eids, 0), dev)
            trailer_all = torch.index_select(self.crc_dev, 0, idx)
            if not present_all.all():  # missing entry: a bad CRC, the receiver re-fetches from the CDN
                trailer_all[torch.from_numpy(np.flatnonzero(~present_all)).to(dev)] = -1
            spans = self._views(srun[:, 4].tolist(), srun[:, 5].tolist()) \
                if spans_plane is None and len(srun) and (srun[:, 3] == 0).all() else None
            for k, (dst, a, b, mode, off, total) in enumerate(srun.tolist() if spans_plane is None else ()):
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
            if spans_plane is None:
                views = self._views(rrun[:, 3].tolist(), rrun[:, 4].tolist())
                for (src, a, b, _, _), view in zip(rrun.tolist(), views):
                    recvs.append((src, view))
                    recvs.append((src, trailers[a:b]))
            h.hold.append(rid_a)  # pinned by p2p_layout until complete_round
            # segment bytes per source run (a run's span also holds alignment gaps)
            np.add.at(self.p2p_from, rrun[:, 0], np.add.reduceat(recv_rows[:, 4], rrun[:, 1]))
            self._grow_crc(int(rid_a.max()) + 1)
            h.recv = (np.ascontiguousarray(recv_rows[:, 7]), np.ascontiguousarray(recv_rows[:, 5]), rid_a, roff_a,
                      np.ascontiguousarray(recv_rows[:, 4]), np.ascontiguousarray(recv_rows[:, :4]))
        self.timer.add("p2p_prep", time.perf_counter() - t_prep)
        t = time.perf_counter()
        h.t_post = t
        if self.is_cuda:
            start = self._events.get(True)
            end = self._events.get(True)
            start.record(self.stream)  # launch_round runs this phase on the node stream
        try:
            if spans_plane is not None:
                spans_plane(*_span_columns(self.arena.data_ptr(), srun, trailer_all, rrun, trailers))
            else:
                self.comm.exchange(sends, recvs)
        except Exception as e:  # noqa: BLE001 - e.g. gloo's "connection closed by peer"
            raise self._peer_lost("data-plane exchange", e) from e
        if self.is_cuda:
            end.record(self.stream)
            h.ev_p2p = (start, end)
        else:
            h.p2p_ms = (time.perf_counter() - t) * 1e3
        if h.recv is None:
            return
        if self.corrupt_next_recv > 0:  # fault injection: transport corruption
            self.corrupt_next_recv -= 1
            o, n = int(roff_a[0]), int(recv_rows[0, 4])
            if n:
                self.arena[o + n // 2] ^= 0x5A
        defer = None
        if self.verify_deferred:  # rows whose consumer checks the CRC (no Python-side origin state)
            wf = self._wt.info(np.ascontiguousarray(recv_rows[:, 7]))[:, 7]
            d = (wf & (W_PY | W_PREFETCH)) == 0
            defer = d if d.any() else None
        if defer is None:
            # verify against the senders' trailers, keyed with the key this rank asked for (a
            # segment sent under another key fails, even when its bytes match its own CRC);
            # the combine kernel also scatters the keyed CRCs into the per-entry table (ids
            # and keys ride the descriptor H2D): a mismatching entry is dropped in
            # complete_round, so the table only ever serves verified values
            _, ok = _crc.crc32_batch(self.arena, roff_a, recv_rows[:, 4], expect_dev=trailers,
                                     scatter_to=self.crc_dev, scatter_idx=rid_a, keys=recv_rows[:, :4])
        else:
            ok = self._defer_verify(h, defer, trailers, roff_a, recv_rows, rid_a)
        if isinstance(ok, np.ndarray):  # decided on the host (every row's check deferred)
            h.ok_host = ok
        elif self.is_cuda:
            h.ok_host = torch.empty(ok.numel(), dtype=torch.uint8, pin_memory=True)
            h.ok_host.copy_(ok, non_blocking=True)
        else:
            h.ok_host = ok
        # wire-level only: peer bytes count as delivered P2P once their CRC check passed
        self.stats["p2p_wire"] += int(recv_rows[:, 4].sum())
        self.stats["p2p_links"] += len(rrun)

    def _defer_verify(self, h: RoundHandle, defer: np.ndarray, trailers, roff_a: np.ndarray, recv_rows: np.ndarray,
                      rid_a: np.ndarray):
        """Received rows under deferred verification (``verify_deferred``): their trailers go
        into the CRC table now (the entries are announced only after the check) and to the
        host with the delivery; the other rows are CRC-read as usual.  Returns the per-row ok
        flags on the node's device (deferred rows: provisionally 1), or on the host when every
        row is deferred (the fleet's common case: one index H2D, one table write, one D2H of the
        trailers -- no flags tensor, no copy back)."""
        dev = self.device
        nd, dd = np.flatnonzero(~defer), np.flatnonzero(defer)
        h.defer = defer
        if not len(nd):
            self.crc_dev.index_copy_(0, _dev_index(rid_a, dev), trailers)
            self._expect_to_host(h, trailers)
            return np.ones(len(recv_rows), dtype=np.uint8)
        if self.is_cuda:
            from ..ops.desc import pack_to_device

            ix = pack_to_device({"nd": nd, "dd": dd, "rd": np.ascontiguousarray(rid_a[dd])}, dev)
        else:
            ix = {"nd": torch.from_numpy(nd), "dd": torch.from_numpy(dd), "rd": torch.from_numpy(rid_a[dd])}
        ok = torch.ones(len(recv_rows), dtype=torch.uint8, device=dev)
        if len(nd):
            _, ok_nd = _crc.crc32_batch(self.arena, roff_a[nd], recv_rows[nd, 4],
                                        expect_dev=torch.index_select(trailers, 0, ix["nd"]),
                                        scatter_to=self.crc_dev, scatter_idx=rid_a[nd], keys=recv_rows[nd, :4])
            ok.index_copy_(0, ix["nd"], ok_nd)
        if len(dd):
            self.crc_dev.index_copy_(0, ix["rd"], torch.index_select(trailers, 0, ix["dd"]))
        self._expect_to_host(h, trailers)
        return ok

    def _expect_to_host(self, h: RoundHandle, trailers) -> None:
        """The senders' (keyed) trailers of a round's receives, to the host for delivery
        (asynchronous on the GPU: read after the host waited on the round)."""
        if self.is_cuda:
            h.expect_host = torch.empty(trailers.numel(), dtype=torch.int32, pin_memory=True)
            h.expect_host.copy_(trailers, non_blocking=True)
        else:
            h.expect_host = trailers.clone()

    def _settle_deferred(self, h: RoundHandle, good: tuple, dgood: np.ndarray, exp_good: np.ndarray,
                         tok: np.ndarray, idx: np.ndarray, winfo: np.ndarray):
        """Delivery-time bookkeeping of received rows whose CRC the consumer checks.  A row
        only bulk (fleet) tokens wait for is delivered with its expected CRC and stays
        pending (one extra pin) until :meth:`verify_done`; a row an in-process request (or
        nobody) waits for is verified here, synchronously, as the loader contract delivers
        checked bytes.  Returns the delivery's ``tok``, ``idx`` and per-token expected CRCs
        (-1: none).  Vectorised: no per-row Python on the common path (every row bulk)."""
        wids, _, eids, offs, lens, _ = good
        n = len(wids)
        info = np.zeros((n, winfo.shape[1]), dtype=winfo.dtype)
        info[dgood] = winfo
        now = dgood & (np.bincount(idx, minlength=n) == 0)
        neg = tok < 0
        if neg.any() and not self.defer_inproc:
            now |= dgood & (np.bincount(idx[neg], minlength=n) > 0)
        keep = None
        if now.any():
            nr = np.flatnonzero(now)
            exp = (exp_good[nr] & _M32).tolist()
            if self.is_cuda:
                with self._on_node_stream():
                    _, okd = _crc.crc32_batch(self.arena, offs[nr], lens[nr], expect=exp)
                    ok_now = okd.cpu().numpy().astype(bool)
            else:
                ok_now = _crc.crc32_batch(self.arena, offs[nr], lens[nr], expect=exp)[1].numpy().astype(bool)
            if ok_now.any():
                self.store.commit(eids[nr[ok_now]])
            bad = nr[~ok_now]
            if len(bad):
                self.store.drop(eids[bad])
                self.stats["crc_failures"] += len(bad)
                self._reject_p2p(lens[bad])
                keep = np.ones(len(tok), dtype=bool)
                for r in bad.tolist():
                    sel = idx == r
                    self._retry_cdn(info[r], tok[sel])
                    keep &= ~sel
            dgood = dgood & ~now
        pend = np.flatnonzero(dgood)
        if len(pend):
            pe = eids[pend]
            self.store.pin(pe)  # held until verify_done
            self._vpend_add(pe, info[pend], exp_good[pend])
        exp_row = np.full(n, -1, dtype=np.int64)
        exp_row[pend] = exp_good[pend] & _M32
        if keep is not None:
            tok, idx = tok[keep], idx[keep]
        return tok, idx, exp_row[idx]

    def _misroute(self, send_rows: np.ndarray, send_eids: np.ndarray) -> None:
        """Fault injection (``misroute_next_send``): send row i's bytes from another resident
        entry of the same length -- the receiver's keyed CRC check must reject it."""
        ids, keys = self.store.resident()
        if not len(ids):
            return
        lens = self.store.entries(ids)[:, 1]
        for i in np.flatnonzero(send_eids >= 0).tolist():
            same = np.flatnonzero((lens == send_rows[i, 4]) & (keys != send_rows[i, :4]).any(axis=1))
            if len(same):
                send_eids[i] = ids[same[0]]
                self.misroute_next_send -= 1
                return

    def _count_p2p(self, lens: np.ndarray, passed: bool) -> None:
        """Account peer copies: delivered P2P bytes (``passed``), or rejected bytes of copies
        that failed their CRC check before delivery (the segment is then re-fetched, and
        counted, from the CDN)."""
        n = len(lens)
        if not n:
            return
        b = int(np.asarray(lens, dtype=np.int64).sum())
        if passed:
            self.stats["p2p"] += b
            self.stats["p2p_segments"] += n
        else:
            self.stats["p2p_rejected"] += b
            self.stats["p2p_rejected_segments"] += n

    def _reject_p2p(self, lens: np.ndarray) -> None:
        """Copies counted as delivered P2P whose deferred check failed: P2P -> rejected."""
        n = len(lens)
        if not n:
            return
        b = int(np.asarray(lens, dtype=np.int64).sum())
        self.stats["p2p"] -= b
        self.stats["p2p_segments"] -= n
        self.stats["p2p_rejected"] += b
        self.stats["p2p_rejected_segments"] += n

    def _vpend_add(self, eids: np.ndarray, info: np.ndarray, expect: np.ndarray) -> None:
        need = int(eids.max()) + 1
        if need > len(self._vflag):
            cap = max(need, 2 * len(self._vflag), 1024)
            flag = np.zeros(cap, dtype=bool)
            flag[:len(self._vflag)] = self._vflag
            vinfo = np.zeros((cap, self._vinfo.shape[1]), dtype=np.int64)
            vinfo[:len(self._vinfo)] = self._vinfo
            vround = np.zeros(cap, dtype=np.int64)
            vround[:len(self._vround)] = self._vround
            vexp = np.zeros(cap, dtype=np.int64)
            vexp[:len(self._vexp)] = self._vexp
            self._vflag, self._vinfo, self._vround, self._vexp = flag, vinfo, vround, vexp
        self._vflag[eids] = True
        self._vinfo[eids] = info
        self._vround[eids] = self.round
        self._vexp[eids] = expect

    VERIFY_STALE_ROUNDS = 32  # a pending entry nobody reported on for this long is checked by the node

    def _sweep_pending(self) -> int:
        """Check, on the node, deferred entries whose consumer never reported (an in-process
        fragment dropped before its transmux: a seek, an abort, a stale level); their entries
        would otherwise stay pinned and unannounced.  Synchronous CRC kernel; rare."""
        stale = np.flatnonzero(self._vflag & (self._vround < self.round - self.VERIFY_STALE_ROUNDS))
        if not len(stale):
            return 0
        ent = self.store.entries(stale)
        offs, lens = ent[:, 0].copy(), ent[:, 1].copy()
        exp = (self._vexp[stale] & _M32).tolist()
        if self.is_cuda:
            with self._on_node_stream():
                _, okd = _crc.crc32_batch(self.arena, offs, lens, expect=exp)
                ok = okd.cpu().numpy().astype(bool)
        else:
            ok = _crc.crc32_batch(self.arena, offs, lens, expect=exp)[1].numpy().astype(bool)
        self.verify_done(stale, ok, np.full(len(stale), self.rt.NO_TOKEN, dtype=np.int64))
        self.stats["verify_swept"] = self.stats.get("verify_swept", 0) + len(stale)
        return len(stale)

    def pending_verify(self) -> int:
        """Entries delivered under deferred verification whose check has not come back."""
        return int(self._vflag.sum())

    def _retry_cdn(self, info: np.ndarray, tokens: np.ndarray) -> None:
        """Ask again, from the CDN, for a segment whose peer copy failed its CRC."""
        tokens = np.ascontiguousarray(tokens, dtype=np.int64)
        if not len(tokens):
            return
        n = len(tokens)
        rep = np.repeat(info.reshape(1, -1), n, axis=0)
        self._wt.add(np.ascontiguousarray(rep[:, :4]), np.ascontiguousarray(rep[:, 4]), np.ascontiguousarray(rep[:, 5]),
                     np.ascontiguousarray(rep[:, 6]), np.ascontiguousarray(rep[:, 7] | W_FORCE_CDN), tokens)
        self._schedule()

    def invalidate(self, keys) -> int:
        """A consumer found the cached copy of these segments unusable (its decrypt or demux
        failed): detach each from the cache -- the removal goes out with the next round's
        control message, so peers stop asking this rank for it -- and take the next request
        for the key from the CDN.  ``keys``: int64[n, 4] ``(swarm, level, urlId, sn)``.
        Returns the number of cached copies detached."""
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.int64).reshape(-1, 4) & _M32)
        if not len(keys):
            return 0
        eids = self.store.lookup(keys, False)
        held = eids[eids >= 0]
        if len(held):
            self.store.detach(held)
        for row in keys.tolist():
            self._force_cdn_keys.add(tuple(row))
        self.stats["invalidated"] = self.stats.get("invalidated", 0) + len(held)
        return len(held)

    def verify_done(self, eids: np.ndarray, ok: np.ndarray, tokens: np.ndarray) -> int:
        """Outcome of deferred CRC checks (fragment columns: the entry each was read from,
        passed, its token).  A passing entry is committed (announced next round, served to
        peers); a failing one is detached (its readers' pins drain) and its tokens are asked
        again from the CDN.  Returns the number of failed entries."""
        eids = np.asarray(eids, dtype=np.int64)
        ok = np.asarray(ok, dtype=bool)
        tokens = np.asarray(tokens, dtype=np.int64)
        if not len(eids):
            return 0
        ue, inv = np.unique(eids, return_inverse=True)
        uok = np.ones(len(ue), dtype=bool)
        np.logical_and.at(uok, inv, ok)
        inside = ue < len(self._vflag)
        pend = np.zeros(len(ue), dtype=bool)
        pend[inside] = self._vflag[ue[inside]]
        good = ue[pend & uok]
        if len(good):
            self._vflag[good] = False
            self.store.commit(good)
            self.store.unpin(good)
            if self._vwait:
                for e in good.tolist():
                    if e in self._vwait:
                        self._release_parked(e, True)
        bad = np.flatnonzero(pend & ~uok)
        for k in bad.tolist():
            e = int(ue[k])
            self._vflag[e] = False
            arr = np.array([e], dtype=np.int64)
            self.store.detach(arr)
            self.store.unpin(arr)
            self.stats["crc_failures"] += 1
            self._reject_p2p(self._vinfo[e:e + 1, 4])
            toks = tokens[inv == k]
            self._retry_cdn(self._vinfo[e], toks[toks >= 0])  # bulk (fleet) tokens: asked again here
            if e in self._vwait:
                self._release_parked(e, False)
            if (toks <= -2).any():  # in-process request tokens (NO_TOKEN = -1: a node sweep)
                # in-process requests were answered already: their players ask again, from the
                # CDN.  (Bulk-only entries are re-fetched above; a key nobody will ask for again
                # must not sit in the set: request_batch checks every key while it is non-empty)
                self._force_cdn_keys.add(tuple(int(v) & _M32 for v in self._vinfo[e][:4]))
        return len(bad)

    # ------------------------------------------------------------------ delivery
    def _deliver_cols(self, tok: np.ndarray, src: np.ndarray, nbytes: np.ndarray, cdn_ms: np.ndarray,
                      p2p_ms: np.ndarray, offs: np.ndarray, eids: np.ndarray, peers: Optional[np.ndarray] = None,
                      delay: Any = None, expect: Optional[np.ndarray] = None) -> None:
        """Answer waiting tokens.  Entries stay pinned ``PIN_DELAY_ROUNDS`` launches (their
        consumers read the arena asynchronously); shaped / slowed transfers are answered
        after their modelled duration.  ``expect`` (bulk tokens only): the CRC the consumer
        must find in the bytes (-1: already verified), see ``verify_deferred``."""
        if delay is not None and not (np.isscalar(delay) and delay <= 0):
            d = np.broadcast_to(np.asarray(delay, dtype=np.float64), tok.shape)
            later = d > 0
            if later.any():
                li = np.flatnonzero(later)
                le = eids[li]
                le = le[le >= 0]
                if len(le):
                    self.store.pin(le)
                self._delayed_seq += 1
                self._delayed[self._delayed_seq] = (le, tok[li])
                self.loop.set_timeout(self._deliver_deferred, float(d[li].max()),
                                      (tok[li], src[li], nbytes[li], cdn_ms[li], p2p_ms[li], offs[li], eids[li],
                                       None if peers is None else peers[li], None,
                                       None if expect is None else expect[li]), le, self._delayed_seq)
                if later.all():
                    return
                ni = np.flatnonzero(~later)
                tok, src, nbytes, cdn_ms, p2p_ms, offs, eids = (tok[ni], src[ni], nbytes[ni], cdn_ms[ni], p2p_ms[ni],
                                                                offs[ni], eids[ni])
                peers = None if peers is None else peers[ni]
                expect = None if expect is None else expect[ni]
        pin = eids[eids >= 0]
        if len(pin):
            self.store.pin(pin)
            self._pins.append((self.round + PIN_DELAY_ROUNDS, pin))
        bulk = tok >= 0
        nb = int(bulk.sum())
        if nb:
            self.stats["segments"] += nb
            if self._bulk is not None:
                ex = {} if expect is None else {"expect": expect if nb == len(tok) else expect[bulk]}
                if nb == len(tok):
                    self._bulk.deliver(tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, **ex)
                else:
                    self._bulk.deliver(tok[bulk], src[bulk], nbytes[bulk], cdn_ms[bulk], p2p_ms[bulk], offs[bulk],
                                       eids[bulk], **ex)
        if nb == len(tok):
            return
        obj = np.flatnonzero(~bulk)
        reqs = [self._tok_req.pop(t, None) for t in tok[obj].tolist()]
        live = [i for i, r in zip(obj.tolist(), reqs) if r is not None]
        if not live:
            return
        views = self._views(offs[live].tolist(), nbytes[live].tolist())
        for i, r, view in zip(live, [r for r in reqs if r is not None], views):
            if expect is not None and expect[i] >= 0:  # deferred check: the consumer's transmux verifies
                view.swarm_verify = VerifyTicket(self, int(eids[i]), int(expect[i]), r.token)
            self._deliver_req(r, SOURCE_NAMES[int(src[i])], int(nbytes[i]), float(cdn_ms[i]), float(p2p_ms[i]), view,
                              self.rank if peers is None else int(peers[i]), int(eids[i]), pin=False)

    def _deliver_deferred(self, cols, ids: np.ndarray, seq: int = 0) -> None:
        self._delayed.pop(seq, None)
        try:
            self._deliver_cols(*cols)
        finally:
            if len(ids):
                self.store.unpin(ids)

    def _deliver_req(self, req: Request, source: str, nbytes: int, cdn_ms: float, p2p_ms: float, data: Any,
                     peer: int, eid: int, pin: bool = True) -> None:
        """Loader callbacks of one in-process request: ``onProgress`` then ``onSuccess``."""
        if req.aborted or req.done:
            return
        if pin and eid >= 0:
            arr = np.array([eid], dtype=np.int64)
            self.store.pin(arr)
            self._pins.append((self.round + PIN_DELAY_ROUNDS, arr))
        req.done = True
        self.stats["segments"] += 1
        trace = self.trace
        if trace is not None:
            now = self.loop.now()
            xfer = p2p_ms if source == "p2p" else cdn_ms
            trace.add(RequestTrace(req.key, req.t_submit, max(req.t_submit, now - xfer), now, source, nbytes,
                                   peer if source == "p2p" else self.rank, self.round))
        if req.agent is not None:
            req.agent._account(source, nbytes)
        cb = req.callbacks
        if isinstance(cb, dict):
            on_progress, on_success = cb.get("onProgress"), cb.get("onSuccess")
        else:
            delivered = getattr(cb, "onDelivered", None)
            if delivered is not None:  # one call instead of a progress event + onSuccess
                delivered(source, nbytes, cdn_ms, p2p_ms, data)
                return
            on_progress, on_success = getattr(cb, "onProgress", None), getattr(cb, "onSuccess", None)
        if on_progress is not None:
            p2p = source in ("p2p", "cache")
            on_progress({"cdnDownloaded": 0 if p2p else nbytes, "p2pDownloaded": nbytes if p2p else 0,
                         "cdnDuration": 0.0 if p2p else cdn_ms, "p2pDuration": p2p_ms if p2p else 0.0})
        if req.aborted:
            return
        if on_success is not None:
            on_success(data)

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


def _span_columns(arena_ptr: int, srun: np.ndarray, trailer_all, rrun: np.ndarray, trailers):
    """A round's transfers as pointer columns ``(send_ptr, send_bytes, send_peer, recv_ptr,
    recv_bytes, recv_peer)`` for the native RCCL group call: per peer its arena span, then
    its CRC-trailer slice -- the same per-pair order on both sides, as RCCL point-to-point
    matches the i-th send with the i-th receive.  ``srun`` rows: (dst, a, b, mode 0, arena
    offset, bytes); ``rrun`` rows: (src, a, b, arena offset, bytes); trailers are int32."""
    def cols(runs, span_off, span_len, tr):
        n = len(runs)
        ptr = np.empty(2 * n, dtype=np.int64)
        nb = np.empty(2 * n, dtype=np.int64)
        peer = np.empty(2 * n, dtype=np.int64)
        if n:
            ptr[0::2] = arena_ptr + runs[:, span_off]
            nb[0::2] = runs[:, span_len]
            ptr[1::2] = tr.data_ptr() + 4 * runs[:, 1]
            nb[1::2] = 4 * (runs[:, 2] - runs[:, 1])
            peer[0::2] = peer[1::2] = runs[:, 0]
        return ptr, nb, peer

    sp, sb, sd = cols(srun, 4, 5, trailer_all)
    rp, rb, rs = cols(rrun, 3, 4, trailers)
    return sp, sb, sd, rp, rb, rs


def _dev_index(idx: np.ndarray, dev: torch.device) -> torch.Tensor:
    """int64 index array on ``dev`` (pinned staging + one async H2D on GPUs)."""
    if dev.type == "cuda":
        from ..ops.desc import pack_to_device

        return pack_to_device({"i": np.ascontiguousarray(idx, dtype=np.int64)}, dev)["i"]
    return torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int64))


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
    ``prefetchSeconds`` / ``prefetchMaxSegments``.  ``roundTimeoutMs`` (default 60 000) /
    ``controlTimeoutMs`` (default 300 000): how long a round may wait for its transfers and the
    control all-gather for every peer before the rank raises :class:`SwarmPeerLost` with its
    plan (a dead peer fails the job in a minute instead of hanging it).  ``deferVerify``: segments received from
    peers reach in-process players before their CRC check, which the player's transmux batch
    runs fused into its decrypt (:class:`VerifyTicket`).  ``numaBind``: run this process on the CPUs
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

        node = RemoteNode(cfg["conn"], world=int(cfg.get("world", 1)), rank=int(cfg.get("rank", 0)),
                          payload=bool(cfg.get("fleetPayload", False)))
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
    if cfg.get("audit"):
        node.audit_on = True
    if cfg.get("roundTimeoutMs") is not None:
        node.round_timeout_s = float(cfg["roundTimeoutMs"]) / 1e3
    if cfg.get("controlTimeoutMs") is not None and hasattr(comm, "control_timeout_s"):
        comm.control_timeout_s = float(cfg["controlTimeoutMs"]) / 1e3
    if cfg.get("deferVerify"):  # in-process players verify received segments in their transmux
        node.verify_deferred = node.defer_inproc = True
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
