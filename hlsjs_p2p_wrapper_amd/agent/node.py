"""SwarmNode — one MI355X (or CPU) peer of the swarm: HBM segment cache + exchange rounds.

This is the engine behind the peer agent's ``getSegment`` (the closed-source
``streamroot-p2p`` module in the reference), designed for the hardware:

* **Cache**: one ``uint8`` arena tensor in HBM (sized for the 288 GB part) whose layout
  is managed by the native ``SegmentStore`` ring allocator; segments received in a round
  land contiguously.
* **Rounds** (SURVEY §5.8): requests accumulate; every rank then runs one collective
  round — all-gather of a small control message (wants, cache delta, flags, counters) on
  the control plane, identical deterministic planning everywhere (native
  ``plan_round``), a CDN phase (pinned-host → HBM ``hipMemcpyAsync`` on a side stream)
  with ingest CRC on the MFMA CRC kernel, and a P2P phase: ONE contiguous buffer per peer
  pair over RCCL (``batch_isend_irecv``), with the sender's CRCs as a trailer, verified on
  device by the receiver.
* **Faults**: a peer copy failing its CRC is dropped and re-requested from the CDN next
  round; churn is modelled by ranks announcing ``online=False`` (they still join the
  collectives, as an RCCL communicator cannot shrink).

Completion semantics match the reference loader contract: ``onProgress({cdnDownloaded,
p2pDownloaded, cdnDuration, p2pDuration})`` then ``onSuccess(data)`` where ``data`` is a
zero-copy ``uint8`` view of the arena (valid until the next round), or
``onError(HttpError)`` (``p2p-loader-generator.js:164-208``).
"""
from __future__ import annotations

import logging
import threading
import time
import zlib
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..net import http
from ..net.event_loop import get_event_loop
from ..ops import crc as _crc
from ..ops import segment as _seg
from ..ops._native import runtime as _rt
from ..parallel.comm import LocalComm, SwarmComm

log = logging.getLogger("hlsjs_p2p_wrapper_amd.node")

MAGIC = 0x48505032  # "HPP2"
HDR = 16
ALIGN = 256
SLACK = 4096


def swarm_id_for(content_id: str) -> int:
    return zlib.crc32(content_id.encode()) & 0x7FFFFFFF


@dataclass(eq=False)
class Request:
    node: "SwarmNode"
    key: Tuple[int, int, int, int]
    url: str
    headers: Dict[str, str]
    callbacks: Any
    agent: Any = None
    aborted: bool = False
    done: bool = False
    t_submit: float = 0.0

    def abort(self) -> None:
        self.aborted = True


@dataclass(eq=False)
class _Want:
    key: Tuple[int, int, int, int]
    url: str
    headers: Dict[str, str]
    size: int
    want_id: int
    waiters: List[Request] = field(default_factory=list)
    force_cdn: bool = False
    attempts: int = 0


class _Completion:
    __slots__ = ("req", "data", "source", "nbytes", "cdn_ms", "p2p_ms", "error", "entry", "delay")

    def __init__(self, req, data, source, nbytes, cdn_ms, p2p_ms, error=None, entry=-1):
        self.req = req
        self.data = data
        self.source = source
        self.nbytes = nbytes
        self.cdn_ms = cdn_ms
        self.p2p_ms = p2p_ms
        self.error = error
        self.entry = entry
        self.delay = 0.0


class SwarmNode:
    def __init__(self, comm: Optional[SwarmComm] = None, device: Any = "auto", cache_bytes: int = 1 << 30,
                 loop=None, cdn_dedup: bool = True, round_interval_ms: Optional[float] = None,
                 auto_tick: bool = True) -> None:
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
        self.crc_dev = torch.zeros(1024, dtype=torch.int32, device=self.device)  # ingest CRC per entry id
        self.cdn_stream = torch.cuda.Stream(self.device) if self.is_cuda else None
        self.online = True
        self.upload_on = True
        self.download_on = True
        self.cdn_dedup = cdn_dedup
        self.round = 0
        self.round_interval_ms = round_interval_ms
        self.auto_tick = auto_tick
        self.leaving = False
        self.closed = False
        self._wants: Dict[Tuple[int, int, int, int], _Want] = {}
        self._next_want_id = 1
        self._tick_scheduled = False
        self._timer = None
        self._pinned_last: List[int] = []
        self._agents: List[Any] = []
        self.peer_online = np.ones(self.world, dtype=bool)
        self.stats = {"cdn": 0, "p2p": 0, "upload": 0, "cache": 0, "rounds": 0, "crc_failures": 0,
                      "segments": 0, "cdn_segments": 0, "p2p_segments": 0}
        self.swarm_stats = {"cdn": 0, "p2p": 0, "upload": 0}
        self.last_round: Dict[str, Any] = {}
        self.corrupt_next_recv = 0  # fault injection: flip a byte in the next N received rounds
        self._cdn_shaped_ms = 0.0
        self._lock = threading.RLock()
        if self.world > 1 and auto_tick:
            self._timer = self.loop.set_interval(self._timer_tick, round_interval_ms or 10.0)

    # ------------------------------------------------------------------ agents
    def attach(self, agent: Any) -> None:
        self._agents.append(agent)

    def detach(self, agent: Any) -> None:
        if agent in self._agents:
            self._agents.remove(agent)
        for w in list(self._wants.values()):
            w.waiters = [r for r in w.waiters if r.agent is not agent]

    @property
    def flags(self) -> int:
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
                callbacks: Any, agent: Any = None) -> Request:
        req = Request(self, tuple(int(k) & 0xFFFFFFFF for k in key), url, dict(headers or {}), callbacks, agent,
                      t_submit=self.loop.now())
        eid = self.store.lookup1(*req.key)
        if eid >= 0:  # local cache hit
            self.store.pin(np.array([eid], dtype=np.int64))
            self.loop.call_soon(self._serve_local, req, eid)
            return req
        w = self._wants.get(req.key)
        if w is None:
            try:
                size = http.head(url, req.headers)
            except http.HttpError as e:
                self.loop.call_soon(self._fail, req, e)
                return req
            w = _Want(req.key, url, req.headers, int(size), self._next_want_id)
            self._next_want_id += 1
            self._wants[req.key] = w
        w.waiters.append(req)
        self._schedule()
        return req

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
            self.stats["cache"] += n
            self._deliver([_Completion(req, self.arena[off:off + n], "cache", n, 0.0, 0.0)])
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

    # ------------------------------------------------------------------ round protocol
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
        w = np.zeros((len(wants), 6), dtype=np.int64)
        for i, x in enumerate(wants):
            w[i, :4] = x.key
            w[i, 4] = x.size
            w[i, 5] = x.want_id | ((1 if x.force_cdn else 0) << 62)
        return np.concatenate([hdr, w.reshape(-1), adds.reshape(-1).astype(np.int64),
                               rms.reshape(-1).astype(np.int64)])

    @staticmethod
    def _decode(msg: np.ndarray):
        if msg.size < HDR or msg[0] != MAGIC:
            raise RuntimeError("bad swarm control message")
        nw, na, nr = int(msg[2]), int(msg[3]), int(msg[4])
        p = HDR
        w = msg[p:p + 6 * nw].reshape(nw, 6)
        p += 6 * nw
        a = msg[p:p + 5 * na].reshape(na, 5)
        p += 5 * na
        r = msg[p:p + 4 * nr].reshape(nr, 4)
        return msg[:HDR], w, a, r

    def _grow_crc(self, n: int) -> None:
        if n > self.crc_dev.numel():
            new = torch.zeros(max(n, 2 * self.crc_dev.numel()), dtype=torch.int32, device=self.device)
            new[:self.crc_dev.numel()] = self.crc_dev
            self.crc_dev = new

    def _sync(self) -> None:
        if self.is_cuda:
            torch.cuda.current_stream(self.device).synchronize()

    def tick(self) -> bool:
        """One collective exchange round.  Returns True when every rank is leaving."""
        with self._lock:
            return self._round()

    def _round(self) -> bool:
        rt = self.rt
        t0 = time.perf_counter()
        self._cdn_shaped_ms = 0.0
        if self._pinned_last:
            self.store.unpin(np.asarray(self._pinned_last, dtype=np.int64))
            self._pinned_last = []
        # ---------------- 1. control plane
        wants = [w for w in self._wants.values() if any(not r.aborted for r in w.waiters)]
        for k in [k for k, w in self._wants.items() if w not in wants]:
            del self._wants[k]
        adds, rms = self.store.take_delta()
        msg = self._encode(wants, adds, rms)
        parts = self.comm.allgather_control(msg)
        self.round += 1
        self.stats["rounds"] += 1
        all_leaving = True
        flags = np.zeros(self.world, dtype=np.int64)
        want_rows = []
        swarm_tot = np.zeros(3, dtype=np.int64)
        for r, part in enumerate(parts):
            hdr, w, a, rm = self._decode(part)
            flags[r] = hdr[1]
            all_leaving = all_leaving and bool(hdr[5])
            swarm_tot += hdr[7:10]
            if len(a) or len(rm):
                self.directory.apply(r, np.ascontiguousarray(a), np.ascontiguousarray(rm))
            if len(w):
                rows = np.zeros((len(w), 8), dtype=np.int64)
                rows[:, :5] = w[:, :5]
                rows[:, 5] = w[:, 5] & ((1 << 62) - 1)
                rows[:, 6] = r
                rows[:, 7] = (w[:, 5] >> 62) & 1
                want_rows.append(rows)
        self.peer_online = (flags & rt.FLAG_ONLINE) != 0
        self.swarm_stats = {"cdn": int(swarm_tot[0]), "p2p": int(swarm_tot[1]), "upload": int(swarm_tot[2])}
        if not want_rows:
            self.last_round = {"wants": 0, "ms": (time.perf_counter() - t0) * 1e3}
            return all_leaving
        all_wants = np.ascontiguousarray(np.concatenate(want_rows))
        plan = rt.plan_round(self.directory, all_wants, flags, self.world)
        me = self.rank
        by_id = {w.want_id: w for w in wants}
        cdn_rows = plan[(plan[:, 5] == -1) & (plan[:, 6] == me)]
        send_rows = plan[plan[:, 5] == me]
        recv_rows = plan[(plan[:, 6] == me) & (plan[:, 5] >= 0)]
        # ---------------- 2. pin what we send from cache (seeded rows are fetched below)
        cached_send = send_rows[send_rows[:, 8] == 0]
        send_ids: Dict[Tuple[int, int, int, int], int] = {}
        if len(cached_send):
            ids = self.store.lookup(np.ascontiguousarray(cached_send[:, :4]), False)
            for row, eid in zip(cached_send, ids):
                send_ids[tuple(int(x) for x in row[:4])] = int(eid)
            valid = ids[ids >= 0]
            if len(valid):
                self.store.pin(valid)
        # ---------------- 3. CDN phase (pinned host -> HBM on the side stream)
        t_cdn0 = time.perf_counter()
        completions: List[_Completion] = []
        cdn_entries: List[Tuple[_Want, int, int, int]] = []  # (want, entry, off, n)
        cdn_ms = 0.0
        ev_cdn = None
        if len(cdn_rows):
            cdn_entries, cdn_ms, ev_cdn = self._cdn_phase(cdn_rows, by_id, completions)
            for w, eid, off, n in cdn_entries:
                send_ids.setdefault(w.key, eid)
        # ---------------- 4. P2P phase
        t_p2p0 = time.perf_counter()
        recv_entries, p2p_ms, ev_p2p, recv_meta = self._p2p_phase(send_rows, recv_rows, send_ids)
        # ---------------- 5. verify + commit
        ok_host = None
        if recv_entries:
            offs = [off for _, off, _ in recv_entries]
            lens = [n for _, _, n in recv_entries]
            _, ok = _crc.crc32_batch(self.arena, offs, lens, expect_dev=recv_meta)
            ok_host = ok.cpu().numpy() if ok is not None else None  # sync point
        else:
            self._sync()
        if ev_cdn is not None:
            cdn_ms = ev_cdn[0].elapsed_time(ev_cdn[1])
        if ev_p2p is not None:
            p2p_ms = ev_p2p[0].elapsed_time(ev_p2p[1])
        if cdn_entries:
            self.store.commit(np.asarray([e for _, e, _, _ in cdn_entries], dtype=np.int64))
        good_recv, bad_recv = [], []
        for i, (row, off, n) in enumerate(recv_entries):
            (good_recv if ok_host is None or ok_host[i] else bad_recv).append((row, off, n))
        if good_recv:
            self.store.commit(np.asarray([r[-1] for r, _, _ in good_recv], dtype=np.int64))
        if bad_recv:
            self.store.drop(np.asarray([r[-1] for r, _, _ in bad_recv], dtype=np.int64))
            self.stats["crc_failures"] += len(bad_recv)
        if len(cached_send):
            ids = np.asarray([send_ids[tuple(int(x) for x in r[:4])] for r in cached_send], dtype=np.int64)
            ids = ids[ids >= 0]
            if len(ids):
                self.store.unpin(ids)
        # ---------------- 6. completions
        sent_bytes = int(send_rows[:, 4].sum()) if len(send_rows) else 0
        self.stats["upload"] += sent_bytes
        shaped_ms = self._cdn_shaped_ms
        for w, eid, off, n in cdn_entries:
            if w.key in self._wants and self._wants[w.key] is w:
                del self._wants[w.key]
                for req in w.waiters:
                    c = _Completion(req, self.arena[off:off + n], "cdn", n, max(cdn_ms, shaped_ms), 0.0, entry=eid)
                    c.delay = shaped_ms
                    completions.append(c)
        for row, off, n in good_recv:
            wid = int(row[7])
            w = by_id.get(wid)
            if w is None or self._wants.get(w.key) is not w:
                continue
            del self._wants[w.key]
            for req in w.waiters:
                completions.append(_Completion(req, self.arena[off:off + n], "p2p", n, 0.0, p2p_ms, entry=row[-1]))
        for row, off, n in bad_recv:
            w = by_id.get(int(row[7]))
            if w is not None:
                w.force_cdn = True  # corrupted peer copy: go to the CDN next round
                w.attempts += 1
        self._deliver(completions)
        self.last_round = {"wants": int(len(all_wants)), "cdn": int(len(cdn_rows)), "send": int(len(send_rows)),
                           "recv": int(len(recv_rows)), "cdn_ms": cdn_ms, "p2p_ms": p2p_ms,
                           "ms": (time.perf_counter() - t0) * 1e3}
        if self._wants:
            self._schedule()
        return all_leaving

    def _cdn_phase(self, cdn_rows: np.ndarray, by_id: Dict[int, _Want], completions: List[_Completion]):
        wants = []
        sources = []
        for row in cdn_rows:
            w = by_id.get(int(row[7]))
            if w is None:
                continue
            try:
                origin, path = http.resolve(w.url)
                data, off, n, _ = origin.resource(path)
                rng = http.parse_range(w.headers)
                if rng is not None:
                    s, e = rng
                    e = n - 1 if e is None else min(e, n - 1)
                    off, n = off + s, max(0, e - s + 1)
                corrupt = origin.should_corrupt(path)
            except http.HttpError as e:
                del self._wants[w.key]
                for req in w.waiters:
                    self.loop.call_soon(self._fail, req, e)
                continue
            wants.append(w)
            sources.append((data, off, n, corrupt))
        if not wants:
            return [], 0.0, None
        keys = np.asarray([w.key for w in wants], dtype=np.int64)
        lens = np.asarray([s[2] for s in sources], dtype=np.int64)
        res = self.store.reserve_run(keys, lens, self.round)
        if res is None:
            raise RuntimeError("segment cache cannot make room (pinned entries block eviction)")
        _, ids, offs = res
        self._grow_crc(int(ids.max()) + 1)
        ev = None
        if self.is_cuda:
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            cur = torch.cuda.current_stream(self.device)
            self.cdn_stream.wait_stream(cur)
            with torch.cuda.stream(self.cdn_stream):
                start.record()
                for (data, off, n, _), doff in zip(sources, offs):
                    self.arena[doff:doff + n].copy_(data[off:off + n], non_blocking=True)
                end.record()
            cur.wait_stream(self.cdn_stream)
            ev = (start, end)
        else:
            t = time.perf_counter()
            for (data, off, n, _), doff in zip(sources, offs):
                self.arena[doff:doff + n].copy_(data[off:off + n])
            ms = (time.perf_counter() - t) * 1e3
        for (_, _, n, corrupt), doff in zip(sources, offs):
            if corrupt and n:
                self.arena[doff + n // 2] ^= 0xFF
        crc, _ = _crc.crc32_batch(self.arena, offs.tolist(), lens.tolist())
        self.crc_dev[torch.from_numpy(ids).to(self.device)] = crc
        # CDN bandwidth shaping (xhr-shaper analog): completions are deferred by the modelled
        # transfer time of this round's CDN bytes
        self._cdn_shaped_ms = http.Shaper.transfer_ms(int(lens.sum()))
        nbytes = int(lens.sum())
        self.stats["cdn"] += nbytes
        self.stats["cdn_segments"] += len(wants)
        entries = [(w, int(eid), int(o), int(n)) for w, eid, o, n in zip(wants, ids, offs, lens)]
        return entries, (0.0 if self.is_cuda else ms), ev

    def _p2p_phase(self, send_rows: np.ndarray, recv_rows: np.ndarray, send_ids: Dict):
        if not len(send_rows) and not len(recv_rows):
            return [], 0.0, None, None
        sends: List[Tuple[int, torch.Tensor]] = []
        recvs: List[Tuple[int, torch.Tensor]] = []
        # --- sends: one contiguous buffer (+ CRC trailer) per destination
        for dst in np.unique(send_rows[:, 6]) if len(send_rows) else []:
            rows = send_rows[send_rows[:, 6] == dst]
            ids = np.asarray([send_ids.get(tuple(int(x) for x in r[:4]), -1) for r in rows], dtype=np.int64)
            present = ids >= 0
            if present.all():
                ent = self.store.entries(ids)
                offs, lens = ent[:, 0], ent[:, 1]
                contiguous = bool(np.all(offs[1:] == offs[:-1] + (lens[:-1] + ALIGN - 1) // ALIGN * ALIGN)) \
                    and np.all(lens == rows[:, 4])
            else:
                contiguous = False
            sizes = rows[:, 4]
            if contiguous:
                total = int(offs[-1] + lens[-1] - offs[0])
                buf = self.arena[int(offs[0]):int(offs[0]) + total]
                trailer = self.crc_dev[torch.from_numpy(ids).to(self.device)]
            else:
                layout = np.zeros(len(rows), dtype=np.int64)
                if len(rows) > 1:
                    layout[1:] = np.cumsum((sizes[:-1] + ALIGN - 1) // ALIGN * ALIGN)
                total = int(layout[-1] + sizes[-1])
                buf = torch.zeros(total, dtype=torch.uint8, device=self.device)
                trailer = torch.full((len(rows),), 0, dtype=torch.int32, device=self.device)
                if present.any():
                    ent = self.store.entries(ids[present])
                    n_copy = np.minimum(ent[:, 1], sizes[present])
                    _seg.copy_segments(self.arena, buf, ent[:, 0], layout[present], n_copy)
                    pidx = torch.from_numpy(np.nonzero(present)[0]).to(self.device)
                    trailer[pidx] = self.crc_dev[torch.from_numpy(ids[present]).to(self.device)]
                if (~present).any():  # stale directory: send a guaranteed-bad CRC
                    midx = torch.from_numpy(np.nonzero(~present)[0]).to(self.device)
                    trailer[midx] = -1
            sends.append((int(dst), buf))
            sends.append((int(dst), trailer.contiguous()))
        # --- recvs: reserve one contiguous run per source
        recv_entries = []
        trailers = []
        for src in np.unique(recv_rows[:, 5]) if len(recv_rows) else []:
            rows = recv_rows[recv_rows[:, 5] == src]
            keys = np.ascontiguousarray(rows[:, :4])
            lens = np.ascontiguousarray(rows[:, 4])
            res = self.store.reserve_run(keys, lens, self.round)
            if res is None:
                raise RuntimeError("segment cache cannot make room for peer data")
            base, ids, offs = res
            self._grow_crc(int(ids.max()) + 1)
            total = int(offs[-1] + lens[-1] - offs[0])
            recvs.append((int(src), self.arena[int(base):int(base) + total]))
            tr = torch.empty(len(rows), dtype=torch.int32, device=self.device)
            recvs.append((int(src), tr))
            trailers.append(tr)
            for r, eid, o, n in zip(rows, ids, offs, lens):
                row = np.concatenate([r, [eid]])
                recv_entries.append((row, int(o), int(n)))
        ev = None
        t = time.perf_counter()
        if self.is_cuda:
            start = torch.cuda.Event(enable_timing=True)
            end = torch.cuda.Event(enable_timing=True)
            start.record()
        self.comm.exchange(sends, recvs)
        if self.is_cuda:
            end.record()
            ev = (start, end)
        ms = (time.perf_counter() - t) * 1e3
        if self.corrupt_next_recv > 0 and recv_entries:  # fault injection: transport corruption
            self.corrupt_next_recv -= 1
            _, o, n = recv_entries[0]
            if n:
                self.arena[o + n // 2] ^= 0x5A
        expect = torch.cat(trailers) if trailers else None
        if recv_entries:
            ids = torch.from_numpy(np.asarray([r[-1] for r, _, _ in recv_entries], dtype=np.int64)).to(self.device)
            self.crc_dev[ids] = expect
        nbytes = int(recv_rows[:, 4].sum()) if len(recv_rows) else 0
        self.stats["p2p"] += nbytes
        self.stats["p2p_segments"] += len(recv_rows)
        return recv_entries, ms, ev, expect

    # ------------------------------------------------------------------ delivery
    def _deliver(self, completions: List[_Completion]) -> None:
        now_list = [c for c in completions if c.delay <= 0]
        later = [c for c in completions if c.delay > 0]
        if later:  # shaped CDN transfers complete after their modelled duration
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
            self._pinned_last.extend(pin)
        for c in completions:
            req = c.req
            if req.aborted or req.done:
                continue
            req.done = True
            self.stats["segments"] += 1
            if req.agent is not None:
                req.agent._account(c.source, c.nbytes)
            cb = req.callbacks
            get = cb.get if isinstance(cb, dict) else (lambda k, _cb=cb: getattr(_cb, k, None))
            on_progress = get("onProgress")
            if on_progress is not None:
                evt = {"cdnDownloaded": c.nbytes if c.source == "cdn" else 0,
                       "p2pDownloaded": c.nbytes if c.source in ("p2p", "cache") else 0,
                       "cdnDuration": c.cdn_ms if c.source == "cdn" else 0.0,
                       "p2pDuration": c.p2p_ms if c.source == "p2p" else 0.0}
                on_progress(evt)
            if req.aborted:
                continue
            on_success = get("onSuccess")
            if on_success is not None:
                on_success(c.data)

    # ------------------------------------------------------------------ lifecycle
    def set_online(self, online: bool) -> None:
        self.online = bool(online)

    def close(self, timeout_rounds: int = 100000) -> None:
        """Collective shutdown: keep running rounds until every rank is leaving."""
        self.leaving = True
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        if self.world > 1:
            for _ in range(timeout_rounds):
                if self.tick():
                    break
        self.closed = True

    def swarm_offload_ratio(self) -> float:
        c, p = self.swarm_stats["cdn"], self.swarm_stats["p2p"]
        return p / (p + c) if (p + c) else 0.0


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
    ``roundIntervalMs``, ``autoTick``.
    """
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
    else:
        raise ValueError(f"unknown gpuSwarm backend {backend!r}")
    node = SwarmNode(comm, device=cfg.get("device", "auto"), cache_bytes=int(cfg.get("cacheBytes", 1 << 30)),
                     cdn_dedup=bool(cfg.get("cdnDedup", True)), round_interval_ms=cfg.get("roundIntervalMs"),
                     auto_tick=bool(cfg.get("autoTick", True)))
    set_current_node(node)
    return node
