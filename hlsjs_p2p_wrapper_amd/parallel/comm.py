"""Swarm communication backends (the WebRTC-DataChannel + tracker analog).

Interface used by the swarm node (every method is *collective*: all ranks call it in the
same order, like an RCCL communicator):

* ``allgather_control(msg: np.int64[n]) -> list[np.int64[...]]`` — control plane: the
  per-round wants / cache deltas / flags.  Tiny and latency bound.
* ``exchange(sends, recvs)`` — data plane: ``sends = [(dst, tensor)]``,
  ``recvs = [(src, tensor)]``; per (src, dst) pair the i-th send matches the i-th recv
  (two-sided, ordered — RCCL point-to-point semantics).
* ``allreduce_sum(np.int64[n])`` — swarm-wide counters (stats offload ratio, K8).

Backends:

* :class:`LocalComm`  — world of one.
* :class:`ThreadHub` / :class:`ThreadComm` — N peers as N threads of one process sharing
  queues and a barrier (the CPU "fake swarm" of SURVEY §4.3); tensors may live on the
  CPU or all on one GPU (then a transfer is an HBM->HBM copy).
* :class:`DistComm` — ``torch.distributed``: the control plane runs on the host, never
  on a GPU stream — through the native shared-memory all-gather (``runtime/shm_control``)
  when every rank is on one host (a node of 8 MI355X: the benchmark's case), over a
  **gloo** group otherwise.  Segment bytes move over **RCCL on xGMI** when the default
  group is nccl: by default through the native data plane (``kernels/rccl_comm.cpp``: the
  node's own RCCL communicator, one ``ncclGroupStart / ncclSend* / ncclRecv* /
  ncclGroupEnd`` call per round enqueued on the node stream, one contiguous buffer per peer
  pair), or with ``HLSP2P_NATIVE_RCCL=0`` through torch's ``batch_isend_irecv``; gloo in
  CPU tests.  ``HLSP2P_CONTROL=gloo`` forces the gloo control plane.  With
  ``HLSP2P_DATA_PLANE=ipc`` on a gloo group whose ranks share a host, GPU segment bytes move
  device to device through HIP-IPC outboxes (:class:`_IpcOutbox`): the multi-rank
  rehearsal on one MI355X, where RCCL refuses two ranks per device.
"""
from __future__ import annotations

import atexit
import logging
import os
import secrets
import socket
import threading
from typing import Any, List, Optional, Sequence, Tuple

import numpy as np
import torch

log = logging.getLogger("hlsjs_p2p_wrapper_amd.comm")


RCCL_CU_RESERVE = 64  # CUs the decrypt grid leaves free while the native RCCL plane is live


class SwarmComm:
    rank: int = 0
    world_size: int = 1

    def allgather_control(self, msg: np.ndarray) -> List[np.ndarray]:
        raise NotImplementedError

    def exchange(self, sends: Sequence[Tuple[int, torch.Tensor]], recvs: Sequence[Tuple[int, torch.Tensor]]) -> None:
        raise NotImplementedError

    def allreduce_sum(self, values: np.ndarray) -> np.ndarray:
        parts = self.allgather_control(np.asarray(values, dtype=np.int64))
        return np.sum(np.stack(parts), axis=0)

    def barrier(self) -> None:
        self.allgather_control(np.zeros(1, dtype=np.int64))

    def close(self) -> None:
        pass

    def abort(self) -> None:
        """Error path: stop the data plane without waiting on peers (no-op by default)."""


class LocalComm(SwarmComm):
    def __init__(self) -> None:
        self.rank = 0
        self.world_size = 1

    def allgather_control(self, msg: np.ndarray) -> List[np.ndarray]:
        return [np.asarray(msg, dtype=np.int64).copy()]

    def exchange(self, sends, recvs) -> None:
        if sends or recvs:
            raise RuntimeError("LocalComm has no peers")


class ThreadHub:
    """Shared state of an in-process swarm of ``world_size`` peer threads."""

    def __init__(self, world_size: int, timeout: float = 120.0) -> None:
        self.world_size = world_size
        self.timeout = timeout
        self._barrier = threading.Barrier(world_size)
        self._slots: List[Optional[np.ndarray]] = [None] * world_size
        self._mail: dict = {}
        self._lock = threading.Lock()

    def comm(self, rank: int) -> "ThreadComm":
        return ThreadComm(self, rank)

    def wait(self) -> None:
        self._barrier.wait(self.timeout)

    def abort(self) -> None:
        self._barrier.abort()


class ThreadComm(SwarmComm):
    def __init__(self, hub: ThreadHub, rank: int) -> None:
        self.hub = hub
        self.rank = rank
        self.world_size = hub.world_size

    def allgather_control(self, msg: np.ndarray) -> List[np.ndarray]:
        hub = self.hub
        hub._slots[self.rank] = np.asarray(msg, dtype=np.int64).copy()
        hub.wait()
        out = [s.copy() for s in hub._slots]  # type: ignore[union-attr]
        hub.wait()
        return out

    def exchange(self, sends, recvs) -> None:
        hub = self.hub
        with hub._lock:
            for dst, t in sends:
                hub._mail.setdefault((self.rank, dst), []).append(t)
        hub.wait()
        per_src: dict = {}
        for src, t in recvs:
            q = hub._mail.get((src, self.rank), [])
            i = per_src.get(src, 0)
            if i >= len(q):
                raise RuntimeError(f"rank {self.rank}: no matching send from {src}")
            s = q[i]
            per_src[src] = i + 1
            if s.numel() != t.numel():
                raise RuntimeError(f"rank {self.rank}: size mismatch from {src}: {s.numel()} != {t.numel()}")
            t.copy_(s.to(t.device), non_blocking=False)
        hub.wait()
        with hub._lock:
            for src in range(self.world_size):
                hub._mail.pop((src, self.rank), None)
        hub.wait()


class DistComm(SwarmComm):
    """torch.distributed backend: gloo control group + default (RCCL/gloo) data group."""

    def __init__(self, control_group=None, data_group=None) -> None:
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("torch.distributed is not initialized")
        self.dist = dist
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        backend = dist.get_backend(data_group)
        plane = os.environ.get("HLSP2P_DATA_PLANE", "")
        if control_group is None:
            control_group = dist.new_group(backend="gloo") if backend != "gloo" else None
        self.control_group = control_group
        self.data_group = data_group
        self.data_backend = backend
        self._cap = 64  # int64 words per rank in the one-shot control all-gather
        # a control all-gather waits this long for every peer before raising (gpuSwarm.
        # controlTimeoutMs; HLSP2P_CONTROL_TIMEOUT seconds): long enough for a cold box's start-up
        # skew, short enough that a dead peer fails the job instead of hanging it
        self.control_timeout_s = float(os.environ.get("HLSP2P_CONTROL_TIMEOUT", str(self.CONTROL_TIMEOUT_S)))
        # shared-memory slot per rank and round: a message larger than it makes every rank
        # take the gloo all-gather for that round (~3.4 ms at 8 ranks instead of ~10 us):
        # counted, and warned about once, never silent (bench.py sizes the slot)
        self.shm_slot_words = max(1024, int(os.environ.get("HLSP2P_SHM_SLOT_WORDS", str(self.SHM_SLOT_WORDS))))
        self.control_fallbacks = 0
        self._shm = self._open_shm_control() if self.world_size > 1 else None
        self.control_transport = "shm" if self._shm is not None else "gloo"
        self._rccl = None
        self.rehearsal = None
        self.rccl_log: Optional[str] = None  # RCCL's connection log of this rank (parallel/wire.py)
        self.peer_devices: dict = {}  # rank -> (host id, PCI bus id, device index), native RCCL plane
        self._ipc: Optional[_IpcOutbox] = None
        if backend == "gloo" and plane == "ipc" and self.world_size > 1 and torch.cuda.is_available():
            self._ipc = _IpcOutbox.open(self)
        # RCCL data plane: on a gloo default group with HLSP2P_DATA_PLANE=rccl (bench.py's GPU
        # launch: the node's native communicator is then the ONLY RCCL communicator of the
        # rank -- no idle torch one doubling channel buffers and proxy threads), or on an nccl
        # default group (torch's communicator exists anyway: the fallback transport)
        want_rccl = (backend == "nccl" or plane == "rccl") and torch.cuda.is_available()
        if want_rccl and os.environ.get("HLSP2P_NATIVE_RCCL", "1") != "0":
            self._rccl = self._open_native_rccl()
        if want_rccl and self._rccl is None:
            if backend != "nccl":  # torch's batch_isend_irecv needs an nccl group (collective)
                self.data_group = dist.new_group(backend="nccl")
                self.data_backend = "nccl"
            # batch_isend_irecv runs on the group's full communicator; when that is created
            # lazily every rank must take part in its first use.  Node construction is
            # collective, so create it here rather than at the first (partial) exchange.
            t = torch.zeros(1, dtype=torch.int64, device=torch.device("cuda", torch.cuda.current_device()))
            dist.all_reduce(t, group=self.data_group)
            torch.cuda.synchronize()
        if self._rccl is not None and torch.cuda.is_available():
            # the persistent decrypt grid leaves CUs to the node stream's RCCL kernels: 64 (8 per
            # XCD) measured best for the bench's lag-2 pipeline of a 7-peer round beside the
            # transmux batches (1,330 us a step against 1,409 at 8; the round completes 2.5x
            # sooner; profiles/r5_overlap)
            try:
                from ..ops._native import device as _dev

                _dev().set_cu_reserve(int(os.environ.get("HLSP2P_RCCL_CU_RESERVE", str(RCCL_CU_RESERVE))))
            except Exception:  # noqa: BLE001 - older extension without the knob: full grid
                pass
        self.data_transport = ("rccl-native" if self._rccl is not None else
                               "rccl-torch" if self.data_backend == "nccl" else
                               "hip-ipc" if self._ipc is not None else backend)

    def _open_native_rccl(self):
        """The node's own RCCL communicator (collective).  Every rank first reports whether
        the native module and RCCL are usable; only if all are does any rank enter
        ``ncclCommInitRank`` (a rank that cannot join would leave the others blocked in it).
        Otherwise every rank stays on torch's ``batch_isend_irecv``.

        ``HLSP2P_RCCL_REHEARSAL=socket``: ranks that share one GPU still get the real native
        RCCL plane -- each rank presents RCCL a host id of its own (``NCCL_HOSTID``), so RCCL
        sees N "hosts" and connects them over its socket transport on the loopback instead
        of refusing duplicate devices.  Everything above the wire (one group call per round,
        send / recv matching, the pointer columns, async-error polling) is the production
        path; only the transport differs from xGMI.  For one-GPU rehearsals only."""
        dist, g = self.dist, self.control_group
        dev = None
        ok = True
        uid: List[object] = [None]
        gpu = None
        self.rehearsal = os.environ.get("HLSP2P_RCCL_REHEARSAL") or None
        if self.rehearsal is not None and self.data_backend != "gloo":
            # the rehearsal's per-rank host id must reach RCCL before its first call; an nccl
            # default group may have initialised RCCL (and hashed the real host id) already.
            # The default group's backend is the same on every rank: all raise here together
            raise RuntimeError("HLSP2P_RCCL_REHEARSAL needs a gloo default group with HLSP2P_DATA_PLANE=rccl "
                               "(bench.py's GPU launch), not an nccl one")
        if self.rehearsal == "socket":  # before any RCCL call: the host hash is computed once
            os.environ["NCCL_HOSTID"] = f"hlsp2p-rehearsal-{os.getpid()}-{self.rank}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")
        elif self.rehearsal is not None:
            raise ValueError(f"unknown HLSP2P_RCCL_REHEARSAL {self.rehearsal!r} (expected 'socket')")
        # RCCL's per-peer connection log (which wire each pair runs on: parallel/wire.py), set
        # before the process's first RCCL call, which reads the debug variables once
        from .wire import configure_rccl_log

        self.rccl_log = configure_rccl_log(self.rank)
        dev_index = torch.cuda.current_device()
        try:
            from ..ops._native import device as _dev

            dev = _dev()
            dev.rccl_version()
            gpu = dev.pci_bus_id(dev_index)
            if self.rank == 0:  # a failure here is reported through the all-gather below
                uid[0] = dev.rccl_unique_id()
        except Exception:  # noqa: BLE001 - no native module / RCCL: torch's path
            ok = False
        flags: List[object] = [None] * self.world_size
        dist.all_gather_object(flags, (ok, _host_id(), gpu, self.rehearsal, dev_index), group=g)
        if not all(f[0] for f in flags):  # type: ignore[index]
            return None
        # every rank must agree on the rehearsal mode: a rank that skips the duplicate-device
        # check below while another raises would leave the others blocked in the next collective
        modes = [f[3] for f in flags]  # type: ignore[index]
        if len(set(modes)) > 1:
            raise RuntimeError(f"ranks disagree on HLSP2P_RCCL_REHEARSAL: {modes}")
        self.peer_devices = {r: (f[1], f[2], f[4]) for r, f in enumerate(flags)}  # type: ignore[index]
        # one GPU per rank: RCCL cannot place two ranks of a communicator on one device (it
        # fails deep inside ncclCommInitRank, or worse, a launcher mapped ranks onto a shared
        # card silently); every rank sees the same table, so every rank raises here together
        seen: dict = {}
        for r, (_, host, bus, _, _) in enumerate(flags):  # type: ignore[misc]
            if (host, bus) in seen and self.rehearsal is None:
                raise RuntimeError(f"RCCL data plane: ranks {seen[(host, bus)]} and {r} would share GPU {bus} on "
                                   f"host {host[0]}; RCCL needs one GPU per rank (rehearse ranks that share a "
                                   "GPU with --dist-backend ipc or gloo)")
            seen[(host, bus)] = r
        dist.broadcast_object_list(uid, src=0, group=g)
        comm, err = None, ""
        try:
            comm = dev.RcclComm(uid[0], self.world_size, self.rank, torch.cuda.current_device())
        except Exception as e:  # noqa: BLE001 - agreed on below: nobody keeps a half-built group
            err = f"{type(e).__name__}: {e}"
        dist.all_gather_object(flags, err, group=g)  # second agreement: every rank joined
        if any(flags):
            if comm is not None:
                comm.abort()
            raise RuntimeError(f"native RCCL communicator init failed on some rank: {flags}")
        atexit.register(comm.abort)  # no-op once closed
        return comm

    SHM_SLOT_WORDS = 16384  # int64 words per rank and round (128 KiB); larger -> gloo
    CONTROL_TIMEOUT_S = 300.0  # library default of the control all-gather's deadline

    def _open_shm_control(self):
        """Shared-memory control plane when every rank runs on this host (collective).

        Rank 0 creates the mapping under a random name, the others attach, and rank 0
        unlinks the name once all are attached (nothing is left in /dev/shm, even after a
        crash).  Any failure on any rank -> every rank stays on gloo."""
        if os.environ.get("HLSP2P_CONTROL", "auto") == "gloo":
            return None
        dist, g = self.dist, self.control_group
        hosts: List[object] = [None] * self.world_size
        dist.all_gather_object(hosts, _host_id(), group=g)
        if any(h != hosts[0] for h in hosts):
            return None
        from ..ops._native import runtime as _rt

        rt = _rt()
        name = [f"/hlsp2p_{os.getpid()}_{secrets.token_hex(6)}" if self.rank == 0 else None]
        dist.broadcast_object_list(name, src=0, group=g)
        shm, ok = None, True
        if self.rank == 0:
            try:
                shm = rt.ShmControl(name[0], 0, self.world_size, self.shm_slot_words, True)
            except Exception:  # noqa: BLE001 - any failure: stay on gloo
                ok = False
        flags: List[object] = [None] * self.world_size
        dist.all_gather_object(flags, ok, group=g)
        if self.rank != 0 and all(flags):
            try:
                shm = rt.ShmControl(name[0], self.rank, self.world_size, self.shm_slot_words, False)
            except Exception:  # noqa: BLE001
                ok = False
        dist.all_gather_object(flags, ok, group=g)
        if shm is not None and self.rank == 0:
            shm.unlink()
        return shm if all(flags) else None

    def allgather_control(self, msg: np.ndarray) -> List[np.ndarray]:
        if self._shm is not None:
            out = self._shm.allgather(np.ascontiguousarray(msg, dtype=np.int64).reshape(-1), self.control_timeout_s)
            if out is not None:
                return out
            # some rank's message exceeded a slot: every rank saw that and falls back here
            self.control_fallbacks += 1
            if self.control_fallbacks == 1:
                log.warning("rank %d: a control message exceeded the %d-word shared-memory slot; this round's "
                            "all-gather fell back to gloo (raise HLSP2P_SHM_SLOT_WORDS; counted in "
                            "control_fallbacks)", self.rank, self.shm_slot_words)
        return self._allgather_gloo(msg)

    def _allgather_gloo(self, msg: np.ndarray) -> List[np.ndarray]:
        """Variable-length all-gather in ONE collective on the common path: each rank sends
        ``[len, payload...]`` padded to a shared capacity.  Only when some rank's message
        exceeds it does a second all-gather move the full padded messages; the capacity
        then grows so the following rounds fit again."""
        dist = self.dist
        msg = np.asarray(msg, dtype=np.int64).reshape(-1)
        cap = self._cap
        buf = torch.zeros(cap + 1, dtype=torch.int64)
        buf[0] = msg.size
        k = min(msg.size, cap)
        buf[1:1 + k] = torch.from_numpy(msg[:k])
        outs = [torch.empty(cap + 1, dtype=torch.int64) for _ in range(self.world_size)]
        dist.all_gather(outs, buf, group=self.control_group)
        sizes = [int(o[0]) for o in outs]
        mx = max(sizes)
        if mx <= cap:
            return [o[1:1 + n].numpy().copy() for o, n in zip(outs, sizes)]
        full = torch.zeros(mx, dtype=torch.int64)
        full[:msg.size] = torch.from_numpy(msg)
        outs = [torch.empty(mx, dtype=torch.int64) for _ in range(self.world_size)]
        dist.all_gather(outs, full, group=self.control_group)
        self._cap = max(cap, int(mx * 1.5) + 16)
        return [o[:n].numpy().copy() for o, n in zip(outs, sizes)]

    def exchange(self, sends, recvs) -> None:
        dist = self.dist
        if self._rccl is not None:
            self._exchange_native(sends, recvs)
            return
        if self._ipc is not None:
            self._ipc.exchange(sends, recvs)
            return
        if self.data_backend == "gloo" and any(t.is_cuda for _, t in list(sends) + list(recvs)):
            self._exchange_staged(sends, recvs)
            return
        ops = []
        for dst, t in sends:
            ops.append(dist.P2POp(dist.isend, t, dst, group=self.data_group))
        for src, t in recvs:
            ops.append(dist.P2POp(dist.irecv, t, src, group=self.data_group))
        if not ops:
            return
        reqs = dist.batch_isend_irecv(ops)
        for r in reqs:
            r.wait()

    @property
    def exchange_spans(self):
        """Pointer-column form of :meth:`exchange` for the native RCCL plane (None on the
        other planes): ``(send_ptr, send_bytes, send_peer, recv_ptr, recv_bytes, recv_peer)``
        int64 columns, one RCCL group call on the current stream.  The caller keeps the
        buffers alive and stream-ordered, as for :meth:`exchange`."""
        if self._rccl is None:
            return None
        return self._exchange_spans

    def _exchange_spans(self, sp, sb, sd, rp, rb, rs) -> None:
        if len(sp) or len(rp):
            self._rccl.exchange(sp, sb, sd, rp, rb, rs, torch.cuda.current_stream().cuda_stream)

    def _exchange_native(self, sends, recvs) -> None:
        """One RCCL group call on the current stream (the swarm node's stream)."""
        if not sends and not recvs:
            return
        ns, nr = len(sends), len(recvs)
        ptr = np.empty(ns + nr, dtype=np.int64)
        nbytes = np.empty(ns + nr, dtype=np.int64)
        peer = np.empty(ns + nr, dtype=np.int64)
        for i, (p, t) in enumerate(list(sends) + list(recvs)):
            if not (t.is_cuda and t.is_contiguous()):
                raise ValueError("native RCCL exchange needs contiguous GPU tensors")
            ptr[i] = t.data_ptr()
            nbytes[i] = t.numel() * t.element_size()
            peer[i] = p
        stream = torch.cuda.current_stream().cuda_stream
        self._rccl.exchange(ptr[:ns], nbytes[:ns], peer[:ns], ptr[ns:], nbytes[ns:], peer[ns:], stream)

    def async_error(self) -> str:
        """The data plane's asynchronous error ("" = none): RCCL reports a failed peer here
        while the transfers waiting on it never complete (the node polls this instead of
        blocking on a round that cannot finish)."""
        if self._rccl is not None:
            return self._rccl.async_error()
        return ""

    def close(self) -> None:
        """Release the native RCCL communicator.  Callers close after their last round has
        completed on the device, so this aborts (returns without waiting on peers) rather
        than runs ncclCommDestroy's finalize, which a rank that already left could hang."""
        if self._rccl is not None:
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            self._rccl.abort()
        if self._ipc is not None:
            self._ipc.close()

    def abort(self) -> None:
        """Error path (e.g. replicated state diverged): abort the native RCCL communicator
        without synchronising the device -- transfers already posted may never be matched, so
        waiting for them would hang; ``ncclCommAbort`` returns regardless.  The IPC rehearsal
        plane's buffers stay mapped until the process exits (peers may still be copying)."""
        if self._rccl is not None:
            self._rccl.abort()

    def topology(self) -> dict:
        """What the data plane reports about itself: for the native RCCL communicator, the
        rank count and rank RCCL holds (``ncclCommCount`` / ``ncclCommUserRank``), the HIP
        device it runs on (``ncclCommCuDevice``), the rounds posted and the RCCL version."""
        out = {"transport": self.data_transport, "world": self.world_size, "rank": self.rank}
        if getattr(self, "rehearsal", None):
            out["rehearsal"] = self.rehearsal  # RCCL's socket transport between ranks sharing a GPU
        if self._rccl is not None and not self._rccl.closed:
            from ..ops._native import device as _dev

            out["rccl"] = {"count": int(self._rccl.comm_count()), "rank": int(self._rccl.comm_user_rank()),
                           "device": int(self._rccl.comm_device()), "rounds": int(self._rccl.rounds),
                           "version": _dev().rccl_version()}
            out["wire"] = self.wire()
        if self._ipc is not None:
            out["ipc_exchanges"] = int(self._ipc.exchanges)
        return out

    def wire(self) -> dict:
        """Which wire this rank's RCCL connections run on (parallel/wire.py): RCCL's own
        per-peer transport from its connection log, its view of the group (ranks / nodes /
        local ranks), and HIP's link type to each peer's device on this host.  Read after the
        exchanges ran: RCCL connects a pair at its first send / receive."""
        from .wire import link_types, read_rccl_log, summarize

        rep = read_rccl_log(self.rccl_log, self.rank)
        out: dict = {"transport": summarize(rep, self.world_size)}
        if rep is not None:
            out.update(peers=rep["peers"], n_ranks=rep["n_ranks"], n_nodes=rep["n_nodes"],
                       local_ranks=rep["local_ranks"], connections=rep["connections"], log_bytes=rep["log_bytes"])
        else:
            out["peers"] = None
        me = self.peer_devices.get(self.rank)
        if me is not None:
            same_host = {r: d[2] for r, d in self.peer_devices.items() if r != self.rank and d[0] == me[0]}
            try:
                out["links"] = link_types(me[2], same_host) if same_host else {}
            except Exception as e:  # noqa: BLE001 - diagnostic only
                out["links"] = f"error: {e}"
        return out

    def _exchange_staged(self, sends, recvs) -> None:
        """gloo data plane with GPU tensors (several ranks sharing one GPU, e.g. rehearsing
        the multi-rank path on a single MI355X): stage through host memory.  Synchronous
        and slow by design; production multi-GPU runs use RCCL."""
        dist = self.dist
        torch.cuda.current_stream().synchronize()  # payloads/trailers are produced on this stream
        ops, staged = [], []
        for dst, t in sends:
            ops.append(dist.P2POp(dist.isend, t.detach().to("cpu"), dst, group=self.data_group))
        for src, t in recvs:
            h = torch.empty(t.numel(), dtype=t.dtype)
            staged.append((t, h))
            ops.append(dist.P2POp(dist.irecv, h, src, group=self.data_group))
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        for t, h in staged:
            t.view(-1).copy_(h, non_blocking=False)

    def allreduce_sum(self, values: np.ndarray) -> np.ndarray:
        if self._shm is not None:
            return SwarmComm.allreduce_sum(self, values)
        t = torch.from_numpy(np.asarray(values, dtype=np.int64).copy())
        self.dist.all_reduce(t, group=self.control_group)
        return t.numpy()

    def barrier(self) -> None:
        if self._shm is not None:
            self._shm.barrier(self.control_timeout_s)
            return
        self.dist.barrier(group=self.control_group)


def _host_id() -> Tuple[str, str]:
    """``(hostname, boot id)``: ranks with equal ids share a host (and its /dev/shm)."""
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            boot = f.read().strip()
    except OSError:
        boot = ""
    return socket.gethostname(), boot


def _as_bytes(t: torch.Tensor) -> torch.Tensor:
    """A contiguous tensor's bytes as a flat uint8 view (no copy)."""
    if not t.is_contiguous():
        raise ValueError("IPC data plane needs contiguous tensors")
    return t.reshape(-1).view(torch.uint8)


def _outbox_slots(table: np.ndarray, me: int, align: int) -> List[Tuple[int, int]]:
    """``(offset, nbytes)`` in a peer's outbox of each of its sends to rank ``me``, in send
    order, from its table ``[outbox bytes, n, (dst, nbytes) * n]`` (sends are packed in
    order at ``align``-byte boundaries)."""
    k = int(table[1])
    out, o = [], 0
    for d, n in zip(table[2:2 + 2 * k:2].tolist(), table[3:3 + 2 * k:2].tolist()):
        if d == me:
            out.append((o, n))
        o += (n + align - 1) // align * align
    return out


class _IpcOutbox:
    """Device-resident data plane for ranks that share one host but no RCCL communicator.

    This is the multi-rank rehearsal on a single MI355X: RCCL refuses two ranks on one
    device, and the gloo data plane stages every byte through host memory.  Here each rank
    packs its sends into an HBM "outbox" that is exported once over HIP IPC (dmabuf).  Peers
    copy their receives straight out of it, device to device, on their node stream, so the
    rest of the round stays stream-ordered exactly as with RCCL.

    Protocol, per exchange (collective, like an RCCL group):

    1. Wait for this rank's receive copies of the previous exchange.  After that, no peer
       can still be reading an outbox that is about to be rewritten.
    2. All-gather the send tables ``[outbox bytes, n, (dst, nbytes) * n]`` (a round larger
       than the fixed outbox fails on every rank).
    3. Pack the sends into the outbox (256-byte aligned, in order) on the node stream, wait
       for the packing copies on the host, then barrier.
    4. For the k-th receive from ``src``, copy the k-th of ``src``'s sends addressed to this
       rank (two-sided, ordered, as RCCL point-to-point) on the node stream.  An event
       recorded after the copies serves step 1.

    Interprocess events recorded after packing replace the host wait of step 3 (the default;
    ``HLSP2P_IPC_EVENTS=0`` restores the wait: the event mode measured +15 % on the 4-rank
    soak).  Peers' node streams wait on them before copying, so the host
    never waits, as with an RCCL group.  A peer's event is re-recorded only in a later
    exchange, after the all-gather of step 2, which this rank joins only once its copies
    (and the wait before them) have run.

    Event lifetime (root cause of the round-2 soak failure, ``tools/ipc_event_probe.py``,
    ``profiles/r3_ipc_events``): on ROCm 7.2 an interprocess event survives exactly 32
    records — the peer's ``hipStreamWaitEvent`` after the 33rd fails with ``invalid
    argument``, whatever the rank count, record density or handle re-opening.  So each rank
    cycles a ring of ``EVENT_RING`` events (exchange ``x`` uses slot ``x % EVENT_RING``) and
    the whole set is re-created and re-shared (a collective at the same exchange number on
    every rank) before any event reaches ``EVENT_RECORDS`` records; the previous set stays
    alive for one generation, as waits queued on the streams may still reference it.

    Enabled with ``HLSP2P_DATA_PLANE=ipc`` on a gloo group (``bench.py --dist-backend
    ipc``).  Every rank must be on the same host; otherwise every rank keeps gloo."""

    ALIGN = 256
    EVENT_RING = 8       # interprocess events per rank, used round-robin
    EVENT_RECORDS = 30   # records per event before the set is renewed (the runtime allows 32)

    def __init__(self, comm: "DistComm") -> None:
        self.comm = comm
        self.cap = 0
        self.buf: Optional[torch.Tensor] = None
        self.peers: List[torch.Tensor] = []
        self._pending = None
        self._ev: Optional[List[Any]] = None  # this rank's event ring: recorded after packing
        self._peer_ev: Optional[List[List[Any]]] = None  # every rank's ring (None: host-side waits)
        self._ev_prev = None  # the previous generation, alive until the next renewal
        self._ev_gen_start = 0
        self.exchanges = 0

    @classmethod
    def open(cls, comm: "DistComm") -> Optional["_IpcOutbox"]:
        dist, g = comm.dist, comm.control_group
        hosts: List[object] = [None] * comm.world_size
        dist.all_gather_object(hosts, _host_id(), group=g)
        if any(h != hosts[0] for h in hosts):
            return None
        box = cls(comm)
        return box if box._share(int(os.environ.get("HLSP2P_IPC_OUTBOX_BYTES", str(1 << 30)))) else None

    def _share(self, cap: int) -> bool:
        """Collective, once: allocate this rank's outbox and open every peer's.  Each local
        step that can fail sits between two all-gathers that report success, so a rank
        that fails never leaves the others blocked in a collective: either every rank ends
        up with every outbox, or every rank returns False (and keeps gloo).

        The capacity is fixed for the communicator's life.  Re-exporting a fresh allocation
        while peers still mapped the old one proved unreliable (CRC failures: a peer kept
        reading through its mapping of the old handle), so a round that needs more fails
        loudly instead (``HLSP2P_IPC_OUTBOX_BYTES``; ``bench.py`` sizes it from the
        workload)."""
        from torch.multiprocessing.reductions import reduce_tensor

        comm = self.comm
        dist, g, me = comm.dist, comm.control_group, comm.rank
        cap = (max(cap, 1 << 20) + (1 << 20) - 1) // (1 << 20) * (1 << 20)
        handle = None
        try:
            self.buf = torch.empty(cap, dtype=torch.uint8, device=torch.device("cuda", torch.cuda.current_device()))
            torch.cuda.synchronize()
            handle = reduce_tensor(self.buf)
        except Exception:  # noqa: BLE001 - reported to every rank below
            handle = None
        handles: List[object] = [None] * comm.world_size
        dist.all_gather_object(handles, handle, group=g)
        ok = all(h is not None for h in handles)
        if ok:
            try:
                self.peers = [self.buf if r == me else h[0](*h[1])  # type: ignore[index]
                              for r, h in enumerate(handles)]
            except Exception:  # noqa: BLE001
                ok = False
        flags: List[object] = [None] * comm.world_size
        dist.all_gather_object(flags, ok, group=g)  # also: every rank holds every outbox
        if not all(flags):
            self.peers, self.buf = [], None
            return False
        self.cap = cap
        if os.environ.get("HLSP2P_IPC_EVENTS", "1") == "1":  # default since the event-ring fix (+15 %)
            self._share_events()
        return True

    def _share_events(self) -> None:
        """Collective: export a fresh ring of interprocess events per rank (optional: on any
        failure every rank packs with a host-side wait instead).  Called once at set-up and
        again every ``EVENT_RING * EVENT_RECORDS`` exchanges (see the class notes)."""
        comm = self.comm
        dist, g, me = comm.dist, comm.control_group, comm.rank
        dev = torch.cuda.current_device()
        self._ev_prev = (self._ev, self._peer_ev)
        handle = None
        own: Optional[List[Any]] = None
        try:
            own = [torch.cuda.Event(enable_timing=False, interprocess=True) for _ in range(self.EVENT_RING)]
            for e in own:
                e.record()
            torch.cuda.synchronize()
            handle = [e.ipc_handle() for e in own]
        except Exception:  # noqa: BLE001 - reported to every rank below
            handle = None
        handles: List[object] = [None] * comm.world_size
        dist.all_gather_object(handles, handle, group=g)
        evs: Optional[List[List[Any]]] = None
        if all(h is not None for h in handles):
            try:
                opened = torch.cuda.Event.from_ipc_handle
                evs = [own if r == me else [opened(dev, x) for x in h]  # type: ignore[union-attr]
                       for r, h in enumerate(handles)]
            except Exception:  # noqa: BLE001
                evs = None
        flags: List[object] = [None] * comm.world_size
        dist.all_gather_object(flags, evs is not None, group=g)
        if all(flags):
            self._ev, self._peer_ev = own, evs
        else:
            self._ev, self._peer_ev = None, None
        self._ev_gen_start = self.exchanges

    def exchange(self, sends, recvs) -> None:
        comm = self.comm
        if self._pending is not None:
            self._pending.synchronize()
            self._pending = None
        A = self.ALIGN
        sizes = [int(t.numel()) * t.element_size() for _, t in sends]
        offs, pos = [], 0
        for n in sizes:
            offs.append(pos)
            pos += (n + A - 1) // A * A
        msg = np.empty(2 + 2 * len(sends), dtype=np.int64)
        msg[0], msg[1] = pos, len(sends)
        msg[2::2] = [d for d, _ in sends]
        msg[3::2] = sizes
        parts = comm.allgather_control(msg)
        need = max(int(p[0]) for p in parts)
        if need > self.cap:  # every rank sees the same tables: all raise together
            raise RuntimeError(f"IPC outbox of {self.cap} bytes cannot hold a round of {need} bytes "
                               "(raise HLSP2P_IPC_OUTBOX_BYTES)")
        stream = torch.cuda.current_stream()
        if self._peer_ev is not None and self.exchanges - self._ev_gen_start >= self.EVENT_RING * self.EVENT_RECORDS:
            self._share_events()  # collective at the same exchange number on every rank
        slot = self.exchanges % self.EVENT_RING
        if sends:
            buf = self.buf
            for (_, t), o, n in zip(sends, offs, sizes):
                if n:
                    buf[o:o + n].copy_(_as_bytes(t), non_blocking=True)
            if self._peer_ev is not None:
                self._ev[slot].record(stream)  # type: ignore[index]
            else:
                stream.synchronize()
        comm.barrier()  # every outbox's packing is enqueued (or done) and its event recorded
        peer_ev = self._peer_ev
        me = comm.rank
        mine: dict = {}  # src -> [(offset, nbytes)] of src's sends to this rank, in order
        cursor: dict = {}
        for src, t in recvs:
            lst = mine.get(src)
            if lst is None:
                lst = mine[src] = _outbox_slots(parts[src], me, A)
                if peer_ev is not None and lst:
                    stream.wait_event(peer_ev[src][slot])  # src's packing has run
            i = cursor.get(src, 0)
            if i >= len(lst):
                raise RuntimeError(f"rank {me}: no matching send from {src}")
            cursor[src] = i + 1
            o, n = lst[i]
            dst = _as_bytes(t)
            if dst.numel() != n:
                raise RuntimeError(f"rank {me}: size mismatch from {src}: {n} != {dst.numel()}")
            if n:
                dst.copy_(self.peers[src][o:o + n], non_blocking=True)
        if recvs:
            ev = torch.cuda.Event()
            ev.record(stream)
            self._pending = ev
        self.exchanges += 1

    def close(self) -> None:
        if self._pending is not None:
            self._pending.synchronize()
            self._pending = None
        self.peers = []
        self.buf = None
