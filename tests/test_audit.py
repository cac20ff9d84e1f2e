"""The node's replicated-state invariants are executable (round-5 VERDICT Weak 6 / Next 4;
SURVEY §5.2): ``HLSP2P_AUDIT=1`` (on in this whole suite, ``tests/conftest.py``) checks them
after every ``launch_round`` / ``complete_round`` (``agent/audit.py``).  Here: the audit passes
on clean and faulty-but-correct runs, and trips within a few rounds when two of round 5's
fixed bugs are put back -- the fleet's early unpin of delivered entries and the node's
``W_ON_DEV`` flag aliasing the want table's "held" bit -- and on a leaked pin, an over-claimed
directory key and a store unpinned more often than pinned."""
import collections
import multiprocessing as mp
import threading
import time

import numpy as np
import pytest
import torch

from hlsjs_p2p_wrapper_amd.agent import node as node_mod
from hlsjs_p2p_wrapper_amd.agent import node_for_config, set_current_node
from hlsjs_p2p_wrapper_amd.agent.audit import AuditError, audit_node
from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub
from hlsjs_p2p_wrapper_amd.parallel.fleet import FleetServer, RemoteNode
from hlsjs_p2p_wrapper_amd.player.transmux import pipeline_for


@pytest.fixture(autouse=True)
def fresh(monkeypatch):
    monkeypatch.setenv("HLSP2P_AUDIT", "1")
    clear_origins()
    set_current_node(None)
    yield
    clear_origins()
    set_current_node(None)


def _origin(n=16, base="http://cdn.audit/vod/"):
    return SyntheticHlsOrigin(base, renditions=[Rendition(1_000_000, 640, 360)], num_segments=n, encrypted=False)


def _two_ranks(rounds, body, corrupt=0):
    """Two ThreadHub ranks, each running ``body(rank, node, step)`` before every round."""
    hub = ThreadHub(2, timeout=60)
    nodes, errs = {}, []

    def rank(r):
        try:
            new_event_loop("virtual")
            node = SwarmNode(hub.comm(r), device="cpu", cache_bytes=64 << 20, auto_tick=False)
            nodes[r] = node
            node.corrupt_next_recv = corrupt
            for step in range(rounds):
                body(r, node, step)
                node.complete_round(node.launch_round())
                node.loop.run_until(lambda: False, timeout_ms=1)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    return nodes, errs


class _Sink:
    def __init__(self):
        self.got = {}

    def deliver(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect=None):
        self.got.update(zip(tok.tolist(), src.tolist()))

    def fail(self, tok, status):
        raise AssertionError("failed requests")


def _requests(origin, sns, tok0=0):
    urls = [origin.base_url + origin.segment_path(0, sn) for sn in sns]
    keys = np.array([[5, 0, 0, sn] for sn in sns], dtype=np.int64)
    return keys, urls, None, np.arange(tok0, tok0 + len(sns), dtype=np.int64)


def test_clean_and_corrupted_swarm_passes_the_audit():
    origin = _origin()
    sinks = {0: _Sink(), 1: _Sink()}

    def body(r, node, step):
        if step == 0:
            node.set_bulk_sink(sinks[r])
            node.request_batch(*_requests(origin, range(8)))
        if step == 3:
            node.request_batch(*_requests(origin, range(8, 16), 100))

    nodes, errs = _two_ranks(10, body, corrupt=2)
    assert not errs, errs
    for r in range(2):
        assert len(sinks[r].got) == 16
        assert nodes[r].audits >= 20  # after every launch and every completion
    assert sum(n.stats["crc_failures"] for n in nodes.values()) >= 1


def test_the_w_on_dev_alias_trips_the_audit(monkeypatch):
    """Round 5's alias: the node's W_ON_DEV was 64, the want table's own "held" bit.  A want
    requeued after a corrupted peer copy then looked device-resident.  On a CPU node the copy
    path never reads the flag, so nothing else notices; the audit does."""
    monkeypatch.setattr(node_mod, "W_ON_DEV", node_mod._rt().WANT_HELD)
    origin = _origin(8)

    def body(r, node, step):
        if step == 0:
            node.set_bulk_sink(_Sink())
            node.request_batch(*_requests(origin, range(8)))

    _, errs = _two_ranks(6, body, corrupt=1)
    assert errs and isinstance(errs[0], AuditError), errs
    assert "W_ON_DEV is set but its origin bytes are in host memory" in str(errs[0])


def _fleet_run(rounds_cap, monkeypatch=None):
    """One CPU rank serving one on-demand fleet player (RemoteNode over a pipe)."""
    loop = new_event_loop("real")
    origin = _origin(24, "http://fleet.audit/vod/")
    node = node_for_config({"gpuSwarm": {"backend": "local", "device": "cpu", "cacheBytes": 64 << 20,
                                         "autoTick": False}})
    a, b = mp.Pipe()
    got, errs = {}, []
    sns = list(range(24))
    stop = threading.Event()

    def player():
        rn = RemoteNode(b)

        class Cb:
            def __init__(self, sn):
                self.sn = sn

            def onProgress(self, ev):  # noqa: N802
                pass

            def onSuccess(self, seg):  # noqa: N802
                got[self.sn] = seg.data() is not None

            def onError(self, err):  # noqa: N802
                errs.append(err)

        for sn in sns:
            rn.request((5, 0, 0, sn), origin.base_url + origin.segment_path(0, sn), None, Cb(sn))
        rn.flush()
        while len(got) + len(errs) < len(sns) and not stop.is_set():
            rn.poll(0.002)
            rn.flush()
        rn.close()

    pipe = pipeline_for(torch.device("cpu"), loop)
    pipe.auto_flush = False
    server = FleetServer(node, pipe, [a])
    t = threading.Thread(target=player, daemon=True)
    t.start()
    try:
        hs, tb = collections.deque(), None
        end = time.monotonic() + 60
        n = 0
        while t.is_alive() and n < rounds_cap:
            assert time.monotonic() < end, f"the player got {len(got)} of {len(sns)}"
            if n % 50 == 49:
                time.sleep(0.002)  # let the player thread run on a loaded machine
            while loop._ready:
                loop.run_once(block=False)
            server.poll()
            server.admit(4)
            hs.append(node.launch_round())
            if len(hs) > 1:
                node.complete_round(hs.popleft())
            nb = server.launch_transmux()
            server.complete_transmux(tb)
            tb = nb
            server.send()
            n += 1
        return node, got, n
    finally:
        stop.set()
        t.join(5)
        server.close()
        node.close()


def test_fleet_run_passes_the_audit():
    node, got, n = _fleet_run(1 << 30)
    assert len(got) == 24 and all(got.values())
    assert node.audits >= 2 * (n - 1)


def test_the_fleet_early_unpin_trips_the_audit(monkeypatch):
    """Round 5's fleet bug: delivered entries lost their pins when the next round launched,
    before the answer batch went out (a small cache then overwrote them before the player read
    them).  Put back -- ``deliver`` no longer pins -- the audit sees entries the server holds
    with fewer pins than its ledger accounts for, at the first completion that delivers."""
    orig = FleetServer.deliver

    def deliver_without_pin(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect=None):
        store = self.node.store
        try:
            self.node.store = _NoPin(store)
            orig(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect)
        finally:
            self.node.store = store

    monkeypatch.setattr(FleetServer, "deliver", deliver_without_pin)
    with pytest.raises(AuditError, match="holds .* pins, its holders account for"):
        _fleet_run(1 << 30)


class _NoPin:
    """The store as round 5's FleetServer.deliver used it: no pin of its own."""

    def __init__(self, store):
        self._s = store

    def pin(self, ids):
        pass

    def __getattr__(self, k):
        return getattr(self._s, k)


def test_a_leaked_pin_and_an_underflow_trip_the_audit():
    node = SwarmNode(device="cpu", cache_bytes=1 << 20, loop=new_event_loop("virtual"), auto_tick=False)
    keys = np.array([[3, 0, 0, 1], [3, 0, 0, 2]], dtype=np.int64)
    _, eids, _ = node.store.reserve_run(keys, np.array([3000, 3000]), 1)
    node.store.commit(eids)
    audit_node(node, "setup")  # consistent
    node.store.pin(eids[:1])  # nobody accounts for it
    with pytest.raises(AuditError, match="pins no holder accounts for"):
        audit_node(node, "leak")
    node.store.unpin(eids[:1])
    node.store.unpin(eids[1:])  # never pinned: an underflow
    with pytest.raises(AuditError, match="unpins of live entries that held no pin"):
        audit_node(node, "underflow")


def test_a_directory_overclaim_trips_the_audit():
    """A key peers believe this rank holds, with no committed local entry behind it, would
    make a peer plan a send this rank cannot look up."""
    hub = ThreadHub(2)
    node = SwarmNode(hub.comm(0), device="cpu", cache_bytes=1 << 20, loop=new_event_loop("virtual"),
                     auto_tick=False)
    audit_node(node, "setup")
    node.directory.apply(0, np.array([[3, 0, 0, 9, 3000]], dtype=np.int64), np.zeros((0, 4), dtype=np.int64))
    with pytest.raises(AuditError, match="peers will believe this rank holds"):
        audit_node(node, "overclaim")
