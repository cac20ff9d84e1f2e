"""Cross-rank consistency of the replicated swarm state (SURVEY §5.2 state-machine
assertions).

Every rank replays the same control messages into its own ``Directory`` and plans each
round on its own; a two-sided data plane (RCCL send / recv) then needs every rank's plan to
match.  The directory digest (incremental, order independent) and the previous round's
full-plan digest ride every control message; ``ingest_control`` compares them before
applying anything, so a divergence stops every rank with a diagnostic within one round
instead of hanging in a send / recv group nobody matches."""
import threading
import time

import numpy as np
import pytest

from hlsjs_p2p_wrapper_amd.agent.node import RoundHandle, SwarmNode
from hlsjs_p2p_wrapper_amd.net import new_event_loop
from hlsjs_p2p_wrapper_amd.ops._native import runtime
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub

rt = runtime()


def _adds(keys, length=1000):
    return np.array([[*k, length] for k in keys], dtype=np.int64).reshape(-1, 5)


def _rms(keys):
    return np.array(keys, dtype=np.int64).reshape(-1, 4)


def test_directory_digest_is_order_independent_and_exact():
    keys = [(7, 0, 0, sn) for sn in range(40)]
    a, b = rt.Directory(), rt.Directory()
    assert a.digest == b.digest == 0
    a.apply(0, _adds(keys), _rms([]))
    a.apply(1, _adds(keys[::2]), _rms([]))
    b.apply(1, _adds(keys[::2][::-1]), _rms([]))  # other rank order, other key order
    b.apply(0, _adds(keys[::-1]), _rms([]))
    assert a.digest == b.digest != 0
    b.apply(1, _adds(keys[:1]), _rms([]))  # re-adding a held key changes nothing
    assert a.digest == b.digest
    b.apply(1, _adds([keys[1]]), _rms([]))  # a new holder does
    assert a.digest != b.digest
    b.apply(1, _adds([]), _rms([keys[1]]))
    assert a.digest == b.digest
    c = rt.Directory()
    c.apply(0, _adds(keys, length=999), _rms([]))  # lengths are part of the content
    c.apply(1, _adds(keys[::2], length=999), _rms([]))
    assert c.digest != a.digest
    a.apply(0, _adds([]), _rms(keys))
    a.apply(1, _adds([]), _rms(keys[::2]))
    assert a.digest == 0 and a.size == 0
    # drop_rank recomputes the digest from the content: equal to the incremental one
    d, e = rt.Directory(), rt.Directory()
    d.apply(0, _adds(keys), _rms([]))
    d.apply(2, _adds(keys[5:9]), _rms([]))
    e.apply(0, _adds(keys), _rms([]))
    e.apply(2, _adds(keys[5:9]), _rms([]))
    e.apply(3, _adds(keys[:20]), _rms([]))
    e.drop_rank(3)
    assert e.digest == d.digest
    # growth (rehash) keeps it
    f = rt.Directory()
    big = [(9, 1, 0, sn) for sn in range(5000)]
    f.apply(0, _adds(big), _rms([]))
    g = rt.Directory()
    for k in big[::-1]:
        g.apply(0, _adds([k]), _rms([]))
    assert f.digest == g.digest


def test_plan_digest_is_the_full_plan_on_every_rank():
    d = rt.Directory()
    d.apply(1, _adds([(7, 0, 0, sn) for sn in range(8)]), _rms([]))
    wants = np.array([[7, 0, 0, sn, 1000, 100 + sn, r, 0] for r in (0, 2) for sn in range(12)], dtype=np.int64)
    flags = np.full(3, rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD | rt.FLAG_CDN_DEDUP, dtype=np.int64)
    digests = set()
    for me in range(3):
        rows, any_p2p, dig = rt.plan_round_for(d, wants, flags, 3, me)
        assert any_p2p
        digests.add(dig)
    assert len(digests) == 1  # the filtered rows differ per rank; the digest covers the full plan
    other = rt.plan_round_for(d, wants[:-1], flags, 3, 0)[2]
    assert other not in digests


def _two_ranks(fn, timeout=30):
    """Run ``fn(rank, node)`` on 2 in-process ranks (ThreadHub); collect exceptions."""
    hub = ThreadHub(2, timeout=timeout)
    errs, nodes = {}, {}

    def rank(r):
        try:
            new_event_loop("virtual")
            node = SwarmNode(hub.comm(r), device="cpu", cache_bytes=16 << 20, auto_tick=False)
            nodes[r] = node
            fn(r, node)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    t0 = time.monotonic()
    [t.start() for t in ts]
    [t.join(timeout + 10) for t in ts]
    return errs, nodes, time.monotonic() - t0


@pytest.fixture
def origin():
    from hlsjs_p2p_wrapper_amd.net import clear_origins
    from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin

    clear_origins()
    o = SyntheticHlsOrigin("http://cdn.div/vod/", renditions=[Rendition(400_000, 320, 180)], num_segments=16,
                           encrypted=False, pin_memory=False)
    yield o
    clear_origins()


class _Sink:
    def __init__(self):
        self.got = 0

    def deliver(self, tok, *a, **k):
        self.got += len(tok)

    def fail(self, *a):
        pass


def _urls(origin, sns):
    return [origin.base_url + origin.segment_path(0, sn) for sn in sns]


def test_directory_divergence_stops_every_rank_with_a_diagnostic(origin):
    """Rank 1's replica gets an entry no control message carried (a local eviction or add
    applied on one rank only): the next round's all-gather shows two directory digests and
    BOTH ranks raise, naming which ranks hold which replica -- within seconds, before the
    diverged plan could post a send / receive group."""
    def body(r, node):
        sink = _Sink()
        node.set_bulk_sink(sink)
        ks = np.array([[5, 0, 0, sn] for sn in range(4)], dtype=np.int64)
        if r == 0:
            node.request_batch(ks, _urls(origin, range(4)), None, np.arange(4, dtype=np.int64))
        for step in range(6):
            if r == 1 and step == 3:
                node.directory.apply(0, np.array([[5, 0, 0, 99, 1234]], dtype=np.int64),
                                     np.zeros((0, 4), dtype=np.int64))
            node.complete_round(node.launch_round())

    errs, nodes, took = _two_ranks(body)
    assert set(errs) == {0, 1}, errs
    for e in errs.values():
        assert isinstance(e, rt.SwarmDivergence) and isinstance(e, RuntimeError)
        msg = str(e)
        assert "directory diverged before round 4" in msg and "ranks [0]" in msg and "ranks [1]" in msg
    assert took < 20


def test_plan_divergence_is_caught_in_the_next_round(origin):
    """A rank whose planner produced a different plan (simulated: its plan digest is
    altered) is caught at the next round's control all-gather -- with asynchronous rounds
    that is before the host waits on the diverged round's transfers."""
    def body(r, node):
        node.set_bulk_sink(_Sink())
        ks = np.array([[5, 0, 0, sn] for sn in range(4)], dtype=np.int64)
        node.request_batch(ks, _urls(origin, range(4)), None, np.arange(4, dtype=np.int64))
        h = node.launch_round()
        if r == 1:
            node._plan_digest ^= 1
        node.complete_round(h)
        node.complete_round(node.launch_round())

    errs, _, took = _two_ranks(body)
    assert set(errs) == {0, 1}, errs
    for e in errs.values():
        assert isinstance(e, rt.SwarmDivergence)
        assert "plans diverged in round 1" in str(e)
    assert took < 20


def test_consistent_ranks_pass_the_check(origin):
    def body(r, node):
        sink = _Sink()
        node.set_bulk_sink(sink)
        ks = np.array([[5, 0, 0, sn] for sn in range(8)], dtype=np.int64)
        node.request_batch(ks, _urls(origin, range(8)), None, np.arange(8, dtype=np.int64))
        for _ in range(4):
            node.complete_round(node.launch_round())
        assert sink.got == 8
        assert node.divergence_check

    errs, nodes, _ = _two_ranks(body)
    assert not errs, errs
    assert nodes[0].directory.digest == nodes[1].directory.digest != 0
    # every byte rank r received came from the other rank
    assert nodes[0].p2p_from[0] == 0 and nodes[1].p2p_from[1] == 0
    assert nodes[0].p2p_from[1] + nodes[1].p2p_from[0] == nodes[0].stats["p2p_wire"] + nodes[1].stats["p2p_wire"] > 0


def test_round_timeout_reports_and_dumps_the_plan(tmp_path, monkeypatch):
    node = SwarmNode(device="cpu", cache_bytes=64 << 10, loop=new_event_loop("virtual"), auto_tick=False)
    monkeypatch.setattr(SwarmNode, "ROUND_SPIN_S", 0.001)
    monkeypatch.setenv("HLSP2P_ROUND_TIMEOUT", "0.01")
    monkeypatch.setenv("HLSP2P_PLAN_DUMP", str(tmp_path))

    class Never:
        def query(self):
            return False

    h = RoundHandle(9, False)
    h.done = Never()
    send = np.array([[5, 0, 0, 1, 100, 0, 1, 3, 0, 0], [5, 0, 0, 2, 50, 0, 1, 4, 0, 0],
                     [5, 0, 0, 2, 70, 0, 2, 4, 0, 0]], dtype=np.int64)
    recv = np.array([[5, 0, 0, 7, 30, 2, 0, 11, 0, 0]], dtype=np.int64)
    h.plan = (send, recv)
    assert SwarmNode.plan_summary(h) == {"round": 9, "send": {1: [2, 150], 2: [1, 70]}, "recv": {2: [1, 30]}}
    with pytest.raises(TimeoutError, match=r"round 9 did not complete.*'send': \{1: \[2, 150\]"):
        node._wait_round(h)
    dump = np.load(tmp_path / "plan.r9.rank0.npz")
    assert (dump["send"] == send).all() and (dump["recv"] == recv).all()


def test_planner_grouping_fast_path_matches_the_general_path():
    """The planner groups wants by key with a counting sort over the sn window when the input
    is rank-major (as ingest_control emits it) and with a hash table otherwise; both must give
    the identical plan (and digest) for the same set of wants."""
    rng = np.random.default_rng(11)
    flags = np.full(4, rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD | rt.FLAG_CDN_DEDUP, dtype=np.int64)
    for trial in range(20):
        d = rt.Directory()
        held = [(7, lvl, 0, sn) for lvl in range(3) for sn in range(100, 140) if rng.random() < 0.3]
        for k in held:
            d.apply(int(rng.integers(0, 4)), _adds([k], length=int(rng.integers(1000, 5000))), _rms([]))
        rows = []
        for r in range(4):
            lvl = int(rng.integers(0, 3))
            sns = rng.choice(np.arange(100, 160), size=int(rng.integers(5, 40)), replace=False)
            for i, sn in enumerate(sorted(sns.tolist())):
                rows.append([7, (lvl + i) % 3, 0, sn, int(rng.integers(1000, 5000)), 1000 * r + i, r, 0])
        wants = np.array(rows, dtype=np.int64)
        shuffled = wants[rng.permutation(len(wants))]  # not rank-major: the hash path
        a = rt.plan_round_for(d, wants, flags, 4, 0)
        b = rt.plan_round_for(d, np.ascontiguousarray(shuffled), flags, 4, 0)
        assert np.array_equal(a[0], b[0]) and a[1] == b[1] and a[2] == b[2], trial
        assert np.array_equal(rt.plan_round(d, wants, flags, 4), rt.plan_round(d, np.ascontiguousarray(shuffled),
                                                                               flags, 4))
