"""The node's byte counters count a peer copy only once its CRC check passed (round-5
VERDICT Weak 5 / Next 3).  A corrupted copy is rejected (``p2p_rejected``) and re-fetched from
the CDN (``cdn``), so ``cdn + p2p`` equals the bytes the players were actually served and the
offload ratio -- the bench's and the swarm totals' -- is exact under injected corruption,
with the check run by the node (``complete_round``) or deferred to the consumer's decrypt
(``verify_done``).  Reference: the ``stats`` definition (``README.md:232-237``,
``lib/hlsjs-p2p-wrapper.js:14-18``)."""
import threading
import zlib

import numpy as np
import pytest

from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub


@pytest.fixture(autouse=True)
def fresh():
    clear_origins()
    yield
    clear_origins()


class _Consumer:
    """A fleet-like bulk sink: records every delivery and, for rows delivered before their
    check (``expect >= 0``), runs the check on the bytes and reports it like the transmux."""

    def __init__(self, node):
        self.node = node
        self.accepted = {}  # token -> (source, bytes)
        self.rejected = 0  # bytes of deliveries whose deferred check failed
        self.pending = []

    def deliver(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect=None):
        ex = np.full(len(tok), -1, dtype=np.int64) if expect is None else np.asarray(expect)
        self.pending.append((tok.copy(), src.copy(), nbytes.copy(), offs.copy(), eids.copy(), ex.copy()))

    def fail(self, tok, status):
        raise AssertionError(f"requests failed: {tok} {status}")

    def drain(self):
        arena = self.node.arena.numpy()
        for tok, src, nbytes, offs, eids, ex in self.pending:
            ok = np.ones(len(tok), dtype=bool)
            for i, (o, n, e) in enumerate(zip(offs.tolist(), nbytes.tolist(), ex.tolist())):
                if e >= 0:
                    ok[i] = (zlib.crc32(arena[o:o + n].tobytes()) & 0xFFFFFFFF) == e
            chk = ex >= 0
            if chk.any():
                self.node.verify_done(eids[chk], ok[chk], tok[chk])
            for t, s, n, good in zip(tok.tolist(), src.tolist(), nbytes.tolist(), ok.tolist()):
                if good:
                    assert t not in self.accepted, "a token was answered twice"
                    self.accepted[t] = (("cdn", "p2p", "cache")[s], n)
                else:
                    self.rejected += n
        self.pending = []


@pytest.mark.parametrize("deferred", [False, True])
def test_offload_counts_only_verified_peer_bytes(deferred):
    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode

    origin = SyntheticHlsOrigin("http://cdn.vc/vod/", renditions=[Rendition(1_000_000, 640, 360)], num_segments=12,
                                encrypted=False)
    seg = origin.pools[0].lengths
    urls = [f"http://cdn.vc/vod/r0/seg{i}.ts" for i in range(12)]
    keys = np.array([[9, 0, 0, i] for i in range(12)], dtype=np.int64)
    hub = ThreadHub(2)
    nodes, sinks, errs = {}, {}, []

    def rank(r):
        try:
            new_event_loop("virtual")
            node = SwarmNode(hub.comm(r), device="cpu", cache_bytes=64 << 20, auto_tick=False)
            node.verify_deferred = deferred
            nodes[r] = node
            sinks[r] = sink = _Consumer(node)
            node.set_bulk_sink(sink)
            node.corrupt_next_recv = 3  # the first three rounds with receives: one byte flipped each
            for step in range(12):
                if step in (0, 2):  # the second half is wanted later: served from the first ranks' caches
                    half = slice(0, 6) if step == 0 else slice(6, 12)
                    node.request_batch(keys[half], urls[half], None, np.arange(12, dtype=np.int64)[half])
                node.complete_round(node.launch_round())
                node.loop.run_until(lambda: False, timeout_ms=1)
                sink.drain()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(120) for t in ts]
    assert not errs, errs
    total = sum(seg)
    rejected = 0
    for r in range(2):
        st, acc = nodes[r].stats, sinks[r].accepted
        assert sorted(acc) == list(range(12)), (r, sorted(acc))  # every request answered once, with good bytes
        served = {s: sum(n for src, n in acc.values() if src == s) for s in ("cdn", "p2p")}
        assert sum(served.values()) == total
        # the node's counters are exactly what its players were served
        assert (st["cdn"], st["p2p"]) == (served["cdn"], served["p2p"]), (r, st, served)
        assert st["p2p_segments"] == sum(1 for src, _ in acc.values() if src == "p2p")
        # every byte that crossed the wire was either accepted or rejected
        assert st["p2p_wire"] == st["p2p"] + st["p2p_rejected"]
        if deferred:
            assert st["p2p_rejected"] == sinks[r].rejected
        rejected += st["p2p_rejected"]
        assert nodes[r].pending_verify() == 0
    assert rejected > 0 and sum(n.stats["crc_failures"] for n in nodes.values()) >= 2
    # the swarm-wide offload (control-header totals of the last round) uses the same counters
    cdn = sum(n.stats["cdn"] for n in nodes.values())
    p2p = sum(n.stats["p2p"] for n in nodes.values())
    assert cdn + p2p == 2 * total
    assert nodes[0].swarm_stats["p2p"] <= p2p
