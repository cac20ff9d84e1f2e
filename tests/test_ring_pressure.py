"""The HBM ring under pressure across ranks.

A rank admits its round's wants only as far as its ring can place them (the oldest, unpinned
entries at the ring's head get overwritten).  A peer may want exactly those oldest segments
in the same round: the plan then has the rank SEND entries its own reservation is about to
overwrite.  The send pins them after admission, so the reservation found them pinned and the
rank failed ("segment cache cannot make room", seen at N=8 on a 4 GB arena).  The rank now
announces those entries' removal in the same round's control message, so no peer plans a
transfer from them."""
import threading

import numpy as np

from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub


class _Sink:
    def __init__(self):
        self.tokens = []

    def deliver(self, tok, *a, **k):
        self.tokens.extend(np.asarray(tok).tolist())

    def fail(self, *a):
        pass


def _two_ranks(fn, caches, timeout=30):
    hub = ThreadHub(2, timeout=timeout)
    errs, nodes = {}, {}

    def rank(r):
        try:
            new_event_loop("virtual")
            node = SwarmNode(hub.comm(r), device="cpu", cache_bytes=caches[r], auto_tick=False)
            nodes[r] = node
            fn(r, node)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(timeout + 10) for t in ts]
    return errs, nodes


def test_a_peer_wanting_the_segments_a_rank_overwrites_this_round():
    clear_origins()
    try:
        origin = SyntheticHlsOrigin("http://cdn.ring/vod/", renditions=[Rendition(400_000, 320, 180)],
                                    num_segments=16, encrypted=False, pin_memory=False)
        lens = [int(origin.pools[0].lengths[sn % origin.pool_size]) for sn in range(16)]
        al = [(n + 255) // 256 * 256 for n in lens]
        cap = sum(al[:6]) + 256  # rank 0's ring holds sns 0-5; sns 6-7 wrap over sns 0-1

        def keys(sns):
            return np.array([[5, 0, 0, sn] for sn in sns], dtype=np.int64)

        def urls(sns):
            return [origin.base_url + origin.segment_path(0, sn) for sn in sns]

        def body(r, node):
            sink = _Sink()
            node.set_bulk_sink(sink)
            if r == 0:
                node.request_batch(keys(range(6)), urls(range(6)), None, np.arange(6, dtype=np.int64))
            for _ in range(3):
                node.complete_round(node.launch_round())
            # one round: rank 0 wants sns 6-7 (its reservation overwrites sns 0-1), rank 1
            # wants sns 0-1 (held by rank 0 until then)
            sns = [6, 7] if r == 0 else [0, 1]
            node.request_batch(keys(sns), urls(sns), None, np.array(sns, dtype=np.int64) + 100)
            for _ in range(4):
                node.complete_round(node.launch_round())
            node.result = sorted(sink.tokens)

        errs, nodes = _two_ranks(body, {0: cap, 1: 16 << 20})
        assert not errs, errs
        assert nodes[0].result == [0, 1, 2, 3, 4, 5, 106, 107]
        assert nodes[1].result == [100, 101]
        assert nodes[0].directory.digest == nodes[1].directory.digest
    finally:
        clear_origins()


def test_a_rounds_several_runs_wrap_together():
    """A round reserves a CDN run and one run per source peer.  Runs that wrapped one by one
    skipped the ring's tail in the middle of the round, and the runs after the wrap could land
    on the round's own, pinned, earlier runs: admission's single-run check passed and the third
    reservation failed (a 3-segment cache in tests/swarm_chaos.py, seed 153).  The round now
    wraps before its first run when its admitted total would cross the end (``wrap_for``)."""
    from hlsjs_p2p_wrapper_amd.ops._native import runtime

    rt = runtime()

    def fresh():
        st = rt.SegmentStore(1024, 16)
        _, ids, _ = st.reserve_run(np.array([[9, 0, 0, 0]], dtype=np.int64), np.array([320]), 0)
        st.commit(ids)  # head -> 320; the entry stays unpinned (evictable)
        return st

    def run(st, sn, n):
        r = st.reserve_run(np.array([[9, 0, 0, sn]], dtype=np.int64), np.array([n], dtype=np.int64), 0)
        if r is not None:
            st.pin(r[1])  # in flight: pinned until its round completes
        return r

    st = fresh()
    assert st.fits(896)  # admission: 896 bytes, wrapping past the 320-byte head
    # runs placed one by one: 512 before the end, 320 wraps to 0, 64 lands on the first run
    assert run(st, 1, 512) is not None and run(st, 2, 320) is not None and run(st, 3, 64) is None
    st = fresh()
    assert st.wrap_for(896)  # the round wraps first: its runs fill [0, 896)
    assert all(run(st, sn, n) is not None for sn, n in ((1, 512), (2, 320), (3, 64)))
    assert st.wrap_for(64) and st.wrap_for(0)  # (no-ops: 64 fits before the end)
