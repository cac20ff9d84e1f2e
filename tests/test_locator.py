"""Native batch locator of fixed-address origins (``runtime/locator.cpp``): a fleet rank's
``request_batch`` resolves its URLs in one native call.  The answers must be the per-request
Python path's (``SwarmNode._resolve``) exactly; byte ranges, live windows and injected faults
must keep taking the Python path."""
import numpy as np
import pytest

from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops._native import runtime


@pytest.fixture(autouse=True)
def fresh():
    clear_origins()
    yield
    clear_origins()


def test_locator_parses_names_and_slots():
    L = runtime().SegmentLocator()
    L.add_dir("http://a/r0/", "seg", ".ts", 10, 100, 1000, 64, np.array([0, 10, 20]), np.array([5, 6, 7]))
    urls = ["http://a/r0/seg11.ts", "http://a/r0/seg100.ts", "http://a/r1/seg11.ts", "http://a/r0/segx.ts",
            "http://a/r0/seg12.ts", "http://a/r0/seg9.ts", "http://a/r0/seg12.tsx", "noslash"]
    size, ptr, base, flags, ok, found = L.resolve(urls)
    assert ok.tolist() == [True, False, False, False, True, False, False, False] and found == 2
    assert size[ok].tolist() == [7, 5] and ptr[ok].tolist() == [1020, 1000]  # 11 % 3 = 2, 12 % 3 = 0
    assert base[ok].tolist() == [1000, 1000] and flags[ok].tolist() == [64, 64]
    assert size[~ok].tolist() == [0] * 6


class Sink:
    def __init__(self):
        self.fails = []

    def deliver(self, *a):
        pass

    def fail(self, tok, status):
        self.fails += list(zip(np.asarray(tok).tolist(), np.asarray(status).tolist()))


def _node():
    node = SwarmNode(device="cpu", cache_bytes=256 << 20, loop=new_event_loop("virtual"), auto_tick=False)
    node.set_bulk_sink(Sink())
    return node


def test_batch_matches_per_request_resolution():
    origin = SyntheticHlsOrigin("http://cdn.loc/vod/", renditions=[Rendition(400_000, 640, 360)] * 2,
                                num_segments=40, pool_size=7, redundant=2, pin_memory=False)
    node = _node()
    urls = [origin.base_url + origin.segment_path(lvl, sn) for lvl in (0, 1) for sn in range(0, 40, 3)]
    ref = [node._resolve(u, None)[:4] for u in urls]  # the Python path (also registers the origin)
    assert len(node._locator) > 0
    node._locs.clear()
    size, ptr, base, flags, ok, found = node._locator.resolve(urls)
    assert ok.all() and found == len(urls)
    assert [tuple(int(v) for v in t) for t in zip(size, ptr, base, flags)] == [tuple(r) for r in ref]
    # a whole batch: no per-URL Python resolution at all
    calls = []
    real = node._resolve
    node._resolve = lambda u, h: calls.append(u) or real(u, h)
    keys = np.array([[1, lvl, 0, sn] for lvl in (0, 1) for sn in range(0, 40, 3)], dtype=np.int64)
    node.request_batch(keys, urls, None, np.arange(len(urls), dtype=np.int64))
    assert calls == [] and node.pending() == len(urls)
    # byte ranges and unknown URLs go the general way
    more = [origin.base_url + origin.segment_path(0, 1), origin.base_url + "r0/seg999.ts"]
    node.request_batch(np.array([[1, 0, 0, 1], [1, 0, 0, 999]], dtype=np.int64), more,
                       [{"Range": "bytes=0-99"}, None], np.array([100, 101], dtype=np.int64))
    assert calls == more
    assert node._bulk.fails == [(101, 404)]


def test_faults_and_live_take_the_python_path():
    origin = SyntheticHlsOrigin("http://cdn.loc/vod2/", renditions=[Rendition(400_000, 640, 360)],
                                num_segments=20, pin_memory=False)
    node = _node()
    u = [origin.base_url + origin.segment_path(0, sn) for sn in range(4)]
    node._resolve(u[0], None)
    assert node._locator_usable()
    origin.fail(r"seg2\.ts$", 503)
    assert not node._locator_usable() and len(node._locator) == 0
    calls = []
    real = node._resolve
    node._resolve = lambda url, h: calls.append(url) or real(url, h)
    node.request_batch(np.array([[1, 0, 0, sn] for sn in range(4)], dtype=np.int64), u, None,
                       np.arange(4, dtype=np.int64))
    assert calls == u and node._bulk.fails == [(2, 503)]
    # once the faults are cleared, the origin returns to the native fast path (it was not
    # locked out by the refusal while faults were active)
    origin.clear_faults()
    node._resolve(origin.base_url + origin.segment_path(0, 7), None)
    assert node._locator_usable() and len(node._locator) > 0
    live = SyntheticHlsOrigin("http://cdn.loc/live/", renditions=[Rendition(400_000, 640, 360)], live=True,
                              pin_memory=False)
    assert live.segment_dirs() is None
