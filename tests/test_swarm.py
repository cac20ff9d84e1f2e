"""In-process multi-peer swarm (the CPU analog of N MI355X peers): P2P
exchange + CDN de-duplication, offload ratio, CRC fault injection -> CDN fallback,
churn (offline peer), P2P toggles, live streams."""
import threading

import numpy as np

import pytest

from hlsjs_p2p_wrapper_amd import Hls
from hlsjs_p2p_wrapper_amd.agent import current_node, node_for_config, set_current_node
from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub
from hlsjs_p2p_wrapper_amd.player import MediaElement
from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine


@pytest.fixture(autouse=True)
def fresh():
    clear_origins()
    yield
    clear_origins()


def run_swarm(n, origin, until=38.0, before=None, cfg_extra=None, hls_cfg=None, start_delay=None, timeout=120_000):
    hub = ThreadHub(n)
    out, errs = {}, []

    def peer(r):
        try:
            set_current_node(None)
            loop = new_event_loop("virtual")
            w = HlsjsP2PWrapper(Engine)
            gs = {"backend": "thread", "hub": hub, "rank": r, "device": "cpu", "cacheBytes": 128 << 20,
                  "roundIntervalMs": 20}
            gs.update(cfg_extra or {})
            node_for_config({"gpuSwarm": gs})  # join the swarm's rounds from the start
            hls = w.createPlayer(dict(hls_cfg or {}), {"gpuSwarm": gs})
            media = MediaElement()
            delay = start_delay(r) if start_delay else 0
            if delay:  # keeps joining the rounds, but only starts playing later
                loop.set_timeout(hls.loadSource, delay, origin.master_url())
            else:
                hls.loadSource(origin.master_url())
            hls.attachMedia(media)
            hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
            node = current_node()
            if before:
                before(r, node, w)
            if callable(until):
                ok = loop.run_until(lambda: until(media), timeout_ms=timeout)
            else:
                ok = loop.run_until(lambda: media.currentTime > until, timeout_ms=timeout)
            out[r] = {"ok": ok, "t": media.currentTime, "stats": dict(w.stats), "node": dict(node.stats),
                      "offload": None}
            node.close()
            out[r]["offload"] = node.swarm_offload_ratio()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=peer, args=(r,)) for r in range(n)]
    [t.start() for t in ts]
    [t.join(300) for t in ts]
    if errs:
        raise errs[0]
    return out


@pytest.fixture
def vod():
    return SyntheticHlsOrigin("http://cdn.test/vod/", renditions=[Rendition(1_000_000, 640, 360)], num_segments=10,
                              encrypted=True)


def test_two_peers_share_cdn_fetches(vod):
    out = run_swarm(2, vod)
    total_cdn = sum(o["stats"]["cdn"] for o in out.values())
    total_p2p = sum(o["stats"]["p2p"] for o in out.values())
    seg_total = sum(vod.pools[0].lengths)
    assert all(o["ok"] for o in out.values())
    assert total_cdn == seg_total  # every segment fetched from the CDN exactly once
    assert total_p2p == seg_total  # ... and delivered to the other peer over P2P
    assert out[0]["stats"]["upload"] == out[1]["stats"]["p2p"]
    assert out[0]["stats"]["peers"] == 1
    assert out[0]["offload"] == pytest.approx(0.5)


def test_four_peers_offload(vod):
    out = run_swarm(4, vod)
    cdn = sum(o["stats"]["cdn"] for o in out.values())
    p2p = sum(o["stats"]["p2p"] for o in out.values())
    assert all(o["ok"] for o in out.values())
    assert p2p / (p2p + cdn) == pytest.approx(0.75)  # (N-1)/N with de-duplication


def test_staggered_peers_with_tiny_caches_play_through():
    """Four peers whose caches hold ~5 segments each, started 16 s apart: a lagging peer keeps
    wanting the segments a leader is about to overwrite (the ring-retire path,
    tests/test_ring_pressure.py; without it this run failed with "cannot make room"),
    in-flight windows of 4, 30 segments -- everyone plays to the end, nothing fails."""
    origin = SyntheticHlsOrigin("http://cdn.test/tiny/", renditions=[Rendition(1_000_000, 640, 360)],
                                num_segments=30, encrypted=True)
    seg = max(origin.pools[0].lengths)
    out = run_swarm(4, origin, until=110.0, cfg_extra={"cacheBytes": 5 * ((seg + 255) // 256 * 256)},
                    hls_cfg={"maxFragLoadsInFlight": 4, "maxBufferLength": 12},
                    start_delay=lambda r: 16000.0 * r, timeout=400_000)
    assert all(o["ok"] for o in out.values()), {r: o["t"] for r, o in out.items()}
    assert sum(o["stats"]["p2p"] for o in out.values()) > 0


def test_late_joiner_served_from_peers_cache(vod):
    # peer 1 starts 60 s later: everything it needs is already cached on peer 0
    out = run_swarm(2, vod, start_delay=lambda r: 60_000 if r == 1 else 0, timeout=400_000)
    assert out[1]["stats"]["cdn"] == 0
    assert out[1]["stats"]["p2p"] == sum(vod.pools[0].lengths)


def test_crc_failure_falls_back_to_cdn(vod):
    def corrupt(r, node, w):
        if r == 1:
            node.corrupt_next_recv = 2
    out = run_swarm(2, vod, before=corrupt)
    assert all(o["ok"] for o in out.values())
    assert out[1]["node"]["crc_failures"] >= 1
    assert out[1]["stats"]["cdn"] > 0  # refetched from the CDN after the bad peer copy


def test_deferred_receive_check_in_the_players_transmux(vod):
    """gpuSwarm.deferVerify: a peer copy reaches the in-process player before its CRC check;
    the player's transmux batch verifies it and reports back (VerifyTicket).  Corrupted copies
    are dropped before anything is buffered, the node detaches them, the player reloads the
    fragment from the CDN -- no player error -- and good copies are committed and announced."""
    errors = {}

    def corrupt(r, node, w):
        assert node.verify_deferred and node.defer_inproc
        if r == 1:
            node.corrupt_next_recv = 2
        hls = w._wrapper.hls
        errors[r] = []
        hls.on(Hls.Events.ERROR, lambda e, d: errors[r].append(d.get("details")))

    out = run_swarm(2, vod, before=corrupt, cfg_extra={"deferVerify": True})
    assert all(o["ok"] for o in out.values())
    assert errors == {0: [], 1: []}
    assert out[1]["node"]["crc_failures"] >= 1
    assert out[1]["stats"]["cdn"] > 0  # the corrupted fragments came again from the CDN
    seg_total = sum(vod.pools[0].lengths)
    assert out[0]["stats"]["p2p"] + out[1]["stats"]["p2p"] > 0
    assert sum(o["stats"]["cdn"] + o["stats"]["p2p"] for o in out.values()) >= 2 * seg_total


def test_deferred_check_of_a_dropped_fragment_is_swept_by_the_node():
    """A received segment whose consumer never reports (dropped before its transmux) is
    checked by the node after VERIFY_STALE_ROUNDS rounds: committed when good, detached when
    not -- never left pinned and unannounced."""
    import zlib

    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode

    node = SwarmNode(device="cpu", cache_bytes=1 << 20, loop=new_event_loop("virtual"), auto_tick=False)
    data = np.arange(3000, dtype=np.uint8)
    keys = np.array([[3, 0, 0, 1, 3000], [3, 0, 0, 2, 3000]], dtype=np.int64)
    res = node.store.reserve_run(np.ascontiguousarray(keys[:, :4]), keys[:, 4], 1)
    _, eids, offs = res
    for o in offs.tolist():
        node.arena[o:o + 3000] = torch_from(data)
    good = zlib.crc32(data.tobytes())
    node.store.pin(eids)
    node._vpend_add(eids, np.zeros((2, 10), dtype=np.int64), np.array([good, good ^ 1], dtype=np.int64))
    node.verify_deferred = True
    node.round = 100
    assert node.pending_verify() == 2
    assert node._sweep_pending() == 2
    assert node.pending_verify() == 0 and node.stats["crc_failures"] == 1
    assert node.store.lookup1(3, 0, 0, 1) >= 0 and node.store.lookup1(3, 0, 0, 2) < 0
    # nobody requested the swept copy: its key must not force a later request to the CDN
    # (the sweep's NO_TOKEN (-1) was read as an in-process request)
    assert not node._force_cdn_keys


def test_a_late_ticket_report_after_the_sweep_is_ignored():
    """A consumer that reports after the node swept its entry must not decide the check of
    whatever segment the entry id holds by then."""
    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode, VerifyTicket

    node = SwarmNode(device="cpu", cache_bytes=1 << 20, loop=new_event_loop("virtual"), auto_tick=False)
    keys = np.array([[3, 0, 0, 1]], dtype=np.int64)
    _, eids, _ = node.store.reserve_run(keys, np.array([3000]), 1)
    node.store.pin(eids)
    node.round = 5
    node._vpend_add(eids, np.zeros((1, 10), dtype=np.int64), np.array([0], dtype=np.int64))
    late = VerifyTicket(node, int(eids[0]), 0, 7)
    node.round = 200  # swept, then (as if evicted and reused) pending again on a newer delivery
    node.verify_done(eids, np.array([True]), np.array([node.rt.NO_TOKEN]))
    node.store.pin(eids)
    node._vpend_add(eids, np.zeros((1, 10), dtype=np.int64), np.array([0], dtype=np.int64))
    late.report(False)
    assert node.pending_verify() == 1 and node.stats["crc_failures"] == 0
    fresh = VerifyTicket(node, int(eids[0]), 0, 8)
    fresh.report(True)
    assert node.pending_verify() == 0


class _ColSink:
    def __init__(self):
        self.got = []

    def deliver(self, tok, src, *a, **k):
        self.got.extend(zip(np.asarray(tok).tolist(), np.asarray(src).tolist()))

    def fail(self, *a):
        pass


@pytest.mark.parametrize("passes", [True, False])
def test_a_request_for_a_copy_awaiting_its_check_waits_for_the_check(passes):
    """A fleet request for a segment whose received copy was delivered and awaits its deferred
    check waits for that check instead of fetching the segment again (the second fetch
    replaced the copy in the index while the first players still read it; their on-demand
    bytes came back empty): answered from the copy when it passes, from the CDN when not."""
    from hlsjs_p2p_wrapper_amd.agent.node import SRC_CACHE, SwarmNode

    loop = new_event_loop("virtual")
    node = SwarmNode(device="cpu", cache_bytes=1 << 20, loop=loop, auto_tick=False)
    sink = _ColSink()
    node.set_bulk_sink(sink)
    node.verify_deferred = True
    key = np.array([[3, 0, 0, 1]], dtype=np.int64)
    _, eids, _ = node.store.reserve_run(key, np.array([3000]), 1)
    node.store.pin(eids)
    info = np.zeros((1, 10), dtype=np.int64)
    info[0, :4] = key[0]
    info[0, 4] = 3000
    node._vpend_add(eids, info, np.array([0], dtype=np.int64))
    node.request_batch(key, ["http://cdn.test/vod/x.ts"], None, np.array([42], dtype=np.int64))
    assert node.stats["parked"] == 1 and len(node._wt) == 0
    node.verify_done(eids, np.array([passes]), np.array([7], dtype=np.int64))
    loop.run_until(lambda: False, timeout_ms=10)
    if passes:
        assert (42, SRC_CACHE) in sink.got and len(node._wt) == 0
    else:
        assert not any(t == 42 for t, _ in sink.got) and len(node._wt) == 1  # asked again, from the CDN
    assert not node._vwait


def torch_from(a):
    import torch

    return torch.from_numpy(a)


def test_offline_peer_neither_serves_nor_receives(vod):
    def offline(r, node, w):
        if r == 1:
            node.set_online(False)
    out = run_swarm(2, vod, before=offline)
    seg_total = sum(vod.pools[0].lengths)
    assert out[1]["stats"]["p2p"] == 0 and out[1]["stats"]["cdn"] == seg_total
    assert out[0]["stats"]["p2p"] == 0 and out[0]["stats"]["cdn"] == seg_total


def test_p2p_download_toggle(vod):
    def no_dl(r, node, w):
        if r == 1:
            node.download_on = False
    out = run_swarm(2, vod, before=no_dl)
    assert out[1]["stats"]["p2p"] == 0


def test_live_stream_swarm():
    origin = SyntheticHlsOrigin("http://cdn.test/live/", renditions=[Rendition(800_000, 640, 360)], live=True,
                                window=6, num_segments=None, pool_size=8, encrypted=True)
    origin.advance(4)  # live edge at sn 9: window sn 4..9 = 24 s of media (frozen clock)
    # live start = 24 - 2 * targetduration = 16 s; play to the live edge
    out = run_swarm(2, origin, until=lambda m: m.currentTime > 22.0, hls_cfg={"liveSyncDurationCount": 2})
    assert all(o["ok"] for o in out.values())
    assert sum(o["stats"]["p2p"] for o in out.values()) > 0
    assert sum(o["stats"]["cdn"] for o in out.values()) == sum(o["stats"]["p2p"] for o in out.values())


def test_request_trace_records(vod):
    # per-request {trequest, tfirst, tload, source, bytes, peer} records
    traces = {}

    def grab(r, node, w):
        traces[r] = node.trace

    out = run_swarm(2, vod, before=grab, cfg_extra={"trace": True})
    assert all(o["ok"] for o in out.values())
    for r, tr in traces.items():
        assert len(tr) > 0
        for rec in tr.records:
            assert rec.trequest <= rec.tfirst <= rec.tload
            assert rec.source in ("cdn", "p2p", "cache")
            assert rec.peer == (1 - r if rec.source == "p2p" else r)
        by = tr.by_source()
        assert by.get("cdn", (0, 0))[1] == out[r]["stats"]["cdn"]
        assert by.get("p2p", (0, 0))[1] == out[r]["stats"]["p2p"]
        assert tr.latency_ms(0.5) >= 0
        assert tr.to_dicts()[0]["bytes"] > 0


def test_agent_prefetch_fills_cache_ahead_of_player(vod):
    # the late joiner prefetches ahead of its playhead; its player's requests then hit
    # the local cache, and the bytes are still accounted as P2P (where they came from)
    out = run_swarm(2, vod, start_delay=lambda r: 60_000 if r == 1 else 0, timeout=400_000,
                    cfg_extra={"prefetchSeconds": 16.0}, hls_cfg={"maxBufferLength": 4})
    assert all(o["ok"] for o in out.values())
    assert out[1]["node"]["prefetched"] > 0
    seg_total = sum(vod.pools[0].lengths)
    assert out[1]["stats"]["cdn"] == 0
    assert out[1]["stats"]["p2p"] == seg_total  # every segment played once, counted once
    assert out[0]["stats"]["cdn"] == seg_total


def test_slow_link_fault_injection(vod):
    # a slow peer link delays P2P completions by their modelled transfer time
    def lat(out_traces, r):
        return out_traces[r].latency_ms(0.5, source="p2p")

    fast, slow = {}, {}
    run_swarm(2, vod, before=lambda r, node, w: fast.__setitem__(r, node.trace), cfg_extra={"trace": True})
    out = run_swarm(2, vod, before=lambda r, node, w: slow.__setitem__(r, node.trace),
                    cfg_extra={"trace": True, "linkKbps": {0: 8000, 1: 8000}})
    assert all(o["ok"] for o in out.values())
    # ~250 KB segments over an 8 Mb/s link: >= 250 ms each, far above the unshaped case.  The
    # receiving rank: whichever the planner's seeding left behind (its rotation starts at a
    # key-drawn rank, and the rank a slow link delays keeps trailing)
    rx = max(slow, key=lambda r: sum(1 for x in slow[r].records if x.source == "p2p"))
    assert lat(slow, rx) > 200 and lat(slow, rx) > 5 * max(lat(fast, rx), 1.0)
    recs = [r for r in slow[rx].records if r.source == "p2p"]
    assert recs and all(r.tload - r.tfirst >= r.bytes * 8 / 8000 - 1e-6 for r in recs)


def test_small_cache_backpressure():
    # SURVEY config 5 analog: a cache far smaller than the stream, and many fragments in
    # flight: wants are deferred (never evicting in-flight / being-consumed segments) and
    # playback completes with correct bytes
    origin = SyntheticHlsOrigin("http://cdn.test/small/", renditions=[Rendition(4_000_000, 1280, 720)],
                                num_segments=12, encrypted=True)
    seg = max(origin.pools[0].lengths)
    out = run_swarm(2, origin, until=44.0, cfg_extra={"cacheBytes": 3 * (seg + 4096), "maxWantsPerRound": 8},
                    hls_cfg={"maxFragLoadsInFlight": 6, "maxBufferLength": 60})
    assert all(o["ok"] for o in out.values())
    assert sum(o["node"].get("deferred", 0) for o in out.values()) > 0
    total = sum(origin.pools[0].lengths[i % len(origin.pools[0].lengths)] for i in range(12))
    for o in out.values():
        assert o["stats"]["cdn"] + o["stats"]["p2p"] == total


def test_segment_larger_than_cache_fails_cleanly():
    # a segment that can never fit the cache fails its request with an HTTP-like error
    # (the loader contract: errors surface as {status}) instead of waiting forever
    from hlsjs_p2p_wrapper_amd.agent import SwarmNode

    origin = SyntheticHlsOrigin("http://cdn.test/huge/", renditions=[Rendition(2_000_000, 640, 360)],
                                num_segments=2, encrypted=False)
    loop = new_event_loop("virtual")
    node = SwarmNode(device="cpu", cache_bytes=64 << 10, loop=loop)
    got = {}
    url = origin.base_url + origin.segment_path(0, 0)
    node.request((1, 0, 0, 0), url, {}, {"onSuccess": lambda d: got.setdefault("ok", d),
                                          "onError": lambda e: got.setdefault("err", e)})
    loop.run_until(lambda: got, timeout_ms=5_000)
    assert "err" in got and getattr(got["err"], "status", None) == 507


def test_abr_ladder_track_switching_under_churn():
    # BASELINE config 3 analog: 3 peers on a 3-rendition ladder; level switches mid-stream
    # (track-view changes reach the agents through PlayerInterface 'onTrackChange') while
    # peer 2 churns offline and back.  Everyone plays through, P2P keeps flowing, and no
    # peer receives P2P bytes while it is masked offline.
    origin = SyntheticHlsOrigin("http://cdn.test/abr/", renditions=[Rendition(400_000, 480, 270),
                                                                    Rendition(800_000, 640, 360),
                                                                    Rendition(1_600_000, 960, 540)],
                                num_segments=12, encrypted=True)
    hub = ThreadHub(3)
    out, errs = {}, []

    def peer(r):
        try:
            set_current_node(None)
            loop = new_event_loop("virtual")
            gs = {"backend": "thread", "hub": hub, "rank": r, "device": "cpu", "cacheBytes": 256 << 20,
                  "roundIntervalMs": 20}
            node = node_for_config({"gpuSwarm": gs})
            w = HlsjsP2PWrapper(Engine)
            hls = w.createPlayer({"startLevel": 0}, {"gpuSwarm": gs})
            media = MediaElement()
            hls.loadSource(origin.master_url())
            hls.attachMedia(media)
            hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
            tracks, offline_p2p = [], []
            agent = node._agents[0]
            agent.player.addEventListener("onTrackChange", lambda d: tracks.append(d["video"].level))
            loop.set_timeout(lambda: setattr(hls, "nextLevel", 2), 8_000)
            loop.set_timeout(lambda: setattr(hls, "nextLevel", 1), 20_000)
            if r == 2:
                def go_offline():
                    node.set_online(False)
                    offline_p2p.append(node.stats["p2p"])

                def back_online():
                    offline_p2p.append(node.stats["p2p"])
                    node.set_online(True)
                loop.set_timeout(go_offline, 6_000)
                loop.set_timeout(back_online, 16_000)
            ok = loop.run_until(lambda: media.currentTime > 44.0, timeout_ms=200_000)
            out[r] = {"ok": ok, "tracks": tracks, "stats": dict(w.stats), "offline_p2p": offline_p2p,
                      "agent_track": agent.currentTrack.level if agent.currentTrack else None}
            node.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=peer, args=(r,)) for r in range(3)]
    [t.start() for t in ts]
    [t.join(300) for t in ts]
    if errs:
        primary = [e for e in errs if not isinstance(e, threading.BrokenBarrierError)]
        raise (primary or errs)[0]
    for r, o in out.items():
        assert o["ok"], r
        assert 2 in o["tracks"] and o["tracks"][-1] == 1 and o["agent_track"] == 1
    assert sum(o["stats"]["p2p"] for o in out.values()) > 0
    a, b = out[2]["offline_p2p"]
    assert a == b  # masked offline: no P2P bytes received in that window


def test_live_window_eviction():
    # the live window slides with sn; segments that left the playlist can no
    # longer be requested and are evicted from the cache (and the swarm is told)
    from hlsjs_p2p_wrapper_amd.agent import SwarmNode

    set_current_node(None)
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.test/slide/", renditions=[Rendition(800_000, 640, 360)], live=True,
                                window=5, num_segments=None, pool_size=8, encrypted=True, loop=loop)
    node = SwarmNode(device="cpu", cache_bytes=256 << 20, loop=loop)
    set_current_node(node)
    w = HlsjsP2PWrapper(Engine)
    hls = w.createPlayer({"liveSyncDurationCount": 2}, {})
    media = MediaElement()
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    assert loop.run_until(lambda: media.currentTime > 60.0, timeout_ms=400_000)
    agent = node._agents[0]
    assert agent.evicted > 0
    ids, keys = node.store.resident()
    first = hls.levels[0].details.fragments[0].sn
    assert len(keys) and keys[:, 3].min() >= agent._evicted_below and agent._evicted_below <= first
    hls.destroy()
    set_current_node(None)


def test_origin_resolution_and_vod_locate():
    """``http.resolve`` picks the longest registered base (cached per URL directory, so nested
    bases keep working), and a VOD origin locates a (ranged) segment's bytes once."""
    from hlsjs_p2p_wrapper_amd.net import http
    from hlsjs_p2p_wrapper_amd.net.origin import _seg_path

    clear_origins()
    try:
        outer = SyntheticHlsOrigin(base_url="http://nest.test/", renditions=[Rendition(100_000, 320, 180)],
                                   num_segments=4, pin_memory=False)
        inner = SyntheticHlsOrigin(base_url="http://nest.test/live/", renditions=[Rendition(100_000, 320, 180)],
                                   num_segments=4, pin_memory=False)
        for _ in range(2):  # second pass: from the directory cache
            assert http.resolve("http://nest.test/live/r0/seg1.ts") == (inner, "r0/seg1.ts")
            assert http.resolve("http://nest.test/r0/seg2.ts") == (outer, "r0/seg2.ts")
            assert http.resolve("http://nest.test/live/r0/seg3.ts?tok=a/b") == (inner, "r0/seg3.ts?tok=a/b")
        with pytest.raises(http.HttpError):
            http.resolve("http://elsewhere.test/r0/seg1.ts")
        assert _seg_path("a/r3/seg17.ts") == (3, 17) and _seg_path("x/a/r3/seg17.ts") is None
        data, off, n, _ = inner.resource("r0/seg1.ts")
        assert inner.locate("r0/seg1.ts") == (data, off, n)
        assert inner.locate("r0/seg1.ts", rng=(10, 19))[1:] == (off + 10, 10)
        assert inner.locate("r0/index.m3u8") is None
        with pytest.raises(http.HttpError):
            inner.locate("r0/seg4.ts")  # past the VOD's last segment
    finally:
        clear_origins()


def test_round_wait_reports_a_dead_peer_instead_of_hanging(monkeypatch):
    """SURVEY §5.3 failure detection: a round whose transfers wait on a crashed peer never
    completes on the device.  The node polls the round instead of blocking on it, and raises
    on the data plane's asynchronous error (RCCL's ncclCommGetAsyncError) or on the
    HLSP2P_ROUND_TIMEOUT deadline.  A round that finishes late is simply waited for."""
    from hlsjs_p2p_wrapper_amd.agent.node import RoundHandle, SwarmNode

    node = SwarmNode(device="cpu", cache_bytes=64 << 10, loop=new_event_loop("virtual"), auto_tick=False)
    monkeypatch.setattr(SwarmNode, "ROUND_SPIN_S", 0.001)

    class Never:
        def query(self):
            return False

    class Later:
        def __init__(self):
            self.n = 0

        def query(self):
            self.n += 1
            return self.n > 3

    h = RoundHandle(7, False)
    h.done = Never()
    node.comm.async_error = lambda: "unhandled system error (remote process exited)"
    with pytest.raises(RuntimeError, match="round 7 failed in the data plane"):
        node._wait_round(h)
    node.comm.async_error = lambda: ""
    monkeypatch.setenv("HLSP2P_ROUND_TIMEOUT", "0.01")
    with pytest.raises(TimeoutError, match="round 7 did not complete"):
        node._wait_round(h)
    h.done = Later()
    node._wait_round(h)  # completes once the event reports done
    assert h.done.n == 4


class _Sink:
    def __init__(self):
        self.got = {}
        self.failed = {}

    def deliver(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids):
        for t, s, n in zip(tok.tolist(), src.tolist(), nbytes.tolist()):
            self.got[t] = ("cdn", "p2p", "cache")[s], n

    def fail(self, tok, status):
        self.failed.update(zip(tok.tolist(), status.tolist()))


def test_per_session_download_toggle_on_one_node(vod):
    """Columnar requests of two sessions on ONE node (a fleet's players): the session with P2P
    download off gets its fragments from the CDN, the other one from the peer that holds
    them; the node keeps uploading (``lib/hlsjs-p2p-wrapper.js:20-36`` toggles the session's
    own agent, not the machine)."""
    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode

    hub = ThreadHub(2)
    urls = [f"http://cdn.test/vod/r0/seg{i}.ts" for i in range(10)]
    ks = np.array([[7, 0, 0, i] for i in range(10)], dtype=np.int64)
    sinks, errs = [_Sink(), _Sink()], []
    nodes = {}

    def rank(r):
        try:
            new_event_loop("virtual")
            node = SwarmNode(hub.comm(r), device="cpu", cache_bytes=64 << 20, auto_tick=False)
            nodes[r] = node
            node.set_bulk_sink(sinks[r])
            if r == 0:  # the holder: fetches everything first
                node.request_batch(ks, urls, None, np.arange(10, dtype=np.int64))
            for step in range(4):
                if r == 1 and step == 2:
                    node.set_session_flags(("fleet", 0), False, True)
                    node.set_session_flags(("fleet", 1), True, True)
                    node.request_batch(ks[:5], urls[:5], None, np.arange(5, dtype=np.int64),
                                       force_cdn=np.ones(5, dtype=bool))  # session 0: download off
                    node.request_batch(ks[5:], urls[5:], None, np.arange(5, 10, dtype=np.int64) | (1 << 40))
                node.complete_round(node.launch_round())
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    assert not errs, errs
    assert all(v[0] == "cdn" for v in sinks[0].got.values()) and len(sinks[0].got) == 10
    s1 = sinks[1].got
    assert [s1[t][0] for t in range(5)] == ["cdn"] * 5  # download off: CDN only
    assert [s1[t | (1 << 40)][0] for t in range(5, 10)] == ["p2p"] * 5  # the other session: peers
    assert nodes[1].download_on and nodes[1].upload_on and nodes[1].session_flags(("fleet", 0)) == (False, True)


def _agent_of(w):
    return w._wrapper.peerAgentModule


def test_agent_negotiates_the_live_buffer_margin():
    """On a live stream the agent asks the bridge ``isLive()`` and sets the player's buffer
    target to ``getBufferLevelMax() - liveMinBufferMargin`` through ``setBufferMarginLive``
    (``lib/integration/player-interface.js:31-66``, ``CHANGELOG.md:15``); on VOD it leaves the
    player's config alone."""
    live = SyntheticHlsOrigin("http://cdn.test/live/", renditions=[Rendition(800_000, 640, 360)], live=True,
                              window=6, num_segments=None, pool_size=8, encrypted=True)
    live.advance(4)
    seen = {}

    def grab(r, node, w):
        seen[r] = w

    out = run_swarm(1, live, until=lambda m: m.currentTime > 18.0, before=grab,
                    cfg_extra={"liveMinBufferMargin": 6.0})
    assert out[0]["ok"]
    agent = _agent_of(seen[0])
    assert agent.is_live is True and agent.live_buffer_level == pytest.approx(30.0 - 6.0)
    cfg = agent.player.hls.config
    assert cfg.maxBufferLength == pytest.approx(24.0) and cfg.maxBufferSize == 0

    vod = SyntheticHlsOrigin("http://cdn.test/vod2/", renditions=[Rendition(800_000, 640, 360)], num_segments=6)
    out = run_swarm(1, vod, until=10.0, before=grab)
    agent = _agent_of(seen[0])
    assert out[0]["ok"] and agent.is_live is False and agent.live_buffer_level is None
    assert agent.player.hls.config.maxBufferLength == 30  # the wrapper default, untouched


def test_node_reports_a_saturated_ingest_link_to_the_planner(monkeypatch):
    """FLAG_CDN_BOUND (the planner's CDN balance relieves only such ranks) follows the share of
    the rank's rounds its CDN copies keep the ingest link busy, averaged over rounds, and is
    only ever set with the balance on (HLSP2P_CDN_BALANCE=1; off by default)."""
    from hlsjs_p2p_wrapper_amd.agent import node as node_mod
    from hlsjs_p2p_wrapper_amd.agent.node import RoundHandle, SwarmNode

    assert not SwarmNode(device="cpu", cache_bytes=64 << 10, loop=new_event_loop("virtual"),
                         auto_tick=False).cdn_balance
    monkeypatch.setenv("HLSP2P_CDN_BALANCE", "1")
    node = SwarmNode(device="cpu", cache_bytes=64 << 10, loop=new_event_loop("virtual"), auto_tick=False)
    bound = node.rt.FLAG_CDN_BOUND
    assert not node.flags & bound
    clock = [100.0]
    monkeypatch.setattr(node_mod.time, "perf_counter", lambda: clock[0])
    for _ in range(20):  # 10 ms rounds, 9.6 ms of CDN copies each: a saturated link
        clock[0] += 0.010
        h = RoundHandle(node.round, np.zeros(0, dtype=np.int64), t0=clock[0])
        h.empty, h.cdn_ms = False, 9.6
        node.complete_round(h)
    assert node._cdn_busy > node_mod.CDN_BOUND_BUSY and node.flags & bound
    for _ in range(20):  # 2 ms of copies per 10 ms round (an HBM origin): the flag clears
        clock[0] += 0.010
        h = RoundHandle(node.round, np.zeros(0, dtype=np.int64), t0=clock[0])
        h.empty, h.cdn_ms = False, 2.0
        node.complete_round(h)
    assert not node.flags & bound
    for _ in range(40):  # bursts: rounds completing back to back after a long gap do not read as saturated
        clock[0] += 0.020
        for dt in (0.0, 0.0001):
            clock[0] += dt
            h = RoundHandle(node.round, np.zeros(0, dtype=np.int64), t0=clock[0])
            h.empty, h.cdn_ms = False, 2.0
            node.complete_round(h)
    assert node._cdn_busy < 0.3 and not node.flags & bound
    node._cdn_busy = 0.95
    node.cdn_balance = False
    assert not node.flags & bound


def test_live_level_switch_lands_on_the_playback_timeline():
    """A live level's first playlist starts its own timeline at 0.  Loaded for the first time
    after the window slid (a level switch), it must be put on the timeline playback is on
    through the sn the levels share (hls.js alignStream): unaligned, the switched-to level's
    fragments sat 8 segments early and the player stalled at its buffer end waiting for them
    (tests/fleet_chaos.py --live, seed 10)."""
    from hlsjs_p2p_wrapper_amd.agent import SwarmNode

    set_current_node(None)
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.test/lsw/", renditions=[Rendition(400_000, 320, 180),
                                                                    Rendition(800_000, 640, 360)],
                                live=True, window=5, num_segments=None, pool_size=8, encrypted=True, loop=loop)
    node = SwarmNode(device="cpu", cache_bytes=256 << 20, loop=loop)
    set_current_node(node)
    w = HlsjsP2PWrapper(Engine)
    hls = w.createPlayer({"liveSyncDurationCount": 2, "startLevel": 0}, {})
    media = MediaElement()
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    hls.currentLevel = 0
    assert loop.run_until(lambda: media.currentTime > 40.0, timeout_ms=400_000)
    assert hls.levels[1].details is None  # never loaded: its first playlist comes after the slide
    hls.currentLevel = 1
    t = media.currentTime
    assert loop.run_until(lambda: media.currentTime > t + 40.0, timeout_ms=400_000), media.currentTime
    off = {lv: {round(f.start - 4.0 * f.sn, 6) for f in hls.levels[lv].details.fragments} for lv in (0, 1)}
    assert off[0] == off[1] and len(off[0]) == 1
    hls.destroy()
    set_current_node(None)


def test_live_seek_behind_the_window_resets_to_the_live_sync_point():
    """A live playhead seeked back past the sliding window (or paused until the window left
    it) cannot be fed: it is reset to the live sync position, as hls.js does; before, it sat
    seeking forever in front of the buffered window (tests/fleet_chaos.py --live, seeds 8, 18)."""
    from hlsjs_p2p_wrapper_amd.agent import SwarmNode

    set_current_node(None)
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.test/lsk/", renditions=[Rendition(400_000, 320, 180)],
                                live=True, window=5, num_segments=None, pool_size=8, encrypted=True, loop=loop)
    node = SwarmNode(device="cpu", cache_bytes=256 << 20, loop=loop)
    set_current_node(node)
    w = HlsjsP2PWrapper(Engine)
    hls = w.createPlayer({"liveSyncDurationCount": 2}, {})
    media = MediaElement()
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    assert loop.run_until(lambda: media.currentTime > 60.0, timeout_ms=400_000)
    first = hls.levels[0].details.fragments[0].start
    assert first > 10.0
    media.currentTime = 1.0  # behind the window
    assert loop.run_until(lambda: media.currentTime > first + 30.0, timeout_ms=400_000), media.currentTime
    hls.destroy()
    set_current_node(None)
