"""Metrics export: the reference ``stats`` counters, swarm offload ratio, HBM
cache occupancy, phase timings and request-latency quantiles in the Prometheus text format,
checked against a 2-peer in-process swarm (CPU, ThreadHub)."""
import re
import urllib.request

import pytest

from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.utils.metrics import MetricsServer, agent_metrics, node_metrics, render

from test_swarm import fresh, run_swarm  # noqa: F401 - fixture re-export

_LV = r'"(?:[^"\\]|\\.)*"'  # a label value with escapes
_SAMPLE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{([a-z_]+=' + _LV + r'(,[a-z_]+=' + _LV + r')*)\})?'
                     r' (-?[0-9.e+-]+|NaN)$')


def parse(text):
    """``{name: [(labels, value)]}``; asserts every line is valid exposition syntax and
    that each family has exactly one HELP and one TYPE line, before its samples."""
    fams, seen_help, seen_type, summaries = {}, set(), set(), set()
    for line in text.strip().split("\n"):
        if line.startswith("# HELP "):
            name = line.split()[2]
            assert name not in seen_help, f"duplicate HELP for {name}"
            seen_help.add(name)
        elif line.startswith("# TYPE "):
            _, _, name, kind = line.split()
            assert kind in ("counter", "gauge", "summary"), line
            if kind == "summary":
                summaries.add(name)
            assert name not in seen_type, f"duplicate TYPE for {name}"
            seen_type.add(name)
        else:
            m = _SAMPLE.match(line)
            assert m, f"bad sample line {line!r}"
            name = m.group(1)
            base = name[:-4] if name.endswith("_sum") else name[:-6] if name.endswith("_count") else None
            assert name in seen_type or (base in seen_type and base in summaries), f"sample before TYPE: {line!r}"
            labels = dict(re.findall(r'([a-z_]+)="((?:[^"\\]|\\.)*)"', m.group(3) or ""))
            fams.setdefault(name, []).append((labels, float(m.group(5))))
    return fams


def value(fams, name, **labels):
    hits = [v for lab, v in fams[name] if all(lab.get(k) == str(x) for k, x in labels.items())]
    assert len(hits) == 1, (name, labels, fams.get(name))
    return hits[0]


@pytest.fixture
def vod():
    return SyntheticHlsOrigin("http://cdn.metrics/vod/", renditions=[Rendition(1_000_000, 640, 360)],
                              num_segments=10, encrypted=True)


def test_render_format_and_merge():
    fams = [("x_total", "counter", "h", [({"a": 'q"\\'}, 3.0)]), ("x_total", "counter", "h", [({"a": "b"}, 1.5)]),
            ("y", "gauge", "g", [({}, 0.25)])]
    text = render(fams)
    parsed = parse(text)
    assert parsed["x_total"] == [({"a": 'q\\"\\\\'}, 3.0), ({"a": "b"}, 1.5)]
    assert "y 0.25\n" in text and "x_total{a=\"b\"} 1.5" in text


def test_swarm_metrics_match_stats(vod):
    nodes, wrappers = {}, {}

    def before(r, node, w):
        node.enable_trace()
        nodes[r], wrappers[r] = node, w

    out = run_swarm(2, vod, before=before)
    seg_total = sum(vod.pools[0].lengths)
    texts = {r: render(node_metrics(nodes[r]) + [f for a in nodes[r]._agents for f in agent_metrics(a)])
             for r in nodes}
    per = {r: parse(t) for r, t in texts.items()}
    cdn = sum(value(per[r], "hlsp2p_cdn_bytes_total", rank=r) for r in per)
    p2p = sum(value(per[r], "hlsp2p_p2p_bytes_total", rank=r) for r in per)
    assert cdn == seg_total and p2p == seg_total  # each segment: one CDN fetch, one peer transfer
    for r, f in per.items():
        st = nodes[r].stats
        assert value(f, "hlsp2p_upload_bytes_total", rank=r) == st["upload"]
        assert value(f, "hlsp2p_rounds_total", rank=r) == st["rounds"] > 0
        assert value(f, "hlsp2p_crc_failures_total", rank=r) == 0
        assert value(f, "hlsp2p_swarm_offload_ratio", rank=r) == pytest.approx(out[r]["offload"]) == pytest.approx(0.5)
        assert value(f, "hlsp2p_world_size", rank=r) == 2
        assert value(f, "hlsp2p_cache_capacity_bytes", rank=r) == 128 << 20
        assert 0 < value(f, "hlsp2p_cache_used_bytes", rank=r) <= 128 << 20
        assert value(f, "hlsp2p_cache_entries", rank=r) >= 1
        assert sum(v for _, v in f["hlsp2p_phase_calls_total"]) > 0
        srcs = {lab["source"] for lab, _ in f["hlsp2p_request_latency_seconds"]}
        assert srcs and srcs <= {"cdn", "p2p", "cache"}
        for lab, v in f["hlsp2p_request_latency_seconds"]:
            assert v >= 0
        # summary _sum / _count per source, consistent with the trace log
        summ = nodes[r].trace.latency_summary()
        for src in srcs:
            assert value(f, "hlsp2p_request_latency_seconds_count", source=src) == summ[src].count > 0
            assert value(f, "hlsp2p_request_latency_seconds_sum", source=src) == pytest.approx(summ[src].sum_ms / 1e3)
        # the reference stats object, exported per agent (labelled by rank and attach index)
        assert value(f, "hlsp2p_agent_bytes_total", source="cdn", rank=r, agent=0) == out[r]["stats"]["cdn"]
        assert value(f, "hlsp2p_agent_bytes_total", source="p2p", rank=r, agent=0) == out[r]["stats"]["p2p"]


def test_agent_labels_distinguish_players_on_one_node():
    """Two agents on one node watching the same content: distinct label sets per agent."""

    class _A:
        def __init__(self, cdn):
            self.stats = {"cdn": cdn, "p2p": 0, "upload": 0, "peers": 1}
            self.contentId = "http://same/stream.m3u8"

    fams = parse(render(agent_metrics(_A(1), 0, rank=3) + agent_metrics(_A(2), 1, rank=3)))
    assert value(fams, "hlsp2p_agent_bytes_total", source="cdn", agent=0, rank=3) == 1
    assert value(fams, "hlsp2p_agent_bytes_total", source="cdn", agent=1, rank=3) == 2
    labs = [tuple(sorted(lab.items())) for lab, _ in fams["hlsp2p_agent_peers"]]
    assert len(set(labs)) == 2


def test_scrape_while_rounds_run(vod, monkeypatch):
    """The endpoint is scraped from its own thread while the swarm keeps running rounds
    (and appending trace records): every scrape parses, none raises."""
    import threading

    scrapes, errors, stop = [], [], threading.Event()

    def scraper(node):
        while not stop.is_set():
            try:
                scrapes.append(parse(render(node_metrics(node))))
            except Exception as e:  # noqa: BLE001
                errors.append(e)
                return
            stop.wait(0.002)  # a scrape every few ms: far more often than any real scraper

    ths = []

    def before(r, node, w):
        node.enable_trace()
        if r == 0:
            t = threading.Thread(target=scraper, args=(node,), daemon=True)
            t.start()
            ths.append(t)

    try:
        run_swarm(2, vod, before=before)
    finally:
        stop.set()
        for t in ths:
            t.join(10)
    assert not errors, errors
    assert len(scrapes) >= 2
    assert any("hlsp2p_request_latency_seconds" in f for f in scrapes)


def test_metrics_port_taken_does_not_fail_the_node(vod):
    """A taken metricsPort logs a warning and the node runs on without the endpoint."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen(1)
    taken = s.getsockname()[1]
    nodes = {}
    try:
        # rank r binds taken + r: rank 0 collides, rank 1 (taken + 1) is most likely free
        out = run_swarm(2, vod, before=lambda r, node, w: nodes.setdefault(r, node),
                        cfg_extra={"metricsPort": taken})
    finally:
        s.close()
    assert all(o["ok"] for o in out.values())
    assert nodes[0].closed and nodes[0].metrics_server is None


def test_metrics_server_scrape(vod):
    nodes = {}
    run_swarm(2, vod, before=lambda r, node, w: nodes.setdefault(r, node))
    srv = MetricsServer(nodes[0], port=0, agents=[])
    try:
        with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/metrics", timeout=10) as resp:
            assert resp.status == 200
            assert resp.headers["Content-Type"].startswith("text/plain; version=0.0.4")
            fams = parse(resp.read().decode())
        assert value(fams, "hlsp2p_rounds_total", rank=0) == nodes[0].stats["rounds"]
        with pytest.raises(urllib.error.HTTPError) as ei:
            urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/nope", timeout=10)
        assert ei.value.code == 404
    finally:
        srv.close()


def test_metrics_port_from_p2p_config(vod):
    """``p2pConfig.gpuSwarm.metricsPort`` starts the endpoint with the node and ``close()``
    stops it."""
    scraped, nodes = {}, {}

    def before(r, node, w):
        nodes[r] = node
        assert node.metrics_server is not None
        with urllib.request.urlopen(f"http://127.0.0.1:{node.metrics_server.port}/metrics", timeout=10) as resp:
            scraped[r] = parse(resp.read().decode())

    run_swarm(2, vod, before=before, cfg_extra={"metricsPort": 0})
    for r in (0, 1):
        assert value(scraped[r], "hlsp2p_world_size", rank=r) == 2
        assert nodes[r].closed and nodes[r].metrics_server is None


@pytest.mark.gpu
def test_metrics_on_gpu_node():
    """A 1-rank node on the MI355X (HBM arena, native kernels): scrape after a 4-segment AES
    playback; the counters match the node and the arena is reported as device memory."""
    import torch

    from hlsjs_p2p_wrapper_amd import Hls
    from hlsjs_p2p_wrapper_amd.agent import current_node, set_current_node
    from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
    from hlsjs_p2p_wrapper_amd.ops import _native
    from hlsjs_p2p_wrapper_amd.player import MediaElement

    _native.device()  # the gfx950 kernels must load
    clear_origins()
    set_current_node(None)
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.gpumetrics/vod/", renditions=[Rendition(2_000_000, 1280, 720)],
                                num_segments=4, encrypted=True, pin_memory=True)
    p2p = {"streamrootKey": "m", "gpuSwarm": {"device": "cuda:0", "cacheBytes": 64 << 20, "metricsPort": 0,
                                              "trace": True}}
    hls = Hls({"transmuxDevice": "cuda:0"}, p2p)
    node = current_node()
    try:
        media = MediaElement()
        buffered = []
        hls.on(Hls.Events.FRAG_BUFFERED, lambda e, d: buffered.append(d["frag"].sn))
        hls.loadSource(origin.master_url())
        hls.attachMedia(media)
        hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
        assert loop.run_until(lambda: len(buffered) == 4, timeout_ms=120_000), buffered
        torch.cuda.synchronize()
        node = current_node()
        assert node.arena.is_cuda
        with urllib.request.urlopen(f"http://127.0.0.1:{node.metrics_server.port}/metrics", timeout=10) as resp:
            fams = parse(resp.read().decode())
        assert value(fams, "hlsp2p_cdn_bytes_total", rank=0) == node.stats["cdn"] == sum(origin.pools[0].lengths)
        assert value(fams, "hlsp2p_cdn_segments_total", rank=0) == 4
        assert value(fams, "hlsp2p_cache_used_bytes", rank=0) >= node.stats["cdn"]
        assert {lab["source"] for lab, _ in fams["hlsp2p_request_latency_seconds"]} == {"cdn"}
        assert value(fams, "hlsp2p_request_latency_seconds_count", source="cdn") == 4
    finally:
        hls.destroy()
        if node is not None:
            node.close()
            assert node.metrics_server is None
        clear_origins()
        set_current_node(None)


def test_healthz_reports_rounds_and_failures():
    """``GET /healthz`` (a serving fleet's liveness probe): ``starting`` before the first round,
    ``ok`` once rounds complete, and HTTP 503 ``failed`` with the reason once the node saw a
    divergence; the ``node_failed`` / ``seconds_since_last_round`` gauges follow."""
    import json
    import urllib.error

    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
    from hlsjs_p2p_wrapper_amd.parallel.comm import LocalComm

    node = SwarmNode(LocalComm(), device="cpu", cache_bytes=1 << 24, auto_tick=False)
    srv = MetricsServer(node, port=0, agents=[])

    def get():
        try:
            with urllib.request.urlopen(f"http://127.0.0.1:{srv.port}/healthz", timeout=10) as resp:
                return resp.status, json.loads(resp.read())
        except urllib.error.HTTPError as e:
            return e.code, json.loads(e.read())

    try:
        code, h = get()
        assert code == 200 and h["status"] == "starting" and h["seconds_since_last_round"] is None
        node.tick()
        code, h = get()
        assert code == 200 and h["status"] == "ok" and h["round"] == 1 and h["seconds_since_last_round"] >= 0
        fams = parse(srv.text())
        assert value(fams, "hlsp2p_node_failed", rank=0) == 0
        assert value(fams, "hlsp2p_seconds_since_last_round", rank=0) >= 0
        node._diverged("replica digest mismatch (test)")
        code, h = get()
        assert code == 503 and h["status"] == "failed" and "digest mismatch" in h["reason"]
        assert value(parse(srv.text()), "hlsp2p_node_failed", rank=0) == 1
    finally:
        srv.close()
        node.close()
