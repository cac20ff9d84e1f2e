"""Real-CDN path (``net/network.py``): the swarm in front of an actual HTTP server.

A ``ThreadingHTTPServer`` on 127.0.0.1 serves a packaged HLS stream (the synthetic origin's
playlists, key and MPEG-TS segments, with ``Range`` support) and counts the bytes it sends
per resource, so the tests can check what crossed the "network": the player plays it
through ``HttpOrigin``, and a swarm downloads every segment from it exactly once (the
planner's STAGE rows), the other peers getting their copies over the swarm.
"""
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import numpy as np
import pytest
import torch

from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net import http as nhttp
from hlsjs_p2p_wrapper_amd.net.network import HttpOrigin
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops._native import runtime

from test_swarm import run_swarm


class _Cdn:
    """HTTP server in front of a synthetic origin; ``sent[path]`` = body bytes sent."""

    def __init__(self, num_segments=10):
        cdn = self
        self.sent = {}
        self.ignore_range = False  # answer a Range request with 200 and the whole resource
        self.bad_content_range = False  # answer 206 with a Content-Range of other bytes
        self.lock = threading.Lock()

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def do_GET(self):  # noqa: N802 - http.server API
                path = self.path.split("?")[0]
                rel = path[len("/vod/"):] if path.startswith("/vod/") else None
                rng = None
                r = self.headers.get("Range")
                if r and not cdn.ignore_range:
                    s, e = r.split("=")[1].split("-")
                    rng = (int(s), int(e) if e else None)
                try:
                    if rel is None:
                        raise nhttp.HttpError(404, path)
                    resp = cdn.origin.serve(rel, cdn.base + rel, rng, {}, False)
                except nhttp.HttpError as e:
                    self.send_response(e.status)
                    self.send_header("Content-Length", "0")
                    self.end_headers()
                    return
                body = resp.body
                if isinstance(body, str):
                    data = body.encode()
                elif isinstance(body, torch.Tensor):
                    data = body.numpy().tobytes()
                else:
                    data = bytes(body)
                self.send_response(resp.status)
                if rng is not None:
                    s0 = rng[0] + (1 if cdn.bad_content_range else 0)
                    self.send_header("Content-Range", f"bytes {s0}-{s0 + len(data) - 1}/*")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)
                with cdn.lock:
                    cdn.sent[rel] = cdn.sent.get(rel, 0) + len(data)

            def log_message(self, *args):
                pass

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.srv.daemon_threads = True
        self.base = f"http://127.0.0.1:{self.srv.server_address[1]}/vod/"
        self.origin = SyntheticHlsOrigin(self.base, renditions=[Rendition(1_000_000, 640, 360)],
                                         num_segments=num_segments, encrypted=True, register=False,
                                         pin_memory=False)
        self.thread = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.thread.start()

    def ts_bytes(self):
        with self.lock:
            return sum(v for k, v in self.sent.items() if k.endswith(".ts"))

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


@pytest.fixture
def cdn():
    clear_origins()
    c = _Cdn()
    yield c
    c.close()
    nhttp.enable_network(False)
    clear_origins()


def test_http_origin_text_binary_range_and_errors(cdn):
    o = HttpOrigin(cdn.base, pin_memory=False, register=False, workers=2)
    try:
        r = o.serve("master.m3u8", cdn.base + "master.m3u8", None, {}, False)
        assert r.status == 200 and r.body.startswith("#EXTM3U")
        key = o.serve("key.bin", cdn.base + "key.bin", None, {}, False)
        assert key.body.numpy()[:16].tobytes() == cdn.origin.key
        path = "r0/seg3.ts"
        data, off, n, _ = cdn.origin.resource(path)
        ref = data[off:off + n].numpy()
        done = threading.Event()
        res = {}

        def cb(length, err):
            res["n"], res["err"] = length, err
            done.set()

        o.stage(path, cdn.base + path, None, {}, cb)
        assert done.wait(10) and res["err"] is None and res["n"] == n
        t, toff, tn, _ = o.resource_range(path, None)
        assert np.array_equal(t[toff:toff + tn].numpy(), ref)
        done.clear()
        o.stage(path, cdn.base + path, (188, 188 * 4 - 1), {}, cb)  # inclusive range
        assert done.wait(10) and res["n"] == 188 * 3
        t, toff, tn, _ = o.resource_range(path, (188, 188 * 4 - 1))
        assert np.array_equal(t[:tn].numpy(), ref[188:188 * 4])
        o.release(path, None)
        assert o.staged_size(path) is None
        with pytest.raises(nhttp.HttpError) as e:
            o.resource_range(path)
        assert e.value.status == 503
        done.clear()
        o.stage("r0/seg999.ts", cdn.base + "r0/seg999.ts", None, {}, cb)
        assert done.wait(10) and res["n"] is None and res["err"].status == 404
    finally:
        o.close()


def test_range_request_against_a_cdn_that_ignores_range(cdn):
    """A CDN answering a Range request with 200 + the whole file: only the requested bytes are
    staged; a 206 whose Content-Range names other bytes is an error, not silent corruption."""
    o = HttpOrigin(cdn.base, pin_memory=False, register=False, workers=2)
    path = "r0/seg2.ts"
    data, off, n, _ = cdn.origin.resource(path)
    ref = data[off:off + n].numpy()
    done = threading.Event()
    res = {}

    def cb(length, err):
        res["n"], res["err"] = length, err
        done.set()

    try:
        cdn.ignore_range = True
        rng = (376, 376 + 188 * 5 - 1)
        o.stage(path, cdn.base + path, rng, {}, cb)
        assert done.wait(10) and res["err"] is None and res["n"] == 188 * 5
        t, toff, tn, _ = o.resource_range(path, rng)
        assert tn == 188 * 5 and np.array_equal(t[toff:toff + tn].numpy(), ref[376:376 + 188 * 5])
        cdn.ignore_range = False
        cdn.bad_content_range = True
        done.clear()
        o.stage(path, cdn.base + path, (0, 187), {}, cb)
        assert done.wait(10) and res["n"] is None and res["err"].status == 502
    finally:
        o.close()


def test_stage_after_close_completes_with_an_error(cdn):
    """Work submitted to (or cancelled by) a closed origin still calls back, so the node's loop
    hold is always released."""
    o = HttpOrigin(cdn.base, pin_memory=False, register=False, workers=1)
    o.close()
    got = []
    o.stage("r0/seg1.ts", cdn.base + "r0/seg1.ts", None, {}, lambda n, e: got.append((n, e)))
    o.serve_async("master.m3u8", cdn.base + "master.m3u8", None, {}, False, lambda r, e: got.append((r, e)))
    assert len(got) == 2 and all(x is None and e.status == 0 for x, e in got)


def test_network_error_is_status_zero():
    o = HttpOrigin("http://127.0.0.1:9/", pin_memory=False, register=False, workers=1, timeout_s=2)
    try:
        with pytest.raises(nhttp.HttpError) as e:
            o.serve("x.m3u8", "http://127.0.0.1:9/x.m3u8", None, {}, False)
        assert e.value.status == 0
    finally:
        o.close()


def test_loop_waits_for_threadsafe_work_on_a_virtual_clock():
    loop = new_event_loop("virtual")
    fired = []
    loop.set_timeout(lambda: fired.append("timer"), 1000)
    loop.hold()

    def worker():
        loop.call_soon_threadsafe(fired.append, "net")
        loop.release()

    threading.Timer(0.05, worker).start()
    assert loop.run_until(lambda: len(fired) == 2, timeout_ms=5000)
    assert fired == ["net", "timer"]  # the clock did not jump past the outstanding work


def test_planner_stage_rows():
    rt = runtime()
    d = rt.Directory()
    key = [7, 0, 0, 42]
    flags = np.array([rt.FLAG_ONLINE | 2 | 4 | 8] * 2, dtype=np.int64)  # online, up, down, dedup

    def plan(rows):
        return rt.plan_round(d, np.array(rows, dtype=np.int64).reshape(-1, 8), flags, 2)

    # nobody staged: the seeder stages it (src -2), the other wanter waits
    p = plan([key + [0, 1, 0, 2], key + [0, 5, 1, 2]])
    assert p.shape[0] == 1 and p[0, 5] == -2
    # rank 1 staged (size known): it fetches (CDN row); rank 0 reserved nothing for the body
    # (size 0), so it is not sent a copy this round -- it waits and reserves next round
    p = plan([key + [0, 1, 0, 2], key + [3000, 5, 1, 0]])
    cdn = p[p[:, 5] == -1]
    fwd = p[p[:, 5] == 1]
    assert cdn.tolist() == [key + [3000, -1, 1, 5, 0, 0]]
    assert fwd.tolist() == []
    # once rank 0 announces the length it reserved (its node read it from the directory),
    # the seeder forwards in the same round
    p = plan([key + [3000, 1, 0, 2], key + [3000, 5, 1, 0]])
    assert p[p[:, 5] == 1].tolist() == [key + [3000, 1, 0, 1, 1, 0]]
    # a lone unstaged want without de-duplication: stage row for itself
    p = plan([key + [0, 9, 0, 2]])
    assert p.tolist() == [key + [0, -2, 0, 9, 0, 0]]
    # one wanter is downloading it (staging): nobody else is told to, everybody waits
    assert plan([key + [0, 1, 0, 2 | 4], key + [0, 5, 1, 2]]).shape[0] == 0
    assert plan([key + [0, 9, 0, 2 | 4]]).shape[0] == 0
    # a holder exists: an unstaged wanter that reserved too little waits, one that reserved
    # enough gets the P2P copy
    d.apply(1, np.array([key + [3000]], dtype=np.int64), np.zeros((0, 4), dtype=np.int64))
    assert plan([key + [0, 1, 0, 2]]).shape[0] == 0
    assert plan([key + [3000, 1, 0, 2]]).tolist() == [key + [3000, 1, 0, 1, 0, 0]]


def test_player_plays_from_an_http_cdn(cdn):
    out = run_swarm(1, cdn.origin, until=39.0, cfg_extra={"network": {"pin_memory": False, "workers": 4}})
    assert out[0]["ok"]
    seg_total = sum(cdn.origin.pools[0].lengths)
    assert cdn.ts_bytes() == seg_total and out[0]["stats"]["cdn"] == seg_total
    assert cdn.sent.get("master.m3u8") and cdn.sent.get("key.bin") == 16


def test_swarm_downloads_each_segment_once(cdn):
    out = run_swarm(3, cdn.origin, until=39.0, cfg_extra={"network": {"pin_memory": False, "workers": 4}})
    assert all(o["ok"] for o in out.values())
    seg_total = sum(cdn.origin.pools[0].lengths)
    assert cdn.ts_bytes() == seg_total  # the network carried every segment once
    assert sum(o["stats"]["cdn"] for o in out.values()) == seg_total
    assert sum(o["stats"]["p2p"] for o in out.values()) == 2 * seg_total
    assert out[0]["offload"] == pytest.approx(2 / 3)


@pytest.mark.gpu
def test_swarm_on_gpu_from_an_http_cdn(cdn):
    """Two GPU peers (one MI355X, thread backend) behind the HTTP CDN: staged bodies land in
    pinned host memory on the worker threads and reach HBM through the round's CDN DMA."""
    out = run_swarm(2, cdn.origin, until=30.0,
                    cfg_extra={"device": "cuda:0", "network": {"pin_memory": True, "workers": 4}})
    assert all(o["ok"] for o in out.values())
    seg_total = sum(cdn.origin.pools[0].lengths)
    assert cdn.ts_bytes() == seg_total
    assert sum(o["stats"]["p2p"] for o in out.values()) == seg_total
