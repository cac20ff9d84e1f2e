"""P2PLoader contract: port of ``test/html/p2p-loader-generator.js`` (real engine + CDN-only
agent over a bandwidth-shaped origin) plus unit tests of every SURVEY §A.3 rule."""
from types import SimpleNamespace

import numpy as np
import pytest

from hlsjs_p2p_wrapper_amd.integration.p2p_loader import p2p_loader_generator
from hlsjs_p2p_wrapper_amd.net import Shaper, clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import StaticOrigin
from hlsjs_p2p_wrapper_amd.player.hls import Hls
from hlsjs_p2p_wrapper_amd.utils.events import JsObject
from mocks import HlsjsWrapperMock, HlsMock

FRAG_SIZE = 245528  # test/html/p2p-loader-generator.js:82
BASE = "http://www.streambox.test/playlists/test_001/"
URL1 = BASE + "stream_110k_48k_416x234_000.ts"


@pytest.fixture
def origin():
    clear_origins()
    data = np.random.default_rng(3).integers(0, 256, FRAG_SIZE, dtype=np.uint8)
    o = StaticOrigin(BASE, {"stream_110k_48k_416x234_000.ts": data})
    yield o
    clear_origins()
    Shaper.reset()


def _create_hls():
    wrapper = HlsjsWrapperMock()
    P2PLoader = p2p_loader_generator(wrapper)
    hls = Hls({"fLoader": P2PLoader, "debug": True})
    wrapper.hls = hls
    return hls, wrapper


def _frag(url, level=0):
    return SimpleNamespace(loadCounter=1, url=url, level=level, sn=None, start=0.0, duration=10.0, loaded=0,
                           byteRangeStartOffset=None, byteRangeEndOffset=None, decryptdata=None)


def test_load_success_events_stats_and_abr(origin):
    loop = new_event_loop("virtual")
    Shaper.maxBandwidth = 512  # kbit/s (test/html/p2p-loader-generator.js:37)
    hls, _ = _create_hls()
    hls.levelController._levels = HlsMock(1, False).levels
    frag = _frag(URL1)
    loaded_events, progress = [], []
    hls.on(Hls.Events.FRAG_LOADED, lambda e, d: loaded_events.append(d))
    hls.on(Hls.Events.FRAG_LOAD_PROGRESS, lambda e, d: progress.append(d["frag"] is frag))
    hls.trigger(Hls.Events.FRAG_LOADING, {"frag": frag})
    assert loop.run_until(lambda: loaded_events, timeout_ms=60_000)
    d = loaded_events[0]
    st = d["stats"]
    assert d["payload"].numel() == FRAG_SIZE
    assert st.trequest >= 0 and st.tfirst > st.trequest and st.tload > st.tfirst
    assert st.loaded == FRAG_SIZE and d["frag"].loaded == FRAG_SIZE
    assert progress and all(progress)
    assert len(loaded_events) == 1
    est_bw = 8 * FRAG_SIZE / ((st.tload - st.trequest) / 1000.0)
    assert hls.abrController.bwEstimator.getEstimate() / est_bw == pytest.approx(1, abs=0.01)


def test_load_failure_triggers_error(origin):
    loop = new_event_loop("virtual")
    hls, _ = _create_hls()
    hls.levelController._levels = HlsMock(1, False).levels
    errors = []
    hls.on(Hls.Events.ERROR, lambda e, d: errors.append(d))
    hls.trigger(Hls.Events.FRAG_LOADING, {"frag": _frag(URL1 + "foo")})
    assert loop.run_until(lambda: errors, timeout_ms=600_000)
    assert len(errors) == 1
    assert errors[0]["details"] == Hls.ErrorDetails.FRAG_LOAD_ERROR
    assert errors[0]["response"].target.status == 404


# ---------------------------------------------------------------- scripted-agent unit tests
class ScriptedAgent:
    StreamTypes = JsObject(HLS="hls")

    def __init__(self):
        self.calls = []
        self.aborted = 0

    def getSegment(self, reqInfo, callbacks, segmentView):
        self.calls.append((reqInfo, callbacks, segmentView))
        agent = self

        class H:
            def abort(self_inner):
                agent.aborted += 1
        return H()


def _unit():
    loop = new_event_loop("virtual")
    loop.advance(1000)
    agent = ScriptedAgent()
    wrapper = SimpleNamespace(peerAgentModule=agent,
                              hls=SimpleNamespace(levels=[SimpleNamespace(urlId=1), SimpleNamespace(urlId=0)]))
    L = p2p_loader_generator(wrapper)
    return loop, agent, wrapper, L


def _load(L, frag=None, **kw):
    rec = JsObject(success=[], error=[], timeout=[], progress=[])
    ldr = L({"xhrSetup": kw.get("xhrSetup")})
    frag = frag or SimpleNamespace(sn=7, level=0, start=28.0, byteRangeStartOffset=None, byteRangeEndOffset=None)
    ldr.load("http://x/seg7.ts", "arraybuffer", lambda e, s: rec.success.append((e, dict(s))),
             lambda e: rec.error.append(e), lambda e, s: rec.timeout.append(dict(s)), kw.get("timeout", 20000),
             kw.get("maxRetry", 2), kw.get("retryDelay", 1000), lambda e, s: rec.progress.append(dict(s)), frag)
    return ldr, rec


def test_guards():
    loop, agent, wrapper, L = _unit()
    ldr = L(None)
    with pytest.raises(Exception, match="expects progress-callback"):
        ldr.load("u", "arraybuffer", None, None, None, 1, 0, 0, None, object())
    with pytest.raises(Exception, match="can only be used for media fragments"):
        ldr.load("u", "arraybuffer", None, None, None, 1, 0, 0, lambda *a: None, None)
    wrapper.peerAgentModule = None
    with pytest.raises(Exception, match="Peer agent is not existing yet"):
        ldr.load("u", "arraybuffer", None, None, None, 1, 0, 0, lambda *a: None, object())


def test_segment_view_track_and_request_info():
    loop, agent, wrapper, L = _unit()
    _load(L, xhrSetup=lambda xhr, url: xhr.setRequestHeader("X-Token", "abc"))
    reqInfo, callbacks, sv = agent.calls[0]
    assert reqInfo["url"] == "http://x/seg7.ts" and reqInfo["headers"] == {"X-Token": "abc"}
    assert sv.sn == 7 and sv.time == 28.0 and sv.trackView.level == 0 and sv.trackView.urlId == 1
    assert sv.viewToString() == "L0U1S7"


def test_byte_range_header_exclusive_to_inclusive():
    loop, agent, wrapper, L = _unit()
    frag = SimpleNamespace(sn=1, level=1, start=0.0, byteRangeStartOffset=100, byteRangeEndOffset=600)
    ldr, _ = _load(L, frag)
    assert agent.calls[0][0]["headers"]["Range"] == "bytes=100-599"
    assert ldr.byteRange == "100-600"


def test_p2p_timing_rewrite():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L)
    cb = agent.calls[0][1]
    loop.advance(500)
    now = loop.now()
    cb.onProgress({"p2pDownloaded": 3000, "cdnDownloaded": 0, "p2pDuration": 30.0, "cdnDuration": 0.0})
    st = rec.progress[-1]
    assert st["loaded"] == 3000
    assert st["trequest"] == pytest.approx(now - 30.0)
    assert st["tfirst"] == pytest.approx(now - 30.0 + 10)  # min(round(30/2), 10)
    # a second progress event does not rewrite again
    loop.advance(5)
    cb.onProgress({"p2pDownloaded": 3000, "cdnDownloaded": 100, "p2pDuration": 30.0, "cdnDuration": 1.0})
    assert rec.progress[-1]["tfirst"] == st["tfirst"]
    assert rec.progress[-1]["loaded"] == 3100
    loop.advance(1)
    cb.onSuccess("DATA")
    e, s = rec.success[0]
    assert e.currentTarget.response == "DATA" and s["tload"] == loop.now()
    assert s["trequest"] < s["tfirst"] < s["tload"]


def test_small_p2p_duration_rtt_is_half():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L)
    now = loop.now()
    agent.calls[0][1].onProgress({"p2pDownloaded": 10, "p2pDuration": 6.0, "cdnDuration": 0.0})
    assert rec.progress[-1]["tfirst"] == pytest.approx(now - 6.0 + 3)


def test_cdn_progress_sets_tfirst_now():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L)
    loop.advance(200)
    agent.calls[0][1].onProgress({"cdnDownloaded": 500})
    assert rec.progress[-1]["tfirst"] == loop.now()
    assert rec.progress[-1]["trequest"] == pytest.approx(1000.0)


def test_retry_with_exponential_backoff_then_error():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L, maxRetry=3, retryDelay=40000)
    delays = []
    for i in range(3):
        t0 = loop.now()
        agent.calls[-1][1].onError(SimpleNamespace(status=503))
        assert ldr.peerAgentLoader is None and ldr.retryTimeout is not None
        n = len(agent.calls)
        loop.run_until(lambda: len(agent.calls) > n, timeout_ms=200_000)
        delays.append(loop.now() - t0)
    assert delays == [40000, 64000, 64000]  # x2 per retry, capped at 64 s
    assert ldr.stats.retry == 3
    agent.calls[-1][1].onError(SimpleNamespace(status=503))
    assert len(rec.error) == 1 and rec.error[0].target.status == 503


def test_abort_ignores_late_callbacks_and_cancels_retry():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L)
    cb = agent.calls[0][1]
    ldr.abort()
    assert agent.aborted == 1 and ldr.stats.aborted is True
    cb.onSuccess("late")
    cb.onError(SimpleNamespace(status=500))
    assert rec.success == [] and rec.error == []
    # abort during a retry wait cancels the pending retry
    ldr2, rec2 = _load(L)
    agent.calls[-1][1].onError(SimpleNamespace(status=500))
    n = len(agent.calls)
    ldr2.abort()
    loop.run_for(100_000)
    assert len(agent.calls) == n


def test_unfinalized_request_is_detected():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L)
    with pytest.raises(Exception, match="P2P loader was not reset correctly"):
        ldr.loadInternal()


def test_timeout_calls_on_timeout_without_aborting():
    loop, agent, wrapper, L = _unit()
    ldr, rec = _load(L, timeout=500)
    loop.run_for(600)
    assert len(rec.timeout) == 1 and agent.aborted == 0


def test_generator_returns_new_class_each_time():
    _, _, wrapper, _ = _unit()
    assert p2p_loader_generator(wrapper) is not p2p_loader_generator(wrapper)
