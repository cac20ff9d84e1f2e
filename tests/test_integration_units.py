"""Ports of ``test/player-interface.js``, ``test/xhr-setup.js``, ``test/api.js`` and
``test/hls-controllers.js`` (the stats-contract anchors of BASELINE.md)."""
import pytest

from hlsjs_p2p_wrapper_amd.api.wrapper_private import HlsjsP2PWrapperPrivate
from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
from hlsjs_p2p_wrapper_amd.integration.player_interface import PlayerInterface
from hlsjs_p2p_wrapper_amd.net import new_event_loop
from hlsjs_p2p_wrapper_amd.player.abr import AbrController
from hlsjs_p2p_wrapper_amd.player.controllers import StreamController
from hlsjs_p2p_wrapper_amd.player.events import Events
from hlsjs_p2p_wrapper_amd.utils.events import JsObject
from hlsjs_p2p_wrapper_amd.utils.xhr import extractInfoFromXhrSetup
from mocks import HlsMock


# --- test/player-interface.js:12-30 ------------------------------------------------------
def test_is_live_false_for_vod():
    pi = PlayerInterface(HlsMock(3, False, 1), Events, lambda: None, {}, None, None)  # stale 6-arg call
    assert pi.isLive() is False


def test_is_live_throws_before_master():
    with pytest.raises(Exception, match="Called isLive before the master playlist was parsed"):
        PlayerInterface(HlsMock(0, False), Events, lambda: None).isLive()


def test_is_live_throws_before_level_playlist():
    with pytest.raises(Exception, match="Called isLive before any levelplaylist was parsed"):
        PlayerInterface(HlsMock(3, None), Events, lambda: None).isLive()


def test_buffer_level_max_and_margin():
    hls = HlsMock(3, True, 0)
    pi = PlayerInterface(hls, Events, lambda: None)
    hls.config.liveSyncDuration = None
    hls.config.maxBufferLength = 42
    assert pi.getBufferLevelMax() == 42
    hls.config.liveSyncDuration = 30
    assert pi.getBufferLevelMax() == 30
    pi.setBufferMarginLive(12)
    assert hls.config.maxBufferSize == 0 and hls.config.maxBufferLength == 12
    hls.config.liveSyncDuration = None
    hls.config.maxBufferLength = -1
    with pytest.raises(Exception, match=r"hlsjsConfig.maxBufferLength must be greater than "
                                        r"p2pConfig.liveMinBufferMargin"):
        pi.getBufferLevelMax()


def test_track_change_and_dispose_events():
    class H(HlsMock):
        def __init__(self):
            super().__init__(3, False, 1)
            self.handlers = {}

        def on(self, ev, fn):
            self.handlers[ev] = fn

    h = H()
    disposed = []
    pi = PlayerInterface(h, Events, lambda: disposed.append(1))
    seen = []
    pi.addEventListener("onTrackChange", lambda d: seen.append(d["video"].viewToString()))
    pi.addEventListener("somethingElse", lambda d: seen.append("bad"))  # silently ignored
    h.levels[2].urlId = 1
    h.handlers[Events.LEVEL_SWITCH](Events.LEVEL_SWITCH, {"level": 2})
    assert seen == ["L2U1"]
    h.handlers[Events.DESTROYING](Events.DESTROYING, {})
    assert disposed == [1]


# --- test/xhr-setup.js:3-64 --------------------------------------------------------------
def test_xhr_forbidden_method():
    with pytest.raises(Exception, match="forbidden property/method of XHR mock"):
        extractInfoFromXhrSetup(lambda xhr, url: xhr.open())


def test_xhr_forbidden_write():
    def setup(xhr, url):
        xhr.onloadend = lambda: None
    with pytest.raises(Exception):
        extractInfoFromXhrSetup(setup)


def test_xhr_forbidden_read():
    with pytest.raises(Exception):
        extractInfoFromXhrSetup(lambda xhr, url: xhr.response)


def test_xhr_headers_and_credentials():
    def setup(xhr, url):
        assert xhr.withCredentials is False
        xhr.withCredentials = True
        xhr.setRequestHeader("SomeHeader", "SomeValue")
    info = extractInfoFromXhrSetup(setup)
    assert info["headers"] == {"SomeHeader": "SomeValue"}
    assert info["withCredentials"] is True


def test_xhr_url_passthrough_and_base_headers():
    urls = []

    def setup(xhr, url):
        xhr.setRequestHeader("bla", "bla")
        urls.append(url)
    info = extractInfoFromXhrSetup(setup, "foobar", {"foo": "bar"})
    assert urls == ["foobar"]
    assert info["headers"] == {"foo": "bar", "bla": "bla"}


def test_xhr_no_setup():
    assert extractInfoFromXhrSetup(None, "u") == {"headers": {}, "withCredentials": False}


# --- test/api.js ---------------------------------------------------------------------------
def test_version_property(monkeypatch):
    monkeypatch.setenv("HLSJS_P2P_VERSION", "foobar")
    assert HlsjsP2PWrapperPrivate.version == "foobar"
    assert HlsjsP2PWrapper.version == "foobar"


# --- test/hls-controllers.js:11-82 ---------------------------------------------------------
class _HlsForAbr(HlsMock):
    def __init__(self, loop):
        super().__init__(5, False, 0, False)
        self.loop = loop


def test_abr_estimate_from_loader_stats():
    loop = new_event_loop("virtual")
    loop.advance(5000)
    abr = AbrController(_HlsForAbr(loop))
    frag = JsObject(loadCounter=1, url="http://foo.bar/foo", level=1)
    stats = JsObject(trequest=loop.now() - 1000, loaded=128000)
    abr.onFragLoading({"frag": frag})
    abr.onFragLoaded({"frag": frag, "stats": stats})
    assert abr.bwEstimator.getEstimate() == pytest.approx(1024000, abs=4000)
    assert abr.lastLoadedFragLevel == frag.level


def test_abr_ignores_reloaded_fragment():
    loop = new_event_loop("virtual")
    loop.advance(5000)
    abr = AbrController(_HlsForAbr(loop))
    default = abr.bwEstimator.getEstimate()
    abr.onFragLoaded({"frag": JsObject(loadCounter=2, level=0), "stats": JsObject(trequest=4990, loaded=1 << 30)})
    assert abr.bwEstimator.getEstimate() == default


def test_stream_controller_frag_last_kbps():
    """fragLastKbps = 8 * length / (tbuffered - tfirst) on buffering (≈1024 ± 8)."""
    from hlsjs_p2p_wrapper_amd.player.hls import Hls

    loop = new_event_loop("virtual")
    loop.advance(10_000)
    hls = Hls({})
    sc: StreamController = hls.streamController
    frag = type("F", (), {"level": 0, "sn": 0, "start": 0.0, "duration": 4.0, "decryptdata": None})()
    stats = JsObject(trequest=loop.now() - 1000, tfirst=loop.now() - 1000, loaded=128000, length=128000)
    sc.inflight[(0, 0)] = frag
    import torch
    z = torch.zeros(0, dtype=torch.uint8)
    sc._on_parsed(frag, stats, {"status": 0, "info": {"video_pid": 256, "video_type": 27, "audio_pid": 257,
                                                     "audio_type": 15, "video_first_pts": -1, "video_last_pts": -1,
                                                     "n_video_pes": 0, "n_audio_pes": 0, "audio_first_pts": -1,
                                                     "audio_last_pts": -1},
                               "video": z, "audio": z, "id3": z, "plain_bytes": 0})
    assert sc.fragLastKbps == pytest.approx(1024, abs=8)
    assert sc.stats is None or True


def test_event_loop_sweeps_cancelled_timers():
    """A long-running peer cancels one fragment-timeout timer per fragment: the timer heap
    must stay bounded by the live timers, and live timers must still fire in order."""
    from hlsjs_p2p_wrapper_amd.net.event_loop import EventLoop

    loop = EventLoop("virtual")
    fired = []
    for i in range(50_000):
        h = loop.set_timeout(lambda: None, 60_000)
        loop.clear_timeout(h)
    for i in range(3):
        loop.set_timeout(fired.append, 10 * (3 - i), i)
    assert len(loop._heap) < 2 * 4096 + 3
    loop.advance(100)
    loop.run_once(block=False)
    assert fired == [2, 1, 0]
