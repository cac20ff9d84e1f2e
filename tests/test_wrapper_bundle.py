"""Wrapper orchestration (C3/C4), bundle (C1/C2) and the full-stack playback tests
ported from ``test/html/bundle.js`` (play, seek, ABR under throttling) — on the CPU
swarm node with a virtual clock."""
import logging

import pytest

from hlsjs_p2p_wrapper_amd import Hls, HlsjsP2PWrapper, HlsjsP2PWrapperPrivate
from hlsjs_p2p_wrapper_amd.agent import set_current_node
from hlsjs_p2p_wrapper_amd.net import Shaper, clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.player import MediaElement
from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine
from hlsjs_p2p_wrapper_amd.utils import ua
from mocks import PeerAgentMock

P2P = {"streamrootKey": "ry-v7xuywnt", "debug": True, "gpuSwarm": {"device": "cpu", "cacheBytes": 96 << 20}}


@pytest.fixture(autouse=True)
def fresh():
    clear_origins()
    set_current_node(None)
    Shaper.reset()
    yield
    Shaper.reset()
    clear_origins()
    set_current_node(None)
    ua.set_user_agent(None)


@pytest.fixture
def vod():
    return SyntheticHlsOrigin("http://cdn.test/vod/", renditions=[Rendition(600_000, 640, 360)], num_segments=20,
                              segment_duration=4.0, encrypted=True)


# ---------------------------------------------------------------- orchestrator errors (§A.1)
def test_private_requires_peer_agent():
    with pytest.raises(Exception, match="Constructor needs DI of PeerAgent"):
        HlsjsP2PWrapperPrivate(Engine, None)


def test_new_media_engine_errors_and_defaults():
    w = HlsjsP2PWrapperPrivate(None, PeerAgentMock)
    with pytest.raises(Exception, match="Can not create Hls.js instance: dependency was not injected"):
        w.newMediaEngine({})
    new_event_loop("virtual")
    w = HlsjsP2PWrapperPrivate(Engine, PeerAgentMock)
    with pytest.raises(Exception, match="`fLoader` in Hls.js config must not be defined"):
        w.newMediaEngine({"fLoader": object})
    user = {"maxBufferLength": 12}
    hls = w.newMediaEngine(user)
    assert user["maxBufferLength"] == 12 and user["maxBufferSize"] == 0 and user["liveSyncDuration"] == 30
    assert hls.config.fLoader is user["fLoader"]  # lodash.defaults mutated the user dict
    user2 = {"liveSyncDurationCount": 5}
    w.newMediaEngine(user2)
    assert "liveSyncDuration" not in user2


def test_start_session_and_create_peer_agent_errors():
    new_event_loop("virtual")
    w = HlsjsP2PWrapperPrivate(Engine, PeerAgentMock)
    hls = w.newMediaEngine({})
    with pytest.raises(Exception, match="p2pConfig must be a valid config object"):
        w.startSession(hls, {}, None, "http://x")
    for bad in ("", 0, "cfg", 5):  # JS `!p2pConfig || typeof p2pConfig !== 'object'`
        with pytest.raises(Exception, match="p2pConfig must be a valid config object"):
            w.startSession(hls, {}, bad, "http://x")
    # ... but an EMPTY object is a valid config in JS ({} is truthy): no Python-falsy rejection
    w2 = HlsjsP2PWrapperPrivate(Engine, PeerAgentMock)
    assert w2.startSession(w2.newMediaEngine({}), {}, {}, "http://x") is not None
    assert w2.hasSession()
    with pytest.raises(Exception, match="Hls.js instance must have valid `url` property"):
        w.createPeerAgent({}, hls, Engine.Events, None)
    with pytest.raises(Exception, match="Need valid Hls.js Events enumeration"):
        w.createPeerAgent({}, hls, None, "http://x")
    w.createPeerAgent({}, hls, Engine.Events, "http://x")
    assert w.hasSession()
    with pytest.raises(Exception, match="Streamroot session already started"):
        w.createPeerAgent({}, hls, Engine.Events, "http://x")
    # startSession with no engine creates one (the reference's latent crash is fixed)
    w2 = HlsjsP2PWrapperPrivate(Engine, PeerAgentMock)
    eng = w2.startSession(None, {}, {"a": 1}, "http://x")
    assert isinstance(eng, Engine) and w2.hasSession()


def test_set_media_element_now_or_on_attaching():
    new_event_loop("virtual")
    w = HlsjsP2PWrapperPrivate(Engine, PeerAgentMock)
    hls = w.newMediaEngine({})
    m = MediaElement()
    hls.attachMedia(m)
    w.createPeerAgent({}, hls, Engine.Events, "http://x")
    assert w.peerAgentModule.media is m
    w.stopSession()
    hls2 = w.newMediaEngine({})
    w.createPeerAgent({}, hls2, Engine.Events, "http://y")
    assert w.peerAgentModule.media is None
    m2 = MediaElement()
    hls2.attachMedia(m2)
    assert w.peerAgentModule.media is m2


def test_media_engine_error_logging(caplog):
    with caplog.at_level(logging.WARNING):
        HlsjsP2PWrapperPrivate.onMediaEngineError("hlsError", {"fatal": True, "type": "networkError",
                                                               "details": "fragLoadError"})
        HlsjsP2PWrapperPrivate.onMediaEngineError("hlsError", {"fatal": False, "type": "mediaError",
                                                               "details": "bufferStalledError"})
    text = caplog.text
    assert "Hls.js fatal error: networkError - fragLoadError" in text
    assert "Hls.js non-fatal error: mediaError - bufferStalledError" in text


# ---------------------------------------------------------------- facade (C3)
def test_facade_stats_toggles_and_loader_snapshot(vod):
    loop = new_event_loop("virtual")
    w = HlsjsP2PWrapper(Engine)
    with pytest.raises(TypeError):
        _ = w.stats  # no session yet
    assert w.P2PLoader is w.P2PLoader  # snapshot taken once
    assert w._wrapper.P2PLoader is not w._wrapper.P2PLoader  # private getter: fresh class
    hls = w.createPlayer({}, P2P)
    media = MediaElement()
    hls.loadSource(vod.master_url())
    hls.attachMedia(media)
    hls.on(Engine.Events.MANIFEST_PARSED, lambda e, d: media.play())
    loop.run_until(lambda: media.currentTime > 2.0, timeout_ms=60_000)
    s = w.stats
    assert set(s) == {"cdn", "p2p", "upload", "peers"} and s["cdn"] > 0 and s["peers"] == 0
    w.p2pDownloadOn = False
    w.p2pUploadOn = False
    assert w.p2pDownloadOn is False and w.p2pUploadOn is False
    hls.destroy()
    assert not w._wrapper.hasSession()  # DESTROYING disposed the agent


def test_legacy_create_sr_module(vod):
    loop = new_event_loop("virtual")
    w = HlsjsP2PWrapper()  # legacy: no DI of the engine
    hls = Engine({"fLoader": w.P2PLoader})
    cfg = {"streamrootKey": "k", "contentId": "mine", "gpuSwarm": P2P["gpuSwarm"]}
    hls.on(Engine.Events.MANIFEST_LOADING, lambda e, d: w.createSRModule(cfg, hls, Engine.Events))
    media = MediaElement()
    hls.loadSource(vod.master_url())
    hls.attachMedia(media)
    hls.on(Engine.Events.MANIFEST_PARSED, lambda e, d: media.play())
    loop.run_until(lambda: media.currentTime > 1.0, timeout_ms=60_000)
    assert cfg["contentId"] is None  # overwritten by the legacy signature (private.js:64)
    assert w._wrapper.peerAgentModule.contentUrl == vod.master_url()
    assert media.currentTime > 1.0


# ---------------------------------------------------------------- bundle (C1/C2)
def test_bundle_statics_read_only_and_support_gate():
    assert Hls.Events is Engine.Events and Hls.ErrorTypes is Engine.ErrorTypes
    assert Hls.DefaultConfig["maxBufferLength"] == 30
    with pytest.raises(AttributeError):
        Hls.Events = None
    ua.set_user_agent("Mozilla/5.0 (Macintosh; Intel Mac OS X 10_12) AppleWebKit/603 (KHTML, like Gecko) "
                      "Version/10.1 Safari/603.1.30")
    assert Hls.isSupported() is False and Hls.getBrowserName() == "Safari"
    ua.set_user_agent("Mozilla/5.0 (Linux; Android 7.0; SM-G930V) AppleWebKit/537.36 Chrome/59.0 Mobile Safari/537.36")
    assert Hls.isSupported() is False
    ua.set_user_agent("Mozilla/5.0 (iPad; CPU OS 10_3 like Mac OS X) AppleWebKit/603 Version/10.0 Mobile Safari/602.1")
    assert Hls.isSupported() is False
    ua.set_user_agent("Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 Chrome/120.0 Safari/537.36")
    assert Hls.isSupported() is True and Hls.getBrowserName() == "Chrome"


def test_bundle_constructor_returns_engine_instance(vod):
    new_event_loop("virtual")
    hls = Hls({"debug": True}, P2P)
    assert isinstance(hls, Engine) and not isinstance(hls, Hls)
    assert hls.config.fLoader.__name__ == "P2PLoader"
    assert hls.config.maxBufferSize == 0 and hls.config.liveSyncDuration == 30


def _start(hls, media, url, cb=None):
    hls.loadSource(url)
    hls.attachMedia(media)

    def parsed(e, d):
        media.volume = 0
        media.play()
        if cb:
            cb()
    hls.on(Hls.Events.MANIFEST_PARSED, parsed)


def test_bundle_plays_from_start(vod):
    loop = new_event_loop("virtual")
    hls = Hls({"debug": True}, P2P)
    media = MediaElement()
    _start(hls, media, vod.master_url())
    assert loop.run_until(lambda: media.currentTime > 1.0, timeout_ms=30_000)


def test_a_fragment_that_never_decrypts_is_retried_with_backoff_then_fatal(vod):
    """Bytes that fail to decrypt (here: a wrong key) are retried like a load error -- back-off,
    up to fragLoadingMaxRetry, then a fatal FRAG_DECRYPT_ERROR -- instead of being reloaded at
    once forever; on each failure the wrapper has the node drop its cached copy, so every retry
    is a fresh CDN fetch."""
    loop = new_event_loop("virtual")
    hls = Hls({"debug": True, "fragLoadingMaxRetry": 2, "fragLoadingRetryDelay": 100}, P2P)
    media = MediaElement()
    errors = []
    hls.on(Hls.Events.ERROR, lambda e, d: errors.append((d.get("details"), d.get("fatal"))))

    def wrong_key(e, d):
        for uri in list(hls.keyLoader.keys):
            hls.keyLoader.keys[uri] = bytes(16)
    hls.on(Hls.Events.KEY_LOADED, wrong_key)
    _start(hls, media, vod.master_url())
    t0 = loop.now()
    assert loop.run_until(lambda: any(f for _, f in errors), timeout_ms=60_000)
    assert errors[-1] == ("fragDecryptError", True) and len(errors) == 3
    assert [f for _, f in errors] == [False, False, True]
    assert loop.now() - t0 >= 300  # two back-offs: 100 ms, then 200 ms
    from hlsjs_p2p_wrapper_amd.agent import current_node

    node = current_node()
    assert node.stats["invalidated"] >= 2 and node.stats["cdn_segments"] >= 3
    hls.destroy()


def test_bundle_recovers_from_a_media_error_and_keeps_playing(vod):
    """hls.js's ``recoverMediaError()`` (detach + re-attach the media element) mid-playback:
    buffering and the playback clock resume; the level statics of hls.js answer."""
    loop = new_event_loop("virtual")
    hls = Hls({"debug": True}, P2P)
    media = MediaElement()
    _start(hls, media, vod.master_url())
    assert loop.run_until(lambda: media.currentTime > 5.0, timeout_ms=30_000)
    assert hls.firstLevel == 0 and hls.startLevel == 0
    hls.startLevel = 0
    hls.recoverMediaError()
    assert hls.media is media
    assert loop.run_until(lambda: media.currentTime > 20.0, timeout_ms=60_000)
    hls.swapAudioCodec()
    assert hls.audioCodecSwap
    hls.destroy()


def test_bundle_seeks_to_30s(vod):
    loop = new_event_loop("virtual")
    hls = Hls({"debug": True}, P2P)
    media = MediaElement()
    state = {"seeking": False, "seeked": False}

    def on_time():
        if media.currentTime > 1 and not state["seeking"]:
            state["seeking"] = True
            media.currentTime = 30
    media.addEventListener("timeupdate", on_time)
    media.addEventListener("seeked", lambda: state.update(seeked=True))
    _start(hls, media, vod.master_url())
    assert loop.run_until(lambda: state["seeked"] and media.currentTime > 31, timeout_ms=30_000)


def test_bundle_abr_settles_low_under_throttling():
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.test/abr/", renditions=[Rendition(40_000, 320, 180),
                                                                    Rendition(800_000, 640, 360),
                                                                    Rendition(3_000_000, 1280, 720)],
                                num_segments=30, segment_duration=2.0)
    Shaper.maxBandwidth = 64  # kbit/s (test/html/bundle.js:82)
    hls = Hls({"debug": True}, P2P)
    media = MediaElement()
    done = {}

    def later():
        loop.set_timeout(lambda: setattr(media, "currentTime", 30), 1000)
    media.addEventListener("seeked", lambda: done.update(levels=(hls.loadLevel, hls.nextLoadLevel)))
    _start(hls, media, origin.master_url(), later)
    assert loop.run_until(lambda: "levels" in done and media.currentTime >= 30, timeout_ms=600_000)
    assert done["levels"] == (0, 0)
