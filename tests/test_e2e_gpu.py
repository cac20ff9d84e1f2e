"""End-to-end on the MI355X: bundle playback with the HBM node, an in-process 2-peer
swarm on one GPU (HBM->HBM transfers), and the smoke entry point.  All ``gpu``."""
import threading

import pytest

from hlsjs_p2p_wrapper_amd import Hls
from hlsjs_p2p_wrapper_amd.agent import current_node, node_for_config, set_current_node
from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub
from hlsjs_p2p_wrapper_amd.player import MediaElement
from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine
from hlsjs_p2p_wrapper_amd.player.transmux import pipeline_for

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def fresh():
    clear_origins()
    set_current_node(None)
    yield
    clear_origins()
    set_current_node(None)


def test_bundle_plays_encrypted_vod_on_gpu(cuda):
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.gpu/vod/", renditions=[Rendition(3_000_000, 1280, 720)],
                                num_segments=8, encrypted=True, pin_memory=True)
    hls = Hls({}, {"gpuSwarm": {"device": "cuda:0", "cacheBytes": 128 << 20}})
    media = MediaElement()
    got = []
    hls.on(Hls.Events.FRAG_PARSING_DATA, lambda e, d: got.append(d) if d["type"] == "video" else None)
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    assert loop.run_until(lambda: media.currentTime > 30.0, timeout_ms=120_000)
    assert got and got[0]["data1"].is_cuda and got[0]["nb"] == 100  # 25 fps x 4 s video PES
    node = current_node()
    assert node.arena.is_cuda and node.stats["cdn"] == sum(origin.pools[0].lengths[:node.stats["cdn_segments"]])
    assert pipeline_for(cuda, loop).segments >= 8


def test_two_peers_on_one_gpu(cuda):
    origin = SyntheticHlsOrigin("http://cdn.gpu/swarm/", renditions=[Rendition(2_000_000, 1280, 720)],
                                num_segments=10, encrypted=True, pin_memory=True)
    hub = ThreadHub(2)
    out, errs = {}, []

    def peer(r):
        try:
            set_current_node(None)
            loop = new_event_loop("virtual")
            gs = {"backend": "thread", "hub": hub, "rank": r, "device": "cuda:0", "cacheBytes": 128 << 20,
                  "roundIntervalMs": 20}
            node_for_config({"gpuSwarm": gs})
            w = HlsjsP2PWrapper(Engine)
            hls = w.createPlayer({}, {"gpuSwarm": gs})
            media = MediaElement()
            hls.loadSource(origin.master_url())
            hls.attachMedia(media)
            hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
            ok = loop.run_until(lambda: media.currentTime > 38.0, timeout_ms=200_000)
            node = current_node()
            out[r] = (ok, dict(w.stats), dict(node.stats))
            node.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=peer, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(300) for t in ts]
    if errs:
        raise errs[0]
    assert all(o[0] for o in out.values())
    seg_total = sum(origin.pools[0].lengths)
    assert sum(o[1]["cdn"] for o in out.values()) == seg_total
    assert sum(o[1]["p2p"] for o in out.values()) == seg_total
    assert all(o[2]["crc_failures"] == 0 for o in out.values())


def test_smoke_entry_point(cuda):
    import __graft_entry__

    __graft_entry__.smoke()
