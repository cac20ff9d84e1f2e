"""Warm restart of the HBM segment cache: a node checkpoints what it played,
a fresh node restores it (CRC re-verified, eviction order kept) and its player is then
served entirely from the restored cache.  Safetensors only: loading executes nothing."""
import pytest
import torch

from hlsjs_p2p_wrapper_amd import Hls
from hlsjs_p2p_wrapper_amd.agent import SwarmNode, set_current_node
from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.player import MediaElement
from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine


def _play(origin, device, cache_path=None, save_path=None, seconds=38.0, corrupt=False):
    set_current_node(None)
    loop = new_event_loop("virtual")
    node = SwarmNode(device=device, cache_bytes=64 << 20, loop=loop)
    set_current_node(node)
    restored = None
    if cache_path:
        if corrupt:  # flip one payload byte in the file's data section
            from safetensors.torch import load_file, save_file
            from safetensors import safe_open

            with safe_open(cache_path, framework="pt") as f:
                meta = f.metadata()
            t = load_file(cache_path)
            t["data"][int(t["offs"][1]) + 100] ^= 0xFF
            save_file(t, cache_path, metadata=meta)
        restored = node.load_cache(cache_path)
    w = HlsjsP2PWrapper(Engine)
    hls = w.createPlayer({}, {})
    media = MediaElement()
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    ok = loop.run_until(lambda: media.currentTime > seconds, timeout_ms=200_000)
    saved = node.save_cache(save_path) if save_path else None
    stats = dict(node.stats)
    hls.destroy()
    set_current_node(None)
    return ok, stats, restored, saved


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_checkpoint_restore_serves_from_cache(tmp_path, device, request):
    if device == "cuda":
        request.getfixturevalue("cuda")
    clear_origins()
    origin = SyntheticHlsOrigin("http://cdn.ckpt/vod/", renditions=[Rendition(1_000_000, 640, 360)],
                                num_segments=10, encrypted=True, pin_memory=(device == "cuda"))
    path = str(tmp_path / "cache.safetensors")
    ok, stats, _, saved = _play(origin, device, save_path=path)
    assert ok and saved["segments"] == 10 and saved["bytes"] == stats["cdn"]
    ok2, stats2, restored, _ = _play(origin, device, cache_path=path)
    assert ok2 and restored == {"restored": 10, "skipped": 0, "bad_crc": 0}
    assert stats2["cdn"] == 0 and stats2["cache"] == stats["cdn"]  # every segment from the warm cache
    # a corrupted checkpoint segment is dropped by the CRC re-check and re-fetched
    ok3, stats3, restored3, _ = _play(origin, device, cache_path=path, corrupt=True)
    assert ok3 and restored3["restored"] == 9 and restored3["bad_crc"] == 1
    assert 0 < stats3["cdn"] < stats["cdn"]
    clear_origins()


def test_checkpoint_rejects_foreign_files(tmp_path):
    from safetensors.torch import save_file

    p = str(tmp_path / "x.safetensors")
    save_file({"data": torch.zeros(4, dtype=torch.uint8)}, p, metadata={"format": "other"})
    node = SwarmNode(device="cpu", cache_bytes=1 << 20, loop=new_event_loop("virtual"))
    with pytest.raises(ValueError, match="not a segment-cache checkpoint"):
        node.load_cache(p)


def test_one_rank_node_skips_the_ingest_crc(monkeypatch):
    """The ingest CRC only produces the trailers peers check; a one-rank swarm never sends, so
    it skips the pass (the checkpoint above then computes the CRCs it saves), a multi-rank
    node keeps it, and HLSP2P_INGEST_CRC=1 forces it."""
    from hlsjs_p2p_wrapper_amd.parallel import ThreadHub

    loop = new_event_loop("virtual")
    assert not SwarmNode(device="cpu", cache_bytes=1 << 20, loop=loop, auto_tick=False).ingest_crc
    hub = ThreadHub(2)
    assert SwarmNode(hub.comm(0), device="cpu", cache_bytes=1 << 20, loop=loop, auto_tick=False).ingest_crc
    monkeypatch.setenv("HLSP2P_INGEST_CRC", "1")
    assert SwarmNode(device="cpu", cache_bytes=1 << 20, loop=loop, auto_tick=False).ingest_crc
