"""Shared configuration + runner for the three integration examples.

The analog of the reference's ``example/config.js`` (p2pConfig / hlsjsConfig /
contentUrl, WebRTC capability detection, ``example/config.js:5-17``).  In this framework a
"peer" is a GPU (or a CPU thread in tests), so the capability check is "can this process
join a swarm" and the stream is a synthetic HLS origin served from pinned host memory, or
with ``--url`` a real HLS stream from its CDN (``p2pConfig.gpuSwarm.network``).

Every example runs as:

* one process, ``--peers N``: N peers as N threads sharing one device (ThreadHub);
* ``torchrun --nproc-per-node N examples/<mode>/play.py``: one peer per rank/GPU over
  ``torch.distributed`` (RCCL on MI355X, gloo with ``--cpu``).
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
from pathlib import Path
from typing import Any, Callable, Dict

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
# torchrun peers share RCCL buffers across processes: this ROCm stack needs the dmabuf IPC
# mode, chosen before the HSA runtime starts (unless the environment already set it)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

from hlsjs_p2p_wrapper_amd.agent import current_node, node_for_config, set_current_node  # noqa: E402
from hlsjs_p2p_wrapper_amd.net import new_event_loop  # noqa: E402
from hlsjs_p2p_wrapper_amd.net.http import enable_network  # noqa: E402
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin  # noqa: E402
from hlsjs_p2p_wrapper_amd.player import MediaElement  # noqa: E402

STREAMROOT_CONFIG: Dict[str, Any] = {
    "p2pConfig": {
        "streamrootKey": "example-key",
        "debug": True,
        "contentId": None,
    },
    "hlsjsConfig": {
        "debug": False,
    },
    "contentUrl": "http://cdn.example/live/master.m3u8",
}


def has_swarm() -> bool:
    """Capability detection (the ``hasWebRTC`` analog): can this process exchange
    segments with peers?"""
    try:
        import torch.distributed as dist

        return dist.is_available()
    except Exception:  # noqa: BLE001
        return False


def make_origin(live: bool = False, encrypted: bool = True, num_segments: int = 30) -> SyntheticHlsOrigin:
    return SyntheticHlsOrigin("http://cdn.example/live/", renditions=[Rendition(2_000_000, 1280, 720),
                                                                      Rendition(800_000, 640, 360)],
                              num_segments=num_segments, encrypted=encrypted, live=live,
                              pin_memory=torch.cuda.is_available())


def parse_args(description: str) -> argparse.Namespace:
    p = argparse.ArgumentParser(description=description)
    p.add_argument("--peers", type=int, default=1, help="in-process peers (threads) when not under torchrun")
    p.add_argument("--seconds", type=float, default=20.0, help="media seconds to play per peer")
    p.add_argument("--live", action="store_true")
    p.add_argument("--clear", action="store_true", help="unencrypted stream")
    p.add_argument("--cpu", action="store_true", help="CPU only (no GPU)")
    p.add_argument("--no-p2p", action="store_true", help="play with P2P disabled (plain engine)")
    p.add_argument("--url", default=None,
                   help="play this http(s):// master playlist from the real CDN (net/network.py) "
                        "instead of the synthetic origin")
    return p.parse_args()


PlayFn = Callable[[Dict[str, Any], MediaElement, bool], Any]


def _peer(play: PlayFn, args, origin, gpu_swarm: Dict[str, Any], out: Dict[int, Any], rank: int) -> None:
    set_current_node(None)
    # a real CDN plays on the wall clock; the synthetic origin on a virtual one (fast)
    loop = new_event_loop("real" if args.url else "virtual")
    if args.url:
        gpu_swarm = dict(gpu_swarm, network=True)
        enable_network()  # also for --no-p2p: the plain engine's loaders need the CDN too
    cfg = {
        "p2pConfig": dict(STREAMROOT_CONFIG["p2pConfig"], gpuSwarm=gpu_swarm),
        "hlsjsConfig": dict(STREAMROOT_CONFIG["hlsjsConfig"]),
        "contentUrl": args.url or origin.master_url(),
    }
    p2p_enabled = has_swarm() and not args.no_p2p
    if p2p_enabled:
        node_for_config(cfg["p2pConfig"])  # join the swarm's rounds before playback starts
    media = MediaElement()
    hls = play(cfg, media, p2p_enabled)
    ok = loop.run_until(lambda: media.currentTime >= args.seconds, timeout_ms=600_000)
    node = current_node()
    stats = dict(node.stats) if (p2p_enabled and node is not None) else {}
    if node is not None:
        node.close()
    out[rank] = {"ok": ok, "currentTime": round(media.currentTime, 2), "level": hls.currentLevel,
                 "cdn": stats.get("cdn", 0), "p2p": stats.get("p2p", 0), "upload": stats.get("upload", 0)}
    hls.destroy()


def main(play: PlayFn, description: str) -> Dict[int, Any]:
    args = parse_args(description)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    device = "cpu" if (args.cpu or not torch.cuda.is_available()) else "cuda"
    origin = None if args.url else make_origin(live=args.live, encrypted=not args.clear)
    out: Dict[int, Any] = {}
    if world > 1:  # torchrun: one peer per rank (one GPU each)
        import torch.distributed as dist

        rank = int(os.environ["RANK"])
        if device == "cuda":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
            dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
        else:
            dist.init_process_group("gloo")
        _peer(play, args, origin, {"backend": "dist", "device": device, "roundIntervalMs": 20}, out, rank)
        print(f"rank {rank}: {out[rank]}", flush=True)
        dist.destroy_process_group()
        return out
    if args.peers == 1:
        _peer(play, args, origin, {"backend": "local", "device": device}, out, 0)
    else:
        from hlsjs_p2p_wrapper_amd.parallel import ThreadHub

        hub = ThreadHub(args.peers)
        ts = [threading.Thread(target=_peer, args=(play, args, origin, {"backend": "thread", "hub": hub, "rank": r,
                                                                        "device": device, "roundIntervalMs": 20},
                                                   out, r)) for r in range(args.peers)]
        [t.start() for t in ts]
        [t.join() for t in ts]
    for r in sorted(out):
        print(f"peer {r}: {out[r]}", flush=True)
    return out
