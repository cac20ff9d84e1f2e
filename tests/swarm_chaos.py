"""Randomized swarm scenarios ("chaos"): N in-process peers (ThreadHub, CPU) on a VOD or an
ABR ladder with random cache sizes, start delays, in-flight windows, seeks, level switches,
offline periods, P2P download toggles, corrupted peer copies and deferred verification.  A
scenario passes when every peer plays to the end without an exception or a media error.

Used by ``tests/test_swarm_chaos.py`` (a few fixed seeds) and runnable directly for a wider
sweep: ``python tests/swarm_chaos.py 0 200 [--extras] [--gpu]``.
"""
from __future__ import annotations

import os
import sys
import threading

import numpy as np

from hlsjs_p2p_wrapper_amd import Hls
from hlsjs_p2p_wrapper_amd.agent import node_for_config, set_current_node
from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub
from hlsjs_p2p_wrapper_amd.player import MediaElement
from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine

# every node of a scenario checks its replicated-state invariants after each round
# (agent/audit.py); HLSP2P_AUDIT=0 turns it off for a timing sweep
os.environ.setdefault("HLSP2P_AUDIT", "1")


def scenario(seed: int, extras: bool = False, device: str = "cpu") -> dict:
    """``extras``: also pause / resume playback and stop / restart loading at random times
    (drawn from a second generator, so the base scenario of a seed does not change).
    ``device``: where the peers' caches and the transmux live (``cuda:0``: every peer on the
    one GPU, with its streams, events and asynchronous copies)."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 5))
    nseg = int(rng.integers(12, 30))
    ladder = rng.random() < 0.4
    rends = ([Rendition(300_000, 480, 270), Rendition(700_000, 640, 360), Rendition(1_200_000, 960, 540)]
             if ladder else [Rendition(int(rng.integers(300_000, 1_500_000)), 640, 360)])
    clear_origins()
    origin = SyntheticHlsOrigin(f"http://cdn.chaos{seed}/vod/", renditions=rends, num_segments=nseg,
                                encrypted=bool(rng.random() < 0.7))
    seg = max(max(p.lengths) for p in origin.pools)
    duration = nseg * 4.0
    peers = []
    for r in range(n):
        peers.append({
            "cache_segs": int(rng.integers(3, 12)),
            "delay": float(rng.choice([0.0, rng.uniform(0, 30_000)])),
            "inflight": int(rng.choice([1, 2, 4, 8])),
            "buffer": float(rng.choice([8.0, 12.0, 30.0])),
            "defer": bool(rng.random() < 0.5),
            "events": [],
        })
        for _ in range(int(rng.integers(0, 4))):
            t = float(rng.uniform(2_000, duration * 1000 * 0.7))
            kind = str(rng.choice(["seek", "offline", "nodl", "corrupt", "level"]))
            peers[r]["events"].append((t, kind, float(rng.uniform(0, duration * 0.8))))
    if extras:
        rng2 = np.random.default_rng(seed + 1_000_003)
        for r in range(n):
            for _ in range(int(rng2.integers(0, 3))):
                t = float(rng2.uniform(2_000, duration * 1000 * 0.7))
                peers[r]["events"].append((t, str(rng2.choice(["pause", "restart"])), float(rng2.uniform(500, 4_000))))
    hub = ThreadHub(n)
    out, errs = {}, []

    def peer(r):
        p = peers[r]
        try:
            set_current_node(None)
            loop = new_event_loop("virtual")
            gs = {"backend": "thread", "hub": hub, "rank": r, "device": device,
                  "cacheBytes": p["cache_segs"] * ((seg + 255) // 256 * 256), "roundIntervalMs": 20,
                  "deferVerify": p["defer"]}
            node = node_for_config({"gpuSwarm": gs})
            w = HlsjsP2PWrapper(Engine)
            hls = w.createPlayer({"maxFragLoadsInFlight": p["inflight"], "maxBufferLength": p["buffer"],
                                  "startLevel": 0}, {"gpuSwarm": gs})
            media = MediaElement()
            media_errors = []
            hls.on(Hls.Events.ERROR, lambda e, d: media_errors.append(d.get("details")) if d.get("fatal") else None)
            if p["delay"]:
                loop.set_timeout(hls.loadSource, p["delay"], origin.master_url())
            else:
                hls.loadSource(origin.master_url())
            hls.attachMedia(media)
            hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
            for t, kind, arg in p["events"]:
                t += p["delay"] + 1000.0  # after the session started (the reference's toggles throw before)
                if kind == "seek":
                    loop.set_timeout(lambda a=arg: setattr(media, "currentTime", a), t)
                elif kind == "offline":
                    loop.set_timeout(lambda: node.set_online(False), t)
                    loop.set_timeout(lambda: node.set_online(True), t + 5_000)
                elif kind == "nodl":
                    loop.set_timeout(lambda: setattr(w, "p2pDownloadOn", False), t)
                    loop.set_timeout(lambda: setattr(w, "p2pDownloadOn", True), t + 5_000)
                elif kind == "corrupt":
                    loop.set_timeout(lambda: setattr(node, "corrupt_next_recv", 2), t)
                elif kind == "level" and ladder:
                    loop.set_timeout(lambda a=arg: setattr(hls, "nextLevel", int(a) % 3), t)
                elif kind == "pause":
                    loop.set_timeout(media.pause, t)
                    loop.set_timeout(media.play, t + arg)
                elif kind == "restart":
                    loop.set_timeout(hls.stopLoad, t)
                    loop.set_timeout(lambda: hls.startLoad(media.currentTime), t + arg)
            ok = loop.run_until(lambda: media.currentTime >= duration - 4.5, timeout_ms=900_000)
            out[r] = {"ok": ok, "t": media.currentTime, "fatal": media_errors, "stats": dict(w.stats)}
            node.close()
        except BaseException as e:  # noqa: BLE001
            errs.append((r, e))
            hub.abort()

    ts = [threading.Thread(target=peer, args=(r,)) for r in range(n)]
    [t.start() for t in ts]
    [t.join(600) for t in ts]
    clear_origins()
    primary = [e for e in errs if not isinstance(e[1], threading.BrokenBarrierError)]
    return {"seed": seed, "n": n, "peers": peers, "out": out, "errors": primary or errs}


def check(res: dict) -> None:
    if res["errors"]:
        raise AssertionError(f"seed {res['seed']}: {res['errors'][0]!r}") from res["errors"][0][1]
    for r, o in res["out"].items():
        assert o["ok"], (res["seed"], r, o["t"], res["peers"][r])
        assert not o["fatal"], (res["seed"], r, o["fatal"])


if __name__ == "__main__":
    lo, hi = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (0, 20)
    extras = "--extras" in sys.argv
    device = "cuda:0" if "--gpu" in sys.argv else "cpu"
    bad = []
    for s in range(lo, hi):
        try:
            res = scenario(s, extras, device)  # (an AuditError is an AssertionError: a failed seed)
            check(res)
            print(f"seed {s}: ok ({res['n']} peers)", flush=True)
        except AssertionError as e:
            print(f"seed {s}: FAIL {e}", flush=True)
            bad.append(s)
    print("failed seeds:", bad)
    sys.exit(1 if bad else 0)
