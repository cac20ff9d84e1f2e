"""Randomized fleet scenarios: one rank (a CPU ``SwarmNode`` + ``FleetServer``, the bench's
node-side loop) serving 2-3 player threads running ``player_main`` -- the process layout of
``bench.py`` in one process -- with random caches, in-flight windows, payload modes, byte
read-back through ``RemoteSegment.data()`` and scripted seeks, pauses, level switches and
load restarts.  A scenario passes when every player plays to the end of the VOD with no
fatal error, no failed byte read and no exception on either side.

Used by ``tests/test_fleet_chaos.py`` (fixed seeds) and runnable directly for a sweep:
``python tests/fleet_chaos.py 0 100`` (``--gpu``: the node on ``cuda:0``).
"""
from __future__ import annotations

import collections
import multiprocessing as mp
import sys
import threading
import time

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.agent import node_for_config, set_current_node
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel.fleet import FleetServer, player_main
from hlsjs_p2p_wrapper_amd.player.transmux import pipeline_for


def scenario(seed: int, timeout_s: float = 120.0, device: str = "cpu") -> dict:
    """``device``: where the node's segment cache and the transmux live (``cuda:0``: the HBM
    ring, the GPU transmux and the on-demand bytes copied back from the device)."""
    rng = np.random.default_rng(seed)
    nseg = int(rng.integers(10, 24))
    ladder = rng.random() < 0.4
    rends = ([Rendition(300_000, 480, 270), Rendition(700_000, 640, 360), Rendition(1_200_000, 960, 540)]
             if ladder else [Rendition(int(rng.integers(300_000, 1_200_000)), 640, 360)])
    origin_kw = dict(base_url=f"http://fleet.chaos{seed}/vod/", renditions=rends, num_segments=nseg,
                     segment_duration=4.0, encrypted=bool(rng.random() < 0.7), pool_size=min(nseg, 8), seed=seed)
    duration = nseg * 4.0
    W = int(rng.integers(2, 4))
    clear_origins()
    set_current_node(None)
    loop = new_event_loop("real")
    pinned = device != "cpu"  # the GPU CDN phase copies from pinned host buffers
    origin = SyntheticHlsOrigin(**origin_kw, pin_memory=pinned)
    seg = max(max(p.lengths) for p in origin.pools)
    cache = int(rng.integers(4, 24)) * ((seg + 255) // 256 * 256)
    node = node_for_config({"gpuSwarm": {"backend": "local", "device": device, "cacheBytes": cache,
                                         "autoTick": False}})
    players = []
    for w in range(W):
        script = []
        for _ in range(int(rng.integers(0, 4))):
            t = float(rng.uniform(200, 3000))  # real milliseconds: the fleet runs on the real clock
            kind = str(rng.choice(["seek", "pause", "level", "restart"]))
            arg = {"seek": float(rng.uniform(0, duration * 0.8)), "pause": float(rng.uniform(50, 400)),
                   "level": int(rng.integers(0, 3)), "restart": float(rng.uniform(20, 300))}[kind]
            script.append((t, kind, arg))
        players.append({"inflight": int(rng.choice([1, 2, 4, 8])), "payload": bool(rng.random() < 0.3),
                        "read": bool(rng.random() < 0.5), "script": script})
    pairs = [mp.Pipe() for _ in range(W)]
    errs: list = []
    threads = []
    for w, (_, child) in enumerate(pairs):
        p = players[w]
        spec = {"origin": dict(origin_kw, pin_memory=pinned),
                "hls_config": {"maxFragLoadsInFlight": p["inflight"], "maxBufferLength": 1e9,
                               "maxMaxBufferLength": 1e9, "startPosition": 0, "startLevel": 0,
                               "tickInterval": 1e9},
                "p2p_config": {"streamrootKey": "t", "contentId": f"fleet-chaos-{seed}",
                               "gpuSwarm": {"fleetPayload": p["payload"]}},
                "world": 1, "rank": 0, "script": p["script"], "read_bytes": p["read"], "in_process": True}

        def run(c=child, s=spec):
            try:
                player_main(c, s)
            except BaseException as e:  # noqa: BLE001
                errs.append(("player", e))
        t = threading.Thread(target=run, daemon=True)
        t.start()
        threads.append(t)
    conns = [parent for parent, _ in pairs]
    pipe = pipeline_for(torch.device(device), loop)
    pipe.auto_flush = False
    server = None
    result = {"seed": seed, "players": players, "cache_segs": cache // ((seg + 255) // 256 * 256), "W": W,
              "errors": errs, "marks": {}, "duration": duration}
    try:
        server = FleetServer(node, pipe, conns)
        end = time.monotonic() + 30
        while len(server.ready) < W:
            server.poll()
            time.sleep(0.002)
            if time.monotonic() > end:
                raise RuntimeError("players did not start")
        for c in conns:
            c.send(("go",))
        hs, b = collections.deque(), None
        deadline = time.monotonic() + timeout_s
        next_mark, tag = time.monotonic() + 0.5, 0
        while True:
            while loop._ready:
                loop.run_once(block=False)
            server.await_players(timeout_s=0.005)
            server.poll()
            server.admit(8)
            hs.append(node.launch_round())
            if len(hs) > 1:
                node.complete_round(hs.popleft())
            nb = server.launch_transmux()
            server.complete_transmux(b)
            server.send()
            b = nb
            if time.monotonic() > next_mark:  # ask every player where it is
                tag += 1
                for w, c in enumerate(conns):
                    if server.open[w]:
                        c.send(("mark", tag))
                next_mark = time.monotonic() + 0.5
            marks = {}
            for t_ in sorted(server.marks):
                marks.update(server.marks[t_])
            result["marks"] = marks
            if len(marks) == W and all(m["t"] >= duration - 4.5 for m in marks.values()):
                break
            if errs or time.monotonic() > deadline:
                break
    except BaseException as e:  # noqa: BLE001
        errs.append(("node", e))
    finally:
        for w, c in enumerate(conns):
            try:
                c.send(("stop",))
            except (OSError, BrokenPipeError):
                pass
        for t in threads:
            t.join(10)
        if server is not None:
            server.close()
        node.close()
        clear_origins()
        set_current_node(None)
    return result


def check(res: dict) -> None:
    if res["errors"]:
        raise AssertionError(f"seed {res['seed']}: {res['errors'][0]!r}") from res["errors"][0][1]
    marks = res["marks"]
    assert len(marks) == res["W"], (res["seed"], "not every player reported", marks)
    for w, m in marks.items():
        assert m.get("fatal", 0) == 0 and m.get("byte_errors", 0) == 0, (res["seed"], w, m, res["players"][w])
        assert m["t"] >= res["duration"] - 4.5, (res["seed"], w, "stopped at", m["t"], res["players"][w],
                                                 res["cache_segs"])


if __name__ == "__main__":
    device = "cuda:0" if "--gpu" in sys.argv else "cpu"
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    lo, hi = (int(argv[0]), int(argv[1])) if len(argv) > 1 else (0, 20)
    bad = []
    for s in range(lo, hi):
        res = scenario(s, device=device)
        try:
            check(res)
            ends = sorted(round(m["t"], 1) for m in res["marks"].values())
            print(f"seed {s}: ok ({res['W']} players, t {ends})", flush=True)
        except AssertionError as e:
            print(f"seed {s}: FAIL {str(e)[:400]}", flush=True)
            bad.append(s)
    print("failed seeds:", bad)
    sys.exit(1 if bad else 0)
