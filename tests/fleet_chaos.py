"""Randomized fleet scenarios: ranks (a CPU or GPU ``SwarmNode`` + ``FleetServer`` each, the
bench's node-side loop) serving 2-3 player threads running ``player_main`` -- the process
layout of ``bench.py`` in one process -- with random caches, in-flight windows, payload modes,
byte read-back through ``RemoteSegment.data()`` and scripted seeks, pauses, level switches and
load restarts.  With ``ranks`` > 1 the ranks are threads on a ``ThreadHub``: they share one
content, plan peer transfers between their caches each round, and a rank's players are
answered from its peers' caches too.  A scenario passes when every player plays to the end of
the VOD with no fatal error, no failed byte read and no exception on any side.

Used by ``tests/test_fleet_chaos.py`` (fixed seeds) and runnable directly for a sweep:
``python tests/fleet_chaos.py 0 100`` (``--gpu``: the nodes on ``cuda:0``; ``--ranks=N``;
``--faults``: corrupted receives and offline periods; ``--live``: a live channel; ``--ring``:
payloads through a small, growing payload ring).
"""
from __future__ import annotations

import collections
import multiprocessing as mp
import os
import sys
import threading
import time

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
from hlsjs_p2p_wrapper_amd.agent import set_current_node
from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.parallel import LocalComm, ThreadHub
from hlsjs_p2p_wrapper_amd.parallel.fleet import FleetServer, player_main
from hlsjs_p2p_wrapper_amd.player.transmux import pipeline_for

# every node of a scenario checks its replicated-state invariants after each round
# (agent/audit.py); HLSP2P_AUDIT=0 turns it off for a timing sweep
os.environ.setdefault("HLSP2P_AUDIT", "1")


LIVE_SPEED = 20.0  # live scenarios: media seconds per wall second
LIVE_WALL_S = 6.0  # ... and their wall time


def _want_rows(node) -> list:
    """The node's live wants (diagnostics of a stalled scenario): info row + waiters."""
    if not len(node._wt):
        return []
    ids = np.arange(1, 1 << 16, dtype=np.int64)
    info = node._wt.info(ids)
    live = np.flatnonzero(info[:, 0] >= 0)[:8]
    out = [(int(ids[i]), info[i].tolist(), list(node._wt.waiters(int(ids[i])))) for i in live]
    try:  # where the planner routes them now (src -1: CDN; a rank: that rank's cache)
        rt = node.rt
        w = np.zeros((len(live), 8), dtype=np.int64)
        w[:, :5] = info[live, :5]
        w[:, 5] = ids[live]
        w[:, 6] = node.rank
        flags = np.where(np.asarray(node.peer_online, dtype=bool), rt.FLAG_ONLINE, 0).astype(np.int64)
        plan, _, _ = rt.plan_round_for(node.directory, w, flags, node.world, node.rank, None)
        out.append(("plan", plan.tolist()))
    except Exception as e:  # noqa: BLE001
        out.append(("plan error", repr(e)))
    return out


def _draw_rank(rng, duration):
    """One rank's draws: its player count, its cache (in segments) and its players."""
    W = int(rng.integers(2, 4))
    cache_segs = int(rng.integers(4, 24))
    players = []
    for _ in range(W):
        script = []
        for _ in range(int(rng.integers(0, 4))):
            t = float(rng.uniform(200, 3000))  # real milliseconds: the fleet runs on the real clock
            kind = str(rng.choice(["seek", "pause", "level", "restart"]))
            arg = {"seek": float(rng.uniform(0, duration * 0.8)), "pause": float(rng.uniform(50, 400)),
                   "level": int(rng.integers(0, 3)), "restart": float(rng.uniform(20, 300))}[kind]
            script.append((t, kind, arg))
        players.append({"inflight": int(rng.choice([1, 2, 4, 8])), "payload": bool(rng.random() < 0.3),
                        "read": bool(rng.random() < 0.5), "script": script})
    return W, cache_segs, players


def scenario(seed: int, timeout_s: float = 120.0, device: str = "cpu", ranks: int = 1, faults: bool = False,
             live: bool = False, ring: bool = False) -> dict:
    """``device``: where the nodes' segment caches and the transmux live (``cuda:0``: the HBM
    ring, the GPU transmux and the on-demand bytes copied back from the device).  ``ranks``:
    rank 0 draws what the single-rank scenario of the seed draws; later ranks draw after it.
    ``faults`` (ranks > 1): each rank also corrupts received rounds and goes offline for a
    while at random times, and the CDN serves one corrupted copy of 1-2 segments (drawn from a
    second generator: the base scenario does not change).
    ``live``: the channel is live (a sliding window of 6-15 segments published 20x faster than
    real time, players at the live sync point on the channel's clock, live-window eviction on
    the nodes); the scripts' times and pauses are scaled to the channel's clock and their seeks
    go back into the window.  A live scenario runs ``LIVE_WALL_S`` and passes when every player
    is still playing at the end (its media clock advanced over the last second).
    ``ring``: every player takes payloads, through a payload ring that starts at 1 MiB and
    grows by at least 1 MiB (``FleetServer._new_ring``): the ring fills, grows and retires
    rings whose regions players still hold, all through the scenario."""
    rng = np.random.default_rng(seed)
    nseg = int(rng.integers(10, 24))
    ladder = rng.random() < 0.4
    rends = ([Rendition(300_000, 480, 270), Rendition(700_000, 640, 360), Rendition(1_200_000, 960, 540)]
             if ladder else [Rendition(int(rng.integers(300_000, 1_200_000)), 640, 360)])
    origin_kw = dict(base_url=f"http://fleet.chaos{seed}/vod/", renditions=rends, num_segments=nseg,
                     segment_duration=4.0, encrypted=bool(rng.random() < 0.7), pool_size=min(nseg, 8), seed=seed)
    duration = nseg * 4.0
    draws = [_draw_rank(rng, duration) for _ in range(ranks)]
    if ring:
        for _, _, ps in draws:
            for p in ps:
                p["payload"] = True
    speed = LIVE_SPEED
    if live:
        lrng = np.random.default_rng(seed + 9_000_017)
        window = int(lrng.integers(6, 16))
        origin_kw.update(live=True, window=window, num_segments=None, live_speed=speed, pool_size=8)
        for _, _, ps in draws:  # the scripts on the channel's clock (player loop ms = media ms)
            for p in ps:
                p["script"] = [(t * speed, "seek_rel", -float(a % (window * 4.0 * 0.6))) if k == "seek" else
                               (t * speed, k, a * speed if k in ("pause", "restart") else a)
                               for t, k, a in p["script"]]
    frng = np.random.default_rng(seed + 5_000_011)
    faults_at = [sorted((float(frng.uniform(0.2, 3.0)), str(frng.choice(["corrupt", "offline"])),
                         int(frng.integers(1, 4)), float(frng.uniform(0.1, 1.0)))
                        for _ in range(int(frng.integers(1, 4)))) if faults and ranks > 1 else []
                 for _ in range(ranks)]
    # ... and the CDN serves one corrupted copy of 1-2 segments (a flipped byte mid-segment:
    # the decrypt / demux may reject it -> the wrapper drops the cached copy, the retry is a
    # fresh CDN fetch)
    cdn_corrupt = [int(x) for x in frng.integers(0, nseg, size=int(frng.integers(1, 3)))] \
        if faults and ranks > 1 else []
    clear_origins()
    pinned = device != "cpu"  # the GPU CDN phase copies from pinned host buffers
    origin = SyntheticHlsOrigin(**origin_kw, pin_memory=pinned)
    seg_al = (max(max(p.lengths) for p in origin.pools) + 255) // 256 * 256
    hub = ThreadHub(ranks, timeout=60) if ranks > 1 else None
    errs: list = []
    result = {"seed": seed, "ranks": ranks, "duration": duration, "errors": errs, "faults": faults_at,
              "cdn_corrupt": cdn_corrupt,
              "players": [p for _, _, ps in draws for p in ps], "W": sum(d[0] for d in draws),
              "cache_segs": [c for _, c, _ in draws], "marks": {}}
    # the ranks stop together: a collective round needs every rank, so once rank 0 sees every
    # player done it names a step a few rounds ahead (ranks run at most a round apart)
    stop = {"step": None}
    done = [False] * ranks
    marks_all: list = [{} for _ in range(ranks)]
    base = [sum(d[0] for d in draws[:r]) for r in range(ranks)]
    # no rank is done before every scripted action ran (a player at the end that a late
    # seek sends back is not done; the scripts' times are on the players' clocks)
    script_end_s = max([t for _, _, ps in draws for p in ps for t, _, _ in p["script"]] or [0.0]) / 1000.0
    if live:
        script_end_s /= speed
    script_end_s += 0.5
    epoch = time.time() + 0.5  # live: the channel's clock, shared by the nodes and players
    if live:
        origin.live_epoch = epoch
    trail = collections.defaultdict(dict)  # live: player -> {mark tag: media t}
    result["live"] = live
    result["trail"] = trail

    def rank_main(r):
        W, cache_segs, players = draws[r]
        set_current_node(None)
        loop = new_event_loop("real")
        comm = hub.comm(r) if hub is not None else LocalComm()
        node = SwarmNode(comm, device=device, cache_bytes=cache_segs * seg_al, auto_tick=False)
        set_current_node(node)
        pairs = [mp.Pipe() for _ in range(W)]
        threads = []
        for w, (_, child) in enumerate(pairs):
            p = players[w]
            hcfg = ({"maxFragLoadsInFlight": p["inflight"], "fragLoadingTimeOut": 60_000, "startLevel": 0}
                    if live else
                    {"maxFragLoadsInFlight": p["inflight"], "maxBufferLength": 1e9, "maxMaxBufferLength": 1e9,
                     "startPosition": 0, "startLevel": 0, "tickInterval": 1e9})
            spec = {"origin": dict(origin_kw, pin_memory=pinned), "hls_config": hcfg,
                    "p2p_config": {"streamrootKey": "t", "contentId": f"fleet-chaos-{seed}",
                                   "gpuSwarm": {"fleetPayload": p["payload"]}},
                    "world": ranks, "rank": r, "script": p["script"], "read_bytes": p["read"],
                    "in_process": True}
            if live:
                spec.update(clock_speed=speed, media_mode="realtime")

            def run(c=child, s=spec):
                try:
                    player_main(c, s)
                except BaseException as e:  # noqa: BLE001
                    errs.append((f"player {r}", e))
            t = threading.Thread(target=run, daemon=True)
            t.start()
            threads.append(t)
        conns = [parent for parent, _ in pairs]
        pipe = pipeline_for(torch.device(device), loop)
        pipe.auto_flush = False
        server = None
        try:
            server = FleetServer(node, pipe, conns)
            if ring:
                server.RING_MIN = 1 << 20
                server.ring_ack_timeout_s = 0.5  # a player behind by half a second loses its payloads
            end = time.monotonic() + 30
            while len(server.ready) < W:
                server.poll()
                time.sleep(0.002)
                if time.monotonic() > end:
                    raise RuntimeError("players did not start")
            if cdn_corrupt and r == 0:  # (on the origin instance the URLs resolve to)
                from hlsjs_p2p_wrapper_amd.net import http as _http
                served = _http.resolve(origin.base_url + origin.segment_path(0, 0))[0]
                for sn in cdn_corrupt:
                    served.corrupt(rf"r\d+/seg{sn}\.ts$", 1)
            for c in conns:
                c.send(("go", {"live_epoch": epoch} if live else {}))
            hs, b = collections.deque(), None
            deadline = time.monotonic() + timeout_s
            next_mark, tag, step = time.monotonic() + 0.5, 0, 0
            live_end = time.monotonic() + LIVE_WALL_S
            t0, todo, back_online = time.monotonic(), list(faults_at[r]), None
            while True:
                now = time.monotonic() - t0
                while todo and todo[0][0] <= now:  # (at s, kind, rounds to corrupt, offline s)
                    _, kind, k, off_s = todo.pop(0)
                    if kind == "corrupt":
                        node.corrupt_next_recv += k
                    elif back_online is None:
                        node.set_online(False)
                        back_online = now + off_s
                if back_online is not None and now >= back_online:
                    node.set_online(True)
                    back_online = None
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
                step += 1
                if time.monotonic() > next_mark:  # ask every player where it is
                    tag += 1
                    for w, c in enumerate(conns):
                        if server.open[w]:
                            c.send(("mark", tag, {"state": True}))
                    next_mark = time.monotonic() + 0.5
                marks = {}
                for t_ in sorted(server.marks):
                    marks.update(server.marks[t_])
                marks_all[r] = {base[r] + w: m for w, m in marks.items()}
                settled = time.monotonic() - t0 > script_end_s
                if live:  # every mark's t per player, for the end check
                    for t_ in sorted(server.marks)[-3:]:
                        for w, m in server.marks[t_].items():
                            trail[base[r] + w][t_] = m["t"]
                    done[r] = time.monotonic() > live_end
                else:
                    done[r] = settled and len(marks) == W and all(m["t"] >= duration - 4.5 for m in marks.values())
                if r == 0 and stop["step"] is None and (all(done) or errs or time.monotonic() > deadline):
                    stop["step"] = step + 4
                    result["stop"] = ("done" if all(done) else "errors" if errs else "deadline", list(done),
                                      round(time.monotonic() - t0, 1))
                    if not all(done) and not errs:  # a stall: where is every thread?
                        import traceback
                        names = {t.ident: t.name for t in threading.enumerate()}
                        result["stacks"] = {names.get(i, i): "".join(traceback.format_stack(f)[-6:])
                                            for i, f in sys._current_frames().items()}
                if stop["step"] is not None and step >= stop["step"]:
                    break
                if hub is None and (errs or time.monotonic() > deadline):
                    break
        except BaseException as e:  # noqa: BLE001
            errs.append((f"rank {r}", e))
        finally:
            result.setdefault("nodes", {})[r] = {"wants": len(node._wt), "parked": len(node._vwait),
                                                 "evicted": server.evicted if server is not None else 0,
                                                 "ring_cap": server._ring.cap if server is not None and
                                                 server._ring is not None else 0,
                                                 "revoked": len(server.revoked) if server is not None else 0,
                                                 "pending_verify": node.pending_verify(),
                                                 "round": node.round,
                                                 "pending_rows": [(int(e), node._vinfo[e][:4].tolist(),
                                                                   int(node._vround[e]))
                                                                  for e in np.flatnonzero(node._vflag)[:8]],
                                                 "want_rows": _want_rows(node),
                                                 "stats": {k: v for k, v in node.stats.items()
                                                           if isinstance(v, (int, float))}}
            for c in conns:
                try:
                    c.send(("stop",))
                except (OSError, BrokenPipeError):
                    pass
            for t in threads:
                t.join(10)
            if server is not None:
                server.close()
            node.close()
            set_current_node(None)

    saved_ring = os.environ.get("HLSP2P_FLEET_PAYLOAD_BYTES")
    if ring:
        os.environ["HLSP2P_FLEET_PAYLOAD_BYTES"] = str(1 << 20)
    try:
        if ranks == 1:
            rank_main(0)
        else:
            ts = [threading.Thread(target=rank_main, args=(r,), daemon=True) for r in range(ranks)]
            [t.start() for t in ts]
            [t.join(timeout_s + 90) for t in ts]
            if any(t.is_alive() for t in ts):
                errs.append(("scenario", TimeoutError("a rank did not stop")))
    finally:
        clear_origins()
        if ring:
            if saved_ring is None:
                os.environ.pop("HLSP2P_FLEET_PAYLOAD_BYTES", None)
            else:
                os.environ["HLSP2P_FLEET_PAYLOAD_BYTES"] = saved_ring
    for m in marks_all:
        result["marks"].update(m)
    return result


def check(res: dict) -> None:
    if res["errors"]:
        raise AssertionError(f"seed {res['seed']}: {res['errors'][0]!r}") from res["errors"][0][1]
    marks = res["marks"]
    assert len(marks) == res["W"], (res["seed"], "not every player reported", marks)
    for w, m in marks.items():
        assert m.get("fatal", 0) == 0 and m.get("byte_errors", 0) == 0, (res["seed"], w, m, res["players"][w])
        if res["live"]:  # still playing: its clock advanced over the last two marks (1 s of wall)
            ts = [t for _, t in sorted(res["trail"][w].items())][-3:]
            assert len(ts) == 3 and ts[-1] - ts[0] >= 0.25 * LIVE_SPEED, (res["seed"], w, "stalled", ts, m,
                                                                           res["players"][w])
            continue
        assert m["t"] >= res["duration"] - 4.5, (res["seed"], w, "stopped at", m["t"], res["players"][w],
                                                 res["cache_segs"], m.get("state"), res.get("nodes"))


if __name__ == "__main__":
    device = "cuda:0" if "--gpu" in sys.argv else "cpu"
    nranks = next((int(a.split("=", 1)[1]) for a in sys.argv if a.startswith("--ranks=")), 1)
    faults = "--faults" in sys.argv
    live = "--live" in sys.argv
    ring = "--ring" in sys.argv
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    lo, hi = (int(argv[0]), int(argv[1])) if len(argv) > 1 else (0, 20)
    bad = []
    for s in range(lo, hi):
        try:
            res = scenario(s, device=device, ranks=nranks, faults=faults, live=live, ring=ring)
            check(res)  # (an AuditError raised in a scenario is an AssertionError: a failed seed)
            ends = sorted(round(m["t"], 1) for m in res["marks"].values())
            st = [n["stats"] for n in res.get("nodes", {}).values()]
            crc, parked = sum(x.get("crc_failures", 0) for x in st), sum(x.get("parked", 0) for x in st)
            ev = sum(n.get("evicted", 0) for n in res.get("nodes", {}).values())
            inv = sum(x.get("invalidated", 0) for x in st)
            print(f"seed {s}: ok ({res['ranks']} ranks, {res['W']} players, t {ends}, crc failures {crc}, "
                  f"parked {parked}, evicted {ev}, invalidated {inv})", flush=True)
        except AssertionError as e:
            print(f"seed {s}: FAIL {str(e)[:400]}", flush=True)
            bad.append(s)
    print("failed seeds:", bad)
    sys.exit(1 if bad else 0)
