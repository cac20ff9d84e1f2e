"""Multi-process swarm over torch.distributed (gloo here; the same DistComm runs RCCL on
MI355X): control plane all-gather + batch_isend_irecv data plane, world_size 2."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _peer(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hlsjs_p2p_wrapper_amd import Hls
        from hlsjs_p2p_wrapper_amd.agent import node_for_config
        from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
        from hlsjs_p2p_wrapper_amd.net import new_event_loop
        from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
        from hlsjs_p2p_wrapper_amd.player import MediaElement
        from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine

        loop = new_event_loop("virtual")
        origin = SyntheticHlsOrigin("http://cdn.dist/vod/", renditions=[Rendition(1_000_000, 640, 360)],
                                    num_segments=8, encrypted=True, pin_memory=False)
        cfg = {"gpuSwarm": {"backend": "dist", "device": "cpu", "cacheBytes": 64 << 20, "roundIntervalMs": 20}}
        node = node_for_config(cfg)
        w = HlsjsP2PWrapper(Engine)
        hls = w.createPlayer({}, cfg)
        media = MediaElement()
        hls.loadSource(origin.master_url())
        hls.attachMedia(media)
        hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
        ok = loop.run_until(lambda: media.currentTime > 30.0, timeout_ms=300_000)
        stats = dict(w.stats)
        node.close()
        q.put((rank, ok, stats, sum(origin.pools[0].lengths), node.swarm_offload_ratio()))
    finally:
        dist.destroy_process_group()


def test_two_process_gloo_swarm():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        rank, ok, stats, total, offload = q.get(timeout=300)
        out[rank] = (ok, stats, total, offload)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(v[0] for v in out.values())
    total = out[0][2]
    assert out[0][1]["cdn"] + out[1][1]["cdn"] == total
    assert out[0][1]["p2p"] + out[1][1]["p2p"] == total
    assert out[0][1]["peers"] == 1
    assert out[0][3] == pytest.approx(0.5)


def _bench_cpu(port: int, *extra: str, nproc: int = 2, config: str = "abr5") -> dict:
    import json
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(repo / "bench.py"), "--cpu", "--gpus",
           str(nproc), "--config", config, "--steps", "8", "--warmup", "2", "--inflight", "8", "--pool", "8",
           "--cache-gb", "0.5", *extra]
    p = subprocess.run(cmd, cwd=repo, env=dict(os.environ, PYTHONPATH=str(repo)), capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("players", ["0", "2"])
def test_bench_two_ranks_abr_ladder_with_churn(players):
    # BASELINE config 3 through the driver's launch path (torchrun + bench.py), gloo on CPU,
    # with one in-process player and with the fleet (player processes): with churn, a rank
    # masked offline fetches everything from the CDN, so the swarm offload ratio drops below
    # the churn-free run's; nothing errors either way
    calm = _bench_cpu(_free_port(), "--players", players)
    # 14 timed steps: two full offline rotations, so the all-online phases hold enough rounds
    # for peers to share even when a loaded machine slows the fleet's players
    churn = _bench_cpu(_free_port(), "--churn", "2", "--players", players, "--steps", "14")
    assert calm["errors"] == 0 and churn["errors"] == 0
    assert calm["n_gpus"] == 2 and churn["config"]["churn_steps"] == 2
    assert 0 < churn["offload_ratio"] < 0.5  # 2 ranks: at most every segment fetched once, received once
    # The calm run's sharing depends on both ranks' ABR picking the same levels, and the ABR
    # estimates follow the players' timing: on a loaded machine (pytest -n) the ranks can settle
    # on different renditions and share almost nothing.  The ordering is only meaningful when
    # they shared.
    if calm["offload_ratio"] >= 0.2:
        assert churn["offload_ratio"] < calm["offload_ratio"]
    _check_per_rank(calm, 2)


@pytest.mark.parametrize("players", ["2", "0"])
def test_bench_fleet_corrupted_peer_copies_are_refetched(players):
    """Both player modes defer the receive-side CRC to the transmux that decrypts the
    segment (fleet: FleetServer sets verify_deferred; in-process: gpuSwarm.deferVerify, the
    player's batch reports through a VerifyTicket): a peer copy corrupted on arrival in each
    of the first 3 timed rounds is caught there, nothing is buffered from it, the copy is
    re-fetched from the CDN, and every player still buffers its fragments without an error."""
    res = _bench_cpu(_free_port(), "--players", players, "--corrupt-recv", "3", "--steps", "10")
    assert res["errors"] == 0 and res["value"] > 0
    assert res["config"]["receive_verify"] == "fused-decrypt"
    fails = sum(r["crc_failures"] for r in res["per_rank"])
    assert 1 <= fails <= 6  # at most one per corrupted round on each rank
    # rejected copies are counted apart: offload_ratio covers verified peer bytes only
    assert sum(r["p2p_rejected_MB"] for r in res["per_rank"]) > 0


def test_bench_eight_ranks_driver_shape():
    """The driver's N=8 launch (torchrun, 8 ranks, one bench.py each) rehearsed on CPU with
    gloo: shared-memory control plane across 8 processes with 4 player processes each,
    segments fetched from the CDN once and forwarded to the 7 other peers (offload ~7/8),
    no errors."""
    res = _bench_cpu(_free_port(), nproc=8, config="hostcost-micro")  # the default: 4 player processes per rank
    assert res["n_gpus"] == 8 and res["errors"] == 0
    assert res["config"]["players_per_gpu"] == 4 and res["config"]["player_processes"]
    assert res["config"]["global_batch"] == 8 * 4 * 8 and res["config"]["parallelism"] == "swarm8-gloo"
    # players are not in lockstep across ranks: a few segments are fetched from the CDN by a
    # second rank (a player that reached them after the window mark), so offload is ~7/8
    assert 0.75 < res["offload_ratio"] <= 0.9
    assert res["value"] > 0
    _check_per_rank(res, 8)


PER_RANK_KEYS = {"rank", "rounds", "step_ms", "wait_device_us", "exchange_us", "exchange_queued_us", "control_us",
                 "plan_us",
                 "host_round_us", "cdn_GBps", "cdn_dev_ms", "p2p_recv_MB", "p2p_sent_MB", "p2p_dev_ms", "p2p_GBps",
                 "p2p_links", "p2p_link_GBps",
                 "transmux_dev_ms", "transmux_wait_us", "await_players_us", "payload_GBps", "payload_wait_us",
                 "crc_failures", "control_fallbacks",
                 "deferred", "inflight", "cu_reserve", "p2p_rejected_MB", "p2p_link_roof_GBps", "p2p_link_util",
                 "bound"}


def _check_per_rank(res, world):
    """The N>1 record explains its own number: one diagnostics row per rank (bench.py
    PER_RANK_FIELDS) plus the transports actually used."""
    rows = res["per_rank"]
    assert [r["rank"] for r in rows] == list(range(world))
    for r in rows:
        assert set(r) == PER_RANK_KEYS
        assert r["rounds"] >= res["steps"] and r["crc_failures"] == 0 and r["control_fallbacks"] == 0
        assert r["bound"] in ("pcie", "xgmi", "transmux", "pcie_d2h", "players", "host")
        assert 0 <= r["p2p_links"] <= world - 1
    # (which rank receives depends on the players' relative pace: the swarm as a whole does)
    assert sum(r["p2p_recv_MB"] for r in rows) > 0 and sum(r["p2p_sent_MB"] for r in rows) > 0
    dp = res["data_plane"]
    assert dp["data"] == "gloo" and dp["control"] == "shm"
    # topology proof: every rank's row, its data plane's own view of the
    # world, and the bytes it received per source peer (matching the per-rank P2P totals)
    assert dp["world"] == world and [r["rank"] for r in dp["ranks"]] == list(range(world))
    for r, pr in zip(dp["ranks"], rows):
        assert r["comm"]["world"] == world and r["comm"]["rank"] == r["rank"]
        assert len(r["recv_bytes_from"]) == world and r["recv_bytes_from"][r["rank"]] == 0
        assert r["rounds"] >= res["steps"]
        assert sum(r["recv_bytes_from"]) / 1e6 == pytest.approx(pr["p2p_recv_MB"] * pr["rounds"], rel=0.01, abs=0.01)


def _bench_plain(*extra: str, timeout: int = 300):
    """``python bench.py ...`` with NO launcher (the driver's BENCH command shape)."""
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(repo)
    return subprocess.run([sys.executable, str(repo / "bench.py"), *extra], cwd=repo, env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_n_self_launches_n_ranks():
    """a plain ``python bench.py --gpus 4`` (no torchrun) runs 4 ranks --
    the parent starts them as a torch.distributed.run child before touching any device,
    forwards rank 0's JSON line, and the record proves the world it ran: n_gpus 4, four rank
    rows, 3/4 offload, each rank's bytes received per source peer."""
    p = _bench_plain("--cpu", "--gpus", "4", "--players", "2", "--config", "hostcost-micro", "--steps", "8",
                     "--warmup", "2", "--inflight", "8", "--pool", "8", "--cache-gb", "0.5")
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1  # exactly the result line on stdout
    import json

    res = json.loads(lines[0])
    assert res["n_gpus"] == 4 and res["errors"] == 0 and res["value"] > 0
    assert 0.4 < res["offload_ratio"] <= 0.8  # 3/4 when the players keep pace; lower on a loaded machine
    dp = res["data_plane"]
    assert dp["launcher"] == "self" and dp["world"] == 4
    assert [r["rank"] for r in dp["ranks"]] == [0, 1, 2, 3]
    for r in dp["ranks"]:
        assert r["comm"]["world"] == 4 and r["comm"]["rank"] == r["rank"]
        assert len(r["recv_bytes_from"]) == 4 and r["recv_bytes_from"][r["rank"]] == 0
    recv = sum(sum(r["recv_bytes_from"]) for r in dp["ranks"])
    assert recv > 0
    _check_per_rank(res, 4)


def test_bench_gpus_must_match_the_launcher_world():
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parents[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(repo / "bench.py"), "--cpu", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--players", "0", "--config", "hostcost-micro"]
    p = subprocess.run(cmd, cwd=repo, env=dict(os.environ, PYTHONPATH=str(repo)), capture_output=True, text=True,
                       timeout=300)
    assert p.returncode != 0
    assert "--gpus 2 but the launcher started 4 ranks" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_self_launch_reports_a_failing_rank():
    """A rank that fails makes the self-launched job exit non-zero with no result line."""
    p = _bench_plain("--cpu", "--gpus", "2", "--players", "0", "--config", "hostcost-micro", "--steps", "2",
                     "--warmup", "1", "--live-window", "3", "--cache-gb", "-1")
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert "failed" in p.stderr


def _peer4(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hlsjs_p2p_wrapper_amd import Hls
        from hlsjs_p2p_wrapper_amd.agent import node_for_config
        from hlsjs_p2p_wrapper_amd.api.wrapper import HlsjsP2PWrapper
        from hlsjs_p2p_wrapper_amd.net import new_event_loop
        from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
        from hlsjs_p2p_wrapper_amd.player import MediaElement
        from hlsjs_p2p_wrapper_amd.player.hls import Hls as Engine

        loop = new_event_loop("virtual")
        origin = SyntheticHlsOrigin("http://cdn.dist4/vod/", renditions=[Rendition(800_000, 640, 360),
                                                                         Rendition(1_600_000, 960, 540)],
                                    num_segments=8, encrypted=True, pin_memory=False)
        cfg = {"gpuSwarm": {"backend": "dist", "device": "cpu", "cacheBytes": 64 << 20, "roundIntervalMs": 20}}
        node = node_for_config(cfg)
        w = HlsjsP2PWrapper(Engine)
        hls = w.createPlayer({"startLevel": rank % 2}, cfg)
        media = MediaElement()
        start = 20_000 if rank == 3 else 0  # late joiner: served from the others' caches
        loop.set_timeout(hls.loadSource, start, origin.master_url())
        hls.attachMedia(media)
        hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
        if rank == 2:  # churn: masked offline for a while
            loop.set_timeout(node.set_online, 3_000, False)
            loop.set_timeout(node.set_online, 12_000, True)
        ok = loop.run_until(lambda: media.currentTime > 30.0, timeout_ms=400_000)
        stats = dict(w.stats)
        node.close()
        q.put((rank, ok, stats, node.swarm_offload_ratio()))
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_four_process_gloo_swarm_with_churn_and_late_joiner():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_peer4, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(4):
        rank, ok, stats, offload = q.get(timeout=400)
        out[rank] = (ok, stats, offload)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert all(v[0] for v in out.values())
    assert out[3][1]["cdn"] == 0 or out[3][1]["p2p"] > 0  # the late joiner mostly rides the swarm
    assert sum(v[1]["p2p"] for v in out.values()) > 0
    assert 0 < out[0][2] < 1


def test_bench_fleet_two_ranks_two_players():
    """Fleet mode through the driver's launch path: 2 ranks x 2 player processes (gloo, CPU).
    Every player's fragments are counted between the in-band window marks; the swarm still
    fetches each segment from the CDN once (player w plays the same DVR slice on each rank)."""
    res = _bench_cpu(_free_port(), "--players", "2", config="hostcost-micro")
    assert res["errors"] == 0 and res["value"] > 0
    assert res["config"]["players_per_gpu"] == 2 and res["config"]["player_processes"]
    assert res["config"]["global_batch"] == 8 * 2 * 2
    # players on an oversubscribed CPU do not keep the same pace on both ranks, so within the
    # window the rank ahead fetches segments its peer only receives after it (GPU rehearsals,
    # profiles/r2_fleet_validation: exactly 0.50 / 0.75 at 2 / 4 ranks)
    assert 0.3 < res["offload_ratio"] <= 0.52


def test_bench_fleet_payloads_two_ranks():
    """``--fleet-payload`` (``gpuSwarm.fleetPayload``: bytes in every player's ``onSuccess``)
    through the driver's launch path: the fragments' bytes go through each rank's shared
    payload ring, the players finish without errors, and the record shows the payload rate."""
    res = _bench_cpu(_free_port(), "--players", "2", "--fleet-payload", config="hostcost-micro")
    assert res["errors"] == 0 and res["value"] > 0
    _check_per_rank(res, 2)
    assert all(r["payload_GBps"] > 0 for r in res["per_rank"])
    assert res["config"]["ingest_crc"]  # ranks with peers compute the trailers their sends carry


def test_ipc_outbox_slots_follow_the_packing_order():
    """The IPC rehearsal plane (parallel/comm.py:_IpcOutbox): a receiver finds each send
    addressed to it in the sender's outbox from the sender's table alone -- sends packed in
    order at 256-byte boundaries, per (src, dst) pair in send order (RCCL p2p semantics)."""
    import numpy as np

    from hlsjs_p2p_wrapper_amd.parallel.comm import _outbox_slots

    sends = [(1, 1000), (2, 300), (1, 4), (3, 0), (1, 256)]  # (dst, nbytes) of one sender
    table = np.array([0, len(sends)] + [v for s in sends for v in s], dtype=np.int64)
    assert _outbox_slots(table, 1, 256) == [(0, 1000), (1536, 4), (1792, 256)]
    assert _outbox_slots(table, 2, 256) == [(1024, 300)]
    assert _outbox_slots(table, 3, 256) == [(1792, 0)]
    assert _outbox_slots(table, 0, 256) == []
    assert _outbox_slots(np.array([0, 0], dtype=np.int64), 1, 256) == []


def test_bench_live_edge_two_ranks():
    """BASELINE config 2 at the live edge through the driver's launch path (2 ranks x 2
    players, gloo, CPU): a sliding live playlist on a compressed clock, every player in real
    time at the live sync point, playlist reloads, the cache evicting segments that slid out
    of the window inside the timed region; the swarm fetches each segment from the CDN once."""
    res = _bench_cpu(_free_port(), "--players", "2", "--steps", "400", "--live-speed", "100", "--live-window", "10",
                     config="1080p6m-live")
    assert res["errors"] == 0 and res["value"] > 0
    cfg = res["config"]
    assert cfg["live"] is True and "live" in cfg["model"] and cfg["evicted_segments"] > 0
    assert 0.3 < res["offload_ratio"] <= 0.52  # each segment crosses the CDN once per swarm of 2
    assert res["live_latency_s"]["p50"] < 30.0  # well ahead of the 30 s live sync point


def test_bench_self_launch_deadline_stops_the_ranks():
    """A self-launched job that overruns ``--launch-timeout`` is stopped -- launcher and ranks
    -- and the bench exits 124 with no result line."""
    import time

    import psutil

    t0 = time.monotonic()
    p = _bench_plain("--cpu", "--gpus", "2", "--players", "0", "--config", "hostcost-micro", "--steps", "100000",
                     "--warmup", "1", "--inflight", "8", "--pool", "8", "--cache-gb", "0.5", "--launch-timeout", "8")
    assert p.returncode == 124, p.stderr[-2000:]
    assert "overran --launch-timeout" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert time.monotonic() - t0 < 60
    time.sleep(1.0)
    left = [q for q in psutil.process_iter(["cmdline"])
            if q.info["cmdline"] and "--launch-timeout" in q.info["cmdline"] and "100000" in q.info["cmdline"]]
    assert not left, [q.info["cmdline"] for q in left]


def test_killing_the_self_launching_bench_stops_its_ranks():
    """SIGKILL of ``bench.py --gpus 2`` (no signal handler runs): the launcher it started gets
    SIGTERM from the kernel on its parent's death and stops the ranks."""
    import signal
    import subprocess
    import sys
    import time
    from pathlib import Path

    import psutil

    repo = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(repo)
    p = subprocess.Popen([sys.executable, str(repo / "bench.py"), "--cpu", "--gpus", "2", "--players", "0", "--config",
                          "hostcost-micro", "--steps", "100000", "--warmup", "1", "--inflight", "8", "--pool", "8",
                          "--cache-gb", "0.5"], cwd=repo, env=env, stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL)
    kids = []
    try:
        parent = psutil.Process(p.pid)
        deadline = time.monotonic() + 120
        while time.monotonic() < deadline and len(kids) < 3:  # the launcher and its two ranks
            time.sleep(0.5)
            kids = parent.children(recursive=True)
        assert len(kids) >= 3, [k.cmdline() for k in kids]
        time.sleep(2.0)
        p.send_signal(signal.SIGKILL)
        p.wait(timeout=30)
        # the launcher gives its ranks 30 s after SIGTERM before it SIGKILLs them; a loaded
        # machine (the full suite) needs the margin
        gone, alive = psutil.wait_procs(kids, timeout=120)

        def desc(a):
            try:
                return a.pid, a.cmdline()[:4], a.ppid()
            except psutil.Error:
                return a.pid, None, None
        assert not alive, [desc(a) for a in alive]
    finally:
        if p.poll() is None:
            p.kill()
        for k in kids:  # a failed check leaves no process behind (exact PIDs of this test's tree)
            try:
                k.kill()
            except psutil.NoSuchProcess:
                pass


@pytest.mark.parametrize("players", ["2", "0"])
def test_bench_calibrates_the_cu_reserve_before_warmup(players):
    """The RCCL CU reserve is calibrated on the run's own round shape before warmup (round-5
    VERDICT Next 2): every candidate is timed (max over ranks), all ranks keep the same,
    fastest one, and the timed window still has exactly --steps steps.  (On CPU the reserve
    does nothing; ``force`` runs the mechanism, ``auto`` runs it on the native RCCL plane.)"""
    res = _bench_cpu(_free_port(), "--players", players, "--cu-calibrate", "force", "--cu-calib-steps", "2")
    cal = res["calibration"]
    assert cal["source"] == "calibrated" and cal["candidates"] == [0, 32, 64, 96]
    assert len(cal["ms_per_step"]) == 4 and all(t > 0 for t in cal["ms_per_step"])
    fastest = cal["candidates"][cal["ms_per_step"].index(min(cal["ms_per_step"]))]
    t = dict(zip(cal["candidates"], cal["ms_per_step"]))
    # the fastest, unless it is within the margin of the previous (default) reserve
    assert cal["chosen"] == (fastest if t[fastest] <= t[cal["previous"]] * (1 - cal["margin"]) else cal["previous"])
    assert cal["steps_per_candidate"] == 2 and res["steps"] == 8 and res["errors"] == 0
    assert all(r["rounds"] >= 8 for r in res["per_rank"])


def test_bench_cu_reserve_env_pins_it():
    import os

    os.environ["HLSP2P_RCCL_CU_RESERVE"] = "32"
    try:
        res = _bench_cpu(_free_port(), "--players", "0", "--cu-calibrate", "force")
    finally:
        del os.environ["HLSP2P_RCCL_CU_RESERVE"]
    assert res["calibration"] == {"source": "HLSP2P_RCCL_CU_RESERVE", "chosen": 32}
