#!/usr/bin/env python3
"""Headline benchmark: segments/s + P2P offload ratio, 1080p 6 Mb/s HLS, 1/2/4/8 MI355X.

Metric and config come from BASELINE.json.  One rank per GPU (``torchrun``), each rank a
swarm peer; every fragment runs the full public API path:

    Hls(hlsjsConfig, p2pConfig)  (bundle)  ->  P2PLoader (fLoader)  ->  PeerAgent
    ->  SwarmNode round:  CDN phase (pinned host -> HBM, side stream) + MFMA CRC ingest
                          P2P phase (one native RCCL send/recv group over xGMI, CRC-verified)
    ->  onProgress/onSuccess  ->  FRAG_LOADED  ->  batched AES-128-CBC decrypt + TS demux
    ->  buffer append  ->  FRAG_BUFFERED

By default each GPU serves ``--players`` (4) player processes ("fleet", parallel/fleet.py):
each runs the bundle player above its ``PeerAgent`` over a ``RemoteNode`` and plays its
own slice of the DVR window, while the rank process runs the node rounds and the GPU
transmux for all of them (the players never touch the GPU).  ``--players 0`` runs one
player inside the rank process.  Player ``w`` plays the same slice on every rank, so the
swarm shares it as before.

Workload (synthetic, see ``--help``): every peer plays the same 1080p 6 Mb/s AES-128
stream (4 s MPEG-TS segments of ~3.0 MB) as fast as the engine delivers ("drain" media
sink, e.g. an edge/restream node catching up a DVR window), with ``--inflight``
fragments in flight per player and step.  One step = one swarm exchange round.  Per-GPU
work is fixed (weak scaling).

``value`` = completed (loaded + decrypted + demuxed + buffered) segments per second over
all ranks (timed region bracketed by barrier + device sync, max time over ranks).
``offload_ratio`` = sum p2p / (sum p2p + sum cdn) bytes over the timed region.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# multi-process GPU work on this ROCm stack (RCCL peer buffers, HIP-IPC rehearsal outboxes)
# needs the dmabuf IPC mode; set it before the HSA runtime starts (torch import) unless the
# environment already chose
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402

_PROF = None
if os.environ.get("HLSP2P_PROFILE"):  # cProfile the timed steps (host-overhead analysis)
    import cProfile

    _PROF = cProfile.Profile()
_PROF_C3 = _PROF is not None and os.environ.get("HLSP2P_PROFILE_SECTION") == "c3"  # only the post-transmux drain

CONFIGS = {
    # name: (renditions preset, encrypted, segment seconds, description)
    # the swarm drains a live channel's DVR window as fast as it can (a throughput bench: at
    # real-time live pace every peer would take 1 segment per 4 s); the window is served as a
    # complete playlist, so no mid-run playlist reloads (live mode, sliding windows and
    # live-window eviction are covered by tests/test_swarm.py)
    "1080p6m": ("1080p", True, 4.0, "1080p 6 Mb/s HLS live-channel DVR catch-up (AES-128, 4 s TS segments)"),
    "1080p6m-clear": ("1080p", False, 4.0, "1080p 6 Mb/s HLS (clear, 4 s TS segments)"),
    "abr5": ("abr5", True, 4.0, "5-rendition ABR ladder (AES-128, 4 s TS)"),
    "4k25m": ("4k", True, 4.0, "4K 25 Mb/s HLS (AES-128, 4 s TS segments)"),
    # diagnostic only: ~30 KB segments, so per-segment host (Python) cost dominates
    "hostcost": ("tiny", True, 4.0, "60 kb/s HLS (AES-128) - host-overhead probe"),
    "hostcost-abr": ("tiny-abr", True, 4.0, "5 x 20-100 kb/s ABR ladder (AES-128) - host-overhead probe"),
    # diagnostic only: ~4 KB segments, for the CPU host-cost harness (device ops ~free)
    "hostcost-micro": ("micro", True, 4.0, "8 kb/s HLS (AES-128) - host-overhead probe, CPU harness"),
    # BASELINE config 2 at the live edge: a sliding live playlist (reloads, window slides,
    # live-window eviction in the timed region) played in real time by every player, on a
    # clock running --live-speed times faster than the wall; the rate is the channel's
    "1080p6m-live": ("1080p", True, 4.0, "1080p 6 Mb/s live HLS at the live edge (AES-128, 4 s TS segments)"),
}
LIVE = {"1080p6m-live"}


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks (one per GPU); without a launcher, N > 1 starts N rank processes itself "
                        "(a torch.distributed.run child) and forwards rank 0's JSON line; under a launcher "
                        "it must equal WORLD_SIZE (default: the launcher's world, else 1)")
    p.add_argument("--launch-timeout", type=float, default=float(os.environ.get("HLSP2P_LAUNCH_TIMEOUT", "1500")),
                   help="self-launch (--gpus N > 1 without a launcher): kill the rank processes and exit "
                        "non-zero after this many seconds")
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", default="1080p6m", choices=sorted(CONFIGS))
    p.add_argument("--inflight", type=int, default=None,
                   help="fragments in flight per player (per step), default 64 (96 at N >= 8) -- chosen by "
                        "measurement: 128 is flat on the PCIe-bound headline and was -4 %% to +20 %% on the "
                        "device-bound HBM-origin probe across boxes (profiles/r3_inflight, profiles/r4_ab); at "
                        "N=8 96 amortizes the rank's per-step host work (profiles/r6_inflight)")
    p.add_argument("--pool", type=int, default=64, help="distinct packaged segments per rendition")
    p.add_argument("--cache-gb", type=float, default=None,
                   help="segment-cache arena per GPU (default 8 GB)")
    p.add_argument("--no-dedup", action="store_true", help="disable CDN de-duplication (seeding)")
    p.add_argument("--cpu", action="store_true", help="CPU rehearsal (gloo, no GPU)")
    p.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo", "ipc"],
                   help="data-plane backend for N>1 (auto: nccl = RCCL on GPUs; gloo stages GPU "
                        "tensors through host memory; ipc: gloo control with device-to-device "
                        "HIP-IPC outboxes -- both are multi-rank rehearsals on a single GPU)")
    p.add_argument("--sync-steps", action="store_true",
                   help="no software pipelining: each step = load, round, transmux, synchronously")
    p.add_argument("--lag", type=int, default=2,
                   help="swarm rounds in flight on the device before the host completes the oldest "
                        "(2: the next round's CDN DMA is always queued behind the current one)")
    p.add_argument("--churn", type=int, default=0, metavar="N",
                   help="swarm churn (BASELINE config 3): every N steps the next rank goes offline for N "
                        "steps (masked in the control plane: it neither serves nor receives P2P), then "
                        "one all-online period; 0 = off")
    p.add_argument("--no-gc-tune", action="store_true", help="keep Python's default GC settings")
    p.add_argument("--metrics-port", type=int, default=None,
                   help="serve Prometheus GET /metrics on port + rank while the bench runs (idle unless scraped)")
    p.add_argument("--players", type=int, default=4,
                   help="fleet mode: this many player processes per GPU feed the node (each plays its own "
                        "slice of the DVR window with --inflight fragments per step; parallel/fleet.py); 0 = "
                        "one player in the node's process")
    p.add_argument("--numa", default="auto", choices=["auto", "off", "remote"],
                   help="auto: run on (and first-touch pinned buffers from) the CPUs local to the GPU; "
                        "remote: the other socket's CPUs (diagnostic); off: leave the affinity alone")
    p.add_argument("--cpu-place", default=os.environ.get("HLSP2P_CPU_PLACE", "shared"),
                   choices=["shared", "nosmt", "cores"],
                   help="CPU placement of the rank and its players inside the NUMA binding (utils/runtime.py "
                        "place_processes): shared = one common CPU set; nosmt = one thread per physical core "
                        "(no two of them on SMT siblings); cores = a physical core each")
    p.add_argument("--ingest", default="pcie", choices=["pcie", "hbm"],
                   help="pcie: the CDN origin is pinned host memory (the benchmark); hbm: DIAGNOSTIC, the "
                        "origin's segment pools live in HBM, so CDN fetches are device-to-device copies "
                        "standing in for segments that arrive over xGMI (the per-GPU ceiling at N=8 "
                        "without the PCIe bound)")
    p.add_argument("--live-speed", type=float, default=100.0,
                   help="live configs: media seconds per wall second (the channel publishes a segment "
                        "every segment_s / speed seconds; players reload and play on the same clock)")
    p.add_argument("--live-window", type=int, default=15, help="live configs: playlist window in segments")
    p.add_argument("--round-ms", type=float, default=5.0,
                   help="live configs: one node round per this many wall milliseconds (paced)")
    p.add_argument("--playlist-steps", type=int, default=None,
                   help="size the players' DVR window for this many steps instead of --steps (soak analysis)")
    p.add_argument("--fleet-payload", action="store_true",
                   help="fleet players receive every fragment's bytes in onSuccess (gpuSwarm.fleetPayload: "
                        "HBM gather + D2H + shared-memory ring per batch); off: the players get the "
                        "transmux result rows only (the bytes stay in HBM)")
    p.add_argument("--corrupt-recv", type=int, default=0, metavar="N",
                   help="fault injection (SURVEY 5.3): flip a byte in the first segment received from a peer in "
                        "each of the first N timed rounds; the CRC check must drop it and the CDN re-serve it")
    p.add_argument("--cu-calibrate", default=os.environ.get("HLSP2P_CU_CALIBRATE", "auto"),
                   choices=["auto", "off", "force"],
                   help="before warmup, time a few pipelined steps per RCCL CU reserve candidate "
                        "(--cu-candidates) and keep the fastest (max over ranks); auto: only while the "
                        "native RCCL plane is live (the reserve only matters beside its kernels); "
                        "HLSP2P_RCCL_CU_RESERVE set: no calibration, that value")
    p.add_argument("--cu-candidates", default="0,32,64,96",
                   help="CU reserve candidates of the calibration (CUs left free of the decrypt grid)")
    p.add_argument("--cu-calib-steps", type=int, default=6, help="timed steps per calibration candidate")
    p.add_argument("--verbose", action="store_true")
    return p.parse_args()


def _numa(mode: str, dev: int, world: int = 1, players: int = 0):
    from hlsjs_p2p_wrapper_amd.utils.runtime import bind_to_gpu_numa, gpu_local_cpus

    if mode == "off":
        return None
    if mode == "auto":
        # every rank on this GPU's NUMA node brings 1 + players busy processes: bind only when
        # the node's CPUs can hold all of them (else leave the affinity alone)
        node, _ = gpu_local_cpus(dev)
        ranks_here = sum(1 for i in range(min(max(1, world), torch.cuda.device_count()))
                         if node is not None and gpu_local_cpus(i)[0] == node)
        return bind_to_gpu_numa(dev, min_cpus=max(8, max(1, ranks_here) * (1 + players)))
    node, local = gpu_local_cpus(dev)  # remote: every allowed CPU NOT local to the GPU
    other = os.sched_getaffinity(0).difference(local)
    if node is None or len(other) < 8:
        return None
    os.sched_setaffinity(0, other)
    return f"remote-of-{node}"


def _place(mode: str, dev: int, pids):
    """Placement of this GPU's host processes (``--cpu-place``); the slot of a rank is its
    GPU's position among the GPUs on the same NUMA node, so ranks never share cores."""
    from hlsjs_p2p_wrapper_amd.utils.runtime import gpu_local_cpus, place_processes

    if mode == "shared":
        return None
    node, _ = gpu_local_cpus(dev)
    slot = sum(1 for i in range(dev) if node is not None and gpu_local_cpus(i)[0] == node)
    sets = place_processes(pids, mode, slot)
    return None if sets is None else mode


def _workload(args):
    """The synthetic stream and player settings (no GPU needed: fleet players are spawned
    from them before this process touches the GPU)."""
    from hlsjs_p2p_wrapper_amd.net.origin import PRESET_1080P_6M, PRESET_4K_25M, PRESET_ABR5, Rendition

    preset, encrypted, seg_dur, desc = CONFIGS[args.config]
    rends = {"1080p": PRESET_1080P_6M, "4k": PRESET_4K_25M, "abr5": PRESET_ABR5,
             "tiny": [Rendition(60_000, 320, 180, name="180p")],
             "micro": [Rendition(8_000, 160, 90, name="90p")],
             "tiny-abr": [Rendition(20_000 * (i + 1), 160 * (i + 1), 90 * (i + 1), name=f"t{i}")
                          for i in range(5)]}[preset]
    K = args.inflight
    # each player's slice of the DVR window covers the run (--playlist-steps: size it for a
    # longer run, to tell a playlist-size effect from a run-length effect in soaks)
    n_segments = (args.warmup + max(args.steps, args.playlist_steps or 0) + 4 + _calib_steps(args)) * K
    W = max(0, args.players)
    origin_kwargs = dict(base_url="http://cdn.bench/live/", renditions=rends,
                         num_segments=n_segments * max(1, W) + (16 * K if W else 0),
                         segment_duration=seg_dur, encrypted=encrypted, pool_size=args.pool, seed=7)
    depth = 1 if args.sync_steps else args.lag + 2  # rounds a fragment spends in flight (see step())
    hls_config = {"maxFragLoadsInFlight": K * depth, "maxBufferLength": 1e9, "maxMaxBufferLength": 1e9,
                  "startPosition": 0, "fragLoadingTimeOut": 600_000, "tickInterval": 1e9}
    if args.config in LIVE:
        # every player watches the same live channel at the live sync point, in real time on
        # the compressed clock; the agent negotiates its buffer target (live margin)
        origin_kwargs.update(live=True, window=args.live_window, num_segments=None, live_speed=args.live_speed)
        hls_config = {"maxFragLoadsInFlight": 8, "fragLoadingTimeOut": 60_000}
    if preset != "abr5":
        hls_config["startLevel"] = 0
    p2p_base = {"streamrootKey": "bench", "contentId": "bench-1080p"}
    if args.fleet_payload:
        p2p_base["gpuSwarm"] = {"fleetPayload": True}
    return preset, encrypted, seg_dur, desc, K, n_segments, W, origin_kwargs, hls_config, p2p_base


INFLIGHT_N8 = 96  # default fragments in flight per player at N >= 8 (main)
CALIB_SETTLE = 2  # untimed steps after each candidate is set (rounds in flight drain under it)


def _calib_candidates(args) -> list:
    """The CU reserve candidates this run will time (empty: no calibration).  ``auto`` runs it
    for an N > 1 GPU run on the native RCCL plane (the driver's 8-GPU bench, the socket
    rehearsal); ``HLSP2P_RCCL_CU_RESERVE`` pins the reserve instead."""
    if args.cu_calibrate == "off" or os.environ.get("HLSP2P_RCCL_CU_RESERVE"):
        return []
    if args.cu_calibrate == "auto":
        world = int(os.environ.get("WORLD_SIZE", str(args.gpus or 1)))
        if args.cpu or world < 2 or args.dist_backend not in ("auto", "nccl"):
            return []
    return [int(x) for x in str(args.cu_candidates).split(",") if x.strip()]


def _calib_steps(args) -> int:
    return len(_calib_candidates(args)) * (CALIB_SETTLE + max(1, args.cu_calib_steps))


def _calibrate(args, node, step, sync, world: int):
    """Pick the decrypt grid's RCCL CU reserve on the real round shape, before warmup (outside
    the timed window): per candidate, ``CALIB_SETTLE`` untimed steps, then
    ``--cu-calib-steps`` steps timed between two barriers; the slowest rank's time decides
    (the bench's own rule) and every rank keeps the same, fastest, candidate.  The xGMI links'
    real rate decides how long RCCL's kernels hold their CUs, which no one-GPU rehearsal can
    tell (round 5 froze 64 from a one-rank HBM self-exchange: profiles/r5_overlap)."""
    cands = _calib_candidates(args)
    if not cands:
        pinned = os.environ.get("HLSP2P_RCCL_CU_RESERVE")
        return {"source": "HLSP2P_RCCL_CU_RESERVE", "chosen": int(pinned)} if pinned else None
    from hlsjs_p2p_wrapper_amd.ops._native import device as _dev

    dev = _dev()
    before = dev.cu_reserve()
    k = max(1, args.cu_calib_steps)
    table = []
    for c in cands:
        dev.set_cu_reserve(int(c))
        for _ in range(CALIB_SETTLE):
            step()
        sync()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        sync()
        ns = np.array([int((time.perf_counter() - t0) * 1e9)], dtype=np.int64)
        if world > 1:
            ns = np.array([max(int(x[0]) for x in node.comm.allgather_control(ns))], dtype=np.int64)
        table.append(round(float(ns[0]) / 1e6 / k, 3))
    # identical table on every rank: the same choice.  The default reserve stays unless a
    # candidate beats it by more than the margin: a few steps per candidate cannot separate
    # options within noise, and a socket- or PCIe-bound run makes them all equal
    margin = float(os.environ.get("HLSP2P_CU_CALIB_MARGIN", "0.04"))
    best = cands[int(np.argmin(table))]
    if before in cands and table[cands.index(best)] > table[cands.index(before)] * (1.0 - margin):
        best = before
    dev.set_cu_reserve(int(best))
    return {"source": "calibrated", "candidates": cands, "ms_per_step": table, "chosen": int(best),
            "previous": int(before), "margin": margin, "steps_per_candidate": k, "settle_steps": CALIB_SETTLE}


def _spawn_players(W, world, rank, origin_kwargs, hls_config, p2p_base, n_segments, seg_dur):
    """Start the fleet's player processes (spawn: fresh interpreters that never open the GPU;
    started before this process initialises it)."""
    import multiprocessing as mp

    from hlsjs_p2p_wrapper_amd.parallel.fleet import player_main

    ctx = mp.get_context("spawn")
    conns, procs = [], []
    saved = {k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "HLSJS_P2P_PURE")}
    os.environ["HIP_VISIBLE_DEVICES"] = os.environ["CUDA_VISIBLE_DEVICES"] = "-1"
    if os.environ.get("HLSP2P_PLAYER_PROFILE"):  # profiled players run pure Python (compiled frames are opaque)
        os.environ["HLSJS_P2P_PURE"] = "1"
    try:
        for w in range(W):
            parent, child = ctx.Pipe()
            spec = {"origin": dict(origin_kwargs, pin_memory=False),
                    "hls_config": dict(hls_config, startPosition=w * n_segments * seg_dur)
                    if not origin_kwargs.get("live") else dict(hls_config),
                    "p2p_config": dict(p2p_base), "world": world, "rank": rank}
            if origin_kwargs.get("live"):  # the player's loop runs on the channel's clock
                spec["clock_speed"] = float(origin_kwargs["live_speed"])
                spec["media_mode"] = "realtime"
            pr = ctx.Process(target=player_main, args=(child, spec), daemon=True, name=f"hlsp2p-player{w}")
            pr.start()
            child.close()
            conns.append(parent)
            procs.append(pr)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return conns, procs


def _launcher_world():
    """The world size a launcher (torchrun / torch.distributed.run, an MPI-style wrapper that
    exports the same variables) gave this process, or None when started directly."""
    if "WORLD_SIZE" in os.environ and "RANK" in os.environ:
        return int(os.environ["WORLD_SIZE"])
    return None


def _self_launch(args) -> int:
    """``--gpus N > 1`` without a launcher: run the N ranks as children of a
    ``torch.distributed.run`` process (one rank per GPU, rendezvous on 127.0.0.1), forward
    rank 0's JSON line, and exit non-zero if any rank fails, the job overruns
    ``--launch-timeout`` or the record does not report N ranks.  Runs before this process
    touches the GPU -- GPUs are counted from the KFD topology (``visible_gpu_count``), and
    right before the launcher starts, ``gpu_touched`` must report no HIP context and no
    ``/dev/kfd`` mapping or descriptor (exit 5 otherwise) -- and never execs:
    the launcher is a child process in this process group, and dies with this process
    (``PR_SET_PDEATHSIG``), so no rank outlives a killed bench."""
    import signal
    import socket
    import subprocess
    import threading

    from hlsjs_p2p_wrapper_amd.utils.runtime import gpu_touched, visible_gpu_count

    n = args.gpus
    dry = os.environ.get("HLSP2P_LAUNCH_DRYRUN") == "1"  # GPU test of this path: everything but the Popen
    avail = None
    if not args.cpu and args.dist_backend in ("auto", "nccl") and not os.environ.get("HLSP2P_RCCL_REHEARSAL"):
        # counted from the KFD topology, not torch.cuda.device_count(): on this torch that may
        # fall back to hipGetDeviceCount, which starts the HIP runtime in this process, and a
        # process that initialised the GPU must not fork-and-exec the launcher
        avail = visible_gpu_count()
        if 0 < avail < n and not dry:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs for the RCCL data plane (one rank per GPU); "
                  f"{avail} visible.  Rehearse ranks that share a GPU with --dist-backend ipc.", file=sys.stderr)
            return 2
    touched = gpu_touched()
    if any(touched.values()):  # checked right before the fork + exec of the launcher
        print(f"bench.py: refusing to start the launcher from a process that initialised the GPU: {touched}",
              file=sys.stderr)
        return 5
    if dry:
        print(json.dumps({"launch": "dry-run", "gpus": n, "visible_gpus": avail, **touched}), flush=True)
        return 0
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    args_run = ["--nnodes=1", f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
                os.path.abspath(__file__), *sys.argv[1:]]
    # The launcher ends if this process is killed, even by SIGKILL (and through it every rank):
    # it asks for SIGTERM on its parent's death (PR_SET_PDEATHSIG) first thing, then checks
    # that parent is still this process, then runs torch.distributed.run as __main__.  Done
    # in the child itself rather than in a preexec_fn, which is unsafe in a process with threads.
    boot = ("import ctypes, os, runpy, signal, sys\n"
            "ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGTERM)\n"
            "if os.getppid() != int(sys.argv[1]):\n"
            "    sys.exit(125)\n"
            "sys.argv = ['torch.distributed.run'] + sys.argv[2:]\n"
            "runpy.run_module('torch.distributed.run', run_name='__main__', alter_sys=True)\n")
    cmd = [sys.executable, "-c", boot, str(os.getpid()), *args_run]
    env = dict(os.environ, HLSP2P_LAUNCHER="self")
    env.setdefault("OMP_NUM_THREADS", "1")
    print(f"# bench.py: launching {n} ranks: {sys.executable} -m torch.distributed.run {' '.join(args_run)}",
          file=sys.stderr, flush=True)
    # same process group as this one: whatever stops the bench stops its ranks too
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    lines = []

    def pump():  # rank 0's JSON line is kept for the parent's stdout; the rest goes to stderr
        for ln in proc.stdout:
            if ln.startswith("{"):
                lines.append(ln.strip())
            else:
                sys.stderr.write(ln)
                sys.stderr.flush()

    reader = threading.Thread(target=pump, daemon=True)
    reader.start()

    def kill_group(sig=signal.SIGTERM):  # torch.distributed.run stops its workers on SIGTERM
        try:
            proc.send_signal(sig)
        except ProcessLookupError:
            pass

    def on_signal(signum, frame):  # the driver stopping this process stops every rank
        kill_group()
        raise SystemExit(128 + signum)

    prev = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGTERM, signal.SIGINT)}
    try:
        try:
            rc = proc.wait(timeout=args.launch_timeout)
        except subprocess.TimeoutExpired:
            print(f"bench.py: {n}-rank job overran --launch-timeout {args.launch_timeout:.0f} s; killing it",
                  file=sys.stderr, flush=True)
            kill_group()
            try:
                proc.wait(timeout=15)
            except subprocess.TimeoutExpired:
                kill_group(signal.SIGKILL)
                proc.wait()
            return 124
    finally:
        for sg, h in prev.items():
            signal.signal(sg, h)
    reader.join(timeout=10)
    if rc != 0:
        print(f"bench.py: the {n}-rank job failed (exit {rc})", file=sys.stderr)
        return rc if rc > 0 else 1
    if not lines:
        print("bench.py: the rank processes printed no result line", file=sys.stderr)
        return 3
    rec = json.loads(lines[-1])
    if rec.get("n_gpus") != n:
        print(f"bench.py: asked for {n} ranks, the record reports n_gpus={rec.get('n_gpus')}", file=sys.stderr)
        return 4
    print(lines[-1], flush=True)
    return 0


def main() -> int:
    args = parse()
    launched = _launcher_world()
    if launched is None:
        if args.gpus is None:
            args.gpus = 1
        if args.gpus < 1:
            raise SystemExit("--gpus must be >= 1")
        if args.gpus > 1:
            return _self_launch(args)
    elif args.gpus is None:
        args.gpus = launched
    elif args.gpus != launched:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {launched} ranks "
                         f"(WORLD_SIZE={launched}); they must agree")
    # a round whose transfers are never matched (a dead or diverged peer), or a control
    # all-gather a peer never joins, fails the job with the rank's plan in the error: the
    # library's own deadlines (60 s / 300 s: gpuSwarm.roundTimeoutMs / controlTimeoutMs)
    if args.inflight is None:
        # 64, by measurement (profiles/r4_ab): the headline is PCIe-bound and flat at 128; the
        # HBM-origin probe was +10-20 % at 128 on round-3 boxes and -4 % on round 4's.  (The
        # round-3 2-rank fault at 128 was the CRC-table lifetime bug, fixed: profiles/r4_uaf.)
        # 96 from N=8 on: with 1/8 of the bytes on PCIe the rank's per-step host work is
        # co-bound with the DMA at 64, and more fragments per step amortize it (the single-GPU
        # projection of an 8-rank swarm, profiles/r6_inflight)
        world_env = int(os.environ.get("WORLD_SIZE", str(args.gpus or 1)))
        args.inflight = INFLIGHT_N8 if world_env >= 8 else 64
    if args.cache_gb is None:
        args.cache_gb = 8.0
    if args.config in LIVE and args.players < 1:
        raise SystemExit("live configs run in fleet mode: --players >= 1")
    if args.sync_steps and args.players:
        # the fleet's players pace the rounds with batches in flight; an unpipelined step is
        # a diagnostic of the in-process path only
        raise SystemExit("--sync-steps runs one player in the rank process: add --players 0")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    (preset, encrypted, seg_dur, desc, K, n_segments, W, origin_kwargs, hls_config,
     p2p_base) = _workload(args)
    players = _spawn_players(W, world, rank, origin_kwargs, hls_config, p2p_base, n_segments, seg_dur) \
        if W else None
    use_gpu = torch.cuda.is_available() and not args.cpu
    rccl_plane = use_gpu and world > 1 and args.dist_backend in ("auto", "nccl")
    if os.environ.get("HLSP2P_RCCL_REHEARSAL"):  # RCCL ranks sharing a GPU over its socket transport
        rccl_plane = False
    if use_gpu:
        n_dev = torch.cuda.device_count()
        if rccl_plane and local_rank >= n_dev:  # before any stream, event or communicator exists
            raise SystemExit(f"bench.py: rank {rank} (local rank {local_rank}) has no GPU of its own: {n_dev} "
                             f"visible for {os.environ.get('LOCAL_WORLD_SIZE', world)} local ranks.  The RCCL "
                             "data plane needs one GPU per rank; rehearse shared-GPU ranks with --dist-backend ipc.")
        local_dev = local_rank % n_dev  # the ipc / gloo rehearsals may share one GPU
        torch.cuda.set_device(local_dev)
        device = torch.device("cuda", local_dev)
        numa_node = _numa(args.numa, local_dev, world, W)  # before the pinned CDN buffers are allocated
        if players is not None and numa_node is not None:  # the players run next to their node
            for pr in players[1]:
                try:
                    os.sched_setaffinity(pr.pid, os.sched_getaffinity(0))
                except OSError:
                    pass
        pids = [os.getpid()] + ([pr.pid for pr in players[1]] if players else [])
        cpu_place = _place(args.cpu_place, local_dev, pids)
    else:
        device = torch.device("cpu")
        numa_node = None
        cpu_place = None
    args.cpu_place_applied = cpu_place
    import torch.distributed as dist

    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = args.dist_backend if args.dist_backend != "auto" else ("nccl" if use_gpu else "gloo")
        if backend == "ipc":  # rehearsal data plane (parallel/comm.py:_IpcOutbox) on a gloo group
            os.environ["HLSP2P_DATA_PLANE"] = "ipc"
            backend = "gloo"
        elif backend == "nccl":
            # RCCL data plane: the swarm node opens ONE native RCCL communicator per rank
            # (kernels/rccl_comm.cpp) over a gloo default group (rendezvous + control fallback);
            # an nccl default group would add torch's own, idle, communicator
            os.environ["HLSP2P_DATA_PLANE"] = "rccl"
            backend = "gloo"
        dist.init_process_group(backend)

    from hlsjs_p2p_wrapper_amd import Hls
    from hlsjs_p2p_wrapper_amd.agent import node_for_config
    from hlsjs_p2p_wrapper_amd.net import new_event_loop
    from hlsjs_p2p_wrapper_amd.net.origin import SyntheticHlsOrigin
    from hlsjs_p2p_wrapper_amd.player import MediaElement
    from hlsjs_p2p_wrapper_amd.player.transmux import pipeline_for

    loop = new_event_loop("real")
    t_pack = time.perf_counter()
    origin = SyntheticHlsOrigin(**origin_kwargs, pin_memory=use_gpu)
    if args.ingest == "hbm" and use_gpu:
        for pool in origin.pools:
            pool.data = pool.data.to(device)
    t_pack = time.perf_counter() - t_pack
    p2p_config = {**p2p_base,
                  "gpuSwarm": {"backend": "dist" if world > 1 else "local", "device": str(device),
                               "cacheBytes": int(args.cache_gb * (1 << 30)), "autoTick": False,
                               "cdnDedup": not args.no_dedup, "maxWantsPerRound": K}}
    if args.metrics_port is not None:
        p2p_config["gpuSwarm"]["metricsPort"] = args.metrics_port
    if not W and os.environ.get("HLSP2P_DEFER_VERIFY", "1") != "0":
        # the in-process player verifies received segments in its transmux batch (the CRC fused
        # into the decrypt), as the fleet's rank does for its players: no separate CRC pass
        p2p_config["gpuSwarm"]["deferVerify"] = True
    if os.environ.get("HLSP2P_DATA_PLANE") == "ipc" and world > 1:
        # rehearsal outbox (fixed size): a rank forwards at most every peer's wants of a round
        seg = max(max(pool.lengths) for pool in origin.pools)
        per_round = (world - 1) * K * max(1, W) * (seg + 512) + (1 << 20)
        os.environ.setdefault("HLSP2P_IPC_OUTBOX_BYTES", str(per_round))
    if world > 1:
        # the control all-gather's shared-memory slot: a round's message is ~16 + 6 words per
        # want + 5 per add + 4 per remove (agent/node.py:_encode); size it for this step's
        # wants with room for adds / removes of the same order, so no round falls back to gloo
        os.environ.setdefault("HLSP2P_SHM_SLOT_WORDS", str(max(16384, 64 + 20 * K * max(1, W))))
    node = node_for_config(p2p_config)
    if W:
        return _fleet(args, world, rank, device, use_gpu, node, origin, players, desc, encrypted, seg_dur,
                      numa_node, dist, t_pack)
    hls = Hls(hls_config, p2p_config)
    media = MediaElement(mode="drain", loop=loop)
    counters = {"buffered": 0, "errors": 0, "level_switches": 0}
    hls.on(Hls.Events.FRAG_BUFFERED, lambda e, d: counters.__setitem__("buffered", counters["buffered"] + 1))
    hls.on(Hls.Events.ERROR, lambda e, d: counters.__setitem__("errors", counters["errors"] + 1))
    hls.on(Hls.Events.LEVEL_SWITCH, lambda e, d: counters.__setitem__("level_switches", counters["level_switches"] + 1))
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda e, d: media.play())
    sc = hls.streamController
    pipe = pipeline_for(device, loop)

    def drain_ready():
        for _ in range(1000):
            if not loop._ready:
                return
            loop.run_once(block=False)

    # bring the player up to its first fragment requests (manifest, level, key)
    t_end = time.perf_counter() + 60
    while time.perf_counter() < t_end and not sc.inflight:
        loop.run_once(block=False)
        sc.tick()
        drain_ready()
    if not sc.inflight:
        raise RuntimeError("player did not start loading fragments")

    from hlsjs_p2p_wrapper_amd.utils.runtime import tune_gc
    from hlsjs_p2p_wrapper_amd.utils.trace import PhaseTimer

    if not args.no_gc_tune:
        tune_gc()  # freeze the start-up heap (playlists, engine, node): no full-GC pauses mid-round

    bt = PhaseTimer()

    # Software pipeline over steps (steady state, --lag + 2 rounds of fragments per peer):
    #   launch round t+lag (collective; device: H2D on the copy stream, RCCL / CRC on the node
    #     stream), so the DMA engine always has the next round queued behind the current one
    #   complete round t  -> onSuccess -> FRAG_LOADED -> transmux submit
    #   launch transmux batch t (decrypt + demux on the default stream, overlaps the rounds in flight)
    #   complete transmux batch t-1 -> FRAG_BUFFERED -> slots free -> player issues loads
    pipe.auto_flush = args.sync_steps
    import collections

    state = {"hs": collections.deque(), "b": None, "step": 0, "offline_steps": 0}

    def churn():
        # rotation: rank k is offline during the k-th N-step period of every (world + 1) periods
        if args.churn > 0 and world > 1:
            online = (state["step"] // args.churn) % (world + 1) != rank
            if online != node.online:
                node.set_online(online)
            state["offline_steps"] += 0 if online else 1
        state["step"] += 1

    def step():
        churn()
        t0 = time.perf_counter()
        if args.sync_steps:
            sc.tick()
            drain_ready()
            t1 = time.perf_counter()
            node.tick()
            drain_ready()
            t2 = time.perf_counter()
            pipe.flush()
            drain_ready()
        else:
            state["hs"].append(node.launch_round())
            t1 = time.perf_counter()
            if len(state["hs"]) > args.lag:
                node.complete_round(state["hs"].popleft())
            drain_ready()
            t2 = time.perf_counter()
            b = pipe.launch()
            t21 = time.perf_counter()
            pipe.complete(state["b"])
            t22 = time.perf_counter()
            if _PROF_C3:
                _PROF.enable()
            drain_ready()
            if _PROF_C3:
                _PROF.disable()
            t25 = time.perf_counter()
            bt.add("c1_tx_launch", t21 - t2)
            bt.add("c2_tx_complete", t22 - t21)
            bt.add("c3_drain", t25 - t22)
            sc.tick()
            drain_ready()
            state["b"] = b
            bt.add("d_player_loads", time.perf_counter() - t25)
        t3 = time.perf_counter()
        bt.add("a_launch_or_tick", t1 - t0)
        bt.add("b_node", t2 - t1)
        bt.add("c_transmux_player", t3 - t2)

    def sync():
        if use_gpu:
            torch.cuda.synchronize(device)
        if world > 1:
            node.comm.barrier()
        if use_gpu:
            torch.cuda.synchronize(device)

    calib = _calibrate(args, node, step, sync, world)  # before warmup: not in the timed window
    for _ in range(args.warmup):
        step()
    sync()
    bt.reset()
    node.timer.reset()
    pipe.timer.reset()
    b0, s0 = counters["buffered"], dict(node.stats)
    pf0 = node.p2p_from.copy()
    node.corrupt_next_recv = args.corrupt_recv
    t0 = time.perf_counter()
    if _PROF is not None and not _PROF_C3:
        _PROF.enable()
    for _ in range(args.steps):
        step()
    sync()
    if _PROF is not None:
        _PROF.disable()
    elapsed = time.perf_counter() - t0
    done = counters["buffered"] - b0
    d_cdn = node.stats["cdn"] - s0["cdn"]
    d_p2p = node.stats["p2p"] - s0["p2p"]
    d_segs = sum(node.stats[k] - s0[k] for k in ("cdn_segments", "p2p_segments"))
    vals = np.array([done, d_cdn, d_p2p, int(elapsed * 1e9), counters["errors"], d_segs], dtype=np.int64)
    per = _per_rank(node, pipe, s0, dict(node.stats), elapsed, args.steps, K)
    if world > 1:
        parts = node.comm.allgather_control(vals)
        tot = np.sum(np.stack(parts), axis=0)
        max_ns = max(int(p[3]) for p in parts)
        per_parts = node.comm.allgather_control(per)
    else:
        tot, max_ns, per_parts = vals, int(vals[3]), [per]
    max_s = max_ns / 1e9
    result = _result(args, world, tot, max_s, origin, K, desc, encrypted, seg_dur, use_gpu, numa_node, dist,
                     transport=getattr(node.comm, "data_transport", None))
    result["per_rank"] = _per_rank_dicts(per_parts, args.steps)
    result["config"]["receive_verify"] = "fused-decrypt" if getattr(node, "verify_deferred", False) else "node"
    result["data_plane"] = _plane_info(node, dist, world, device, node.p2p_from - pf0)
    if calib is not None:
        result["calibration"] = calib
    _label_rehearsal(result)
    if args.verbose:
        print(f"# rank {rank} pack {t_pack:.2f}s {_mem(use_gpu, device)} counters {counters} level {hls.currentLevel}\n"
              f"#   node stats {node.stats} last round {node.last_round}\n"
              f"#   step ms {bt.summary_ms(args.steps)}\n"
              f"#   node ms {node.timer.summary_ms(args.steps)}\n"
              f"#   transmux ms {pipe.timer.summary_ms(args.steps)}", file=sys.stderr)
    _dump_profile(rank)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        node.comm.barrier()
        node.comm.close()  # the native RCCL communicator (collective, every rank is here)
        dist.destroy_process_group()
    return 0


def _fleet(args, world, rank, device, use_gpu, node, origin, players, desc, encrypted, seg_dur, numa_node, dist,
           t_pack):
    """Fleet mode (``--players W``): W player processes per GPU, each playing its own slice of
    the DVR window through the bundle ``Hls`` over a ``RemoteNode``; this process runs the
    node (rounds, CDN DMA, RCCL, CRC) and the batched GPU transmux (``parallel/fleet.py``).
    The timed window is K node steps; the fragments counted are those the players buffered
    between two in-band marks sent at its edges (a mark follows every answer sent before it
    through the same pipe)."""
    import collections

    from hlsjs_p2p_wrapper_amd.net.event_loop import get_event_loop
    from hlsjs_p2p_wrapper_amd.parallel.fleet import FleetServer
    from hlsjs_p2p_wrapper_amd.player.transmux import pipeline_for
    from hlsjs_p2p_wrapper_amd.utils.runtime import cpu_calibration_us, tune_gc

    W, K = args.players, args.inflight
    conns, procs = players
    loop = get_event_loop()  # the node's loop: cache hits and failures are delivered from it
    pipe = pipeline_for(device, loop)
    pipe.auto_flush = False
    server = FleetServer(node, pipe, conns)
    node.max_wants_per_round = K * W  # every player gets K fragments per round
    state = {"hs": collections.deque(), "b": None}

    def drain_ready():
        for _ in range(1000):
            if not loop._ready:
                return
            loop.run_once(block=False)

    debug = os.environ.get("HLSP2P_FLEET_DEBUG")
    nstep = [0]
    from hlsjs_p2p_wrapper_amd.utils.trace import PhaseTimer

    fleet_timer = PhaseTimer()

    live = args.config in LIVE
    pace = {"next": 0.0}

    def step():
        if live:  # a live channel: rounds at a fixed wall-clock cadence, not as fast as possible
            now = time.perf_counter()
            if pace["next"] > now:
                time.sleep(pace["next"] - now)
            pace["next"] = max(pace["next"], now) + args.round_ms / 1e3
        if args.churn > 0 and world > 1:  # BASELINE config 3: the same rotation as the in-process path
            online = (nstep[0] // args.churn) % (world + 1) != rank
            if online != node.online:
                node.set_online(online)
        pc = time.perf_counter
        t0 = pc()
        drain_ready()
        server.await_players()  # the players' next requests (paces the rounds by the players)
        t1 = pc()
        server.poll()
        server.admit(K)  # K per player and round: players keep the same pace on every rank
        t2 = pc()
        state["hs"].append(node.launch_round())
        if len(state["hs"]) > args.lag:
            node.complete_round(state["hs"].popleft())
        t3 = pc()
        b = server.launch_transmux()
        server.complete_transmux(state["b"])
        t4 = pc()
        server.send()
        state["b"] = b
        t5 = pc()
        # the rank's step split: waiting on players vs its own host work (per phase)
        ft = fleet_timer.total
        ft["await_players"] += t1 - t0
        ft["poll_admit"] += t2 - t1
        ft["rounds"] += t3 - t2
        ft["transmux"] += t4 - t3
        ft["send"] += t5 - t4
        nstep[0] += 1
        if debug and nstep[0] % 20 == 0:
            print(f"# fleet step {nstep[0]} round {node.round} wants {node.pending()} "
                  f"queued {[q.n for q in server._q]} requests {server.requests} sent {server.sent} "
                  f"delivered-queue {len(server._delivered)} last {node.last_round}", file=sys.stderr, flush=True)

    def sync():
        if use_gpu:
            torch.cuda.synchronize(device)
        if world > 1:
            node.comm.barrier()
        if use_gpu:
            torch.cuda.synchronize(device)

    def mark(tag):
        for c, o in zip(conns, server.open):
            if o:
                c.send(("mark", tag, {"calib": args.verbose}))

    try:
        # players start (imports, origin): wait for every player of every rank, then let them
        # all load at once; step until each has sent requests (collective on every rank)
        t_end = time.perf_counter() + 180
        while len(server.ready) < W:
            server.poll()
            time.sleep(0.005)
            if time.perf_counter() > t_end or not all(pr.is_alive() for pr in procs):
                raise RuntimeError("fleet players did not start")
        if world > 1:
            node.comm.barrier()
        go = {}
        if live:  # the channel's epoch: rank 0's clock, shared by every rank's node and players
            ep = np.array([int((time.time() + 0.2) * 1e6)], dtype=np.int64)
            if world > 1:
                ep = node.comm.allgather_control(ep)[0]
            origin.live_epoch = go["live_epoch"] = float(ep[0]) / 1e6
        for c in conns:
            c.send(("go", go))
        while True:
            step()
            up = np.array([int(all(n > 0 or not o for n, o in zip(server.requests, server.open)))],
                          dtype=np.int64)
            if world > 1:
                up = np.array([min(int(x[0]) for x in node.comm.allgather_control(up))], dtype=np.int64)
            if up[0]:
                break
            if time.perf_counter() > t_end or not all(pr.is_alive() for pr in procs):
                raise RuntimeError("fleet players did not start")
            time.sleep(0.002)
        if not args.no_gc_tune:
            tune_gc()
        calib = _calibrate(args, node, step, sync, world)  # before warmup: not in the timed window
        for _ in range(args.warmup):
            step()
        sync()
        node.timer.reset()
        pipe.timer.reset()
        fleet_timer.reset()
        s0 = dict(node.stats)
        pf0 = node.p2p_from.copy()
        pay0 = (server.payload_bytes, server.payload_wait_s)
        node.corrupt_next_recv = args.corrupt_recv
        calib0 = cpu_calibration_us() if args.verbose else 0.0
        mark("t0")
        t0 = time.perf_counter()
        if _PROF is not None:
            _PROF.enable()
        blocks, tb = [], t0  # soak analysis: wall ms per step over blocks of the window
        bs = max(1, args.steps // 10)
        for i in range(args.steps):
            step()
            if (i + 1) % bs == 0:
                tn = time.perf_counter()
                blocks.append(round((tn - tb) * 1e3 / bs, 3))
                tb = tn
        sync()
        elapsed = time.perf_counter() - t0
        fleet_ms = fleet_timer.summary_ms(args.steps)
        node_ms, tm_ms = node.timer.summary_ms(args.steps), pipe.timer.summary_ms(args.steps)
        win_fleet = dict(fleet_timer.total)
        win_fleet["payload_bytes"] = server.payload_bytes - pay0[0]
        win_fleet["payload_wait"] = server.payload_wait_s - pay0[1]
        s1_timers = (dict(node.timer.total), dict(pipe.timer.total))
        if _PROF is not None:
            _PROF.disable()
            _dump_profile(rank)
        calib1 = cpu_calibration_us() if args.verbose else 0.0
        mark("t1")
        s1 = dict(node.stats)
        pf1 = node.p2p_from.copy()
        # keep serving until every player has acknowledged both marks (collective rounds)
        t_end = time.perf_counter() + 120
        while True:
            step()
            got = server.marks.get("t1", {})
            ok = np.array([int(all(not o or w in got for w, o in enumerate(server.open)))], dtype=np.int64)
            if world > 1:
                ok = np.array([min(int(x[0]) for x in node.comm.allgather_control(ok))], dtype=np.int64)
            if ok[0]:
                break
            if time.perf_counter() > t_end:
                raise TimeoutError("fleet players did not acknowledge the window marks")
        m0, m1 = server.marks.get("t0", {}), server.marks["t1"]
        done = sum(m1[w]["buffered"] - m0.get(w, {"buffered": 0})["buffered"] for w in m1)
        lat = [x for w in m1 for x in m1[w].get("live_latency_s", [])]
        errors = sum(m1[w]["errors"] for w in m1)
        d_segs = sum(s1[k] - s0[k] for k in ("cdn_segments", "p2p_segments"))
        vals = np.array([done, s1["cdn"] - s0["cdn"], s1["p2p"] - s0["p2p"], int(elapsed * 1e9), errors, d_segs],
                        dtype=np.int64)
        per = _per_rank(node, pipe, s0, s1, elapsed, args.steps, K * W, fleet_total=win_fleet, timers=s1_timers)
        if world > 1:
            parts = node.comm.allgather_control(vals)
            tot = np.sum(np.stack(parts), axis=0)
            max_ns = max(int(x[3]) for x in parts)
            per_parts = node.comm.allgather_control(per)
        else:
            tot, max_ns, per_parts = vals, int(vals[3]), [per]
        result = _result(args, world, tot, max_ns / 1e9, origin, K, desc, encrypted, seg_dur, use_gpu, numa_node,
                         dist, players=W, transport=getattr(node.comm, "data_transport", None))
        result["per_rank"] = _per_rank_dicts(per_parts, args.steps)
        # how received segments were checked: by the CRC fused into the transmux decrypt
        # (deferred, fleet default) or by the node's own verify pass before delivery
        result["config"]["receive_verify"] = "fused-decrypt" if getattr(node, "verify_deferred", False) else "node"
        # whether CDN fetches get the CRC trailer peers check (a one-rank swarm sends nothing, so
        # it skips that pass; the headline is the same with it forced: profiles/r4_ingestcrc)
        result["config"]["ingest_crc"] = bool(getattr(node, "ingest_crc", True))
        # how a player's onSuccess payload reaches its bytes (RemoteSegment.data()): copied for
        # every fragment into the shared ring, or fetched from the HBM cache when read
        result["config"]["player_bytes"] = "ring" if args.fleet_payload else "on-demand"
        result["data_plane"] = _plane_info(node, dist, world, device, pf1 - pf0)
        if calib is not None:
            result["calibration"] = calib
        _label_rehearsal(result)
        if live:
            result["config"].update(live=True, live_speed=args.live_speed, live_window=args.live_window,
                                    round_ms=args.round_ms, evicted_segments=server.evicted)
            if lat:  # publication -> buffered, in media seconds (the live sync point is 30 s back)
                result["live_latency_s"] = {"p50": round(float(np.percentile(lat, 50)), 2),
                                            "p95": round(float(np.percentile(lat, 95)), 2), "n": len(lat)}
        if args.verbose:
            ipc = getattr(node.comm, "_ipc", None)
            plane = getattr(node.comm, "data_transport", "local") + (
                f" (events: {ipc._peer_ev is not None})" if ipc is not None else "")
            print(f"# rank {rank} pack {t_pack:.2f}s players {W} data plane {plane} {_mem(use_gpu, device)} "
                  f"marks {dict(m1)}\n"
                  f"#   node stats {node.stats} last round {node.last_round}\n"
                  f"#   node ms {node_ms}\n"
                  f"#   transmux ms {tm_ms}\n"
                  f"#   fleet step ms {fleet_ms}\n"
                  f"#   step ms by tenth of the window {blocks}\n"
                  f"#   core speed (fixed loop, us): rank {calib0:.0f} -> {calib1:.0f}; players "
                  f"{[round(m0[w].get('calib_us', 0)) for w in sorted(m0)]} -> "
                  f"{[round(m1[w].get('calib_us', 0)) for w in sorted(m1)]}\n"
                  f"#   player CPU per buffered fragment (us) {_player_cpu(m0, m1)}", file=sys.stderr)
        if rank == 0:
            print(json.dumps(result), flush=True)
    finally:
        for c, o in zip(conns, server.open):
            if o:
                try:
                    c.send(("stop",))
                except (OSError, BrokenPipeError):
                    pass
        for pr in procs:
            pr.join(timeout=20)
            if pr.is_alive():
                pr.kill()
                pr.join(timeout=5)
    if world > 1:
        node.comm.barrier()
        node.comm.close()
        dist.destroy_process_group()
    return 0


def _result(args, world, tot, max_s, origin, K, desc, encrypted, seg_dur, use_gpu, numa_node, dist, players=0,
            transport=None):
    """The JSON line (``tot``: [fragments buffered, cdn bytes, p2p bytes, ns, errors, segments]
    summed over ranks; ``max_s``: the slowest rank's timed window)."""
    # bytes per delivered segment over the timed region (an ABR ladder mixes renditions)
    seg_bytes = int((tot[1] + tot[2]) // max(1, tot[5])) if tot[5] else int(np.mean(origin.pools[0].lengths))
    inflight = K * max(1, players)
    return {
        "metric": "segments/sec + P2P offload ratio, 1080p 6 Mb/s HLS at 1/2/4/8 MI355X",
        "value": round(float(tot[0]) / max_s, 2),
        "unit": "segments/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(max_s * 1e3 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "uint8",
        "data": "synthetic",
        "offload_ratio": round(float(tot[2]) / max(1.0, float(tot[1] + tot[2])), 4),
        "goodput_GBps": round(float(tot[1] + tot[2]) / max_s / 1e9, 3),  # bytes delivered to the players
        "errors": int(tot[4]),
        "config": {"model": f"{desc}, {world} peer{'s' if world > 1 else ''} ({world} x MI355X)" if use_gpu
                   else f"{desc}, {world} peer{'s' if world > 1 else ''} (CPU)",
                   "offload": "measured" if world > 1 else "n/a (no peers: one rank fetches everything from the CDN)",
                   "global_batch": inflight * world, "seq_len": seg_bytes,
                   "parallelism": f"swarm{world}" + (f"-{_data_plane(dist, transport)}" if world > 1 else ""),
                   "inflight_per_gpu": inflight, "players_per_gpu": max(1, players),
                   "player_processes": players > 0, "encrypted": encrypted, "segment_s": seg_dur,
                   "churn_steps": args.churn, "device": "MI355X" if use_gpu else "cpu", "numa": numa_node,
                   "cpu_place": getattr(args, "cpu_place_applied", None) or "shared",
                   "ingest": args.ingest if use_gpu else "host"},
    }


from hlsjs_p2p_wrapper_amd.parallel.wire import XGMI_LINK_GBPS_PER_DIR  # noqa: E402

# per-rank diagnostics of the timed window, all-gathered as int64 milli-units (fixed order)
PER_RANK_FIELDS = ("rank", "rounds", "step_ms", "wait_device_us", "exchange_us", "exchange_queued_us", "control_us",
                   "plan_us",
                   "host_round_us",
                   "cdn_GBps", "cdn_dev_ms", "p2p_recv_MB", "p2p_sent_MB", "p2p_dev_ms", "p2p_GBps",
                   "p2p_links", "p2p_link_GBps", "transmux_dev_ms", "transmux_wait_us", "await_players_us",
                   "payload_GBps", "payload_wait_us", "crc_failures", "control_fallbacks", "deferred", "inflight",
                   "cu_reserve", "p2p_rejected_MB", "p2p_link_roof_GBps", "p2p_link_util")


def _per_rank(node, pipe, s0, s1, elapsed, steps, inflight, fleet_total=None, timers=None) -> np.ndarray:
    """This rank's timed-window diagnostics (``PER_RANK_FIELDS``): per ROUND host phases in
    us (``wait_device`` = host blocked on the round's device event, ``exchange`` = posting
    the data plane: microseconds for RCCL, which only enqueues, but the HIP-IPC rehearsal
    plane blocks there on its peers' packing, ``exchange_queued`` = host time from posting the
    exchange to the node stream reaching it (device event times mapped to host time through
    the last round the host waited on; average over the rounds measured), ``control`` =
    control all-gather + directory
    ingest, ``plan`` = plan_round + pins); the CDN rate over the
    window and the copy-stream (H2D) device ms per round; P2P received / sent MB per round,
    the node-stream exchange device ms per round (a peer's stall included), the received
    GB/s over that time, the source links per round and the GB/s per link (bytes per link
    over the exchange time: a lower bound on each xGMI link's rate); transmux device ms per
    step (default stream) and the host wait for it; fleet: per-step wait on the players, and
    with ``fleetPayload`` the D2H rate of the fragments' bytes into the players' ring and the
    per-step host wait on it."""
    rounds = max(1, s1["rounds"] - s0["rounds"])
    tm, pt = timers if timers is not None else (node.timer.total, pipe.timer.total)
    recv = s1.get("p2p_wire", s1["p2p"]) - s0.get("p2p_wire", s0["p2p"])  # wire bytes (checked or not): link rates
    sent = s1["upload"] - s0["upload"]
    links = s1.get("p2p_links", 0) - s0.get("p2p_links", 0)
    p2p_dev_s = tm.get("dev_p2p_ms", 0.0)  # seconds (PhaseTimer totals)
    host_round = sum(tm.get(k, 0.0) for k in ("control", "plan", "cdn_enqueue", "p2p_enqueue", "commit", "deliver"))
    try:
        from hlsjs_p2p_wrapper_amd.ops._native import device as _dev

        cu_reserve = _dev().cu_reserve() if node.is_cuda else 0
    except Exception:  # noqa: BLE001 - CPU rehearsal without the device module
        cu_reserve = 0
    vals = {
        "rank": node.rank, "rounds": rounds, "step_ms": elapsed * 1e3 / max(1, steps),
        "wait_device_us": tm.get("wait_device", 0.0) * 1e6 / rounds,
        "exchange_us": tm.get("p2p_enqueue", 0.0) * 1e6 / rounds,
        "exchange_queued_us": tm.get("exchange_queued", 0.0) * 1e6 / max(1.0, tm.get("exchange_queued_n", 0.0)),
        "control_us": tm.get("control", 0.0) * 1e6 / rounds,
        "plan_us": tm.get("plan", 0.0) * 1e6 / rounds,
        "host_round_us": host_round * 1e6 / rounds,
        "cdn_GBps": (s1["cdn"] - s0["cdn"]) / max(elapsed, 1e-9) / 1e9,
        "cdn_dev_ms": tm.get("dev_cdn_ms", 0.0) * 1e3 / rounds,
        "p2p_recv_MB": recv / rounds / 1e6, "p2p_sent_MB": sent / rounds / 1e6,
        "p2p_dev_ms": p2p_dev_s * 1e3 / rounds,
        "p2p_GBps": recv / p2p_dev_s / 1e9 if p2p_dev_s > 0 else 0.0,
        "p2p_links": links / rounds,
        "p2p_link_GBps": recv / links / (p2p_dev_s / rounds) / 1e9 if links and p2p_dev_s > 0 else 0.0,
        "transmux_dev_ms": pt.get("dev_transmux", 0.0) * 1e3 / max(1, steps),
        "transmux_wait_us": pt.get("wait_device", 0.0) * 1e6 / max(1, steps),
        "await_players_us": (fleet_total or {}).get("await_players", 0.0) * 1e6 / max(1, steps),
        "payload_GBps": (fleet_total or {}).get("payload_bytes", 0) / max(elapsed, 1e-9) / 1e9,
        "payload_wait_us": (fleet_total or {}).get("payload_wait", 0.0) * 1e6 / max(1, steps),
        "crc_failures": s1["crc_failures"] - s0["crc_failures"],
        "control_fallbacks": getattr(node.comm, "control_fallbacks", 0),
        "deferred": s1.get("deferred", 0) - s0.get("deferred", 0),
        "inflight": inflight, "cu_reserve": cu_reserve,
        # peer bytes whose CRC check failed (re-fetched from the CDN; not in offload_ratio)
        "p2p_rejected_MB": (s1.get("p2p_rejected", 0) - s0.get("p2p_rejected", 0)) / 1e6,
        # the per-direction roofline of one xGMI link beside the measured per-link receive rate
        # (p2p_link_GBps is a lower bound on the link's rate: bytes over the whole exchange time)
        "p2p_link_roof_GBps": XGMI_LINK_GBPS_PER_DIR,
        "p2p_link_util": (recv / links / (p2p_dev_s / rounds) / 1e9 / XGMI_LINK_GBPS_PER_DIR
                          if links and p2p_dev_s > 0 else 0.0),
    }
    return np.array([int(round(float(vals[k]) * 1000)) for k in PER_RANK_FIELDS], dtype=np.int64)


def _per_rank_dicts(parts, steps) -> list:
    """Decode the gathered rows; add each rank's ``bound`` label.

    Rule: the busiest device stream -- ``pcie`` (H2D copy stream), ``xgmi`` (the node
    stream's exchange), ``transmux`` (decrypt + demux), ``pcie_d2h`` (the fleet payload copy;
    its host wait stands for its busy time) -- when it is busy for >= 80 % of a step (the
    pipeline keeps it saturated), or when the host waited on the device for more than 30 % of
    a step (``wait_device`` and ``exchange`` per round x rounds per step + the transmux and
    payload waits); otherwise ``players`` when the fleet's wait on its players exceeds half a
    step, else ``host``."""
    out = []
    for p in parts:
        d = {k: float(v) / 1000 for k, v in zip(PER_RANK_FIELDS, np.asarray(p).tolist())}
        for k in ("rank", "rounds", "crc_failures", "control_fallbacks", "deferred", "inflight", "cu_reserve"):
            d[k] = int(round(d[k]))
        for k, v in list(d.items()):
            if isinstance(v, float):
                d[k] = round(v, 3)
        step = max(d["step_ms"], 1e-9)
        rps = d["rounds"] / max(1, steps)
        waited = ((d["wait_device_us"] + d["exchange_us"]) * rps + d["transmux_wait_us"] + d["payload_wait_us"]) / 1e3
        busy = {"pcie": d["cdn_dev_ms"] * rps, "xgmi": d["p2p_dev_ms"] * rps, "transmux": d["transmux_dev_ms"],
                "pcie_d2h": d["payload_wait_us"] / 1e3}
        top = max(busy, key=busy.get)
        if busy[top] >= 0.8 * step or waited > 0.3 * step:
            d["bound"] = top
        elif d["await_players_us"] / 1e3 > 0.5 * step:
            d["bound"] = "players"
        else:
            d["bound"] = "host"
        out.append(d)
    return out


def _plane_info(node, dist, world: int, device, recv_from=None) -> dict:
    """Which transports the run actually used (the data plane may fall back; see
    parallel/comm.py) and the topology that proves an N > 1 record: per rank (all-gathered,
    collective) its host, local rank, device index and PCI address, what the data plane
    reports about itself (for RCCL: ``ncclCommCount`` / ``ncclCommUserRank`` /
    ``ncclCommCuDevice``, rounds posted, version) and the bytes it received from each source
    peer over the timed window (``recv_from``: the fan-in over the point-to-point links).
    ``distinct_devices``: no two ranks drive the same GPU (required on the RCCL plane: the
    run fails otherwise).  ``hsa_ipc_legacy``: the HSA IPC mode the process started with
    (``0`` = dmabuf: RCCL's intra-node P2P transport and the HIP-IPC rehearsal export device
    buffers with ``hipIpcGetMemHandle``, which fails with ``invalid argument`` under the
    legacy mode on this host driver, ``tools/ipc_probe.py``)."""
    import socket

    comm = node.comm
    ipc = getattr(comm, "_ipc", None)
    transport = getattr(comm, "data_transport", "local")
    bus = None
    if device.type == "cuda":
        try:
            from hlsjs_p2p_wrapper_amd.ops._native import device as _dev

            bus = _dev().pci_bus_id(device.index)
        except Exception:  # noqa: BLE001 - reported as unknown
            bus = None
    me = {"rank": node.rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "host": socket.gethostname(),
          "device": device.index if device.type == "cuda" else None, "pci_bus_id": bus,
          "rounds": int(node.stats["rounds"]),
          "recv_bytes_from": [int(x) for x in (recv_from if recv_from is not None else node.p2p_from)]}
    topo = getattr(comm, "topology", None)
    if topo is not None:
        me["comm"] = topo()
    ranks = [me]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    devs = [(r["host"], r["pci_bus_id"]) for r in ranks if r["pci_bus_id"] is not None]
    distinct = len(set(devs)) == len(devs) if len(devs) == len(ranks) else None
    rehearsal = next((r["comm"].get("rehearsal") for r in ranks if r.get("comm", {}).get("rehearsal")), None)
    if transport.startswith("rccl") and distinct is not True and rehearsal is None:
        raise RuntimeError(f"RCCL data plane without one GPU per rank: {[(r['rank'], r['pci_bus_id']) for r in ranks]}")
    rccl = next((r["comm"]["rccl"] for r in ranks if "rccl" in r.get("comm", {})), None)
    # the wire each rank's RCCL connections actually use (RCCL's own connection log: P2P over
    # xGMI, or a NET fallback) and HIP's link type to its peers (parallel/wire.py)
    from hlsjs_p2p_wrapper_amd.parallel.wire import degraded, link_kinds
    for r in ranks:
        w = r.get("comm", {}).get("wire")
        r["transport"] = w.get("transport") if w else None
    wires = sorted({r["transport"] for r in ranks if r["transport"]})
    return {"data": transport, "control": getattr(comm, "control_transport", "local"),
            "ipc_events": bool(ipc is not None and ipc._peer_ev is not None),
            "shm_slot_words": getattr(comm, "shm_slot_words", None),
            "hsa_ipc_legacy": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY"),
            "launcher": os.environ.get("HLSP2P_LAUNCHER") or ("torchrun" if "TORCHELASTIC_RUN_ID" in os.environ
                                                              else "env" if world > 1 else "none"),
            "world": world, "distinct_devices": distinct, "rccl_rehearsal": rehearsal,
            "rccl_version": rccl["version"] if rccl else None, "wire": wires, "hip_links": link_kinds(ranks),
            "transport_degraded": degraded(transport, distinct, rehearsal, wires), "ranks": ranks}


def _label_rehearsal(result: dict) -> None:
    """A run whose RCCL ranks share GPUs (``HLSP2P_RCCL_REHEARSAL``) says so in its config:
    the model names the devices actually used and the parallelism the transport."""
    dp = result.get("data_plane") or {}
    if dp.get("transport_degraded"):
        # one GPU per rank, yet RCCL connected some pair over a network transport: the number
        # is real but it is not an xGMI number, and the record says so where it is read first
        cfg = result["config"]
        cfg["model"] += f" [RCCL fell back to {'/'.join(dp.get('wire') or [])}: NOT an xGMI run]"
        cfg["parallelism"] += "-degraded"
        print(f"bench.py: WARNING: RCCL transport degraded on a one-GPU-per-rank run: {dp.get('wire')}; "
              "see data_plane.ranks[*].comm.wire", file=sys.stderr, flush=True)
        if os.environ.get("HLSP2P_REQUIRE_XGMI") == "1":
            raise RuntimeError(f"RCCL data plane did not use its P2P transport: {dp.get('wire')}")
    if not dp.get("rccl_rehearsal"):
        return
    devs = {(r["host"], r["pci_bus_id"]) for r in dp.get("ranks", [])}
    cfg = result["config"]
    cfg["model"] = cfg["model"].rsplit(", ", 1)[0] + (f", {result['n_gpus']} peers sharing {len(devs)} MI355X "
                                                  f"(native RCCL over its {dp['rccl_rehearsal']} transport: "
                                                  "a rehearsal, not an xGMI run)")
    cfg["parallelism"] += f"-{dp['rccl_rehearsal']}"
    for r in result.get("per_rank", []):  # the exchange ran over the rehearsal transport, not xGMI
        if r.get("bound") == "xgmi":
            r["bound"] = f"exchange-{dp['rccl_rehearsal']}"


def _mem(use_gpu, device) -> str:
    """Peak memory of this rank (soak runs: the HBM arena is allocated once, so the device
    peak must not grow with the step count; host: the process's peak RSS)."""
    hwm = "?"
    try:
        with open("/proc/self/status") as f:
            hwm = next((ln.split()[1] for ln in f if ln.startswith("VmHWM:")), "?")
    except OSError:
        pass
    dev = f"hbm peak {torch.cuda.max_memory_allocated(device) / 2**30:.2f} GiB " if use_gpu else ""
    return f"{dev}host peak {int(hwm) / 2**20:.2f} GiB" if hwm != "?" else dev


def _data_plane(dist, transport) -> str:
    """Label of the data plane the node's comm actually uses (an IPC request that could not
    be honoured reports gloo)."""
    if transport and transport.startswith("rccl"):
        return "rccl"
    return "ipc" if transport == "hip-ipc" else "gloo"


def _player_cpu(m0: dict, m1: dict) -> list:
    """Per fleet player: CPU seconds spent between the window marks over fragments buffered."""
    out = []
    for w in sorted(m1):
        a, b = m0.get(w, {}), m1[w]
        n = b["buffered"] - a.get("buffered", 0)
        if n > 0 and "cpu_s" in a and "cpu_s" in b:
            out.append(round((b["cpu_s"] - a["cpu_s"]) * 1e6 / n, 1))
    return out


def _dump_profile(rank: int) -> None:
    if _PROF is not None:
        import io
        import pstats

        out = io.StringIO()
        st = pstats.Stats(_PROF, stream=out)
        st.sort_stats("tottime").print_stats(45)
        st.sort_stats("cumtime").print_stats(60)
        with open(os.environ["HLSP2P_PROFILE"] + f".{rank}.txt", "w") as f:
            f.write(out.getvalue())


if __name__ == "__main__":
    sys.exit(main())
