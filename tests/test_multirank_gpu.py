"""multi-rank runs on the GPU box.  The pool's box has ONE MI355X and RCCL
cannot place two ranks on one GPU, so two torchrun ranks share the card with a gloo data
plane (GPU tensors staged through host memory) or the HIP-IPC outbox data plane
(device-to-device copies, ``parallel/comm.py:_IpcOutbox``).  Everything else is the production N>1
path of bench.py: control all-gather, native planning, CDN seeding + same-round
forwarding, per-pair buffers with CRC trailers verified on device, async rounds, batched
decrypt + demux, FRAG_BUFFERED accounting."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("plane", ["gloo", "ipc"])
def test_two_ranks_share_one_gpu_bench_path(cuda, plane):
    """``gloo``: GPU tensors staged through host memory; ``ipc``: device-to-device copies out
    of the peers' HIP-IPC outboxes (parallel/comm.py:_IpcOutbox)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"), "--gpus", "2", "--steps", "4",
           "--warmup", "2", "--inflight", "16", "--pool", "16", "--cache-gb", "1", "--dist-backend", plane]
    env = dict(os.environ, PYTHONPATH=str(REPO))
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert p.returncode == 0, p.stderr[-4000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["errors"] == 0
    assert res["offload_ratio"] == pytest.approx(0.5, abs=0.02)  # every segment fetched once, shared once
    assert res["value"] > 0 and res["config"]["parallelism"] == f"swarm2-{plane}"


@pytest.mark.gpu
def test_two_ranks_ipc_events_bench_scale(cuda):
    """Bench-scale state on the rehearsal plane (round-3 VERDICT weak 3): 4 players x 64 in
    flight per rank (256 wants a round: the store's entry ids pass 1024 by round 5, where the
    old CRC table grew under queued scatters), a 6 GB arena per rank, interprocess events
    on, and 250 timed rounds (the event ring is renewed after 240 exchanges)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"), "--gpus", "2", "--steps", "250",
           "--warmup", "5", "--inflight", "64", "--players", "4", "--cache-gb", "6", "--dist-backend", "ipc"]
    env = dict(os.environ, PYTHONPATH=str(REPO), HLSP2P_IPC_EVENTS="1")
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["errors"] == 0 and res["data_plane"]["ipc_events"]
    assert res["offload_ratio"] == pytest.approx(0.5, abs=0.05)
    for r in res["per_rank"]:
        assert r["rounds"] >= 250 and r["crc_failures"] == 0 and r["control_fallbacks"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("players", ["2", "0"])
def test_two_ranks_corrupted_peer_copies_caught_by_the_fused_verify(cuda, players):
    """Both player modes on the GPU: received segments are verified by the CRC fused into the
    decrypt (profiles/r4_fused) -- the fleet rank's batch for its players, or the in-process
    player's own batch (gpuSwarm.deferVerify).  A peer copy corrupted on arrival in each of
    the first 3 timed rounds must be caught there, detached and re-fetched from the CDN, and
    no player may see an error."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(REPO / "bench.py"), "--gpus", "2", "--steps", "20",
           "--warmup", "4", "--inflight", "16", "--players", players, "--cache-gb", "2", "--dist-backend", "ipc",
           "--ingest", "hbm", "--corrupt-recv", "3"]
    env = dict(os.environ, PYTHONPATH=str(REPO))
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=420)
    assert p.returncode == 0, p.stderr[-4000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["errors"] == 0 and res["value"] > 0
    assert res["config"]["receive_verify"] == "fused-decrypt"
    fails = sum(r["crc_failures"] for r in res["per_rank"])
    assert 1 <= fails <= 6  # at most one per corrupted round on each rank


@pytest.mark.gpu
def test_native_rccl_plane_with_ranks_sharing_the_gpu(cuda):
    """The production native RCCL data plane at N=2 on the one GPU: each rank presents RCCL a
    host id of its own (HLSP2P_RCCL_REHEARSAL=socket), so RCCL connects the ranks over its
    socket transport instead of refusing duplicate devices.  bench.py self-launches the ranks
    (no torchrun); the round's group calls go through the pointer-column path; a corrupted
    peer copy in each of the first 3 timed rounds is caught by the in-process player's fused
    verify and re-fetched; the record shows RCCL's own view (2 ranks, rounds posted)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=str(REPO), HLSP2P_RCCL_REHEARSAL="socket")
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "10", "--warmup", "3",
                        "--cache-gb", "2", "--inflight", "16", "--players", "0", "--ingest", "hbm",
                        "--corrupt-recv", "3"], cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-4000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["errors"] == 0 and res["value"] > 0
    assert res["config"]["receive_verify"] == "fused-decrypt"
    assert res["config"]["parallelism"] == "swarm2-rccl-socket" and "rehearsal" in res["config"]["model"]
    dp = res["data_plane"]
    assert dp["data"] == "rccl-native" and dp["rccl_rehearsal"] == "socket" and dp["launcher"] == "self"
    # the wire, from RCCL's own connection log: every peer over its socket transport (the
    # parser's positive control: on an 8-GPU node the same record must say P2P)
    assert dp["wire"] == ["net"] and dp["transport_degraded"] is False  # a rehearsal, labelled as such
    for r in dp["ranks"]:
        rc = r["comm"]["rccl"]
        assert rc["count"] == 2 and rc["rank"] == r["rank"] and rc["rounds"] > 0
        assert sum(r["recv_bytes_from"]) > 0
        w = r["comm"]["wire"]
        assert r["transport"] == "net" and w["peers"] == {str(1 - r["rank"]): ["NET/Socket"]}, w
        assert w["n_nodes"] == 2 and w["log_bytes"] < (1 << 20), w
        assert w["links"] == {str(1 - r["rank"]): "same-device"}, w
    assert 1 <= sum(r["crc_failures"] for r in res["per_rank"]) <= 6
