"""Which wire an N > 1 run used, and how bench.py's self-launch counts GPUs (round-5 VERDICT
Next 1).  The RCCL log lines below are built from librccl's own format strings
(``strings librccl.so``: ``Channel %02d/%01d : %d[%lx] -> %d[%lx] via P2P/IPC%s%s comm %p
nRanks %02d``, ``... [send] via NET/%s/%d%s%s%s comm %p nRanks %02d``, ``comm %p rank %d
nRanks %d nNodes %d localRanks %d localRank %d MNNVL %d``)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

from hlsjs_p2p_wrapper_amd.parallel import wire
from hlsjs_p2p_wrapper_amd.utils import runtime

REPO = Path(__file__).resolve().parents[1]

XGMI_LOG = """\
host:1234:1250 [0] NCCL INFO comm 0x5600 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0 MNNVL 0
host:1234:1250 [0] NCCL INFO Channel 00/1 : 0[0] -> 1[1] via P2P/IPC comm 0x5600 nRanks 08
host:1234:1250 [0] NCCL INFO Channel 01/1 : 0[0] -> 2[2] via P2P/IPC/read comm 0x5600 nRanks 08
host:1234:1250 [0] NCCL INFO Channel 00/1 : 3[3] -> 0[0] via P2P/direct pointer comm 0x5600 nRanks 08
host:1234:1250 [0] NCCL INFO Channel 00/1 : 0[0] -> 3[3] via P2P/IPC comm 0x5600 nRanks 08
"""

SOCKET_LOG = """\
h:1:2 [0] NCCL INFO comm 0x7f rank 1 nRanks 2 nNodes 2 localRanks 1 localRank 0 MNNVL 0
h:1:2 [0] NCCL INFO Channel 00/1 : 1[c1000] -> 0[c1000] [send] via NET/Socket/0 comm 0x7f nRanks 02
h:1:2 [0] NCCL INFO Channel 00/1 : 0[c1000] -> 1[c1000] [receive] via NET/Socket/0 comm 0x7f nRanks 02
h:1:2 [0] NCCL INFO Connected all trees
"""


def test_parse_xgmi_log():
    rep = wire.parse_rccl_log(XGMI_LOG, 0)
    assert rep["peers"] == {"1": ["P2P/IPC"], "2": ["P2P/IPC"], "3": ["P2P/IPC", "P2P/direct pointer"]}
    assert (rep["n_ranks"], rep["n_nodes"], rep["local_ranks"]) == (8, 1, 8)
    assert rep["connections"] == 4
    assert wire.summarize(rep, 4) == "p2p"
    assert wire.summarize(rep, 8) == "p2p-partial"  # 4 of 7 peers connected so far


def test_parse_socket_log_is_net():
    rep = wire.parse_rccl_log(SOCKET_LOG, 1)
    assert rep["peers"] == {"0": ["NET/Socket"]} and rep["n_nodes"] == 2
    assert wire.summarize(rep, 2) == "net"
    # one GPU per rank, no rehearsal, a NET pair: degraded; a socket rehearsal is not
    assert wire.degraded("rccl-native", True, None, ["net"])
    assert not wire.degraded("rccl-native", None, "socket", ["net"])
    assert not wire.degraded("rccl-native", True, None, ["p2p"])
    assert not wire.degraded("hip-ipc", True, None, ["net"])
    assert wire.degraded("rccl-native", True, None, ["p2p", "shm"])  # P2P refused: through host memory
    ranks = [{"comm": {"wire": {"links": {"1": "XGMI/1", "2": "XGMI/1"}}}},
             {"comm": {"wire": {"links": {"0": "XGMI/1", "2": "PCIE/2"}}}}, {"comm": {}}]
    assert wire.link_kinds(ranks) == ["PCIE", "XGMI"]


def test_world_of_one_is_self_and_missing_log_unknown():
    rep = wire.parse_rccl_log("x NCCL INFO comm 0x1 rank 0 nRanks 1 nNodes 1 localRanks 1 localRank 0 MNNVL 0\n", 0)
    assert rep["peers"] == {} and wire.summarize(rep, 1) == "self"
    assert wire.summarize(None, 2) == "unknown"
    assert wire.read_rccl_log(None, 0) is None
    assert wire.read_rccl_log("/nonexistent/rccl.log", 0) is None


def test_configure_rccl_log(monkeypatch, tmp_path):
    for k in ("NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS", "HLSP2P_RCCL_WIRE_LOG"):
        monkeypatch.delenv(k, raising=False)
    p = wire.configure_rccl_log(3, str(tmp_path))
    assert p == os.environ["NCCL_DEBUG_FILE"] and p.startswith(str(tmp_path)) and p.endswith(".rank3.log")
    assert os.environ["NCCL_DEBUG"] == "INFO" and "COLL" not in os.environ["NCCL_DEBUG_SUBSYS"]
    # the user's own setting wins; a literal file of theirs is still read back
    monkeypatch.setenv("NCCL_DEBUG", "INFO")
    monkeypatch.setenv("NCCL_DEBUG_FILE", str(tmp_path / "mine.%h.%p"))
    assert wire.configure_rccl_log(0) == str(tmp_path / f"mine.{os.uname().nodename}.{os.getpid()}")
    monkeypatch.setenv("NCCL_DEBUG", "INFO")  # INFO on the console: the user's choice, kept
    monkeypatch.delenv("NCCL_DEBUG_FILE")
    assert wire.configure_rccl_log(0) is None
    monkeypatch.setenv("NCCL_DEBUG", "VERSION")  # a lower level (the pool's environment): raised to INFO
    p = wire.configure_rccl_log(2, str(tmp_path))
    assert p.endswith(".rank2.log") and os.environ["NCCL_DEBUG"] == "INFO" and os.environ["NCCL_DEBUG_FILE"] == p
    monkeypatch.delenv("NCCL_DEBUG")
    monkeypatch.setenv("HLSP2P_RCCL_WIRE_LOG", "0")
    assert wire.configure_rccl_log(0) is None
    f = tmp_path / "r.log"
    f.write_text(SOCKET_LOG)
    rep = wire.read_rccl_log(str(f), 1)
    assert rep["peers"] == {"0": ["NET/Socket"]} and rep["log_bytes"] == len(SOCKET_LOG)


def _fake_kfd(tmp_path, nodes):
    topo = tmp_path / "topology" / "nodes"
    dev = tmp_path / "dri"
    dev.mkdir(parents=True)
    for i, (simd, minor, present) in enumerate(nodes):
        d = topo / str(i)
        d.mkdir(parents=True)
        props = f"cpu_cores_count {0 if simd else 64}\nsimd_count {simd}\ngpu_id {1000 + i if simd else 0}\n"
        if minor is not None:
            props += f"drm_render_minor {minor}\n"
        (d / "properties").write_text(props)
        if present and minor is not None:
            (dev / f"renderD{minor}").write_bytes(b"")
    return str(topo), str(dev)


def test_kfd_gpu_count_and_visibility(tmp_path, monkeypatch):
    # two CPU nodes, four GPU nodes, one of them not passed through (no render node)
    topo, dev = _fake_kfd(tmp_path, [(0, None, False), (0, None, False), (1024, 128, True), (1024, 136, True),
                                     (1024, 144, False), (1024, 152, True)])
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(k, raising=False)
    gpus = runtime.kfd_gpus(topo, dev)
    assert [g["render_minor"] for g in gpus] == [128, 136, 144, 152]
    assert [g["usable"] for g in gpus] == [True, True, False, True]
    assert runtime.visible_gpu_count(topo, dev) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,2")
    assert runtime.visible_gpu_count(topo, dev) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "-1")
    assert runtime.visible_gpu_count(topo, dev) == 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,7,0")  # stops at the first invalid index
    assert runtime.visible_gpu_count(topo, dev) == 1
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "1")
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "0,1")
    assert runtime.visible_gpu_count(topo, dev) == 1
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "2")  # HIP indexes the devices ROCr kept: 0 and 1
    assert runtime.visible_gpu_count(topo, dev) == 0
    assert runtime.visible_gpu_count(str(tmp_path / "none"), dev) == 0


def test_gpu_touched_in_a_fresh_process():
    code = ("import torch, json\nfrom hlsjs_p2p_wrapper_amd.utils.runtime import gpu_touched\n"
            "print(json.dumps(gpu_touched()))\n")
    p = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=str(REPO)))
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == {"torch_initialized": False, "kfd_mapped": False,
                                                            "kfd_open": False}


def test_self_launch_dry_run_checks_the_parent():
    """``bench.py --gpus 2`` without a launcher, stopped right before it would start the
    launcher: GPUs counted without HIP, no HIP context and no /dev/kfd in the parent."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=str(REPO), HLSP2P_LAUNCH_DRYRUN="1")
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["launch"] == "dry-run" and rec["gpus"] == 2
    assert not rec["torch_initialized"] and not rec["kfd_mapped"] and not rec["kfd_open"]
    assert rec["visible_gpus"] == runtime.visible_gpu_count()


@pytest.mark.gpu
def test_self_launch_parent_never_touches_the_gpu(cuda):
    """On the GPU box: the self-launch's GPU count (KFD topology) equals what HIP reports in a
    separate process, and the parent reaches the launcher's fork with no HIP context, no
    /dev/kfd mapping and no /dev/kfd descriptor -- with the count faked past the box's one GPU
    (dry run: the refusal for too few GPUs is skipped, the checks run)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(REPO)
    hip = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"], cwd=REPO,
                         env=env, capture_output=True, text=True, timeout=120)
    assert hip.returncode == 0, hip.stderr[-2000:]
    n_hip = int(hip.stdout.strip().splitlines()[-1])
    n = n_hip + 1
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(n)], cwd=REPO,
                       env=dict(env, HLSP2P_LAUNCH_DRYRUN="1"), capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    rec = json.loads(p.stdout.strip().splitlines()[-1])
    assert rec["visible_gpus"] == n_hip, (rec, n_hip)
    assert not rec["torch_initialized"] and not rec["kfd_mapped"] and not rec["kfd_open"], rec


def test_a_degraded_record_says_so(monkeypatch):
    """bench.py's labelling of an N>1 record whose RCCL pairs fell back to a network transport
    with one GPU per rank: the model says it is not an xGMI run, the parallelism ends in
    -degraded; HLSP2P_REQUIRE_XGMI=1 fails the run instead."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def record():
        return {"n_gpus": 8, "config": {"model": "1080p, 8 peers (8 x MI355X)", "parallelism": "swarm8-rccl"},
                "per_rank": [{"bound": "xgmi"}],
                "data_plane": {"wire": ["net", "p2p"], "transport_degraded": True, "rccl_rehearsal": None,
                               "ranks": []}}

    monkeypatch.delenv("HLSP2P_REQUIRE_XGMI", raising=False)
    r = record()
    bench._label_rehearsal(r)
    assert r["config"]["model"].endswith("[RCCL fell back to net/p2p: NOT an xGMI run]")
    assert r["config"]["parallelism"] == "swarm8-rccl-degraded"
    monkeypatch.setenv("HLSP2P_REQUIRE_XGMI", "1")
    with pytest.raises(RuntimeError, match="did not use its P2P transport"):
        bench._label_rehearsal(record())
    ok = record()
    ok["data_plane"].update(wire=["p2p"], transport_degraded=False)
    bench._label_rehearsal(ok)
    assert ok["config"]["parallelism"] == "swarm8-rccl" and "NOT" not in ok["config"]["model"]
