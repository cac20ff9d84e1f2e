"""Library users get the bench's fail-fast deadlines (round-5 VERDICT Weak 7 / Next 5):
``gpuSwarm.roundTimeoutMs`` / ``controlTimeoutMs`` default to 60 s / 300 s in the library,
and a rank whose peer died raises :class:`SwarmPeerLost` with its plan instead of hanging.
Reference: per-attempt timeouts are first-class in the loader
(``lib/integration/p2p-loader-generator.js:163,206-208``)."""
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest

from hlsjs_p2p_wrapper_amd.net import new_event_loop

REPO = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_library_defaults_and_config_keys(monkeypatch):
    from hlsjs_p2p_wrapper_amd.agent import node_for_config, set_current_node
    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
    from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm

    monkeypatch.delenv("HLSP2P_ROUND_TIMEOUT", raising=False)
    assert SwarmNode.ROUND_TIMEOUT_S == 60.0 and DistComm.CONTROL_TIMEOUT_S == 300.0
    new_event_loop("virtual")
    set_current_node(None)
    node = node_for_config({"gpuSwarm": {"backend": "local", "device": "cpu", "cacheBytes": 1 << 20}})
    assert node.round_deadline_s() == 60.0
    monkeypatch.setenv("HLSP2P_ROUND_TIMEOUT", "7")
    assert node.round_deadline_s() == 7.0
    set_current_node(None)
    node = node_for_config({"gpuSwarm": {"backend": "local", "device": "cpu", "cacheBytes": 1 << 20,
                                         "roundTimeoutMs": 2500}})
    assert node.round_deadline_s() == 2.5  # the config key wins over the environment
    set_current_node(None)


@pytest.mark.parametrize("deadline_s", [6])
def test_survivor_of_a_dead_peer_raises_with_its_plan(deadline_s):
    """Two ranks of ``examples/bundle/play.py`` (the user's torchrun path, here started as two
    plain processes so no launcher stops the survivor for us).  Rank 1 dies abruptly at round 40
    (``HLSP2P_FAULT_EXIT``); rank 0 must raise ``SwarmPeerLost`` carrying its plan, within the
    control deadline (``HLSP2P_CONTROL_TIMEOUT``, the env form of ``gpuSwarm.controlTimeoutMs``)
    plus start-up slack -- not hang for the old 10 minutes."""
    port = _free_port()
    base = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    base.update(PYTHONPATH=str(REPO), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
                HLSP2P_CONTROL_TIMEOUT=str(deadline_s), HLSP2P_FAULT_EXIT="1:40")
    procs = []
    for r in range(2):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(REPO / "examples" / "bundle" / "play.py"), "--cpu",
                                       "--seconds", "1000"], cwd=REPO, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    try:
        out1, err1 = procs[1].communicate(timeout=240)
        t_dead = time.monotonic()
        out0, err0 = procs[0].communicate(timeout=deadline_s + 60)
        t_raise = time.monotonic() - t_dead
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert procs[1].returncode == 17, err1[-2000:]  # the injected crash
    assert procs[0].returncode != 0, (out0[-1000:], err0[-2000:])
    assert "SwarmPeerLost" in err0 and "a peer may have stopped" in err0, err0[-3000:]
    assert "Plan of round" in err0 and "'send'" in err0 and "'recv'" in err0, err0[-3000:]
    assert t_raise < deadline_s + 45, t_raise
