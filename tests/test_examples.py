"""The three integration modes of examples/ (bundle / custom / legacy, reference
``example/index.html:11-36``) run end to end: in-process 2-peer swarm, plain-engine
fallback, and one example as 2 torchrun ranks over gloo."""
import ast
import os
import re
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _run(args, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(REPO))
    p = subprocess.run([sys.executable, *args], cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    # ranks share stdout: records may interleave on one line, so match them individually
    return {int(m.group(1)): ast.literal_eval(m.group(2))
            for m in re.finditer(r"(?:peer|rank) (\d+): (\{[^{}]*\})", p.stdout)}


@pytest.mark.parametrize("mode", ["bundle", "custom", "legacy"])
def test_example_two_peers(mode):
    peers = _run([f"examples/{mode}/play.py", "--peers", "2", "--cpu", "--seconds", "8"])
    assert sorted(peers) == [0, 1]
    assert all(p["ok"] and p["currentTime"] >= 8 for p in peers.values())
    cdn = sum(p["cdn"] for p in peers.values())
    p2p = sum(p["p2p"] for p in peers.values())
    assert p2p > 0 and cdn > 0
    assert peers[0]["upload"] == peers[1]["p2p"]


def test_example_plain_engine_fallback():
    peers = _run(["examples/custom/play.py", "--no-p2p", "--cpu", "--seconds", "6"])
    assert peers[0]["ok"] and peers[0]["p2p"] == 0


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.slow
def test_example_torchrun_two_ranks():
    peers = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
                  "127.0.0.1", "--master-port", str(_free_port()), "examples/bundle/play.py", "--cpu", "--seconds",
                  "8"])
    assert sorted(peers) == [0, 1]
    assert all(p["ok"] for p in peers.values())
    assert sum(p["p2p"] for p in peers.values()) > 0


def test_example_plays_a_real_http_cdn():
    """``--url``: the bundle example against a real HTTP server (the local CDN of
    ``test_network_origin.py``), two in-process peers sharing the downloads."""
    from test_network_origin import _Cdn

    cdn = _Cdn(num_segments=4)
    try:
        peers = _run(["examples/bundle/play.py", "--peers", "2", "--cpu", "--seconds", "3",
                      "--url", cdn.origin.master_url()])
        assert sorted(peers) == [0, 1] and all(p["ok"] for p in peers.values())
        assert sum(p["cdn"] for p in peers.values()) == cdn.ts_bytes()  # one download per segment
        assert sum(p["p2p"] for p in peers.values()) > 0
    finally:
        cdn.close()
