"""The single-rank stand-ins for an N-rank swarm (``tools/round_replay.py``,
``tools/project_swarm.py``; ``profiles/r6_replay``, ``profiles/r6_project``).

Both run rank 0 alone against N-1 synthetic peers that want what it wants and hold what it
received the round before, so the native planner builds the real N-rank plan.  The tests pin
the plan's shape (1/N of the wants from the CDN, each forwarded to N-1 peers, the rest
received), that every request is answered, and -- on the GPU -- that the projection's
received segments pass the consumer's fused CRC check with their seeders' keyed trailers."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


def _run(args, timeout=300):
    env = dict(os.environ, PYTHONPATH=str(REPO))
    p = subprocess.run([sys.executable, *args], cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("world", [1, 4, 8])
def test_round_replay_builds_the_n_rank_plan(world):
    res = _run([str(REPO / "tools" / "round_replay.py"), "--world", str(world), "--wants", "64", "--rounds", "30",
                "--warmup", "5"])
    W = 64
    assert res["per_round"] == {"cdn": W / world, "send": (W / world) * (world - 1), "recv": W - W / world}
    # every want of every round answered once (the last `lag` rounds are drained untimed)
    assert res["delivered"] == W * (30 + 5)
    assert res["crc_failures"] == 0
    assert res["p2p_segments"] + res["cdn_segments"] == res["delivered"]
    assert res["launch_us"] > 0 and res["complete_us"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("config,churn", [("1080p6m", 0), ("abr5", 2)])
def test_projection_of_an_eight_rank_swarm_on_one_gpu(cuda, config, churn):
    """The headline shape, and config 3 (the ABR ladder with peers going offline in rotation)."""
    res = _run([str(REPO / "tools" / "project_swarm.py"), "--peers", "8", "--steps", "12", "--warmup", "4",
                "--cache-gb", "2", "--config", config, "--churn", str(churn)], timeout=420)
    rec = res["bench_record"]
    assert rec["n_gpus"] == 1 and res["peers"] == 8
    assert rec["errors"] == 0
    pr = rec["per_rank"][0]
    assert pr["crc_failures"] == 0 and pr["p2p_rejected_MB"] == 0.0
    # ~7/8 of the bytes arrive from the synthetic seeders and pass the fused decrypt CRC (the
    # seeder rotation starts at a key-drawn rank: this rank's share of a short window varies;
    # under churn an offline peer leaves this rank up to 1/7 to seed)
    assert (0.80 if churn else 0.84) <= rec["offload_ratio"] <= 0.91
    assert res["received_rows"] > 0
    assert res["projected_ms_per_step"] >= res["xgmi_receive_roof_ms_per_step"] > 0
    assert set(res["transmux_launch_us_per_call"]) >= {"plan", "decrypt_launch", "demux_launch_d2h"}


def test_round_replay_under_churn_seeds_more_and_answers_everything():
    """bench.py's churn rotation on the synthetic peers (config 3): while one of the 7 peers
    is offline this rank seeds 1/7 of the round instead of 1/8, and every want is still
    answered once."""
    res = _run([str(REPO / "tools" / "round_replay.py"), "--world", "8", "--wants", "64", "--rounds", "36",
                "--warmup", "0", "--churn", "2"])
    assert res["delivered"] == 64 * 36 and res["crc_failures"] == 0
    assert 64 / 8 < res["per_round"]["cdn"] < 64 / 6
    assert res["per_round"]["recv"] == 64 - res["per_round"]["cdn"]
