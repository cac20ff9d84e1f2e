"""Intra-node control plane: the native shared-memory all-gather that DistComm uses when
every rank shares one host (runtime/shm_control.cpp), against the gloo all-gather.

Three spawned ranks all-gather variable-length messages (including empty ones and one
that overflows the slot, which must send EVERY rank to the gloo fallback in step), run
barriers and an all-reduce, and check that nothing is left in /dev/shm."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank: int, world: int, port: int, q) -> None:
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm

        comm = DistComm()
        res = {"transport": comm.control_transport, "slot": comm.shm_slot_words}
        big = comm.shm_slot_words + 5
        rounds = []
        for g in range(40):
            n = 0 if (g + rank) % 7 == 0 else (g * 13 + rank * 5) % 300
            if g == 17 and rank == 1:
                n = big  # overflow: all ranks must fall back to gloo this round
            msg = np.arange(n, dtype=np.int64) * (rank + 1) + g
            parts = comm.allgather_control(msg)
            ok = True
            for r, p in enumerate(parts):
                m = 0 if (g + r) % 7 == 0 else (g * 13 + r * 5) % 300
                if g == 17 and r == 1:
                    m = big
                ok &= p.dtype == np.int64 and np.array_equal(p, np.arange(m, dtype=np.int64) * (r + 1) + g)
            rounds.append(bool(ok))
            if g % 10 == 0:
                comm.barrier()
        res["rounds_ok"] = all(rounds)
        res["fallbacks"] = comm.control_fallbacks
        res["sum"] = comm.allreduce_sum(np.array([rank, 1], dtype=np.int64)).tolist()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_shm_control_allgather_matches_and_falls_back(monkeypatch):
    """(The slot is sized through HLSP2P_SHM_SLOT_WORDS; the one oversized round is counted
    on every rank, not silent.)"""
    monkeypatch.setenv("HLSP2P_SHM_SLOT_WORDS", "2048")
    before = set(os.listdir("/dev/shm")) if os.path.isdir("/dev/shm") else set()
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert out[r]["transport"] == "shm"
        assert out[r]["rounds_ok"], r
        assert out[r]["slot"] == 2048 and out[r]["fallbacks"] == 1
        assert out[r]["sum"] == [0 + 1 + 2, world]
    after = set(os.listdir("/dev/shm")) if os.path.isdir("/dev/shm") else set()
    assert not [n for n in after - before if n.startswith("hlsp2p_")]
