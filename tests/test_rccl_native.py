"""Native RCCL data plane (``kernels/rccl_comm.cpp``).

The pool's GPU box has one MI355X and RCCL refuses two ranks on one device, so the GPU
tests use a one-rank communicator: a rank sending to and receiving from itself runs the
same ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd path, on the caller's stream, as
a round between peers.  The multi-GPU run is the driver's 1/2/4/8-GPU bench."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

REPO = Path(__file__).resolve().parents[1]


def test_unique_id_and_version_without_gpu():
    from hlsjs_p2p_wrapper_amd.ops._native import device

    dev = device()
    uid = dev.rccl_unique_id()
    assert isinstance(uid, bytes) and len(uid) == 128
    assert int(dev.rccl_version()) >= 21800
    with pytest.raises(ValueError):
        dev.RcclComm(b"short", 1, 0, 0)


def test_gloo_world_keeps_torch_data_plane():
    """A gloo default group never opens the native plane (CPU tests, rehearsals)."""
    code = (
        "import torch.distributed as dist\n"
        "from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm\n"
        "dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d', world_size=1, rank=0)\n"
        "c = DistComm()\n"
        "print('RESULT', c.data_transport, c._rccl is None)\n"
        "dist.destroy_process_group()\n" % _free_port())
    p = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PYTHONPATH=str(REPO)))
    assert p.returncode == 0, p.stderr[-2000:]
    assert [ln.split()[1:] for ln in p.stdout.splitlines() if ln.startswith("RESULT")] == [["gloo", "True"]]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_native_rccl_self_exchange_on_stream(cuda):
    from hlsjs_p2p_wrapper_amd.ops._native import device

    dev = device()
    comm = dev.RcclComm(dev.rccl_unique_id(), 1, 0, torch.cuda.current_device())
    try:
        g = torch.Generator(device="cpu").manual_seed(3)
        seg = torch.randint(0, 256, (3_000_017,), dtype=torch.uint8, generator=g).to(cuda)
        trailer = torch.arange(1, 65, dtype=torch.int32, device=cuda) * 0x01010101
        out_seg = torch.zeros_like(seg)
        out_tr = torch.zeros_like(trailer)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            comm.exchange(np.array([seg.data_ptr(), trailer.data_ptr()]), np.array([seg.numel(), 4 * trailer.numel()]),
                          np.array([0, 0]), np.array([out_seg.data_ptr(), out_tr.data_ptr()]),
                          np.array([out_seg.numel(), 4 * out_tr.numel()]), np.array([0, 0]), s.cuda_stream)
            done = torch.cuda.Event()
            done.record(s)
        done.synchronize()
        assert torch.equal(out_seg, seg) and torch.equal(out_tr, trailer)
        assert comm.rounds == 1 and comm.async_error() == ""
        # what RCCL itself reports (the topology record of an N > 1 bench run)
        assert comm.comm_count() == 1 and comm.comm_user_rank() == 0
        assert comm.comm_device() == torch.cuda.current_device()
        bus = dev.pci_bus_id(torch.cuda.current_device())
        assert len(bus.split(":")) == 3 and bus.endswith(".0"), bus
        with pytest.raises(ValueError):  # peer out of range for a world of one
            comm.exchange(np.array([seg.data_ptr()]), np.array([16]), np.array([1]), np.zeros(0, np.int64),
                          np.zeros(0, np.int64), np.zeros(0, np.int64), s.cuda_stream)
    finally:
        comm.close()
    assert comm.closed


@pytest.mark.gpu
@pytest.mark.parametrize("group", ["nccl", "gloo+rccl"])
def test_distcomm_uses_native_rccl(cuda, group):
    """DistComm opens the native plane and moves a round's (segment buffer, CRC trailer) pair
    through it on the node-style side stream: over a one-rank nccl group, and over the gloo
    default group that ``bench.py`` uses (HLSP2P_DATA_PLANE=rccl), where the native
    communicator is the rank's only RCCL communicator and the decrypt grid leaves CUs free."""
    init = ("dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d', world_size=1, rank=0, device_id=dev)"
            if group == "nccl" else
            "dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d', world_size=1, rank=0)") % _free_port()
    code = f"""
import torch, torch.distributed as dist
from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm
from hlsjs_p2p_wrapper_amd.ops._native import device as _dev
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
{init}
c = DistComm()
assert c.data_transport == 'rccl-native', c.data_transport
if '{group}' != 'nccl':
    assert c.data_backend == 'gloo' and c.data_group is None  # no torch RCCL communicator
    assert _dev().cu_reserve() == 64  # parallel/comm.py RCCL_CU_RESERVE (profiles/r5_overlap)
buf = torch.arange(1 << 20, dtype=torch.int32, device=dev).view(torch.uint8)
tr = torch.tensor([7, 8, 9], dtype=torch.int32, device=dev)
rb, rt = torch.empty_like(buf), torch.empty_like(tr)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    c.exchange([(0, buf), (0, tr)], [(0, rb), (0, rt)])
torch.cuda.synchronize()
assert torch.equal(rb, buf) and torch.equal(rt, tr)
t = c.topology()
assert t['transport'] == 'rccl-native' and t['world'] == 1, t
assert t['rccl']['count'] == 1 and t['rccl']['rank'] == 0 and t['rccl']['device'] == 0, t
assert t['rccl']['rounds'] == 1 and int(t['rccl']['version']) >= 21800, t
# the wire: a world of one connects nothing (sends to self are local copies); RCCL's own log
# names the group it built (1 rank, 1 node)
w = t['wire']
if '{group}' == 'nccl':  # torch's eager nccl group started RCCL first: its debug output was set already
    assert w['transport'] == 'unknown' and w['peers'] is None, w
else:
    assert w['transport'] == 'self' and w['peers'] == dict() and w['n_ranks'] == 1 and w['n_nodes'] == 1, w
    assert w['log_bytes'] < (1 << 20), w  # INIT/P2P/NET only: no per-operation lines
c.close()
dist.destroy_process_group()
print('NATIVE_OK')
"""
    env = dict(os.environ, PYTHONPATH=str(REPO))
    if group != "nccl":
        env["HLSP2P_DATA_PLANE"] = "rccl"
    p = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=180,
                       env=env)
    assert p.returncode == 0 and "NATIVE_OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])


@pytest.mark.gpu
def test_bench_refuses_more_rccl_ranks_than_gpus(cuda):
    """``bench.py --gpus N`` on a box with fewer than N GPUs: the RCCL plane needs one GPU per
    rank, so the self-launch refuses before starting any rank (exit 2, a clear message) --
    it never runs ranks that share a card, or fewer ranks than asked."""
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(REPO)
    p = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode == 2, (p.stdout[-2000:], p.stderr[-2000:])
    assert f"--gpus {n} needs {n} visible GPUs" in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_span_columns_pair_each_span_with_its_trailer():
    """The node hands the native RCCL plane a round as pointer columns: per peer its arena span
    then its CRC-trailer slice, on both sides (RCCL matches the i-th send with the i-th
    receive of a pair)."""
    from hlsjs_p2p_wrapper_amd.agent.node import _span_columns

    class T:  # a trailer buffer at a fixed address
        def __init__(self, p):
            self.p = p

        def data_ptr(self):
            return self.p

    srun = np.array([[1, 0, 3, 0, 4096, 9000], [3, 3, 4, 0, 65536, 100]], dtype=np.int64)
    rrun = np.array([[2, 0, 2, 8192, 6000]], dtype=np.int64)
    sp, sb, sd, rp, rb, rs = _span_columns(1 << 40, srun, T(5000), rrun, T(7000))
    assert sp.tolist() == [(1 << 40) + 4096, 5000, (1 << 40) + 65536, 5000 + 12]
    assert sb.tolist() == [9000, 12, 100, 4] and sd.tolist() == [1, 1, 3, 3]
    assert rp.tolist() == [(1 << 40) + 8192, 7000] and rb.tolist() == [6000, 8] and rs.tolist() == [2, 2]
    empty = _span_columns(0, np.zeros((0, 6), dtype=np.int64), None, np.zeros((0, 5), dtype=np.int64), None)
    assert all(len(c) == 0 for c in empty)


@pytest.mark.gpu
def test_exchange_spans_moves_arena_runs_and_trailers(cuda):
    """The pointer-column exchange on a one-rank native communicator: two arena runs and
    their trailer slices sent to self land in the receive runs, byte for byte."""
    code = """
import numpy as np, torch, torch.distributed as dist
from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm
from hlsjs_p2p_wrapper_amd.agent.node import _span_columns
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
dist.init_process_group('gloo', init_method='tcp://127.0.0.1:%d', world_size=1, rank=0)
c = DistComm()
assert c.exchange_spans is not None
g = torch.Generator().manual_seed(5)
arena = torch.zeros(1 << 23, dtype=torch.uint8, device=dev)  # 8 MiB: sources + both receive runs
arena[:3_000_000] = torch.randint(0, 256, (3_000_000,), dtype=torch.uint8, generator=g).to(dev)
tr = torch.tensor([11, 22, 33], dtype=torch.int32, device=dev)
rt = torch.zeros(3, dtype=torch.int32, device=dev)
srun = np.array([[0, 0, 2, 0, 0, 2_000_000], [0, 2, 3, 0, 2_000_000, 1_000_000]], dtype=np.int64)
rrun = np.array([[0, 0, 2, 3_000_064, 2_000_000], [0, 2, 3, 6_000_128, 1_000_000]], dtype=np.int64)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    c.exchange_spans(*_span_columns(arena.data_ptr(), srun, tr, rrun, rt))
torch.cuda.synchronize()
assert torch.equal(arena[3_000_064:5_000_064], arena[:2_000_000])
assert torch.equal(arena[6_000_128:7_000_128], arena[2_000_000:3_000_000])
assert rt.tolist() == [11, 22, 33]
c.close()
dist.destroy_process_group()
print('SPANS_OK')
""" % _free_port()
    env = dict(os.environ, PYTHONPATH=str(REPO), HLSP2P_DATA_PLANE="rccl")
    p = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True, timeout=180, env=env)
    assert p.returncode == 0 and "SPANS_OK" in p.stdout, (p.stdout[-2000:], p.stderr[-4000:])
