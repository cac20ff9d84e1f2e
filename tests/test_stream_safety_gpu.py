"""Stream-ordered lifetime of the swarm node's device tensors (stream-ordered
allocation + events on cache buffers).

The caching allocator returns a freed block to the pool of the stream it was allocated on
without waiting for work other streams still have queued against it.  Round 3's 2-rank
fault was exactly that: the per-entry CRC table, allocated on the default stream, was
replaced from the node stream while a verify CRC that scatters into it was still queued
there; the transmux's descriptor block (a default-stream allocation) took the freed block
and the late scatter overwrote it.  These tests hold the node stream back with a device
sleep so the queued scatter runs only after the default stream has reused whatever it can,
then check a sentinel written on the default stream.
"""
import numpy as np
import pytest
import torch

SENTINEL = 0x5A5A5A5A
LATE = 0x0F0F0F0F  # what the held-back node-stream write stores


def _sleep_cycles(cuda, ms=200.0):
    """``torch.cuda._sleep`` cycles for ~``ms`` of device time (calibrated: the counter it
    spins on is not the shader clock on every part)."""
    s = torch.cuda.Stream(cuda)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        a.record(s)
        torch.cuda._sleep(10_000_000)
        b.record(s)
    b.synchronize()
    per_cycle = max(a.elapsed_time(b), 1e-3) / 10_000_000
    return int(min(ms / per_cycle, 2**31 - 1))


def _concurrent_stream(cuda, tries=8):
    """A new stream the device runs beside the default stream, plus the streams tried (kept
    alive).  HIP maps streams onto a few hardware queues (``GPU_MAX_HW_QUEUES``); a stream
    that shares the default stream's queue runs in order with it, and the race the positive
    control provokes cannot happen there."""
    keep = []
    cycles = _sleep_cycles(cuda, 30.0)
    for _ in range(tries):
        s = torch.cuda.Stream(cuda)
        keep.append(s)
        done = torch.cuda.Event()
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
            done.record(s)
        x = torch.empty(1, dtype=torch.int32, device=cuda)
        x.fill_(1)  # default stream
        mark = torch.cuda.Event()
        mark.record()
        mark.synchronize()
        concurrent = not done.query()  # the default stream finished while s still slept
        torch.cuda.synchronize()
        if concurrent:
            return s, keep
    return None, keep


def _segments(arena, n, seg=4096):
    gen = torch.Generator().manual_seed(3)
    data = torch.randint(0, 256, (n * seg,), dtype=torch.uint8, generator=gen)
    arena[:n * seg].copy_(data.to(arena.device))
    offs = np.arange(n, dtype=np.int64) * seg
    return offs, np.full(n, seg, dtype=np.int64)


@pytest.mark.gpu
def test_old_crc_table_pattern_is_detected(cuda):
    """Positive control: the round-3 pattern (table allocated on the default stream,
    replaced from the node stream without record_stream) lets a default-stream allocation
    take the table's block while a scatter into it is still queued -- the sentinel is
    overwritten.  Shows the check below can see the race."""
    torch.cuda.synchronize()
    node_stream, _streams = _concurrent_stream(cuda)
    if node_stream is None:
        pytest.skip("every new stream ran in order with the default stream (control inconclusive)")
    size = 4100
    table = torch.zeros(size, dtype=torch.int32, device=cuda)  # default-stream allocation
    old_ptr = table.data_ptr()
    torch.cuda.synchronize()
    cycles = _sleep_cycles(cuda)
    with torch.cuda.stream(node_stream):
        torch.cuda._sleep(cycles)
        table[:64].fill_(LATE)  # stands for the queued CRC scatter (plain torch: no host sync)
        new = torch.zeros(2 * size, dtype=torch.int32, device=cuda)
        new[:size] = table
        table = new  # the old block goes back to the default stream's pool right now
    # default-stream allocations until one covers the old table's first entries (the freed
    # block may coalesce with free neighbours, so the first one need not start there)
    probe = _covering_probe(cuda, size, old_ptr)
    torch.cuda.synchronize()
    if probe is None:
        pytest.skip("no default-stream allocation received the freed block (control inconclusive)")
    p, off = probe
    assert (p[off:off + 64] == LATE).all()  # the late write landed in the new owner's memory


def _covering_probe(cuda, size, ptr, tries=256):
    """Allocate sentinel-filled int32 tensors of ``size`` on the default stream until one
    covers ``[ptr, ptr + 256)``; returns (tensor, int32 offset of ptr) or None.  Filling is
    enqueued right away, so it runs while the node stream still sleeps."""
    keep = []
    for _ in range(tries):
        p = torch.empty(size, dtype=torch.int32, device=cuda)
        p.fill_(SENTINEL)
        keep.append(p)
        lo = p.data_ptr()
        if lo <= ptr and ptr + 256 <= lo + 4 * size:
            return p, (ptr - lo) // 4
    return None


@pytest.mark.gpu
def test_node_crc_table_grow_is_stream_safe(cuda):
    """The node's own grow path: the same queued scatter, then ``_grow_crc``; no
    default-stream allocation may receive the old table's block before the scatter ran."""
    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode
    from hlsjs_p2p_wrapper_amd.ops import crc as _crc

    node = SwarmNode(device=str(cuda), cache_bytes=4 << 20, auto_tick=False)
    size = node.crc_dev.numel()
    assert size == 1024  # the small-cache table: a grow is reachable
    offs, lens = _segments(node.arena, 64)
    torch.cuda.synchronize()
    old_table_ptr = node.crc_dev.data_ptr()
    cycles = _sleep_cycles(cuda)
    with torch.cuda.stream(node.stream):  # as launch_round's phases run
        torch.cuda._sleep(cycles)
        _crc.crc32_batch(node.arena, offs, lens, scatter_to=node.crc_dev, scatter_idx=np.arange(64))
        node._grow_crc(size + 1)
    old_ptr = old_table_ptr
    # no default-stream allocation may cover the old table before the scatter ran; any that
    # did would also show the scatter's writes over its sentinel
    probe = _covering_probe(cuda, size, old_ptr)
    torch.cuda.synchronize()
    assert probe is None
    # and the grown table kept the scattered CRCs (copied on the node stream after the scatter)
    want = np.array([_crc.crc32(node.arena[o:o + n].cpu()) for o, n in zip(offs, lens)], dtype=np.uint32)
    got = node.crc_dev[:64].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    assert node.crc_dev.numel() >= 2 * size


@pytest.mark.gpu
def test_node_crc_table_sized_for_the_arena(cuda):
    """The table starts big enough that the hot path never grows it: 8 GiB of arena holds
    >= 2^20 entries only below 8 KiB per segment."""
    from hlsjs_p2p_wrapper_amd.agent.node import SwarmNode

    node = SwarmNode(device=str(cuda), cache_bytes=1 << 30, auto_tick=False)
    assert node.crc_dev.numel() == (1 << 30) // (8 << 10) + 1
