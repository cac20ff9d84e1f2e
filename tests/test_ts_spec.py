"""TS demux against an independent, spec-built stream (``tests/ts_builder.py``, ISO/IEC
13818-1): the host demux and the gfx950 kernels must recover exactly the elementary-stream
bytes and the per-PES ``(es_offset, pts, dts)`` the builder put in, from streams with what the
framework's own muxer never emits -- a network entry ahead of the program in the PAT, PMT
descriptors, a PCR-only PID, adaptation fields with PCR and stuffing, null and SDT packets,
PSI repeated mid-segment, PES_packet_length 0, PTS-only video frames, PES headers longer than
PTS + DTS.

The reference hands demux to hls.js; hls.js is not importable here, so the
ground truth is the builder's, which shares no code with ``runtime/ts.cpp`` or the kernels.
"""
import numpy as np
import pytest
import torch

from hlsjs_p2p_wrapper_amd.ops import tsdemux
from ts_builder import CLASSES, build

CASES = [dict(seed=0), dict(seed=1, with_id3=False), dict(seed=2, video_type=0x24),
         dict(seed=3, n_video=40, n_audio=60), dict(seed=4, n_video=1, n_audio=1)]


def _batch(streams, device="cpu"):
    offs, pos = [], 0
    for s in streams:
        offs.append(pos)
        pos += (len(s) + 255) // 256 * 256
    buf = np.zeros(pos + 256, np.uint8)
    for o, s in zip(offs, streams):
        buf[o:o + len(s)] = np.frombuffer(s, np.uint8)
    es = torch.zeros(pos + 256, dtype=torch.uint8, device=device)
    res = tsdemux.demux_batch(torch.from_numpy(buf).to(device), offs, [len(s) for s in streams], es, offs)
    return res


def _check(res, truths, streams):
    for i, (tr, s) in enumerate(zip(truths, streams)):
        seg = res.segment(i)
        assert seg["status"] == 0, seg["status"]
        assert seg["pmt_pid"] == tr["pmt_pid"]
        assert seg["n_packets"] == len(s) // 188
        assert seg["video_type"] == tr["video_type"] and seg["audio_type"] == tr["audio_type"]
        for name in CLASSES:
            want = tr[name]
            if want["pid"] < 0:
                assert seg[f"{name}_pid"] < 0 or seg[f"n_{name}_pes"] == 0
                continue
            assert seg[f"{name}_pid"] == want["pid"]
            assert seg[f"{name}_bytes"] == len(want["es"])
            assert bytes(seg[name]["es"].cpu().numpy()) == want["es"], name
            got = [tuple(int(v) for v in row) for row in seg[name]["pes"]]
            assert got == want["pes"], name
            assert seg[f"{name}_first_pts"] == want["pes"][0][1]
            assert seg[f"{name}_last_pts"] == want["pes"][-1][1]


def test_builder_streams_are_well_formed():
    s, tr = build(seed=0)
    pk = np.frombuffer(s, np.uint8).reshape(-1, 188)
    assert (pk[:, 0] == 0x47).all()
    pids = ((pk[:, 1].astype(int) & 0x1F) << 8) | pk[:, 2]
    assert {0, 0x11, 0x1F0, 0x1000, 0x1FFF, 0x100, 0x101, 0x102} <= set(pids.tolist())
    # continuity counters advance by one per payload-carrying packet of a PID
    for pid in (0x100, 0x101):
        cc = pk[pids == pid, 3] & 0x0F
        assert ((np.diff(cc.astype(int)) % 16) == 1).all()
    assert any(dts < 0 for _, _, dts in tr["video"]["pes"]) and any(dts >= 0 for _, _, dts in tr["video"]["pes"])


def test_host_demux_recovers_a_spec_built_stream(rt):
    built = [build(**c) for c in CASES]
    streams, truths = [b[0] for b in built], [b[1] for b in built]
    _check(_batch(streams), truths, streams)


@pytest.mark.gpu
def test_gpu_demux_recovers_a_spec_built_stream(cuda):
    built = [build(**c) for c in CASES]
    streams, truths = [b[0] for b in built], [b[1] for b in built]
    res = _batch(streams, cuda)
    _check(res, truths, streams)
    cpu = _batch(streams)
    assert torch.equal(res.info.cpu(), cpu.info) and torch.equal(res.pes.cpu(), cpu.pes)
