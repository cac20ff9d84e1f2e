"""Scatter demux (``kernels/ts_scatter.hip`` + the scatter epilogue of ``aes_cbc.hip``): the
encrypted group is demuxed without a plaintext buffer -- header-only decrypt, scan, prefix,
place, then the bulk decrypt writes payload bytes straight to their ES positions.

Every output word is checked against the host oracle (``runtime/ts.cpp``) and the four-pass
split sequence: info rows, ES bytes, PES tables, plaintext lengths.  Segments cover the
header-group and packet-slot edges (1, 3, 4, 255, 256, 257 packets), a length that is not a
packet multiple, a corrupted sync byte, a PES table overflow, clear segments in the same
batch (they take the four-pass path) and a wrong key."""
import numpy as np
import pytest

from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux

from test_transmux_fused import _launch, _oracle, _same, _segments

pytestmark = pytest.mark.gpu


def _edge_segments():
    key = bytes(range(16, 32))
    out = []
    base, _ = tsdemux.mux_segment(duration=4.0, target_bytes=400_000, with_id3=True, seed=91, sn=3)
    for i, npk in enumerate((1, 3, 4, 255, 256, 257, 1024)):
        seg = base[:188 * npk].copy()
        iv = aes.iv_from_sn(100 + i)
        out.append((seg, aes.cbc_encrypt(key, iv, seg), key, iv))
    tail = np.concatenate([base[:188 * 700], np.full(100, 7, dtype=np.uint8)])  # not a packet multiple
    bad = base[:188 * 600].copy()
    bad[188 * 77] = 0x46  # sync byte
    bad[188 * 301] = 0x00
    for j, seg in enumerate((tail, bad)):
        iv = aes.iv_from_sn(200 + j)
        out.append((seg, aes.cbc_encrypt(key, iv, seg), key, iv))
    return out


@pytest.mark.parametrize("max_pes", [512, 7])
def test_scatter_demux_matches_oracle_and_fourpass(cuda, max_pes):
    jobs = _segments() + _edge_segments()
    scatter, _ = _launch("split", jobs, max_pes, demux="scatter")
    fourpass, _ = _launch("split", jobs, max_pes)
    for i, (seg, _, _, _) in enumerate(jobs):
        ref = _oracle(seg, max_pes)
        assert scatter[i]["plain"] == len(seg) == fourpass[i]["plain"], i
        _same(scatter[i], ref, max_pes)
        _same(scatter[i], fourpass[i], max_pes)
        assert scatter[i]["info"][22] == scatter[i]["info"][6]  # packed classes, as four-pass
    n = len(_segments())
    assert scatter[n + 7]["info"][0] & tsdemux.STATUS["bad_length"]
    assert scatter[n + 8]["info"][0] & tsdemux.STATUS["bad_sync"]
    if max_pes == 7:
        assert scatter[0]["info"][0] & tsdemux.STATUS["pes_overflow"] and scatter[0]["info"][9] > 7


def test_scatter_demux_wrong_key_reports_no_media(cuda):
    jobs = _segments()[:3]
    scatter, _ = _launch("split", jobs, 512, bad=bytes(16), demux="scatter")
    fourpass, _ = _launch("split", jobs, 512, bad=bytes(16))
    assert scatter[0]["plain"] == fourpass[0]["plain"] == -1
    assert scatter[0]["info"].tolist() == fourpass[0]["info"].tolist()
    for i in (1, 2):
        _same(scatter[i], fourpass[i], 512)
