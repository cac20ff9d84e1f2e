"""Fused decrypt + demux (``kernels/transmux_fused.hip``): one pass per segment, the
plaintext never written to HBM, payload offsets from a decoupled look-back across tiles.

Every output word is checked against the host oracle (``runtime/ts.cpp``) and against the
split kernel sequence (decrypt, psi, scan, prefix, gather): info rows, ES bytes, PES
tables, plaintext lengths — on segments that span one tile, many tiles, end exactly on a
tile boundary (the PKCS#7 block alone in a tile of its own), clear ones, a wrong key, id3
streams and a PES table overflow."""
import numpy as np
import pytest
import torch

from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux

pytestmark = pytest.mark.gpu


def _tile_pkts():
    from hlsjs_p2p_wrapper_amd.ops._native import device

    return device().transmux_tile_bytes() // 188  # kernels/transmux_fused.hip kTilePkts


def _segments():
    key = bytes(range(16))
    TILE_PKTS = _tile_pkts()
    out = []
    specs = [(3_000_000, True, False), (300_000, True, True), (50_000, True, False), (188 * 64, False, True),
             (188 * TILE_PKTS, True, False), (188 * TILE_PKTS * 2, True, True), (188 * TILE_PKTS * 3, False, False),
             (1_000_000, False, True), (188 * 5, True, False)]
    for i, (nbytes, enc, id3) in enumerate(specs):
        seg, _ = tsdemux.mux_segment(duration=2.0, target_bytes=nbytes, with_id3=id3, seed=40 + i, sn=i)
        iv = aes.iv_from_sn(i)
        payload = aes.cbc_encrypt(key, iv, seg) if enc else seg
        out.append((seg, payload, key if enc else None, iv))
    return out


def _launch(mode, jobs, max_pes, bad=None, demux="fourpass"):
    from hlsjs_p2p_wrapper_amd.ops._native import device

    dev = device()
    dev.set_transmux_mode(mode)
    dev.set_demux_mode(demux)
    cuda = torch.device("cuda", 0)
    offs, pos = [], 0
    for _, p, _, _ in jobs:
        offs.append(pos)
        pos += (len(p) + 255) // 256 * 256
    arena = torch.zeros(pos + 4096, dtype=torch.uint8)
    for (_, p, _, _), o in zip(jobs, offs):
        arena[o:o + len(p)] = torch.from_numpy(p.copy())
    arena = arena.to(cuda)
    n = len(jobs)
    enc = np.array([1 if k is not None else 0 for _, _, k, _ in jobs], dtype=np.uint8)
    drk = np.zeros((n, 44), dtype=np.uint32)
    ivs = np.zeros((n, 16), dtype=np.uint8)
    for i, (_, _, k, iv) in enumerate(jobs):
        if k is not None:
            drk[i] = aes.round_keys_le(bad if (bad is not None and i == 0) else k)
            ivs[i] = np.frombuffer(iv, dtype=np.uint8)
    td0, isb = aes.device_tables(cuda)
    groups, keep, host = dev.transmux_launch(arena, np.array(offs, dtype=np.int64),
                                             np.array([len(p) for _, p, _, _ in jobs], dtype=np.int64), enc, drk, ivs,
                                             td0, isb, max_pes)
    torch.cuda.synchronize()
    res = [None] * n
    for gidx, info, pes, es, es_offs, hinfo, hlens in groups:
        for k, i in enumerate(gidx.tolist()):
            row = info[k].cpu().numpy()
            base = int(es_offs[k])
            esb = [es[base + o:base + o + int(n)].cpu().numpy() for o, n in ((0, row[6]), (row[22], row[7]),
                                                                                (row[23], row[8]))]
            res[i] = {"info": row, "pes": pes[k].cpu().numpy(), "es": np.concatenate(esb),
                      "plain": int(np.asarray(hlens)[k] if not isinstance(hlens, torch.Tensor) else hlens[k])}
    dev.set_transmux_mode("split")
    dev.set_demux_mode("fourpass")
    return res, keep


def _oracle(seg, max_pes):
    r = tsdemux.demux_batch(torch.from_numpy(seg.copy()), [0], [len(seg)], torch.zeros(len(seg) + 256,
                                                                                     dtype=torch.uint8), [0],
                            max_pes=max_pes)
    info = r.info[0].numpy()
    nbytes = int(info[6] + info[7] + info[8])
    assert info[22] == info[6] and info[23] == info[6] + info[7]  # packed [video | audio | id3]
    return {"info": info, "pes": r.pes[0].numpy(), "es": r.es[:nbytes].numpy()}


def _same(a, b, max_pes):
    # slots 22 / 23 say where audio / id3 start: packed by the oracle and the split kernels,
    # per-class regions in the fused kernel; the bytes there are compared below
    assert a["info"][:22].tolist() == b["info"][:22].tolist()
    assert np.array_equal(a["es"], b["es"])
    for c in range(3):
        k = min(int(a["info"][9 + c]), max_pes)
        assert np.array_equal(a["pes"][c, :k], b["pes"][c, :k]), c


@pytest.mark.parametrize("max_pes", [512, 7])
def test_fused_matches_oracle_and_split(cuda, max_pes):
    jobs = _segments()
    fused, keep = _launch("fused", jobs, max_pes)
    assert int(keep[0][-2].cpu()) >> 32 == 0  # no look-back / PSI hand-off timed out
    split, _ = _launch("split", jobs, max_pes)
    for i, (seg, _, _, _) in enumerate(jobs):
        ref = _oracle(seg, max_pes)
        assert fused[i]["plain"] == len(seg) == split[i]["plain"], i
        _same(fused[i], ref, max_pes)
        _same(fused[i], split[i], max_pes)
    if max_pes == 7:  # the 3 MB segment overflows a 7-entry PES table: flagged, counts exact
        assert fused[0]["info"][0] & tsdemux.STATUS["pes_overflow"] and fused[0]["info"][9] > 7


@pytest.mark.parametrize("max_pes", [512, 7])
def test_split_demux_modes_match_oracle(cuda, max_pes):
    """The split sequence's demux after the decrypt: the four-kernel sequence (the default) and
    the one-pass kernel (scan + prefix + gather in one, decoupled look-back) agree with the
    host oracle byte for byte."""
    jobs = _segments()
    onepass, keep = _launch("split", jobs, max_pes, demux="onepass")
    fourpass, _ = _launch("split", jobs, max_pes)
    for i, (seg, _, _, _) in enumerate(jobs):
        ref = _oracle(seg, max_pes)
        assert onepass[i]["plain"] == len(seg) == fourpass[i]["plain"], i
        _same(onepass[i], ref, max_pes)
        _same(fourpass[i], ref, max_pes)
        assert fourpass[i]["info"][22] == fourpass[i]["info"][6]  # packed classes
        if onepass[i]["info"][5] > 0:  # class regions
            assert onepass[i]["info"][23] == 2 * onepass[i]["info"][22] > 0


def test_fused_wrong_key_reports_no_media(cuda):
    """A wrong key fails the PKCS#7 check (overwhelmingly likely): plaintext length -1 and an
    empty demux, exactly as the split pipeline reports it, though the segment's tiles ran."""
    jobs = _segments()[:3]
    fused, _ = _launch("fused", jobs, 512, bad=bytes(16))
    split, _ = _launch("split", jobs, 512, bad=bytes(16))
    assert fused[0]["plain"] == split[0]["plain"] == -1
    assert fused[0]["info"].tolist() == split[0]["info"].tolist()  # no media: offsets 0 on both
    for i in (1, 2):
        _same(fused[i], split[i], 512)


def test_split_is_the_default_mode(cuda):
    from hlsjs_p2p_wrapper_amd.ops._native import device

    # the split sequence measured faster (profiles/r3_transmux_fused_vs_split.md); fused is opt-in
    assert device().transmux_mode() == "split" and device().transmux_tile_bytes() % (4 * 188) == 0
