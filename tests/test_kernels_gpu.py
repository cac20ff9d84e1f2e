"""Numerics of the gfx950 kernels against host oracles (zlib / FIPS-197-validated AES /
CPU demux).  All marked ``gpu``."""
import zlib

import numpy as np
import pytest
import torch

from hlsjs_p2p_wrapper_amd.ops import aes, crc, segment, tsdemux

pytestmark = pytest.mark.gpu


def _rand(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


@pytest.mark.parametrize("variant", ["fp4", "i8"])
def test_crc32_mfma_matches_zlib(cuda, variant):
    rng = np.random.default_rng(0)
    lens = [0, 1, 15, 16, 255, 256, 257, 4096, 8191, 8192, 8193, 100003, 3_000_064, 1 << 20, 5_000_011]
    offs, blob = [], []
    pos = 0
    for i, n in enumerate(lens):
        offs.append(pos)
        blob.append(_rand(n, i))
        pad = (-(pos + n)) % 256
        blob.append(np.full(pad, 0xA5, np.uint8))  # nonzero: a read past the end must not count
        pos += n + pad
    buf = np.concatenate(blob)
    t = torch.from_numpy(buf).to(cuda)
    expect = [zlib.crc32(buf[o:o + n].tobytes()) for o, n in zip(offs, lens)]
    got, ok = crc.crc32_batch(t, offs, lens, expect=expect, variant=variant)
    got = got.cpu().numpy().view(np.uint32)
    assert [int(x) for x in got] == expect
    assert ok.cpu().numpy().tolist() == [1] * len(lens)
    # corrupt one byte -> mismatch detected
    t[offs[7] + 3] ^= 0x40
    _, ok2 = crc.crc32_batch(t, offs, lens, expect=expect, variant=variant)
    assert ok2.cpu().numpy().tolist()[7] == 0
    _ = rng


@pytest.mark.parametrize("dev", ["cpu", "cuda"])
def test_crc32_scatter_into_entry_table(dev, request):
    # the ingest path writes each CRC to table[entry id] inside the combine kernel; slots not
    # named keep their value, and an out-of-range id is refused on the host before any launch
    device = request.getfixturevalue("cuda") if dev == "cuda" else torch.device("cpu")
    lens = [0, 3, 256, 70001, 4096]
    offs = [i * 81920 for i in range(len(lens))]
    buf = _rand(offs[-1] + 81920, 11)
    t = torch.from_numpy(buf).to(device)
    table = torch.full((40,), 7, dtype=torch.int32, device=device)
    ids = [31, 2, 17, 0, 39]
    crc_t, _ = crc.crc32_batch(t, offs, lens, scatter_to=table, scatter_idx=ids)
    expect = np.array([zlib.crc32(buf[o:o + n].tobytes()) for o, n in zip(offs, lens)], dtype=np.uint32)
    ref = np.full(40, 7, dtype=np.int32)
    ref[ids] = expect.view(np.int32)
    assert np.array_equal(table.cpu().numpy(), ref)
    assert np.array_equal(crc_t.cpu().numpy(), expect.view(np.int32))
    with pytest.raises(ValueError):
        crc.crc32_batch(t, offs[:1], lens[:1], scatter_to=table, scatter_idx=[40])


def test_aes_cbc_decrypt_matches_host(cuda):
    B = 9
    keys = [bytes(np.random.default_rng(100 + i).integers(0, 256, 16, dtype=np.uint8)) for i in range(B)]
    ivs = [aes.iv_from_sn(1000 + i) for i in range(B)]
    plains = [_rand(n, i) for i, n in enumerate([0, 1, 15, 16, 17, 1000, 65536, 188 * 1000, 3_000_001])]
    cts = [aes.cbc_encrypt(k, v, p) for k, v, p in zip(keys, ivs, plains)]
    offs, pos = [], 0
    for c in cts:
        offs.append(pos)
        pos += (len(c) + 255) // 256 * 256
    src = np.zeros(pos, np.uint8)
    for o, c in zip(offs, cts):
        src[o:o + len(c)] = c
    s = torch.from_numpy(src).to(cuda)
    d = torch.zeros_like(s)
    out_len = aes.cbc_decrypt_batch(s, offs, [len(c) for c in cts], keys, ivs, d, offs)
    out_len = out_len.cpu().numpy()
    host = d.cpu().numpy()
    for i, p in enumerate(plains):
        assert out_len[i] == len(p)
        assert np.array_equal(host[offs[i]:offs[i] + len(p)], p)
    # nothing written past a segment's ciphertext: the kernel's buffer ranges drop the stores of
    # the blocks beyond each segment's end (the last chunk of a segment is partial)
    ends = [o + len(c) for o, c in zip(offs, cts)]
    for e, nxt in zip(ends, offs[1:] + [pos]):
        assert not host[e:nxt].any()
    # wrong key -> padding check fails (overwhelmingly likely)
    bad = aes.cbc_decrypt_batch(s, offs[-1:], [len(cts[-1])], [bytes(16)], ivs[-1:], d, offs[-1:])
    assert int(bad.cpu()[0]) == -1 or not np.array_equal(d.cpu().numpy()[offs[-1]:offs[-1] + 64], plains[-1][:64])


def test_ts_demux_matches_cpu_oracle(cuda):
    segs = []
    for i, (tb, id3) in enumerate([(3_000_000, False), (400_000, True), (1_000_000, False), (188 * 300, True)]):
        seg, _ = tsdemux.mux_segment(target_bytes=tb, with_id3=id3, seed=11 + i, sn=i, start_time=4.0 * i)
        segs.append(seg)
    offs, pos = [], 0
    for s in segs:
        offs.append(pos)
        pos += (len(s) + 255) // 256 * 256
    buf = np.zeros(pos + 256, np.uint8)
    for o, s in zip(offs, segs):
        buf[o:o + len(s)] = s
    lens = [len(s) for s in segs]
    cpu = tsdemux.demux_batch(torch.from_numpy(buf), offs, lens, torch.zeros(pos + 256, dtype=torch.uint8), offs)
    g_buf = torch.from_numpy(buf).to(cuda)
    g_es = torch.zeros(pos + 256, dtype=torch.uint8, device=cuda)
    gpu = tsdemux.demux_batch(g_buf, offs, lens, g_es, offs)
    assert torch.equal(gpu.info.cpu(), cpu.info)
    assert torch.equal(gpu.pes.cpu(), cpu.pes)
    ci = cpu.info.numpy()
    for i, o in enumerate(offs):
        n = int(ci[i, 14])
        assert torch.equal(g_es[o:o + n].cpu(), cpu.es[o:o + n])
        assert ci[i, 0] == 0


def _damaged_segments():
    """TS segments with damage on the parse's error paths: adaptation-field lengths (byte 4) up
    to past the packet, broken PES start codes and header lengths, PES headers that run to the
    packet end, and lost sync bytes."""
    rng = np.random.default_rng(7)
    segs = []
    for i in range(6):
        seg, _ = tsdemux.mux_segment(target_bytes=300_000, with_id3=bool(i & 1), seed=40 + i, sn=i, start_time=4.0 * i)
        seg = np.frombuffer(seg, np.uint8).copy()
        pk = seg.reshape(-1, 188)
        n = len(pk)
        adapt = np.flatnonzero((pk[:, 3] & 0x20) != 0)
        pusi = np.flatnonzero((pk[:, 1] & 0x40) != 0)
        if i >= 1 and len(adapt):  # adaptation lengths: random, the largest legal, past the packet
            for j in rng.choice(adapt, min(20, len(adapt)), replace=False):
                pk[j, 4] = rng.choice([0, 1, 182, 183, 184, 200, int(rng.integers(0, 256))])
        if i >= 2 and len(pusi):  # PES start code / header length damaged
            for j in rng.choice(pusi, min(12, len(pusi)), replace=False):
                s0 = 4 + (1 + int(pk[j, 4]) if pk[j, 3] & 0x20 else 0)
                if s0 + 9 <= 188:
                    pk[j, s0 + int(rng.integers(0, 3))] ^= 0xFF if rng.random() < 0.5 else 0
                    if rng.random() < 0.5:
                        pk[j, s0 + 8] = int(rng.integers(0, 256))
        if i >= 3:  # PES headers pushed to the end of their packet
            for j in rng.choice(pusi, min(8, len(pusi)), replace=False) if len(pusi) else []:
                pk[j, 3] |= 0x20
                pk[j, 4] = int(rng.integers(160, 184))
        if i >= 4:  # lost sync
            for j in rng.choice(n, 5, replace=False):
                pk[j, 0] = 0x46
        segs.append(seg.tobytes())
    return segs


def test_ts_demux_matches_cpu_oracle_on_damaged_streams(cuda):
    """Damaged packets take the kernels' error paths exactly as the CPU oracle does."""
    segs = _damaged_segments()
    offs, pos = [], 0
    for sg in segs:
        offs.append(pos)
        pos += (len(sg) + 255) // 256 * 256
    buf = np.zeros(pos + 256, np.uint8)
    for o, sg in zip(offs, segs):
        buf[o:o + len(sg)] = np.frombuffer(sg, np.uint8)
    lens = [len(sg) for sg in segs]
    cpu = tsdemux.demux_batch(torch.from_numpy(buf), offs, lens, torch.zeros(pos + 256, dtype=torch.uint8), offs)
    g_es = torch.zeros(pos + 256, dtype=torch.uint8, device=cuda)
    gpu = tsdemux.demux_batch(torch.from_numpy(buf).to(cuda), offs, lens, g_es, offs)
    assert torch.equal(gpu.info.cpu(), cpu.info)
    assert torch.equal(gpu.pes.cpu(), cpu.pes)
    ci = cpu.info.numpy()
    assert (ci[1:, 0] != 0).any()  # the damage reached the error paths
    for i, o in enumerate(offs):
        n = int(ci[i, 14])
        assert torch.equal(g_es[o:o + n].cpu(), cpu.es[o:o + n])


def test_transmux_with_header_records_matches_cpu_oracle_on_damaged_streams(cuda):
    """The same damage through the encrypted transmux batch, where the scan takes its packet
    headers (and byte 4, unless the header sits at byte 12 of its block) from the records the
    decrypt writes: info rows, PES tables and ES bytes equal the CPU oracle on the plaintext."""
    from hlsjs_p2p_wrapper_amd.ops._native import device

    segs = _damaged_segments()
    key = bytes(range(16, 32))
    cts = [aes.cbc_encrypt(key, aes.iv_from_sn(100 + i), np.frombuffer(sg, np.uint8)) for i, sg in enumerate(segs)]
    offs, pos = [], 0
    for c in cts:
        offs.append(pos)
        pos += (len(c) + 255) // 256 * 256
    src = np.zeros(pos + 256, np.uint8)
    for o, c in zip(offs, cts):
        src[o:o + len(c)] = c
    B = len(cts)
    td0, isb = aes.device_tables(cuda)
    drk = np.tile(aes.round_keys_le(key), (B, 1)).astype(np.uint32)
    iv = np.stack([np.frombuffer(aes.iv_from_sn(100 + i), np.uint8) for i in range(B)])
    groups, keep, _, _ = device().transmux_launch(torch.from_numpy(src).to(cuda), np.asarray(offs, np.int64),
                                                  np.asarray([len(c) for c in cts], np.int64), np.ones(B, np.uint8),
                                                  drk, iv, td0, isb, tsdemux.DEFAULT_MAX_PES)
    torch.cuda.synchronize()
    idx, info, pes, es, eo, _, _ = groups[0]
    assert list(idx) == list(range(B))
    plain_offs, ppos = [], 0
    for sg in segs:
        plain_offs.append(ppos)
        ppos += (len(sg) + 255) // 256 * 256
    pbuf = np.zeros(ppos + 256, np.uint8)
    for o, sg in zip(plain_offs, segs):
        pbuf[o:o + len(sg)] = np.frombuffer(sg, np.uint8)
    cpu = tsdemux.demux_batch(torch.from_numpy(pbuf), plain_offs, [len(sg) for sg in segs],
                              torch.zeros(ppos + 256, dtype=torch.uint8), plain_offs)
    assert torch.equal(info.cpu(), cpu.info)
    assert torch.equal(pes.cpu(), cpu.pes)
    ci = cpu.info.numpy()
    assert (ci[1:, 0] != 0).any()
    es_h = es.cpu()
    for i in range(B):
        n = int(ci[i, 14])
        assert torch.equal(es_h[int(eo[i]):int(eo[i]) + n], cpu.es[plain_offs[i]:plain_offs[i] + n])


def test_decrypt_then_demux_on_device(cuda):
    seg, st = tsdemux.mux_segment(target_bytes=1_500_000, seed=5, sn=42, start_time=168.0)
    key = bytes(range(16))
    iv = aes.iv_from_sn(42)
    ct = aes.cbc_encrypt(key, iv, seg)
    src = torch.zeros(len(ct) + 256, dtype=torch.uint8, device=cuda)
    src[:len(ct)] = torch.from_numpy(ct).to(cuda)
    dec = torch.zeros_like(src)
    out_len = aes.cbc_decrypt_batch(src, [0], [len(ct)], [key], [iv], dec, [0])
    es = torch.zeros_like(src)
    res = tsdemux.demux_batch(dec, [0], out_len, es, [0], caps=[len(ct)])
    info = res.info.cpu().numpy()[0]
    assert info[0] == 0
    assert tuple(info[6:9]) == tuple(st["es_bytes"])
    assert tuple(info[9:12]) == tuple(st["n_pes"])


def test_copy_segments(cuda):
    src = torch.randint(0, 256, (1 << 20,), dtype=torch.uint8, device=cuda)
    dst = torch.zeros_like(src)
    so, do, n = [0, 1000, 70001, 500000], [16, 300000, 400001, 900000], [70000, 3, 200000, 100000]
    segment.copy_segments(src, dst, so, do, n)
    for a, b, c in zip(so, do, n):
        assert torch.equal(dst[b:b + c], src[a:a + c])


def test_pack_to_device_native_dtypes_and_layout(cuda):
    # the native descriptor packer (one pinned block, one H2D): every dtype the launchers
    # use, uint32 as int32 bits, non-contiguous input, odd sizes (16-byte sub-array padding)
    from hlsjs_p2p_wrapper_amd.ops.desc import pack_to_device

    rng = np.random.default_rng(5)
    arrays = {
        "i64": rng.integers(-2**40, 2**40, 7, dtype=np.int64),
        "u32": rng.integers(0, 2**32, 13, dtype=np.uint32),
        "i32": rng.integers(-2**31, 2**31, 3, dtype=np.int32),
        "u8": rng.integers(0, 256, (5, 16), dtype=np.uint8),
        "f64": rng.random(9),
        "strided": np.arange(40, dtype=np.int64)[::3],
        "empty": np.zeros(0, dtype=np.int64),
    }
    out = pack_to_device(arrays, cuda)
    assert list(out) == list(arrays)
    for name, a in arrays.items():
        t = out[name]
        assert t.device.type == "cuda" and t.numel() == a.size
        ref = a.reshape(-1).view(np.int32) if a.dtype == np.uint32 else a.reshape(-1)
        assert np.array_equal(t.cpu().numpy(), ref), name
        if t.numel():
            assert t.data_ptr() % 16 == 0


def test_native_crc_launch_matches_python_assembly(cuda):
    """crc32_launch (one native call) == the Python-assembled launch, incl. verify + scatter."""
    lens = [0, 17, 4096, 8193, 3_000_064, 250_000]
    offs, pos = [], 0
    for n in lens:
        offs.append(pos)
        pos += (n + 255) // 256 * 256 + 256
    buf = torch.from_numpy(_rand(pos, 5)).to(cuda)
    o, n = np.asarray(offs, np.int64), np.asarray(lens, np.int64)
    expect = [zlib.crc32(buf[a:a + b].cpu().numpy().tobytes()) for a, b in zip(offs, lens)]
    exp_dev = torch.from_numpy(np.asarray(expect, np.uint32).view(np.int32).copy()).to(cuda)
    exp_dev[2] ^= 1  # one mismatch
    ids = np.array([9, 3, 7, 0, 5, 11], np.int64)
    t_native = torch.zeros(16, dtype=torch.int32, device=cuda)
    t_py = torch.zeros(16, dtype=torch.int32, device=cuda)
    c1, ok1 = crc.crc32_batch(buf, offs, lens, expect_dev=exp_dev, scatter_to=t_native, scatter_idx=ids)
    c2, ok2 = crc._crc32_batch_py(buf, o, n, None, exp_dev, t_py, ids)
    assert torch.equal(c1, c2) and torch.equal(ok1, ok2) and torch.equal(t_native, t_py)
    assert [int(x) for x in c1.cpu().numpy().view(np.uint32)] == expect
    assert ok1.cpu().tolist() == [1, 1, 0, 1, 1, 1]


def test_arena_views_share_storage(cuda):
    from hlsjs_p2p_wrapper_amd.ops._native import device

    arena = torch.arange(4096, dtype=torch.int32, device=cuda).view(torch.uint8)
    views = device().arena_views(arena, np.array([0, 256, 1000], np.int64), np.array([16, 0, 3000], np.int64))
    assert [v.numel() for v in views] == [16, 0, 3000]
    assert views[2].data_ptr() == arena.data_ptr() + 1000 and torch.equal(views[2], arena[1000:4000])
    with pytest.raises(ValueError):
        device().arena_views(arena, np.array([16000], np.int64), np.array([1000], np.int64))


@pytest.mark.gpu
def test_fused_decrypt_crc_matches_zlib_at_segment_sizes(cuda):
    """The CRC fused into the AES decrypt (aes_cbc.hip AesCrc + crc32_fold_combine_kernel)
    on bench-sized ciphertexts: 50 segments of 16 B .. 3 MB plus a 4K-sized 12.5 MB and a 40 MB
    one (the fold's per-segment workgroup then walks many chunk tiles per wave), every CRC equal
    to zlib's; one corrupted byte fails exactly its segment."""
    import zlib

    from hlsjs_p2p_wrapper_amd.player.transmux import MediaPipeline
    from hlsjs_p2p_wrapper_amd.net import new_event_loop

    rng = np.random.default_rng(11)
    sizes = [16, 4096, 4112] + [int(x) * 16 for x in rng.integers(1, 3_000_000 // 16, 45)] + [12_500_000 // 16 * 16,
                                                                                                40_000_016]
    offs, pos = [], 0
    for n in sizes:
        offs.append(pos)
        pos += (n + 255) // 256 * 256
    host = rng.integers(0, 256, pos, dtype=np.uint8)
    arena = torch.from_numpy(host).to(cuda)
    crcs = np.array([zlib.crc32(host[o:o + n].tobytes()) for o, n in zip(offs, sizes)], dtype=np.int64)
    B = len(sizes)
    drk = np.tile(aes.round_keys_le(bytes(16)), (B, 1)).astype(np.uint32)
    iv = np.zeros((B, 16), dtype=np.uint8)
    pipe = MediaPipeline(cuda, new_event_loop("virtual"))
    o, nb, enc = np.asarray(offs, dtype=np.int64), np.asarray(sizes, dtype=np.int64), np.ones(B, dtype=bool)
    *_, ok = pipe.complete_columns(pipe.launch_columns(arena, o, nb, enc, drk, iv, expect=crcs))
    assert ok.all(), np.flatnonzero(~ok)
    arena[offs[7] + sizes[7] // 2] ^= 0x40
    *_, ok = pipe.complete_columns(pipe.launch_columns(arena, o, nb, enc, drk, iv, expect=crcs))
    assert np.flatnonzero(~ok).tolist() == [7]
