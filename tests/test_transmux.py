"""Batched transmux stage (decrypt + demux between FRAG_LOADED and the buffer): every
fragment's result — status, info row, plaintext length, video/audio/id3 ES views — matches
the per-segment host oracle, for a mixed batch (encrypted + clear, varied sizes, one bad
key) staged from host payloads.  Runs on CPU (host kernels) and on the GPU (HIP kernels)."""
import pytest
import torch

from hlsjs_p2p_wrapper_amd.net import new_event_loop
from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux
from hlsjs_p2p_wrapper_amd.player.transmux import InfoRow, MediaPipeline, TransmuxJob


def _batch():
    key = bytes(range(16))
    jobs = []
    for i, (nbytes, enc) in enumerate([(300_000, True), (188 * 700, False), (1_000_000, True), (50_000, True),
                                       (188 * 64, False)]):
        seg, st = tsdemux.mux_segment(duration=2.0, target_bytes=nbytes, with_id3=(i % 2 == 0), seed=10 + i, sn=i)
        iv = aes.iv_from_sn(i)
        payload = aes.cbc_encrypt(key, iv, seg) if enc else seg
        jobs.append((seg, payload, key if enc else None, iv if enc else None))
    return jobs


def _run(device):
    loop = new_event_loop("virtual")
    pipe = MediaPipeline(torch.device(device), loop)
    out = {}
    jobs = _batch()
    for n, (_, payload, key, iv) in enumerate(jobs):
        pipe.submit(TransmuxJob(torch.from_numpy(payload.copy()), key, iv, lambda r, n=n: out.__setitem__(n, r)))
    bad = jobs[0]
    pipe.submit(TransmuxJob(torch.from_numpy(bad[1].copy()), bytes(16), bad[3], lambda r: out.__setitem__("bad", r)))
    pipe.flush()
    return jobs, out


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_pipeline_results_match_oracle(device, request):
    if device == "cuda":
        request.getfixturevalue("cuda")
    jobs, out = _run(device)
    for n, (seg, _, _, _) in enumerate(jobs):
        r = out[n]
        assert r.get("error") is None and r["status"] == 0
        assert r["plain_bytes"] == len(seg)
        ref = tsdemux.demux_batch(torch.from_numpy(seg.copy()), [0], [len(seg)],
                                  torch.zeros(len(seg) + 256, dtype=torch.uint8), [0]).segment(0)
        info = r["info"]
        assert isinstance(info, InfoRow)
        for k in ("video_pid", "audio_pid", "video_bytes", "audio_bytes", "id3_bytes", "n_video_pes",
                  "video_first_pts", "video_last_pts"):
            assert info[k] == ref[k], k
        assert torch.equal(r["video"].cpu(), ref["video"]["es"])
        assert torch.equal(r["audio"].cpu(), ref["audio"]["es"])
        assert r["id3"].numel() == ref["id3_bytes"]
        assert info.to_dict()["video_bytes"] == ref["video_bytes"] and "status" in info
    # wrong key: bad padding (overwhelmingly likely) or garbage that fails demux
    bad = out["bad"]
    assert bad.get("error") is not None or bad["status"] != 0


def _arena_jobs(device):
    """Payloads as views of one arena (the swarm node's delivery form), 16-byte aligned."""
    jobs = _batch()
    offs, pos = [], 0
    for _, payload, _, _ in jobs:
        offs.append(pos)
        pos += (len(payload) + 255) // 256 * 256
    arena = torch.zeros(pos, dtype=torch.uint8, device=device)
    for (_, payload, _, _), o in zip(jobs, offs):
        arena[o:o + len(payload)] = torch.from_numpy(payload.copy()).to(device)
    views = [arena[o:o + len(p)] for (_, p, _, _), o in zip(jobs, offs)]
    return jobs, arena, views, offs


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_stage_uses_arena_views_in_place(device):
    """Views of one allocation are staged without a copy (base = the arena storage, offsets =
    the views' positions); a payload from another allocation forces the staging copy."""
    _, arena, views, offs = _arena_jobs(device)
    pipe = MediaPipeline(torch.device(device), new_event_loop("virtual"))
    base, got = pipe._stage(views, [v.numel() for v in views])
    assert base.data_ptr() == arena.data_ptr() and got == offs
    other = torch.zeros(4096, dtype=torch.uint8, device=device)
    mixed = views[:2] + [other]
    base2, got2 = pipe._stage(mixed, [v.numel() for v in mixed])
    assert base2.data_ptr() != arena.data_ptr() and got2[0] == 0
    for v, o in zip(mixed, got2):
        assert torch.equal(base2[o:o + v.numel()].cpu(), v.cpu())


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_complete_arrays_matches_per_job_results(device):
    """The fleet's columnar completion (one info-row array per batch) carries the same rows
    and plaintext lengths as the per-fragment results; a rejected job has no row."""
    jobs, _, views, _ = _arena_jobs(device)
    loop = new_event_loop("virtual")
    ref = {}
    pipe = MediaPipeline(torch.device(device), loop)
    for n, ((_, _, key, iv), v) in enumerate(zip(jobs, views)):
        pipe.submit(TransmuxJob(v, key, iv, lambda r, n=n: ref.__setitem__(n, r)))
    pipe.flush()
    pipe.auto_flush = False
    subs = [TransmuxJob(v, key, iv, None, n) for n, ((_, _, key, iv), v) in enumerate(zip(jobs, views))]
    subs.append(TransmuxJob(views[0][:100], bytes(16), bytes(16), None, "odd"))  # not a multiple of 16
    for j in subs:
        pipe.submit(j)
    got_jobs, rows, plain, has = pipe.complete_arrays(pipe.launch())
    assert [j.frag for j in got_jobs] == list(range(len(jobs))) + ["odd"]
    assert rows.shape == (len(subs), tsdemux.INFO_WORDS)
    for n in range(len(jobs)):
        assert has[n] and rows[n].tolist() == ref[n]["info"]._row and plain[n] == ref[n]["plain_bytes"]
    assert not has[-1] and plain[-1] == -1


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_launch_columns_verifies_expected_crcs(device, request):
    """Fragments handed to the transmux with a peer's CRC (``expect``) are verified by the
    batch that decrypts them: on the GPU the CRC is fused into the AES decrypt (encrypted
    fragments) or run by the CRC kernel (clear ones).  A wrong expectation fails exactly that
    fragment, the decrypt + demux results are the same as without verification, and the
    fused CRC matches zlib for sizes around the 4096-byte chunk edges."""
    import zlib

    import numpy as np

    if device == "cuda":
        request.getfixturevalue("cuda")
    jobs, arena, views, offs = _arena_jobs(device)
    # extra encrypted fragments of awkward sizes: 16 B, one chunk, one chunk + 16, 3 chunks - 16
    key = bytes(range(16))
    extra = []
    for i, n in enumerate((16, 4096, 4112, 3 * 4096 - 16)):
        rng = np.random.default_rng(40 + i)
        extra.append(rng.integers(0, 256, n, dtype=np.uint8))
    pos = arena.numel()
    big = torch.zeros(pos + sum((len(e) + 255) // 256 * 256 for e in extra), dtype=torch.uint8, device=device)
    big[:pos] = arena
    for e in extra:
        big[pos:pos + len(e)] = torch.from_numpy(e).to(device)
        offs = offs + [pos]
        pos += (len(e) + 255) // 256 * 256
    payloads = [p for _, p, _, _ in jobs] + extra
    enc = np.array([k is not None for _, _, k, _ in jobs] + [True] * len(extra))
    n = len(payloads)
    drk = np.tile(aes.round_keys_le(key), (n, 1)).astype(np.uint32)
    iv = np.stack([np.frombuffer(j[3] if j[3] is not None else bytes(16), dtype=np.uint8) for j in jobs]
                  + [np.frombuffer(bytes(16), dtype=np.uint8)] * len(extra))
    keys = np.tile(np.frombuffer(key, dtype=np.uint8), (n, 1))
    nb = np.array([len(p) for p in payloads], dtype=np.int64)
    crcs = np.array([zlib.crc32(bytes(p)) for p in payloads], dtype=np.int64)
    expect = crcs.copy()
    expect[1] ^= 0x10  # a clear fragment with a wrong trailer
    expect[2] ^= 1     # an encrypted one
    expect[3] = -1     # not verified
    expect[-1] ^= 1 << 31
    loop = new_event_loop("virtual")
    pipe = MediaPipeline(torch.device(device), loop)
    o = np.asarray(offs, dtype=np.int64)
    tag, rows, plain, has, ok = pipe.complete_columns(pipe.launch_columns(big, o, nb, enc, drk, iv, "t", keys=keys,
                                                                          expect=expect))
    want = np.ones(n, dtype=bool)
    want[[1, 2, n - 1]] = False
    assert tag == "t" and ok.tolist() == want.tolist()
    _, rows0, plain0, has0, ok0 = pipe.complete_columns(pipe.launch_columns(big, o, nb, enc, drk, iv, keys=keys))
    assert ok0.all() and np.array_equal(rows, rows0) and np.array_equal(plain, plain0) and np.array_equal(has, has0)
    # every fused CRC is exact: expecting the true values passes all of them
    *_, ok_all = pipe.complete_columns(pipe.launch_columns(big, o, nb, enc, drk, iv, keys=keys, expect=crcs))
    assert ok_all.all()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_rejected_fragments_with_an_expected_crc_are_still_checked(device, request):
    """an encrypted fragment whose length is not a whole number of AES blocks is
    rejected before the decrypt, so the fused CRC never reads it.  Its expected CRC is checked
    by the CRC kernel instead -- a fragment that asked for a check is reported as passed only
    when a check ran and passed -- also when the whole batch is rejected (no decrypt launch)."""
    import zlib

    import numpy as np

    from hlsjs_p2p_wrapper_amd.player.transmux import _Batch

    if device == "cuda":
        request.getfixturevalue("cuda")
    rng = np.random.default_rng(3)
    payloads = [rng.integers(0, 256, n, dtype=np.uint8) for n in (100, 4004, 33)]  # none a multiple of 16
    offs, pos = [], 0
    for p in payloads:
        offs.append(pos)
        pos += (len(p) + 255) // 256 * 256
    arena = torch.zeros(pos + 256, dtype=torch.uint8)
    for o, p in zip(offs, payloads):
        arena[o:o + len(p)] = torch.from_numpy(p)
    arena = arena.to(device)
    n = len(payloads)
    o = np.asarray(offs, dtype=np.int64)
    nb = np.array([len(p) for p in payloads], dtype=np.int64)
    enc = np.ones(n, dtype=bool)
    key = bytes(range(16))
    drk = np.tile(aes.round_keys_le(key), (n, 1)).astype(np.uint32)
    iv = np.zeros((n, 16), dtype=np.uint8)
    keys = np.tile(np.frombuffer(key, dtype=np.uint8), (n, 1))
    crcs = np.array([zlib.crc32(bytes(p)) for p in payloads], dtype=np.int64)
    expect = crcs.copy()
    expect[1] ^= 4  # the middle one's trailer is wrong
    pipe = MediaPipeline(torch.device(device), new_event_loop("virtual"))
    *_, has, ok = pipe.complete_columns(pipe.launch_columns(arena, o, nb, enc, drk, iv, keys=keys, expect=expect))
    assert ok.tolist() == [True, False, True]
    assert not has.any()  # no decrypt / demux result for a rejected fragment
    # the default is "not verified": a fragment that asked for a check no check covered fails
    b = _Batch(None, n=3, expect_mask=np.array([True, False, True]))
    assert MediaPipeline._verified(b, 3).tolist() == [False, True, False]


class _Ticket:
    def __init__(self, expect):
        self.expect = expect
        self.got = None

    def report(self, ok):
        self.got = ok


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_jobs_with_verify_tickets_are_checked_by_their_batch(device, request):
    """In-process deferred receive checks (agent/node.py VerifyTicket): a job carrying a
    ticket is verified by the batch that transmuxes it -- on the GPU the CRC is fused into the
    AES decrypt -- the outcome is reported to the ticket, and a failed fragment's result is a
    ``verify_failed`` error (nothing of it reaches the buffer).  Jobs without a ticket are
    untouched."""
    import zlib

    if device == "cuda":
        request.getfixturevalue("cuda")
    jobs, arena, views, offs = _arena_jobs(device)
    tickets = []
    subs = []
    out = {}
    for n, ((_, payload, key, iv), v) in enumerate(zip(jobs, views)):
        t = None
        if n % 2 == 0:  # every other fragment arrived from a peer
            crc = zlib.crc32(bytes(payload))
            t = _Ticket(crc ^ (1 if n == 2 else 0))  # fragment 2's copy is "corrupted"
            tickets.append((n, t))
        subs.append(TransmuxJob(v, key, iv, lambda r, n=n: out.__setitem__(n, r), n, t))
    loop = new_event_loop("virtual")
    pipe = MediaPipeline(torch.device(device), loop)
    pipe.auto_flush = False
    for j in subs:
        pipe.submit(j)
    pipe.complete(pipe.launch())
    for n, t in tickets:
        assert t.got is (n != 2), (n, t.got)
    assert out[2].get("verify_failed") and out[2]["error"] is not None
    for n in range(len(subs)):
        if n != 2:
            assert out[n].get("error") is None and not out[n].get("verify_failed"), (n, out[n])
