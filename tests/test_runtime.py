"""Native host runtime: ring-allocated segment store, swarm directory + deterministic
exchange planner, AES known-answer vectors, TS mux/demux oracle."""
import numpy as np

from hlsjs_p2p_wrapper_amd.ops import aes


def keys(*sns, swarm=1, level=0, url=0):
    return np.array([[swarm, level, url, s] for s in sns], dtype=np.int64)


# ---------------------------------------------------------------- store
def test_store_reserve_commit_lookup_delta(rt):
    st = rt.SegmentStore(1 << 20, 256)
    base, ids, offs = st.reserve_run(keys(1, 2, 3), np.array([1000, 300, 256]), 0)
    assert base == 0 and offs.tolist() == [0, 1024, 1536]  # contiguous, 256-aligned
    assert st.lookup(keys(1), False).tolist() == [-1]  # pending entries are invisible
    assert st.lookup(keys(1), True).tolist() == [ids[0]]
    st.commit(ids)
    assert st.lookup(keys(1, 2, 3, 4), False).tolist() == ids.tolist() + [-1]
    add, rm = st.take_delta()
    assert add[:, 3].tolist() == [1, 2, 3] and add[:, 4].tolist() == [1000, 300, 256] and len(rm) == 0
    st.drop(ids[:1])
    add, rm = st.take_delta()
    assert len(add) == 0 and rm[:, 3].tolist() == [1]


def test_store_commit_of_a_replaced_copy_is_not_announced(rt):
    """A received copy awaiting its deferred check (pending, pinned by its readers) is replaced
    in the index when the key is fetched again.  Its check passing later commits it for those
    readers only: announcing it would tell peers this rank holds a key its index maps to a
    copy still in flight (fleet chaos, 3 ranks)."""
    st = rt.SegmentStore(1 << 20, 256)
    _, old, _ = st.reserve_run(keys(1), np.array([1000]), 0)
    st.pin(old)
    _, new, _ = st.reserve_run(keys(1), np.array([1000]), 1)
    st.commit(old)
    add, _ = st.take_delta()
    assert len(add) == 0
    st.commit(new)
    add, _ = st.take_delta()
    assert add[:, 3].tolist() == [1]


def test_store_detach_keeps_pinned_bytes_until_the_ring_reaches_them(rt):
    """A received copy that failed its deferred CRC check is detached: no longer found (nor
    announced: it was never committed), its id stays valid while readers hold pins, the key
    can be reserved again at once, and the ring frees the old bytes only after the pins drop."""
    st = rt.SegmentStore(4 * 1024, 256)
    _, ids, _ = st.reserve_run(keys(1, 2), np.array([1024, 1024]), 0)
    st.commit(ids[1:])
    st.pin(ids[:1])
    st.take_delta()
    st.detach(ids[:1])
    assert st.lookup(keys(1), True).tolist() == [-1]
    add, rm = st.take_delta()
    assert len(add) == 0 and len(rm) == 0  # pending: nobody was told about it
    _, again, _ = st.reserve_run(keys(1), np.array([1024]), 1)
    assert again[0] != ids[0] and st.lookup(keys(1), True).tolist() == again.tolist()
    # the ring is full up to the detached, pinned entry: no room until it is unpinned
    assert st.reserve_run(keys(9), np.array([2048]), 2) is None
    st.unpin(ids[:1])
    assert st.reserve_run(keys(9), np.array([2048]), 3) is not None
    st.detach(np.array([ids[1]]))  # a resident one is announced as removed
    _, rm = st.take_delta()
    assert rm[:, 3].tolist() == [2]


def _plan_rows(ks, lens, src, dst, seeded=0):
    rows = np.zeros((len(ks), 9), dtype=np.int64)
    rows[:, :4] = ks
    rows[:, 4] = lens
    rows[:, 5] = src
    rows[:, 6] = dst
    rows[:, 7] = np.arange(len(ks)) + 100
    rows[:, 8] = seeded
    return rows


def test_store_p2p_layout_sends_and_recv_reservations(rt):
    """One native call lays out a round's P2P buffers (node.py:_p2p_phase): a destination
    whose entries lie back to back sends its arena span as is; one that does not (or misses
    an entry) gets a gather list; each source gets one pinned contiguous reservation."""
    st = rt.SegmentStore(1 << 20, 256)
    _, ids, offs = st.reserve_run(keys(1, 2, 3, 4), np.array([1000, 300, 256, 700]), 0)
    st.commit(ids)
    send = np.concatenate([_plan_rows(keys(1, 2), [1000, 300], 0, 1),     # back to back -> span
                           _plan_rows(keys(1, 3, 9), [1000, 256, 50], 0, 2)])  # gap + missing -> gather
    eids = np.array([ids[0], ids[1], ids[0], ids[2], -1], dtype=np.int64)
    recv = np.concatenate([_plan_rows(keys(20, 21), [400, 500], 1, 0), _plan_rows(keys(30), [90], 3, 0)])
    srun, gath, rrun, rid, roff = st.p2p_layout(send, eids, recv, 5)
    assert srun.tolist() == [[1, 0, 2, 0, 0, 1024 + 300], [2, 2, 5, 1, -1, 1024 + 256 + 50]]
    assert gath.tolist() == [[1, offs[0], 0, 1000], [1, offs[2], 1024, 256]]
    assert rrun[:, 0].tolist() == [1, 3] and rrun[:, 1:3].tolist() == [[0, 2], [2, 3]]
    assert roff[1] == roff[0] + 512 and rrun[0, 3] == roff[0] and rrun[0, 4] == 512 + 500
    ent = st.entries(rid)
    assert ent[:, 3].tolist() == [1, 1, 1]  # pinned until the round completes
    assert st.lookup(keys(20, 21, 30), True).tolist() == rid.tolist()  # pending reservations


def test_store_ring_fifo_eviction_and_pins(rt):
    st = rt.SegmentStore(4096, 256)
    _, a, _ = st.reserve_run(keys(1, 2), np.array([1024, 1024]), 0)
    st.commit(a)
    _, b, _ = st.reserve_run(keys(3), np.array([2048]), 1)
    st.commit(b)
    st.take_delta()
    # full: the next 1 KiB evicts the oldest entry (sn 1)
    res = st.reserve_run(keys(4), np.array([1024]), 2)
    assert res is not None and res[2].tolist() == [0]
    assert st.lookup(keys(1), False).tolist() == [-1] and st.evictions == 1
    _, rm = st.take_delta()
    assert rm[:, 3].tolist() == [1]
    st.commit(res[1])
    # pinned entries block eviction
    st.pin(st.lookup(keys(2), False))
    assert st.reserve_run(keys(5), np.array([1024]), 3) is None
    st.unpin(st.lookup(keys(2), False))
    assert st.reserve_run(keys(5), np.array([1024]), 3) is not None


def test_store_wraps_and_evicts_skipped_tail(rt):
    st = rt.SegmentStore(3000, 256)
    for i in range(10):
        r = st.reserve_run(keys(i), np.array([1000]), i)
        assert r is not None
        st.commit(r[1])
        assert r[2][0] + 1024 <= 3000
    assert st.num_entries <= 2


def test_store_evict_below_live_window(rt):
    st = rt.SegmentStore(1 << 20, 256)
    _, ids, _ = st.reserve_run(keys(*range(10)), np.full(10, 100), 0)
    st.commit(ids)
    assert st.evict_below(1, 6) == 6
    assert (st.lookup(keys(*range(10)), False) >= 0).tolist() == [False] * 6 + [True] * 4


# ---------------------------------------------------------------- planner
F = None


def flags(rt, n, **over):
    base = rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD | rt.FLAG_CDN_DEDUP
    f = np.full(n, base, dtype=np.int64)
    for r, v in over.items():
        f[int(r[1:])] = v
    return f


def wants(rows):
    # (sn, size, want_id, rank, wflags)
    return np.array([[1, 0, 0, sn, size, wid, rank, wf] for sn, size, wid, rank, wf in rows], dtype=np.int64)


def test_planner_p2p_from_holder_and_dedup(rt):
    d = rt.Directory()
    d.apply(0, np.array([[1, 0, 0, 5, 1000]], dtype=np.int64), np.zeros((0, 4), np.int64))
    plan = rt.plan_round(d, wants([(5, 1000, 11, 1, 0), (6, 2000, 12, 1, 0), (6, 2000, 21, 2, 0),
                                   (6, 2000, 31, 3, 0)]), flags(rt, 4), 4)
    rows = {(int(r[3]), int(r[6])): r for r in plan}
    assert rows[(5, 1)][5] == 0  # sn 5 held by rank 0 -> P2P 0 -> 1
    seeder = [int(r[6]) for r in plan if r[3] == 6 and r[5] == -1]
    assert len(seeder) == 1  # sn 6 fetched from the CDN exactly once ...
    fwd = [r for r in plan if r[3] == 6 and r[5] >= 0]
    assert len(fwd) == 2 and all(r[5] == seeder[0] and r[8] == 1 for r in fwd)  # ... and forwarded
    # CDN rows first, then P2P grouped by (src, dst)
    assert all(r[5] == -1 for r in plan[:1])


def test_planner_is_deterministic_and_balances_links(rt):
    d = rt.Directory()
    held = np.array([[1, 0, 0, s, 100, ] for s in range(40)], dtype=np.int64)
    for r in (0, 1, 2):
        d.apply(r, held, np.zeros((0, 4), np.int64))
    w = wants([(s, 100, s, 3, 0) for s in range(40)])
    p1 = rt.plan_round(d, w, flags(rt, 4), 4)
    p2 = rt.plan_round(d, w[::-1].copy(), flags(rt, 4), 4)
    assert np.array_equal(p1, p2)  # input order does not matter
    srcs = np.bincount(p1[:, 5], minlength=3)
    assert srcs.max() - srcs.min() <= 1  # spread across the three holders' links


def test_planner_cdn_balance_holds_a_leaders_lone_want_once(rt):
    """Ranks whose players run a round apart never want a segment in the same round, so the
    rank ahead would fetch every segment from the CDN and the others take its copies.  The
    planner's CDN balance holds a lone, unheld want back once when its rank reports its ingest
    link as its bound (FLAG_CDN_BOUND), is over its share of the swarm's CDN bytes, and another
    rank already asks for an earlier segment of the same track; the follower then fetches it
    itself, and the leader's copy comes from the follower."""
    d = rt.Directory()
    mb = 1 << 20
    w = wants([(10, 1000, 1, 0, 0), (9, 1000, 2, 1, 0)])  # rank 0 one segment ahead of rank 1
    cdn = lambda plan: sorted((int(r[3]), int(r[6])) for r in plan if r[5] == -1)  # noqa: E731
    assert cdn(rt.plan_round(d, w, flags(rt, 2), 2)) == [(9, 1), (10, 0)]  # no balance input
    skew = np.array([600 * mb, 100 * mb], dtype=np.int64)
    assert cdn(rt.plan_round(d, w, flags(rt, 2), 2, skew)) == [(9, 1), (10, 0)]  # rank 0's link is not its bound
    full = rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD | rt.FLAG_CDN_DEDUP
    bound = flags(rt, 2, r0=full | rt.FLAG_CDN_BOUND)
    assert cdn(rt.plan_round(d, w, bound, 2, skew)) == [(9, 1)]  # CDN-bound and over its share: sn 10 held
    held = wants([(10, 1000, 1, 0, 8), (9, 1000, 2, 1, 0)])
    assert cdn(rt.plan_round(d, held, bound, 2, skew)) == [(9, 1), (10, 0)]  # kHeld (8): at most once
    even = np.array([300 * mb, 290 * mb], dtype=np.int64)
    assert cdn(rt.plan_round(d, w, bound, 2, even)) == [(9, 1), (10, 0)]  # within its share
    small = np.array([60 * mb, 10 * mb], dtype=np.int64)
    assert cdn(rt.plan_round(d, w, bound, 2, small)) == [(9, 1), (10, 0)]  # start-up: no decision
    ahead = wants([(10, 1000, 1, 0, 0), (11, 1000, 2, 1, 0)])  # rank 1 is ahead, not following sn 10
    assert cdn(rt.plan_round(d, ahead, bound, 2, skew)) == [(10, 0), (11, 1)]
    nodedup = flags(rt, 2, r0=full | rt.FLAG_CDN_BOUND, r1=rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD)
    assert cdn(rt.plan_round(d, w, nodedup, 2, skew)) == [(9, 1), (10, 0)]  # follower not in the CDN dedup swarm
    # want order does not change the plan (every rank computes the same one)
    assert np.array_equal(rt.plan_round(d, w, bound, 2, skew), rt.plan_round(d, w[::-1].copy(), bound, 2, skew))


def test_planner_respects_flags(rt):
    d = rt.Directory()
    d.apply(0, np.array([[1, 0, 0, 5, 1000]], dtype=np.int64), np.zeros((0, 4), np.int64))
    w = wants([(5, 1000, 1, 1, 0)])
    assert rt.plan_round(d, w, flags(rt, 2, r0=rt.FLAG_ONLINE | rt.FLAG_DOWNLOAD), 2)[0][5] == -1  # no upload
    assert rt.plan_round(d, w, flags(rt, 2, r0=rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD), 2)[0][5] == -1  # offline
    assert rt.plan_round(d, w, flags(rt, 2, r1=rt.FLAG_ONLINE), 2)[0][5] == -1  # wanter: no P2P download
    assert rt.plan_round(d, wants([(5, 1000, 1, 1, 1)]), flags(rt, 2), 2)[0][5] == -1  # force-CDN want
    assert rt.plan_round(d, w, flags(rt, 2), 2)[0][5] == 0
    d.drop_rank(0)
    assert rt.plan_round(d, w, flags(rt, 2), 2)[0][5] == -1


# ---------------------------------------------------------------- AES / TS oracles
def test_aes_known_answer_vectors(rt):
    # FIPS-197 C.1
    assert rt.aes_encrypt_block(bytes(range(16)), bytes.fromhex("00112233445566778899aabbccddeeff")).hex() == \
        "69c4e0d86a7b0430d8cdb78070b4c55a"
    # NIST SP 800-38A F.2.1 CBC-AES128 (first block)
    key = bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c")
    iv = bytes.fromhex("000102030405060708090a0b0c0d0e0f")
    pt = np.frombuffer(bytes.fromhex("6bc1bee22e409f96e93d7e117393172a"), np.uint8)
    ct = aes.cbc_encrypt(key, iv, pt)
    assert ct[:16].tobytes().hex() == "7649abac8119b246cee98e9b12e9197d"
    assert len(ct) == 32  # + one full PKCS#7 padding block
    assert aes.cbc_decrypt(key, iv, ct).tobytes() == pt.tobytes()
    assert aes.iv_from_sn(1) == bytes(15) + b"\x01"


def test_cpu_batch_decrypt_and_bad_padding():
    import torch

    key = bytes(range(16))
    segs = [np.random.default_rng(i).integers(0, 256, n, dtype=np.uint8) for i, n in enumerate([5, 100, 4096])]
    cts = [aes.cbc_encrypt(key, aes.iv_from_sn(i), s) for i, s in enumerate(segs)]
    offs = [0, 256, 512]
    src = torch.zeros(8192, dtype=torch.uint8)
    for o, c in zip(offs, cts):
        src[o:o + len(c)] = torch.from_numpy(c)
    dst = torch.zeros_like(src)
    out = aes.cbc_decrypt_batch(src, offs, [len(c) for c in cts], [key] * 3,
                                [aes.iv_from_sn(i) for i in range(3)], dst, offs)
    assert out.tolist() == [5, 100, 4096]
    for o, s in zip(offs, segs):
        assert dst[o:o + len(s)].numpy().tobytes() == s.tobytes()
    bad = aes.cbc_decrypt_batch(src, offs[:1], [16], [bytes(16)], [bytes(16)], dst, offs[:1])
    assert bad.tolist()[0] in (-1,) or bad.tolist()[0] >= 0


def test_mux_demux_roundtrip_and_pts(rt):
    import torch

    from hlsjs_p2p_wrapper_amd.ops import tsdemux

    seg, st = tsdemux.mux_segment(duration=4.0, fps=25, target_bytes=800_000, with_id3=True, seed=3, sn=10,
                                  start_time=40.0)
    assert len(seg) % 188 == 0 and abs(len(seg) - 800_000) < 40_000
    buf = torch.from_numpy(seg.copy())
    es = torch.zeros(len(seg), dtype=torch.uint8)
    r = tsdemux.demux_batch(buf, [0], [len(seg)], es, [0])
    s = r.segment(0)
    assert s["status"] == 0 and s["video_pid"] == 0x100 and s["audio_pid"] == 0x101 and s["id3_pid"] == 0x102
    assert (s["video_bytes"], s["audio_bytes"], s["id3_bytes"]) == st["es_bytes"]
    assert (s["n_video_pes"], s["n_audio_pes"], s["n_id3_pes"]) == st["n_pes"]
    assert s["video_first_pts"] == st["first_pts"][0] == 900000 + 40 * 90000 + 3600
    v = s["video"]["es"].numpy()
    assert v[:6].tolist() == [0, 0, 0, 1, 0x09, 0xF0]  # AUD NAL at the start of the video ES
    assert s["video"]["pes"][0][0] == 0 and s["video"]["pes"][1][1] - s["video"]["pes"][0][1] == 3600
    # corrupt a sync byte -> flagged, packet skipped
    buf[188 * 50] = 0
    r2 = tsdemux.demux_batch(buf, [0], [len(seg)], es, [0])
    assert r2.segment(0)["status"] & tsdemux.STATUS["bad_sync"]


def test_planner_seeds_contiguous_runs(rt):
    # 4 ranks want the same 64 fresh segments: each seeds ONE contiguous sn run of 16 (a
    # single merged pinned-host -> HBM DMA per rank) and forwards it to the other three
    d = rt.Directory()
    rows = [(sn, 3_000_000, 1000 * r + sn, r, 0) for r in range(4) for sn in range(64)]
    plan = rt.plan_round(d, wants(rows), flags(rt, 4), 4)
    cdn = plan[plan[:, 5] == -1]
    assert len(cdn) == 64
    for r in range(4):
        sns = sorted(int(x) for x in cdn[cdn[:, 6] == r][:, 3])
        assert len(sns) == 16 and sns == list(range(sns[0], sns[0] + 16))
    p2p = plan[plan[:, 5] >= 0]
    assert len(p2p) == 64 * 3 and np.all(p2p[:, 8] == 1)


# ---------------------------------------------------------------- want table
def _add(wt, ks, size=1000, flags=0, tokens=None, ptr=0):
    n = len(ks)
    tok = np.arange(n, dtype=np.int64) if tokens is None else np.asarray(tokens, dtype=np.int64)
    return wt.add(ks, np.full(n, size, dtype=np.int64), np.full(n, ptr, dtype=np.int64),
                  np.zeros(n, dtype=np.int64), np.full(n, flags, dtype=np.int64), tok)


def test_want_table_join_abort_finish(rt):
    """Requests join the want of their key as tokens; aborted tokens are forgotten; a want
    nobody waits for any more is dropped at the next selection; finishing a want returns its
    live tokens (the delivery columns)."""
    wt = rt.WantTable()
    st = rt.SegmentStore(1 << 20, 256)
    ids, created = _add(wt, keys(1, 2, 1), tokens=[10, 11, 12])
    assert created.tolist() == [1, 1, 0] and ids[0] == ids[2] and len(wt) == 2 and wt.num_tokens == 3
    assert wt.abort(np.array([11], dtype=np.int64)) == 1 and wt.abort1(99) is False
    adm, rows, dropped, big, deferred = wt.select(st, None, -1, 1)
    assert adm.tolist() == [ids[0]] and dropped.tolist() == [ids[1]] and len(big) == 0 and deferred == 0
    assert rows[0, :5].tolist() == [1, 0, 0, 1, 1000] and rows[0, 5] == ids[0]
    assert wt.select(st, None, -1, 2)[0].tolist() == []  # in flight: not announced again
    tok, idx, pf = wt.finish(adm)
    assert sorted(tok.tolist()) == [10, 12] and idx.tolist() == [0, 0] and pf.tolist() == [0]
    assert len(wt) == 0 and wt.num_tokens == 0
    # in-process object path: add1 returns -id-1 for a new want, the id when joining
    r = wt.add1(1, 0, 0, 7, 500, 0, 0, 0, -2)
    assert r < 0 and wt.add1(1, 0, 0, 7, 500, 0, 0, 0, -3) == -r - 1 and wt.lookup1(1, 0, 0, 7) == -r - 1


def test_want_table_select_order_cap_and_backpressure(rt):
    """Requested wants go first (FIFO, capped), prefetch-only ones fill the room left; only
    the largest prefix the ring can place now is admitted; a want larger than the whole
    cache is reported, the rest wait; requeued wants keep their place."""
    wt = rt.WantTable()
    st = rt.SegmentStore(8 * 1024, 256)
    pf_ids, _ = _add(wt, keys(100), flags=rt.WANT_PREFETCH, tokens=[rt.NO_TOKEN])
    ids, _ = _add(wt, keys(1, 2, 3), size=2048, tokens=[1, 2, 3])
    assert wt.select(st, None, 0, 1)[0].tolist() == []  # cap 0 (maxWantsPerRound: 0) admits nothing
    adm, _, _, _, _ = wt.select(st, None, 2, 1)
    assert adm.tolist() == ids[:2].tolist()  # cap 2: requests before the prefetch
    wt.requeue(adm, False)
    adm, _, _, _, deferred = wt.select(st, None, -1, 2)
    assert adm.tolist() == ids.tolist() + pf_ids.tolist() and deferred == 0  # 3 x 2 KiB + 1 KiB fits 8 KiB
    wt.requeue(adm, False)
    # fill the ring with a pinned entry: only 2 KiB stay free
    _, e, _ = st.reserve_run(keys(50), np.array([6 * 1024]), 0)
    st.commit(e)
    st.pin(e)
    big, _ = _add(wt, keys(9), size=64 * 1024, tokens=[9])
    adm, _, _, too_big, deferred = wt.select(st, None, -1, 3)
    assert adm.tolist() == ids[:1].tolist() and too_big.tolist() == big.tolist() and deferred == 3
    # a CRC failure requeues with force_cdn (row bit 62) and one more attempt
    wt.requeue(adm, True)
    info = wt.info(adm)
    assert info[0, 7] & rt.WANT_FORCE_CDN and info[0, 9] == 1 and info[0, 8] == -1


def test_want_table_unstaged_size_from_directory(rt):
    """A network want whose body is not staged yet has no size; once a holder announced the
    segment, selection reserves the holder's length (so a peer copy always fits what the
    receiver admitted: never a reservation failure mid-round), and backpressure applies to it."""
    wt = rt.WantTable()
    st = rt.SegmentStore(4096, 256)
    d = rt.Directory()
    ids, _ = _add(wt, keys(5), size=0, flags=rt.WANT_NOT_STAGED, tokens=[1])
    adm, rows, _, _, _ = wt.select(st, d, -1, 1)
    assert adm.tolist() == ids.tolist() and rows[0, 4] == 0 and (rows[0, 5] >> 61) & 1
    wt.requeue(adm, False)
    d.apply(0, np.array([[1, 0, 0, 5, 3000]], dtype=np.int64), np.zeros((0, 4), dtype=np.int64))
    _, e, _ = st.reserve_run(keys(60), np.array([2048]), 0)  # nearly full: 2 KiB free, 3000 B needed
    st.commit(e)
    st.pin(e)
    adm, _, _, _, deferred = wt.select(st, d, -1, 2)
    assert adm.tolist() == [] and deferred == 1  # waits rather than over-commit the ring
    st.unpin(e)
    adm, rows, _, _, _ = wt.select(st, d, -1, 3)
    assert adm.tolist() == ids.tolist() and rows[0, 4] == 3000


def test_the_nodes_want_flags_match_the_want_table_bits(rt):
    """The node ORs its own flags into the want table's (requests, locator, CDN phase): each
    must be the table's bit of that name and none may alias another.  W_ON_DEV once shared
    bit 64 with the table's "held" bit, so a requeued want looked device-resident to the GPU
    CDN phase."""
    from hlsjs_p2p_wrapper_amd.agent import node as n

    assert (n.W_FORCE_CDN, n.W_NOT_STAGED, n.W_STAGING, n.W_PREFETCH, n.W_PY, n.W_CORRUPT, n.W_ON_DEV) == (
        rt.WANT_FORCE_CDN, rt.WANT_NOT_STAGED, rt.WANT_STAGING, rt.WANT_PREFETCH, rt.WANT_PY, rt.WANT_CORRUPT,
        rt.WANT_ON_DEV)
    bits = [rt.WANT_FORCE_CDN, rt.WANT_NOT_STAGED, rt.WANT_STAGING, rt.WANT_PREFETCH, rt.WANT_PY, rt.WANT_CORRUPT,
            rt.WANT_HELD, rt.WANT_ON_DEV]
    assert len(set(bits)) == len(bits) and all(b & (b - 1) == 0 for b in bits)
    wt = rt.WantTable()
    ids, _ = _add(wt, keys(3), size=100, flags=0, tokens=[1])
    wt.requeue(ids, False)
    assert not (wt.info(ids)[0, 7] & n.W_ON_DEV)  # held, not device-resident


def test_planner_never_sends_more_than_the_wanter_admitted(rt):
    """A receive lands in the ring region its wanter's admission retired (the
    round's reservations could reach past it): the planner never sends a copy larger than the
    want's announced size.  A staged want smaller than the holder's copy goes to the CDN, a
    not-staged one (size still unknown) waits for the holder's length; a seeded forward obeys
    the same rule."""
    d = rt.Directory()
    d.apply(0, np.array([[1, 0, 0, 5, 3000]], dtype=np.int64), np.zeros((0, 4), np.int64))
    # holder transfer: sizes 3000 (fits), 2000 (staged, smaller: CDN), 0 (not staged: waits)
    plan = rt.plan_round(d, wants([(5, 3000, 11, 1, 0), (5, 2000, 21, 2, 0), (5, 0, 31, 3, 2)]), flags(rt, 4), 4)
    by = {int(r[6]): (int(r[5]), int(r[4])) for r in plan}
    assert by[1] == (0, 3000) and by[2] == (-1, 2000) and 3 not in by
    assert all(r[4] <= {11: 3000, 21: 2000, 31: 0}[int(r[7])] for r in plan)
    # seeded forwards: the seeder's copy is larger than one wanter's own size
    plan = rt.plan_round(rt.Directory(), wants([(9, 4000, 12, 1, 0), (9, 4000, 22, 2, 0), (9, 3500, 32, 3, 0)]),
                         flags(rt, 4), 4)
    for r in plan:
        assert r[4] <= {12: 4000, 22: 4000, 32: 3500}[int(r[7])]


def test_planner_spreads_lone_seeds_across_the_wanters(rt):
    """The live edge: every rank wants the same one new segment per round and nobody holds it.
    The seeder rotation starts at a rank drawn from the round's first seed key, so over many
    rounds every wanting rank seeds its share (it started at rank 0 every round, which made
    the lowest rank fetch the whole channel from the CDN); every replica draws the same rank."""
    world, rounds = 8, 400
    seeds = np.zeros(world, dtype=np.int64)
    for sn in range(rounds):
        rows = wants([(sn, 3000, 100 * sn + r, r, 0) for r in range(world)])
        plan = rt.plan_round(rt.Directory(), rows, flags(rt, world), world)
        cdn = [int(r[6]) for r in plan if r[5] == -1]
        assert len(cdn) == 1  # one fetch, forwarded to the 7 others
        assert sorted(int(r[6]) for r in plan if r[5] == cdn[0]) == [r for r in range(world) if r != cdn[0]]
        assert np.array_equal(rt.plan_round(rt.Directory(), rows, flags(rt, world), world), plan)
        seeds[cdn[0]] += 1
    assert seeds.min() >= rounds / world / 2, seeds  # ~50 each; rank 0 alone seeded all 400 before
    # a round with many seeds still gives every rank one contiguous run of its quota
    rows = wants([(sn, 3000, 1000 * r + sn, r, 0) for r in range(world) for sn in range(64)])
    plan = rt.plan_round(rt.Directory(), rows, flags(rt, world), world)
    for r in range(world):
        sns = sorted(int(p[3]) for p in plan if p[5] == -1 and p[6] == r)
        assert len(sns) == 8 and sns == list(range(sns[0], sns[0] + 8))


def test_planner_spreads_a_lone_wanters_holders(rt):
    """A late joiner wants segments every other rank already holds: the holders take turns
    across rounds (the holder rotation is shifted by a key-drawn offset) instead of the rank
    after the wanter serving every one."""
    world, n = 8, 400
    d = rt.Directory()
    adds = np.array([[1, 0, 0, sn, 3000] for sn in range(n)], dtype=np.int64)
    for r in range(1, world):
        d.apply(r, adds, np.zeros((0, 4), np.int64))
    served = np.zeros(world, dtype=np.int64)
    for sn in range(n):
        plan = rt.plan_round(d, wants([(sn, 3000, sn, 0, 0)]), flags(rt, world), world)
        assert len(plan) == 1 and plan[0][6] == 0 and plan[0][5] >= 1
        served[int(plan[0][5])] += 1
    assert served[0] == 0 and served[1:].min() >= n / (world - 1) / 2, served
