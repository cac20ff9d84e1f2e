"""Keyed CRCs (SURVEY K2 on the device): the node's CRC table, the trailers peers send and
the receiver's check hold ``crc32 ^ key_digest(key)``, computed in the CRC combine kernel
from the 12-byte keys riding its descriptor block.  A CRC alone only proves that bytes match
the CRC sent with them; a sender whose entry was overwritten by another segment (round 5's
bookkeeping bugs) sends bytes and table CRC that agree with each other and not with the key
the receiver asked for.  Bound to the key, that copy fails the receiver's check and is
re-fetched from the CDN.  Reference: the 12-byte key ``segment-view.js:9-17,59-61``."""
import threading
import zlib

import numpy as np
import pytest
import torch

from hlsjs_p2p_wrapper_amd.net import clear_origins, new_event_loop
from hlsjs_p2p_wrapper_amd.net.origin import Rendition, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import crc as _crc
from hlsjs_p2p_wrapper_amd.parallel import ThreadHub

KEYS = np.array([[7, 0, 0, 1], [7, 0, 0, 2], [7, 1, 0, 1], [7, 0, 1, 1], [8, 0, 0, 1], [0, 0, 0, 0]], dtype=np.int64)


def _mix64(z):
    m = (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def _digest_py(k):
    """Independent Python statement of the digest (the native host and device twins must match)."""
    swarm, level, url, sn = (int(v) & 0xFFFFFFFF for v in k)
    a = level | (url << 32)
    b = sn | (swarm << 32)
    z = _mix64(a ^ _mix64((b + 0x9E3779B97F4A7C15) & ((1 << 64) - 1)))
    return (z ^ (z >> 32)) & 0xFFFFFFFF


def test_host_digest_matches_its_statement_and_separates_keys():
    d = _crc.key_digest(KEYS).view(np.uint32)
    assert d.tolist() == [_digest_py(k) for k in KEYS]
    assert len(set(d.tolist())) == len(KEYS)  # every field of the key changes it


def _buf_and_rows(device):
    g = torch.Generator().manual_seed(11)
    buf = torch.randint(0, 256, (1 << 16,), dtype=torch.uint8, generator=g)
    offs = np.array([0, 4096, 12288, 20480, 40960, 49152], dtype=np.int64)
    lens = np.array([3000, 7000, 1, 17000, 0, 9999], dtype=np.int64)
    raw = np.array([zlib.crc32(buf[o:o + n].numpy().tobytes()) for o, n in zip(offs, lens)], dtype=np.uint32)
    return buf.to(device), offs, lens, raw.view(np.int32)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_keyed_check_and_table(device, request):
    if device == "cuda":
        request.getfixturevalue("cuda")
    buf, offs, lens, raw = _buf_and_rows(device)
    keyed = raw ^ _crc.key_digest(KEYS)
    table = torch.zeros(16, dtype=torch.int32, device=device)
    idx = np.array([3, 5, 7, 9, 11, 13], dtype=np.int64)
    crc, ok = _crc.crc32_batch(buf, offs, lens, expect_dev=torch.from_numpy(keyed.copy()).to(device),
                               scatter_to=table, scatter_idx=idx, keys=KEYS)
    assert crc.cpu().numpy().tolist() == raw.tolist()  # the plain CRC-32 comes back
    assert ok.cpu().numpy().tolist() == [1] * 6
    assert table.cpu().numpy()[idx].tolist() == keyed.tolist()  # the table holds keyed values
    # the same bytes checked under other keys (rows rotated): every row fails
    _, ok2 = _crc.crc32_batch(buf, offs, lens, expect_dev=torch.from_numpy(keyed.copy()).to(device),
                              keys=np.roll(KEYS, 1, axis=0))
    assert ok2.cpu().numpy().tolist() == [0] * 6
    # unkeyed mode is unchanged
    _, ok3 = _crc.crc32_batch(buf, offs, lens, expect=(raw.view(np.uint32)).tolist())
    assert ok3.cpu().numpy().tolist() == [1] * 6


class _Sink:
    def __init__(self):
        self.got = {}
        self.pending = []  # rows delivered before their check: (tok, eids, offs, nbytes, expect)

    def deliver(self, tok, src, nbytes, cdn_ms, p2p_ms, offs, eids, expect=None):
        for t, s in zip(tok.tolist(), src.tolist()):
            self.got[t] = s  # (a re-delivery after a failed check overwrites it)
        if expect is not None:
            chk = np.asarray(expect) >= 0
            if chk.any():
                self.pending.append((tok[chk], eids[chk], offs[chk], nbytes[chk], np.asarray(expect)[chk]))

    def fail(self, tok, status):
        raise AssertionError("failed")


@pytest.mark.parametrize("deferred", [False, True])
def test_a_segment_sent_under_another_key_is_rejected(deferred):
    """Rank 0 holds sn 0-7 of a stream whose sn k and k + 4 have the SAME bytes (pool of 4), so
    a plain CRC cannot tell them apart; it sends rank 1 the entry of sn 0 for sn 4 (injected
    misroute).  The keyed check rejects it -- by the node (``deferred`` False) or by the
    consumer's check of the unbound expectation -- and sn 4 comes again from the CDN."""
    from hlsjs_p2p_wrapper_amd.agent.node import SRC_CDN, SRC_P2P, SwarmNode

    clear_origins()
    origin = SyntheticHlsOrigin("http://cdn.keyed/vod/", renditions=[Rendition(600_000, 320, 180)], num_segments=8,
                                encrypted=False, pool_size=4)
    urls = [origin.base_url + origin.segment_path(0, sn) for sn in range(8)]
    keys = np.array([[5, 0, 0, sn] for sn in range(8)], dtype=np.int64)
    hub = ThreadHub(2, timeout=60)
    nodes, sinks, errs = {}, {0: _Sink(), 1: _Sink()}, []

    def rank(r):
        try:
            new_event_loop("virtual")
            node = SwarmNode(hub.comm(r), device="cpu", cache_bytes=64 << 20, auto_tick=False)
            node.verify_deferred = deferred
            nodes[r] = node
            node.set_bulk_sink(sinks[r])
            for step in range(8):
                if r == 0 and step == 0:
                    node.request_batch(keys, urls, None, np.arange(8, dtype=np.int64))
                if r == 1 and step == 3:
                    node.request_batch(keys[4:], urls[4:], None, np.arange(4, 8, dtype=np.int64))
                if r == 0 and step == 3:
                    node.misroute_next_send = 1
                node.complete_round(node.launch_round())
                node.loop.run_until(lambda: False, timeout_ms=1)
                if deferred:
                    _check_deferred(node, sinks[r])
        except BaseException as e:  # noqa: BLE001
            errs.append(e)
            hub.abort()

    ts = [threading.Thread(target=rank, args=(r,)) for r in range(2)]
    [t.start() for t in ts]
    [t.join(90) for t in ts]
    clear_origins()
    assert not errs, errs
    assert nodes[0].misroute_next_send == 0  # the misroute was injected
    assert nodes[1].stats["crc_failures"] == 1 and nodes[1].stats["p2p_rejected_segments"] == 1
    got = sinks[1].got
    assert sorted(got) == [4, 5, 6, 7]
    assert got[4] == SRC_CDN and [got[t] for t in (5, 6, 7)] == [SRC_P2P] * 3


def _check_deferred(node, sink):
    """What a fleet transmux does with rows delivered before their check: CRC-32 of the bytes
    against the delivered (unbound) expectation, reported to the node."""
    rows, sink.pending = sink.pending, []
    for tok, eids, offs, nbytes, expect in rows:
        a = node.arena.numpy()
        ok = np.array([(zlib.crc32(a[o:o + n].tobytes()) & 0xFFFFFFFF) == (e & 0xFFFFFFFF)
                       for o, n, e in zip(offs.tolist(), nbytes.tolist(), expect.tolist())])
        node.verify_done(eids, ok, tok)
