"""Index math of the decrypt's packet-header records (aes_cbc.hip AesHdr, ts_demux.hip
ts_scan_kernel), checked on the CPU: block b stores record q = ceil(16 b / 188) iff packet q
starts inside it, with the division done as umulhi(16 b + 187, M) >> 7; every packet's header
then sits whole in its record at byte (188 q) mod 16, and every packet gets exactly one record."""
import numpy as np

MAGIC = 2924233053  # aes_cbc.hip kDiv188Magic


def test_header_record_index_math():
    b = np.arange(0, 1 << 20, dtype=np.uint64)  # 16 MiB of blocks, past any HLS segment
    b16 = b << np.uint64(4)
    q = ((b16 + np.uint64(187)) * np.uint64(MAGIC)) >> np.uint64(39)  # umulhi(., M) >> 7
    assert np.array_equal(q, (b16 + np.uint64(187)) // np.uint64(188))
    has = (q * np.uint64(188) - b16) < np.uint64(16)
    recs = q[has]
    # one record per packet, in order, and each header lies inside its block
    assert np.array_equal(recs, np.arange(len(recs), dtype=np.uint64))
    off = (recs * np.uint64(188)) & np.uint64(15)
    assert set(np.unique(off).tolist()) == {0, 4, 8, 12}
    assert np.all(recs * np.uint64(188) + np.uint64(4) <= (b[has] + np.uint64(1)) * np.uint64(16))
