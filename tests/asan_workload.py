"""Exercise every entry point of the native host runtime; run by test_asan_runtime.py
against the ASan/UBSan build (``python -m hlsjs_p2p_wrapper_amd.ops.build --asan``)
under ``LD_PRELOAD=libasan`` (sanitizers on the host-side code).

Usage: python asan_workload.py <path to the sanitizer-built _runtime*.so>
"""
import importlib.util
import sys
import zlib

import numpy as np


def load(path):
    spec = importlib.util.spec_from_file_location("_runtime", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def store_churn(rt, rng):
    st = rt.SegmentStore(1 << 20, 256)
    live = []
    for rnd in range(400):
        n = int(rng.integers(1, 6))
        sns = rng.integers(0, 200, n)
        keys = np.stack([np.ones(n), np.zeros(n), rng.integers(0, 2, n), sns], axis=1).astype(np.int64)
        lens = rng.integers(1, 70_000, n).astype(np.int64)
        res = st.reserve_run(keys, lens, rnd)
        if res is not None:
            _, ids, offs = res
            assert np.all(offs + lens <= st.capacity)
            if rng.random() < 0.2:
                st.drop(ids)
            else:
                st.commit(ids)
                live.extend(ids.tolist())
        if live and rng.random() < 0.3:
            pick = np.asarray(rng.choice(live, size=min(3, len(live)), replace=False), dtype=np.int64)
            st.pin(pick)
            st.unpin(pick)
        if rng.random() < 0.05:
            st.evict_below(1, int(rng.integers(0, 200)))
        st.lookup(keys, False)
        st.take_delta()
    if live:
        st.entries(np.asarray(live[-8:], dtype=np.int64))


def planner(rt, rng):
    world = 8
    d = rt.Directory()
    for r in range(world):
        held = np.stack([np.ones(50), np.zeros(50), np.zeros(50), rng.integers(0, 100, 50),
                         rng.integers(1000, 4_000_000, 50)], axis=1).astype(np.int64)
        d.apply(r, held, np.zeros((0, 4), np.int64))
    flags = np.full(world, rt.FLAG_ONLINE | rt.FLAG_UPLOAD | rt.FLAG_DOWNLOAD | rt.FLAG_CDN_DEDUP, dtype=np.int64)
    for _ in range(50):
        n = 200
        wants = np.stack([np.ones(n), np.zeros(n), np.zeros(n), rng.integers(0, 150, n),
                          rng.integers(1000, 4_000_000, n), np.arange(n), rng.integers(0, world, n),
                          rng.integers(0, 2, n)], axis=1).astype(np.int64)
        plan = rt.plan_round(d, wants, flags, world)
        assert plan.shape[1] == 10
        rm = np.stack([np.ones(5), np.zeros(5), np.zeros(5), rng.integers(0, 100, 5)], axis=1).astype(np.int64)
        d.apply(int(rng.integers(0, world)), np.zeros((0, 5), np.int64), rm)
    d.drop_rank(3)


def crypto_and_crc(rt, rng):
    key = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    iv = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    for n in (0, 1, 15, 16, 17, 4095, 100_000):
        pt = rng.integers(0, 256, n, dtype=np.uint8)
        ct = rt.cbc_encrypt(key, iv, pt)
        assert len(ct) % 16 == 0 and len(ct) > n
        back = rt.cbc_decrypt(key, iv, ct)
        assert back is not None and back.tobytes() == pt.tobytes()
        assert rt.crc32(pt) == zlib.crc32(pt.tobytes())
    junk = rng.integers(0, 256, 64, dtype=np.uint8)
    rt.cbc_decrypt(key, iv, junk)  # bad padding: None or bytes, never a fault
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    offs = np.array([0, 1000, 70_000, 500_000], dtype=np.int64)
    lens = np.array([1000, 0, 300_000, 524_288], dtype=np.int64)
    crc = rt.crc32_batch(buf, offs, lens)
    for o, n, c in zip(offs, lens, crc.view(np.uint32)):
        assert int(c) == zlib.crc32(buf[o:o + n].tobytes())
    rt.crc_mfma_weights()
    rt.crc_shift_tables()
    rt.aes_tables()


def ts_fuzz(rt, rng):
    infow = rt.TS_INFO_WORDS
    seg, _ = rt.mux_segment(4.0, 25.0, 400_000, 128, True, 5, 3, 12.0)
    cases = [seg.copy()]
    for _ in range(30):  # random bit flips / truncations / pure noise
        s = seg.copy()
        idx = rng.integers(0, len(s), 200)
        s[idx] ^= rng.integers(1, 256, 200, dtype=np.uint8)
        cases.append(s[: int(rng.integers(0, len(s)))])
    cases.append(rng.integers(0, 256, 188 * 300, dtype=np.uint8))
    noise = rng.integers(0, 256, 188 * 300, dtype=np.uint8)
    noise[::188] = 0x47  # valid sync, garbage headers
    cases.append(noise)
    for c in cases:
        n = len(c)
        buf = np.zeros(max(n, 1) + 256, dtype=np.uint8)
        buf[:n] = c
        es = np.zeros(max(n, 1) + 256, dtype=np.uint8)
        max_pes = 64
        pes = np.zeros((1, 3, max_pes, 3), dtype=np.int64)
        info = np.zeros((1, infow), dtype=np.int64)
        rt.demux_batch(buf, np.array([0], np.int64), np.array([n], np.int64), es, np.array([0], np.int64),
                       pes, info, max_pes)


def main():
    rt = load(sys.argv[1])
    rng = np.random.default_rng(1234)
    store_churn(rt, rng)
    planner(rt, rng)
    crypto_and_crc(rt, rng)
    ts_fuzz(rt, rng)
    print("ASAN-WORKLOAD-OK")


if __name__ == "__main__":
    main()
