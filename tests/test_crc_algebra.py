"""CPU validation of the MFMA CRC formulation: the host-built weight fragments and shift
tables, evaluated with numpy exactly as the gfx950 kernels evaluate them, reproduce
zlib.crc32 (so a GPU mismatch can only be a kernel bug, not an algebra bug)."""
import zlib

import numpy as np


def _apply(tab, b, v):
    t = tab[b * 1024:(b + 1) * 1024]
    return int(t[v & 0xFF] ^ t[256 + ((v >> 8) & 0xFF)] ^ t[512 + ((v >> 16) & 0xFF)] ^ t[768 + (v >> 24)])


def _emulate(data: bytes, w: np.ndarray, tab: np.ndarray) -> int:
    n = len(data)
    G = (n + 255) // 256
    buf = np.zeros(G * 256, np.uint8)
    buf[:n] = np.frombuffer(data, np.uint8)
    # W fragments [s][lane][e] in the kernel's order: s = 8q + jb, element e = byte
    # 32q + 16h + e of the group masked to bit jb (i8 value 2^jb, -128 for jb = 7)
    wf = w.reshape(64, 64, 16).astype(np.int64)
    residues = []
    for g in range(G):
        grp = buf[g * 256:(g + 1) * 256]
        acc = np.zeros(32, np.int64)
        for s in range(64):
            q, jb = s >> 3, s & 7
            for h in range(2):
                chunk = grp[32 * q + 16 * h:32 * q + 16 * h + 16].astype(np.int64) & (1 << jb)
                a = np.where(chunk >= 128, chunk - 256, chunk)  # signed i8
                for col in range(32):
                    acc[col] += int((a * wf[s, col + 32 * h, :]).sum())
        r = 0
        for col in range(32):
            r |= ((int(acc[col]) >> 7) & 1) << col
        residues.append(r)
    raw = 0
    for r in residues:  # Horner with P_8 = one 256-byte group
        raw = _apply(tab, 8, raw) ^ r
    pad = G * 256 - n
    for b in range(8):
        if (pad >> b) & 1:
            raw = _apply(tab, 40 + b, raw)
    init = 0xFFFFFFFF
    for b in range(40):
        if (n >> b) & 1:
            init = _apply(tab, b, init)
    return raw ^ init ^ 0xFFFFFFFF


def test_mfma_crc_formulation_matches_zlib(rt):
    w = rt.crc_mfma_weights()
    tab = rt.crc_shift_tables()
    assert w.shape == (65536,) and set(np.unique(w)) <= {0, 1, 2, 4, 8, 16, 32, 64, -128}
    rng = np.random.default_rng(1)
    for n in (1, 3, 255, 256, 300, 700):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert _emulate(data, w, tab) == zlib.crc32(data), n


def test_host_crc_matches_zlib(rt):
    rng = np.random.default_rng(2)
    for n in (0, 1, 7, 8, 9, 1000, 65537):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        assert rt.crc32(d) == zlib.crc32(d.tobytes())


_E2M1 = np.array([0, 0.5, 1, 1.5, 2, 3, 4, 6, -0.0, -0.5, -1, -1.5, -2, -3, -4, -6])


def _fp4_elements(words) -> np.ndarray:
    """32 e2m1 values of a 4-dword operand fragment, element j = 8v + e = nibble e of dword v."""
    w = np.asarray(words, dtype=np.uint64).reshape(4, 1)
    nib = (w >> (4 * np.arange(8, dtype=np.uint64))) & 0xF
    return _E2M1[nib.reshape(-1).astype(np.int64)]


def test_fp4_mfma_crc_formulation_matches_zlib(rt):
    """The f8f6f4 path: each step feeds one data dword per lane as four e2m1 operand dwords
    (nibble bits 0/1/2/3 = 0.5/1.0/2.0/2.0) against host B fragments scaled by the inverse;
    the f32 accumulator must be an exact count whose parity is the group's raw CRC bit."""
    w = rt.crc_mfma_weights_fp4().reshape(32, 64, 16)
    b = np.stack([[_fp4_elements(np.frombuffer(w[s, lane].tobytes(), dtype=np.uint32)) for lane in range(64)]
                  for s in range(32)])  # [s][lane][32]
    rng = np.random.default_rng(11)
    groups = rng.integers(0, 256, size=(6, 256), dtype=np.uint8)
    groups[0] = 0xFF  # every nibble bit set: the largest counts
    for grp in groups:
        acc = np.zeros(32)
        for s in range(32):
            q, wd = s >> 2, s & 3
            for h in range(2):
                d = int(np.frombuffer(grp[32 * q + 16 * h + 4 * wd:][:4].tobytes(), dtype=np.uint32)[0])
                a = _fp4_elements([d & 0x11111111, d & 0x22222222, d & 0x44444444, (d >> 1) & 0x44444444])
                acc += b[s, 32 * h:32 * h + 32] @ a
        assert np.all(acc == np.round(acc)) and acc.max() <= 2048  # exact in f32
        par = sum((int(acc[c]) & 1) << c for c in range(32))
        assert par == (~zlib.crc32(grp.tobytes(), 0xFFFFFFFF)) & 0xFFFFFFFF  # zero-init register


def _chunk_rows(chunk: np.ndarray, wf: np.ndarray) -> list:
    """The 32 row residues of one 4096-byte chunk, as the fused decrypt + CRC kernel forms
    them (aes_cbc.hip): lane l holds block 64j + l (chain j); row r = l & 31 and half
    h = l >> 5; step s = 4j + d feeds dword d of that block as four e2m1 operand dwords."""
    words = chunk.view("<u4").reshape(256, 4).astype(np.uint64)
    acc = np.zeros((32, 32))
    for s in range(16):
        j, d = s >> 2, s & 3
        for h in range(2):
            for r in range(32):
                dw = int(words[64 * j + 32 * h + r, d])
                a = _fp4_elements([dw & 0x11111111, dw & 0x22222222, dw & 0x44444444, (dw >> 1) & 0x44444444])
                for col in range(32):
                    b = _fp4_elements(wf[s, col + 32 * h].view("<u4"))
                    acc[r, col] += float((a * b).sum())
    rows = []
    for r in range(32):
        v = 0
        for col in range(32):
            v |= (int(acc[r, col]) & 1) << col
        rows.append(v)
    return rows


def test_fused_chunk_crc_formulation_matches_zlib(rt):
    """The CRC fused into the AES decrypt: per-chunk row residues (host weights from
    crc_chunk_weights_fp4), folded per chunk with the 16-byte shift P_4 (Horner over the 32
    rows), then a Horner over 4096-byte chunks (P_12), the pad removal Q_0..Q_11 and the
    init term -- as crc32_rows_fold + crc32_combine(lg_group=12) compute them."""
    wf = rt.crc_chunk_weights_fp4().reshape(16, 64, 16)
    tab = rt.crc_shift_tables()
    assert rt.CRC_NUM_Q == 12 and len(tab) == (40 + 12) * 1024
    rng = np.random.default_rng(5)
    for n in (16, 4096, 4096 + 48, 2 * 4096 + 4000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        C = (n + 4095) // 4096
        buf = np.zeros(C * 4096, np.uint8)
        buf[:n] = np.frombuffer(data, np.uint8)
        raw = 0
        for c in range(C):
            rows = _chunk_rows(buf[c * 4096:(c + 1) * 4096], wf)
            chunk = 0
            for v in rows:
                chunk = _apply(tab, 4, chunk) ^ v
            raw = _apply(tab, 12, raw) ^ chunk
        pad = C * 4096 - n
        for b in range(12):
            if (pad >> b) & 1:
                raw = _apply(tab, 40 + b, raw)
        init = 0xFFFFFFFF
        for b in range(40):
            if (n >> b) & 1:
                init = _apply(tab, b, init)
        assert raw ^ init ^ 0xFFFFFFFF == zlib.crc32(data), n
