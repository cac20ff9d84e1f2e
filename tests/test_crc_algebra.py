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
