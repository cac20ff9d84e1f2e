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


def _planes(dw: int):
    return [dw & 0x11111111, dw & 0x22222222, dw & 0x44444444, (dw >> 1) & 0x44444444]


def _chunk_masks(chunk: np.ndarray, wa: np.ndarray) -> np.ndarray:
    """The decrypt side (aes_cbc.hip: crc_chunk_masks): lane l holds block 64j + l (chain j);
    chains 2p and 2p + 1 share accumulator set p, step (j & 1, d) feeding dword d of the
    lane's block against the pair-independent B fragments wa[4 (j & 1) + d]; the accumulators
    start at 2^23 (the mantissa LSB is then the parity) and lane l's 16 parities of set p go to
    bits 16 p + i of its mask dword (i = row (i & 3) + 8 (i >> 2) + 4 (l >> 5), column l & 31)."""
    words = chunk.view("<u4").reshape(256, 4).astype(np.uint64)
    b = np.stack([[_fp4_elements(wa[st, lane].view("<u4")) for lane in range(64)] for st in range(8)])
    masks = np.zeros(64, np.uint32)
    for p in range(2):
        acc = np.full((32, 32), 2.0 ** 23, dtype=np.float32)  # [row][col], f32 as the MFMA accumulates
        for jj in range(2):
            j = 2 * p + jj
            for d in range(4):
                for h in range(2):
                    for r in range(32):
                        a = _fp4_elements(_planes(int(words[64 * j + 32 * h + r, d])))
                        acc[r] += np.float32(b[4 * jj + d, 32 * h:32 * h + 32] @ a)
        bits = acc.view(np.uint32) & 1
        assert np.array_equal(bits, (acc.astype(np.int64) - 2 ** 23) & 1)
        for lane in range(64):
            for i in range(16):
                row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5)
                masks[lane] |= int(bits[row, lane & 31]) << (16 * p + i)
    return masks


def _fold(masks: np.ndarray, wf: np.ndarray) -> int:
    """The fold side (crc32_mfma.hip: fold_tile in crc32_fold_combine_kernel): A = host fragments (row = CRC
    bit), B = the chunk's mask dwords (k half hh of step s reads dword s + 32 hh)."""
    acc = np.zeros(32)
    for s in range(32):
        for hh in range(2):
            x = _fp4_elements(_planes(int(masks[s + 32 * hh])))
            for row in range(32):
                acc[row] += float(_fp4_elements(wf[s, row + 32 * hh].view("<u4")) @ x)
    assert np.all(acc == np.round(acc)) and acc.max() <= 2048
    return sum((int(acc[r]) & 1) << r for r in range(32))


def test_fused_chunk_crc_formulation_matches_zlib(rt):
    """The CRC fused into the AES decrypt, two MFMA levels: row parities per chain pair in the
    decrypt (8 pair-independent weight steps), a [32 x 2048] x [2048 x chunks] GF(2) GEMM
    per chunk in the fold, then a Horner over 4096-byte chunks (P_12), the pad removal
    Q_0..Q_11 and the init term -- as crc32_fold_combine_kernel (fold_tile + combine_segment<12>) does."""
    na, nf = rt.CRC_FUSED_AES_STEPS, rt.CRC_FUSED_FOLD_STEPS
    w = rt.crc_chunk_weights_fp4().reshape(na + nf, 64, 16)
    wa, wf = w[:na], w[na:]
    tab = rt.crc_shift_tables()
    assert rt.CRC_NUM_Q == 12 and len(tab) == (40 + 12) * 1024 and rt.CRC_FUSED_MASK_DWORDS == 64
    rng = np.random.default_rng(5)
    for n in (16, 4096 + 48, 2 * 4096 + 4000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        C = (n + 4095) // 4096
        buf = np.zeros(C * 4096, np.uint8)
        buf[:n] = np.frombuffer(data, np.uint8)
        if n == 16:
            buf[:16] = 0xFF  # every nibble bit set: the largest counts
            data = bytes(buf[:16])
        raw = 0
        for c in range(C):
            chunk = buf[c * 4096:(c + 1) * 4096]
            res = _fold(_chunk_masks(chunk, wa), wf)
            assert res == (~zlib.crc32(chunk.tobytes(), 0xFFFFFFFF)) & 0xFFFFFFFF  # zero-init register
            raw = _apply(tab, 12, raw) ^ res
        pad = C * 4096 - n
        for b in range(12):
            if (pad >> b) & 1:
                raw = _apply(tab, 40 + b, raw)
        init = 0xFFFFFFFF
        for b in range(40):
            if (n >> b) & 1:
                init = _apply(tab, b, init)
        assert raw ^ init ^ 0xFFFFFFFF == zlib.crc32(data), n
