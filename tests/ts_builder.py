"""An independent MPEG-TS builder for demux tests (ISO/IEC 13818-1), written from the spec --
not from the framework's muxer (``runtime/ts.cpp``) -- with the stream features real HLS
segments carry that the synthetic packager never emits:

* a PAT listing the network PID (program 0) before the program, a PMT with program-info and
  ES-info descriptors, a separate PCR PID carrying adaptation-only packets with a PCR;
* adaptation fields with a PCR (and stuffing) in payload packets, null packets (PID 0x1FFF)
  and SDT packets (PID 0x11) interleaved, continuity counters per PID;
* H.264 video PES with PTS + DTS and ``PES_packet_length`` 0, AAC audio PES with PTS only and
  a real length, an ID3 (timed metadata, stream type 0x15) PES, and PES headers carrying
  extra optional fields beyond PTS/DTS (``PES_header_data_length`` > 10 with stuffing bytes).

:func:`build` returns the stream and its ground truth: per class the exact elementary-stream
bytes (every PES payload back to back) and the ``(es_offset, pts, dts)`` of each PES, which
is what the demux must recover (``ops/tsdemux.py`` output format).
"""
from __future__ import annotations

import numpy as np

PACKET = 188
CLASSES = ("video", "audio", "id3")


def _crc32_mpeg(data: bytes) -> int:
    crc = 0xFFFFFFFF
    for b in data:
        crc ^= b << 24
        for _ in range(8):
            crc = ((crc << 1) ^ 0x04C11DB7) & 0xFFFFFFFF if crc & 0x80000000 else (crc << 1) & 0xFFFFFFFF
    return crc


def _section(table_id: int, ext: int, body: bytes) -> bytes:
    """A PSI section with the syntax indicator set and its CRC_32."""
    length = 5 + len(body) + 4  # ext(2) version(1) sec(1) last(1) + body + crc
    head = bytes([table_id, 0xB0 | ((length >> 8) & 0x0F), length & 0xFF, ext >> 8, ext & 0xFF, 0xC1, 0x00, 0x00])
    sec = head + body
    return sec + _crc32_mpeg(sec).to_bytes(4, "big")


def _ts_timestamp(prefix: int, t: int) -> bytes:
    t &= (1 << 33) - 1
    return bytes([(prefix << 4) | (((t >> 30) & 0x07) << 1) | 1, (t >> 22) & 0xFF, (((t >> 15) & 0x7F) << 1) | 1,
                  (t >> 7) & 0xFF, ((t & 0x7F) << 1) | 1])


def _pes(stream_id: int, payload: bytes, pts: int, dts: int = -1, length_field: bool = True,
         extra_header: int = 0) -> bytes:
    flags = 0x80 if dts < 0 else 0xC0
    opt = _ts_timestamp(0x3 if dts >= 0 else 0x2, pts) + (_ts_timestamp(0x1, dts) if dts >= 0 else b"")
    opt += b"\xff" * extra_header  # stuffing bytes in the optional header (allowed, 2.4.3.7)
    header = bytes([0x80, flags, len(opt)]) + opt
    n = len(header) + len(payload)
    plen = n if (length_field and n <= 0xFFFF) else 0
    return b"\x00\x00\x01" + bytes([stream_id, plen >> 8, plen & 0xFF]) + header + payload


def _pcr_bytes(pcr: int) -> bytes:
    base, ext = (pcr // 300) & ((1 << 33) - 1), pcr % 300
    return bytes([(base >> 25) & 0xFF, (base >> 17) & 0xFF, (base >> 9) & 0xFF, (base >> 1) & 0xFF,
                  ((base & 1) << 7) | 0x7E | ((ext >> 8) & 1), ext & 0xFF])


class _Muxer:
    def __init__(self) -> None:
        self.packets: list = []
        self.cc: dict = {}

    def _cc(self, pid: int) -> int:
        c = self.cc.get(pid, 0)
        self.cc[pid] = (c + 1) & 0x0F
        return c

    def packet(self, pid: int, payload: bytes, pusi: bool, pcr: int = -1) -> int:
        """One packet with as much of ``payload`` as fits; an adaptation field carries the PCR
        (``pcr`` >= 0, in 27 MHz units) and/or the stuffing that pads a short tail (2.4.3.4).
        Returns the payload bytes consumed."""
        fields = b"" if pcr < 0 else bytes([0x10]) + _pcr_bytes(pcr)  # flags: PCR_flag
        room = PACKET - 4 - (1 + len(fields) if fields else 0)
        take = min(room, len(payload))
        if fields or take < PACKET - 4:
            length = PACKET - 4 - 1 - take  # adaptation_field_length
            if length and not fields:
                fields = b"\x00"  # flags byte, nothing set
            af = bytes([length]) + fields + b"\xff" * (length - len(fields))
            afc = 0x30
        else:
            af, afc = b"", 0x10
        pkt = bytes([0x47, (0x40 if pusi else 0) | ((pid >> 8) & 0x1F), pid & 0xFF, afc | self._cc(pid)]) \
            + af + payload[:take]
        assert len(pkt) == PACKET, len(pkt)
        self.packets.append(pkt)
        return take

    def adaptation_only(self, pid: int, pcr: int) -> None:
        """A packet with no payload (adaptation_field_control '10'), as a PCR-only PID sends."""
        fields = bytes([0x10]) + _pcr_bytes(pcr)
        af = bytes([PACKET - 5]) + fields + b"\xff" * (PACKET - 5 - len(fields))
        self.packets.append(bytes([0x47, (pid >> 8) & 0x1F, pid & 0xFF, 0x20 | self._cc(pid)]) + af)

    def psi(self, pid: int, section: bytes) -> None:
        self.packet(pid, b"\x00" + section, True)  # pointer_field 0

    def pes(self, pid: int, data: bytes, pcr: int = -1) -> None:
        first = True
        while data:
            took = self.packet(pid, data, first, pcr if first else -1)
            data = data[took:]
            first = False


def build(seed: int = 0, n_video: int = 12, n_audio: int = 20, with_id3: bool = True, video_type: int = 0x1B):
    """A segment with the features listed in the module docstring.  Returns ``(stream bytes,
    truth)``; ``truth[cls] = {"es": bytes, "pes": [(es_offset, pts, dts), ...], "pid": int}``
    and ``truth["pmt_pid"]``, ``truth["video_type"]``, ``truth["audio_type"]``."""
    rng = np.random.default_rng(seed)
    VPID, APID, IPID, PCRPID, PMTPID, SDTPID = 0x100, 0x101, 0x102, 0x1F0, 0x1000, 0x11
    m = _Muxer()
    # PAT: program 0 -> network PID 0x10, then program 1 -> the PMT
    pat = _section(0x00, 1, bytes([0, 0, 0xE0, 0x10, 0, 1, 0xE0 | (PMTPID >> 8), PMTPID & 0xFF]))
    m.psi(0, pat)
    # PMT: PCR PID, a program-info descriptor, then video / audio / id3 each with a descriptor
    pinfo = bytes([0x05, 0x04]) + b"HDMV"  # registration descriptor

    def desc(tag: int, body: bytes) -> bytes:
        return bytes([tag, len(body)]) + body

    streams = b""
    for st, pid, d in ((video_type, VPID, desc(0x28, bytes([0x64, 0x00, 0x28, 0x3F]))),  # AVC video descriptor
                       (0x0F, APID, desc(0x0A, b"eng\x00")),  # ISO 639 language
                       (0x15, IPID, desc(0x26, b"\xff\xffID3 \xffID3 \x00\x0f"))):  # metadata descriptor
        if st == 0x15 and not with_id3:
            continue
        streams += bytes([st, 0xE0 | (pid >> 8), pid & 0xFF, 0xF0 | (len(d) >> 8), len(d) & 0xFF]) + d
    body = bytes([0xE0 | (PCRPID >> 8), PCRPID & 0xFF, 0xF0 | (len(pinfo) >> 8), len(pinfo) & 0xFF]) + pinfo + streams
    pmt = _section(0x02, 1, body)
    m.psi(PMTPID, pmt)
    m.psi(SDTPID, _section(0x42, 1, bytes([0xFF, 0x01, 0xFF, 0x00, 0x01, 0xFC, 0x80, 0x00])))
    truth = {c: {"es": b"", "pes": [], "pid": p} for c, p in zip(CLASSES, (VPID, APID, IPID if with_id3 else -1))}
    truth.update(pmt_pid=PMTPID, video_type=video_type, audio_type=0x0F)
    events = []  # (time, class, payload, pts, dts)
    t0 = 900_000 + int(rng.integers(0, 1 << 20))
    for i in range(n_video):
        size = int(rng.integers(900, 6000)) if i else int(rng.integers(15000, 30000))  # a big first frame
        pts = t0 + i * 3600 + 7200
        dts = -1 if i % 3 == 2 else pts - 3600  # some frames carry PTS only (DTS == PTS)
        events.append((pts - 7200, "video", rng.integers(0, 256, size, dtype=np.uint8).tobytes(), pts, dts))
    for i in range(n_audio):
        size = int(rng.integers(200, 700))
        pts = t0 + i * 1920
        events.append((pts, "audio", rng.integers(0, 256, size, dtype=np.uint8).tobytes(), pts, -1))
    if with_id3:
        for i in range(2):
            pts = t0 + i * 90_000
            events.append((pts, "id3", b"ID3\x04\x00\x00\x00\x00\x00\x0f" + rng.integers(0, 256, 15, dtype=np.uint8)
                           .tobytes(), pts, -1))
    events.sort(key=lambda e: (e[0], CLASSES.index(e[1])))
    for k, (t, cls, payload, pts, dts) in enumerate(events):
        if k == len(events) // 2:  # PSI repeats mid-segment, as muxers send it every ~100 ms
            m.psi(0, pat)
            m.psi(PMTPID, pmt)
        if k % 5 == 0:
            m.adaptation_only(PCRPID, (t - 1000) * 300)  # PCR on its own PID
        if k % 7 == 3:
            m.packets.append(bytes([0x47, 0x1F, 0xFF, 0x10]) + b"\xff" * 184)  # null packet
        pid = truth[cls]["pid"]
        sid = {"video": 0xE0, "audio": 0xC0, "id3": 0xBD}[cls]
        extra = 3 if (cls == "video" and k % 4 == 1) else 0
        pes = _pes(sid, payload, pts, dts, length_field=cls != "video", extra_header=extra)
        tr = truth[cls]
        tr["pes"].append((len(tr["es"]), pts, dts))
        tr["es"] += payload
        m.pes(pid, pes, pcr=(t * 300) if (cls == "video" and k % 3 == 0) else -1)
    return b"".join(m.packets), truth
