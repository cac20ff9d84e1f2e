"""Synthetic HLS origin ("CDN"): packager + server for multi-rendition streams.

The reference's tests play a public HLS stream from a real CDN
(``test/html/bundle.js:20-26``) and fetch a 245,528-byte fragment
(``test/html/p2p-loader-generator.js:82``).  There is no network here, so the CDN is an
in-process origin that *packages* a real HLS stream:

* master playlist with ``#EXT-X-STREAM-INF`` per rendition, optionally repeated per
  redundant (backup) URL tree so levels have several ``url[]`` entries → several
  ``urlId`` tracks (``lib/integration/mapping/media-map.js:60-73``);
* media playlists, VOD (``#EXT-X-ENDLIST``) or live sliding window advancing with the
  event-loop clock (``#EXT-X-MEDIA-SEQUENCE``);
* MPEG-TS segments from the native muxer, optionally AES-128-CBC encrypted
  (``#EXT-X-KEY:METHOD=AES-128,URI=...,IV=...``);
* segment bytes held in **pinned host memory** (one tensor per rendition), so the GPU
  node's CDN path is a single ``hipMemcpyAsync`` H2D on a side stream.

Segments come from a pool of ``pool_size`` distinct packaged segments per rendition
(``sn % pool_size``) so long streams do not need gigabytes of host RAM; all pool entries
share one key/IV so any sn decrypts with the playlist's ``IV`` attribute.
Fault injection: :meth:`fail` (HTTP status for matching paths) and :meth:`corrupt`.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import math
import re
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..ops import aes as _aes
from ..ops import tsdemux as _ts
from .http import HttpError, Response, register_origin


@dataclass
class Rendition:
    bandwidth: int                   # bit/s (EXT-X-STREAM-INF BANDWIDTH)
    width: int = 1920
    height: int = 1080
    fps: float = 25.0
    audio_kbps: int = 128
    codecs: str = "avc1.640028,mp4a.40.2"
    name: str = ""

    def segment_bytes(self, duration: float) -> int:
        return int(self.bandwidth * duration / 8)


PRESET_1080P_6M = [Rendition(6_000_000, 1920, 1080, name="1080p")]
PRESET_4K_25M = [Rendition(25_000_000, 3840, 2160, fps=50.0, name="2160p")]
PRESET_ABR5 = [
    Rendition(800_000, 640, 360, name="360p"),
    Rendition(1_600_000, 960, 540, name="540p"),
    Rendition(3_000_000, 1280, 720, name="720p"),
    Rendition(6_000_000, 1920, 1080, name="1080p"),
    Rendition(8_000_000, 1920, 1080, fps=50.0, name="1080p50"),
]


def _seg_path(path: str) -> Optional[Tuple[int, int]]:
    """``(level, sn)`` of a canonical segment path ``[<a-h>/]r<level>/seg<sn>.ts`` without a
    regex (one parse per fragment on the node's request path); None: use the regex."""
    if not path.endswith(".ts"):
        return None
    slash = path.rfind("/")
    if slash <= 0:
        return None
    name = path[slash + 1:-3]
    start = path.rfind("/", 0, slash) + 1
    lvl = path[start:slash]
    if (name[:3] != "seg" or lvl[:1] != "r" or not name[3:].isdecimal() or not lvl[1:].isdecimal()
            or not (start == 0 or (start == 2 and path[0] in "abcdefgh"))):
        return None
    return int(lvl[1:]), int(name[3:])


@dataclass
class _Pool:
    data: torch.Tensor              # pinned uint8
    offsets: List[int]
    lengths: List[int]
    crcs: List[int] = field(default_factory=list)


class SyntheticHlsOrigin:
    def __init__(self, base_url: str = "http://origin.test/live/", renditions: Sequence[Rendition] = (),
                 segment_duration: float = 4.0, num_segments: Optional[int] = 10, live: bool = False,
                 window: int = 6, encrypted: bool = False, pool_size: Optional[int] = None, redundant: int = 1,
                 seed: int = 1, with_id3: bool = False, start_sn: int = 0, pin_memory: Optional[bool] = None,
                 loop=None, register: bool = True, live_speed: float = 1.0,
                 live_epoch: Optional[float] = None) -> None:
        self.base_url = base_url if base_url.endswith("/") else base_url + "/"
        self.renditions = list(renditions) or list(PRESET_1080P_6M)
        self.segment_duration = float(segment_duration)
        self.live = live
        self.num_segments = num_segments
        self.window = window
        self.encrypted = encrypted
        self.redundant = max(1, int(redundant))
        self.seed = seed
        self.with_id3 = with_id3
        self.start_sn = start_sn
        self.live_speed = live_speed
        # live edge from the wall clock (time.time() at which the window was full): every
        # process serving or playing the channel agrees on it without sharing a loop
        self.live_epoch = live_epoch
        self._paths: Dict[str, Tuple[int, int]] = {}  # segment path -> (level, sn)
        if pool_size is None:
            pool_size = num_segments if (num_segments is not None and not live) else 16
        self.pool_size = max(1, int(pool_size))
        if pin_memory is None:
            pin_memory = torch.cuda.is_available()
        self.pin_memory = pin_memory
        self.loop = loop
        self._t0 = loop.now() if loop is not None else 0.0
        self._manual_edge: Optional[int] = None
        h = hashlib.sha256(f"{self.base_url}/{seed}".encode()).digest()
        self.key = h[:16]
        self.iv = h[16:32]
        self.requests: List[str] = []
        self._failures: List[Tuple[re.Pattern, int, int]] = []  # (pattern, status, remaining)
        self._corrupt: List[Tuple[re.Pattern, int]] = []
        self._lock = threading.Lock()
        self.pools: List[_Pool] = [self._package(r, i) for i, r in enumerate(self.renditions)]
        if register:
            register_origin(self.base_url, self)

    # ---------------------------------------------------------------- packaging
    def _package(self, rend: Rendition, level: int) -> _Pool:
        seg_bytes = rend.segment_bytes(self.segment_duration)

        def make(i: int) -> np.ndarray:
            seg, _ = _ts.mux_segment(self.segment_duration, rend.fps, seg_bytes, rend.audio_kbps, self.with_id3,
                                     self.seed * 1000 + level, i, self.segment_duration * i)
            if self.encrypted:
                seg = _aes.cbc_encrypt(self.key, self.iv, seg)
            return seg

        with cf.ThreadPoolExecutor(max_workers=8) as ex:
            segs = list(ex.map(make, range(self.pool_size)))
        offsets, lengths, pos = [], [], 0
        for s in segs:
            offsets.append(pos)
            lengths.append(len(s))
            pos += (len(s) + 255) // 256 * 256
        data = torch.empty(max(pos, 256), dtype=torch.uint8, pin_memory=self.pin_memory)
        dv = data.numpy()
        for o, s in zip(offsets, segs):
            dv[o:o + len(s)] = s
        from ..ops import crc as _crc

        crcs = [_crc.crc32(dv[o:o + n]) for o, n in zip(offsets, lengths)]
        return _Pool(data, offsets, lengths, crcs)

    # ---------------------------------------------------------------- live edge
    def live_edge(self) -> int:
        """Highest available sn."""
        if not self.live:
            return self.start_sn + (self.num_segments or 0) - 1
        if self._manual_edge is not None:
            return self._manual_edge
        if self.live_epoch is not None:
            produced = int(max(0.0, time.time() - self.live_epoch) * self.live_speed / self.segment_duration)
            return self.start_sn + self.window - 1 + produced
        now = self.loop.now() if self.loop is not None else 0.0
        produced = int(((now - self._t0) / 1000.0) * self.live_speed / self.segment_duration)
        return self.start_sn + self.window - 1 + produced

    def advance(self, n: int = 1) -> None:
        """Manually publish ``n`` more live segments (tests / benches)."""
        if self._manual_edge is None:
            self._manual_edge = self.live_edge()
        self._manual_edge += n

    def first_sn(self) -> int:
        if not self.live:
            return self.start_sn
        return max(self.start_sn, self.live_edge() - self.window + 1)

    # ---------------------------------------------------------------- playlists
    def master_url(self) -> str:
        return self.base_url + "master.m3u8"

    def level_path(self, level: int, url_id: int = 0) -> str:
        return f"{'abcdefgh'[url_id]}/r{level}/index.m3u8"

    def segment_path(self, level: int, sn: int) -> str:
        return f"r{level}/seg{sn}.ts"

    def master_playlist(self) -> str:
        lines = ["#EXTM3U"]
        for u in range(self.redundant):
            for i, r in enumerate(self.renditions):
                lines.append(f'#EXT-X-STREAM-INF:PROGRAM-ID=1,BANDWIDTH={r.bandwidth},RESOLUTION={r.width}x{r.height},'
                             f'CODECS="{r.codecs}",NAME="{r.name or i}"')
                lines.append(self.level_path(i, u))
        return "\n".join(lines) + "\n"

    def media_playlist(self, level: int) -> str:
        first = self.first_sn()
        last = self.live_edge()
        td = int(math.ceil(self.segment_duration))
        lines = ["#EXTM3U", "#EXT-X-VERSION:3", f"#EXT-X-TARGETDURATION:{td}", f"#EXT-X-MEDIA-SEQUENCE:{first}"]
        if not self.live:
            lines.append("#EXT-X-PLAYLIST-TYPE:VOD")
        if self.encrypted:
            lines.append(f'#EXT-X-KEY:METHOD=AES-128,URI="../../key.bin",IV=0x{self.iv.hex()}')
        for sn in range(first, last + 1):
            lines.append(f"#EXTINF:{self.segment_duration:.3f},")
            lines.append(f"../../{self.segment_path(level, sn)}")
        if not self.live:
            lines.append("#EXT-X-ENDLIST")
        return "\n".join(lines) + "\n"

    # ---------------------------------------------------------------- faults
    def fail(self, pattern: str, status: int = 404, times: int = -1) -> None:
        with self._lock:
            self._failures.append((re.compile(pattern), status, times))

    def corrupt(self, pattern: str, times: int = -1) -> None:
        with self._lock:
            self._corrupt.append((re.compile(pattern), times))

    def clear_faults(self) -> None:
        with self._lock:
            self._failures.clear()
            self._corrupt.clear()

    def _check_fail(self, path: str) -> None:
        if not self._failures:  # the common case, per request: no lock
            return
        with self._lock:
            for i, (rx, status, times) in enumerate(self._failures):
                if rx.search(path):
                    if times == 0:
                        continue
                    if times > 0:
                        self._failures[i] = (rx, status, times - 1)
                    raise HttpError(status, path)

    def should_corrupt(self, path: str) -> bool:
        if not self._corrupt:
            return False
        with self._lock:
            for i, (rx, times) in enumerate(self._corrupt):
                if rx.search(path) and times != 0:
                    if times > 0:
                        self._corrupt[i] = (rx, times - 1)
                    return True
        return False

    # ---------------------------------------------------------------- serving
    _SEG = re.compile(r"(?:[a-h]/)?r(\d+)/seg(\d+)\.ts$")
    _LVL = re.compile(r"(?:[a-h]/)?r(\d+)/index\.m3u8$")

    def resource(self, path: str) -> Tuple[torch.Tensor, int, int, int]:
        """(pinned tensor, offset, length, crc) of a segment, for zero-copy device fetches."""
        ls = self._paths.get(path)
        if ls is None:  # parse once per path (each is resolved at request and at fetch time)
            ls = _seg_path(path)
            if ls is None:
                m = self._SEG.search(path)
                if not m:
                    raise HttpError(404, path)
                ls = (int(m.group(1)), int(m.group(2)))
            if len(self._paths) > 65536:
                self._paths.clear()
            self._paths[path] = ls
        level, sn = ls
        if level >= len(self.pools):
            raise HttpError(404, path)
        if self.live:
            if sn < self.first_sn() - self.window or sn > self.live_edge() or sn < self.start_sn:
                raise HttpError(404, path)
        elif sn < self.start_sn or sn >= self.start_sn + (self.num_segments or 0):
            raise HttpError(404, path)
        pool = self.pools[level]
        i = sn % self.pool_size
        return pool.data, pool.offsets[i], pool.lengths[i], pool.crcs[i]

    def segment_dirs(self) -> Optional[List[Tuple[str, str, str, int, int, torch.Tensor, List[int], List[int]]]]:
        """Where every segment's bytes live, per URL directory, for the swarm node's native
        batch locator (``runtime/locator.cpp``): ``(directory URL, name prefix, name suffix,
        first sn, end sn, pool tensor, slot offsets, slot lengths)``; the slot of ``sn`` is
        ``sn % pool_size``.  None when the bytes are not fixed per URL: a live window, or
        injected failures / corruption (those go through :meth:`locate` per request)."""
        if self.live or self._failures or self._corrupt or self.num_segments is None:
            return None
        out = []
        trees = [""] + [f"{c}/" for c in "abcdefgh"[:self.redundant]]
        for level, pool in enumerate(self.pools):
            offs, lens = list(pool.offsets[:self.pool_size]), list(pool.lengths[:self.pool_size])
            for t in trees:
                out.append((f"{self.base_url}{t}r{level}/", "seg", ".ts", self.start_sn,
                            self.start_sn + self.num_segments, pool.data, offs, lens))
        return out

    def locate(self, path: str, url: str = "", rng=None) -> Optional[Tuple[torch.Tensor, int, int]]:
        """``(pinned tensor, offset, length)`` of a segment's (ranged) bytes, resolved once
        when the node creates the want: a VOD origin's pools never change, so the CDN phase
        reuses it.  None for a live origin (its window moves: resolved again at fetch time)
        and for non-segment paths.
        Raises like :meth:`size`."""
        if self.live or not path.endswith(".ts"):
            return None
        self._check_fail(path)
        data, off, n, _ = self.resource(path)
        if rng is not None:
            s, e = rng
            e = n - 1 if e is None else min(e, n - 1)
            off, n = off + s, max(0, e - s + 1)
        return data, off, n

    def size(self, path: str, url: str = "", rng=None) -> int:
        self._check_fail(path)
        if path.endswith(".ts"):
            _, _, n, _ = self.resource(path)
        else:
            n = len(self._text(path).encode())
        if rng is not None:
            s, e = rng
            e = n - 1 if e is None else min(e, n - 1)
            return max(0, e - s + 1)
        return n

    def _text(self, path: str) -> str:
        if path.endswith("master.m3u8"):
            return self.master_playlist()
        m = self._LVL.search(path)
        if m:
            level = int(m.group(1))
            if level >= len(self.renditions):
                raise HttpError(404, path)
            return self.media_playlist(level)
        raise HttpError(404, path)

    def serve(self, path: str, url: str, rng, headers: Dict[str, str], with_credentials: bool) -> Response:
        with self._lock:
            self.requests.append(path)
        self._check_fail(path)
        if path.endswith("key.bin"):
            return Response(200, self.key, url, 16)
        if path.endswith(".ts"):
            data, off, n, _ = self.resource(path)
            start, end = 0, n - 1
            status = 200
            if rng is not None:
                start, e = rng
                end = n - 1 if e is None else min(e, n - 1)
                if start >= n or end < start:
                    raise HttpError(416, url)
                status = 206
            body = data[off + start:off + end + 1]
            if self.should_corrupt(path):
                body = body.clone()
                body[len(body) // 2] ^= 0xFF
            return Response(status, body, url, end - start + 1, source=(data, off + start), offset=start)
        text = self._text(path)
        return Response(200, text, url, len(text.encode()))


class StaticOrigin:
    """Serves fixed resources (``path -> bytes/str``) — for tests and hand-made streams."""

    def __init__(self, base_url: str, resources: Optional[Dict[str, object]] = None, register: bool = True,
                 pin_memory: bool = False) -> None:
        self.base_url = base_url if base_url.endswith("/") else base_url + "/"
        self.requests: List[str] = []
        self._res: Dict[str, object] = {}
        self.pin_memory = pin_memory
        for k, v in (resources or {}).items():
            self.put(k, v)
        self._failures: List[Tuple[re.Pattern, int, int]] = []
        if register:
            register_origin(self.base_url, self)

    def put(self, path: str, value) -> None:
        if isinstance(value, (bytes, bytearray, np.ndarray)):
            arr = np.frombuffer(bytes(value), dtype=np.uint8) if not isinstance(value, np.ndarray) else value
            t = torch.empty(max(len(arr), 1), dtype=torch.uint8, pin_memory=self.pin_memory)
            t[:len(arr)] = torch.from_numpy(np.ascontiguousarray(arr))
            self._res[path] = (t, len(arr))
        else:
            self._res[path] = str(value)

    def fail(self, pattern: str, status: int = 404, times: int = -1) -> None:
        self._failures.append((re.compile(pattern), status, times))

    def should_corrupt(self, path: str) -> bool:
        return False

    def _check(self, path: str) -> None:
        for i, (rx, status, times) in enumerate(self._failures):
            if rx.search(path) and times != 0:
                if times > 0:
                    self._failures[i] = (rx, status, times - 1)
                raise HttpError(status, path)
        if path not in self._res:
            raise HttpError(404, path)

    def resource(self, path: str):
        self._check(path)
        v = self._res[path]
        if isinstance(v, str):
            raise HttpError(415, path)
        t, n = v
        return t, 0, n, 0

    def size(self, path: str, url: str = "", rng=None) -> int:
        self._check(path)
        v = self._res[path]
        n = len(v.encode()) if isinstance(v, str) else v[1]
        if rng is not None:
            s, e = rng
            e = n - 1 if e is None else min(e, n - 1)
            return max(0, e - s + 1)
        return n

    def serve(self, path: str, url: str, rng, headers, with_credentials) -> Response:
        self.requests.append(path)
        self._check(path)
        v = self._res[path]
        if isinstance(v, str):
            return Response(200, v, url, len(v.encode()))
        t, n = v
        start, end, status = 0, n - 1, 200
        if rng is not None:
            start, e = rng
            end = n - 1 if e is None else min(e, n - 1)
            status = 206
        return Response(status, t[start:end + 1], url, end - start + 1, source=(t, start), offset=start)
