"""M3U8 parsing (master + media playlists) into :mod:`.level` objects.

Covers what the engine needs from RFC 8216: ``EXT-X-STREAM-INF`` (BANDWIDTH,
RESOLUTION, CODECS, NAME), ``EXTINF``, ``EXT-X-TARGETDURATION``,
``EXT-X-MEDIA-SEQUENCE``, ``EXT-X-KEY`` (METHOD/URI/IV), ``EXT-X-BYTERANGE``,
``EXT-X-DISCONTINUITY``, ``EXT-X-ENDLIST``.  Redundant variants (same BANDWIDTH and
resolution) are grouped into one level with several ``url`` entries, as hls.js's level
controller does — each is a separate ``urlId`` track for the peer agent.
"""
from __future__ import annotations

import re
from typing import Dict, List, Optional, Tuple
from urllib.parse import urljoin

from .level import DecryptData, Fragment, Level, LevelDetails

_ATTR = re.compile(r'([A-Z0-9-]+)=("[^"]*"|[^,]*)')


class PlaylistError(Exception):
    pass


def parse_attrs(s: str) -> Dict[str, str]:
    out = {}
    for k, v in _ATTR.findall(s):
        if v.startswith('"') and v.endswith('"'):
            v = v[1:-1]
        out[k] = v
    return out


def is_master(text: str) -> bool:
    return "#EXT-X-STREAM-INF" in text


def parse_master(text: str, base_url: str) -> List[Level]:
    if not text.lstrip().startswith("#EXTM3U"):
        raise PlaylistError("no EXTM3U delimiter")
    levels: List[Level] = []
    by_key: Dict[Tuple[int, int, int], Level] = {}
    lines = [l.strip() for l in text.splitlines()]
    pending: Optional[Dict[str, str]] = None
    for line in lines:
        if not line:
            continue
        if line.startswith("#EXT-X-STREAM-INF:"):
            pending = parse_attrs(line[len("#EXT-X-STREAM-INF:"):])
            continue
        if line.startswith("#"):
            continue
        if pending is not None:
            url = urljoin(base_url, line)
            bw = int(pending.get("BANDWIDTH", "0") or 0)
            w = h = 0
            res = pending.get("RESOLUTION")
            if res and "x" in res:
                w, h = (int(x) for x in res.lower().split("x", 1))
            key = (bw, w, h)
            if key in by_key:
                by_key[key].url.append(url)
            else:
                codecs = pending.get("CODECS", "")
                vc = next((c for c in codecs.split(",") if c.startswith(("avc", "hvc", "hev"))), None)
                ac = next((c for c in codecs.split(",") if c.startswith("mp4a")), None)
                lvl = Level(url=[url], bitrate=bw, width=w, height=h, name=pending.get("NAME", ""),
                            codecs=codecs, audioCodec=ac, videoCodec=vc)
                by_key[key] = lvl
                levels.append(lvl)
            pending = None
    if not levels:
        raise PlaylistError("no levels found in manifest")
    levels.sort(key=lambda l: l.bitrate)
    return levels


def _resolver(base_url: str):
    """``urljoin(base_url, uri)`` memoized per directory part of ``uri``: a playlist's
    segment URIs share a handful of directories, and urljoin (~10 us) ran once per segment
    (a 2 h VOD playlist at 4 s segments: ~1,800 of them)."""
    dirs = {}

    def resolve(uri: str) -> str:
        if "?" in uri or "#" in uri:  # query / fragment: let urljoin handle it
            return urljoin(base_url, uri)
        d, sep, name = uri.rpartition("/")
        r = dirs.get(d)
        if r is None:
            r = urljoin(base_url, d + "/" if sep else "./")
            dirs[d] = r
        return r + name

    return resolve


def parse_media(text: str, base_url: str, level_index: int) -> LevelDetails:
    if not text.lstrip().startswith("#EXTM3U"):
        raise PlaylistError("no EXTM3U delimiter")
    details = LevelDetails(url=base_url)
    sn = 0
    start = 0.0
    cc = 0
    decrypt: Optional[DecryptData] = None
    duration: Optional[float] = None
    title = ""
    byterange: Optional[Tuple[int, int]] = None
    last_br_end = 0
    live = True
    frags: List[Fragment] = []
    resolve = _resolver(base_url)
    for raw in text.splitlines():
        line = raw.strip()
        if not line:
            continue
        if line.startswith("#EXT-X-TARGETDURATION:"):
            details.targetduration = float(line.split(":", 1)[1])
        elif line.startswith("#EXT-X-MEDIA-SEQUENCE:"):
            sn = int(line.split(":", 1)[1])
            details.startSN = sn
        elif line.startswith("#EXT-X-VERSION:"):
            details.version = int(line.split(":", 1)[1])
        elif line.startswith("#EXT-X-ENDLIST"):
            live = False
        elif line.startswith("#EXT-X-PLAYLIST-TYPE:") and line.split(":", 1)[1].strip() == "VOD":
            pass
        elif line.startswith("#EXT-X-DISCONTINUITY"):
            cc += 1
        elif line.startswith("#EXT-X-KEY:"):
            a = parse_attrs(line[len("#EXT-X-KEY:"):])
            method = a.get("METHOD", "NONE")
            if method == "NONE":
                decrypt = None
            else:
                iv = None
                if "IV" in a:
                    hexs = a["IV"][2:] if a["IV"].lower().startswith("0x") else a["IV"]
                    iv = bytes.fromhex(hexs.rjust(32, "0"))
                decrypt = DecryptData(method=method, uri=urljoin(base_url, a.get("URI", "")), iv=iv)
        elif line.startswith("#EXTINF:"):
            body = line[len("#EXTINF:"):]
            dur, _, title = body.partition(",")
            duration = float(dur)
        elif line.startswith("#EXT-X-BYTERANGE:"):
            v = line.split(":", 1)[1]
            length, _, offset = v.partition("@")
            off = int(offset) if offset else last_br_end
            byterange = (off, off + int(length))
            last_br_end = byterange[1]
        elif line.startswith("#"):
            continue
        else:
            if duration is None:
                raise PlaylistError(f"segment without EXTINF: {line}")
            dd = None
            if decrypt is not None:
                dd = DecryptData(method=decrypt.method, uri=decrypt.uri, iv=decrypt.iv)
            f = Fragment(url=resolve(line), sn=sn, start=start, duration=duration, level=level_index,
                         cc=cc, decryptdata=dd, title=title)
            if byterange is not None:
                f.byteRangeStartOffset, f.byteRangeEndOffset = byterange
            frags.append(f)
            start += duration
            sn += 1
            duration = None
            byterange = None
    details.fragments = frags
    details.live = live
    details.endSN = sn - 1
    details.endCC = cc
    details.totalduration = start
    details.averagetargetduration = (start / len(frags)) if frags else details.targetduration
    return details


def write_media_playlist(frags: List[Tuple[str, float]], target: int, media_sequence: int = 0,
                         endlist: bool = True, key_line: Optional[str] = None) -> str:
    """Small writer used by tests/examples for hand-made playlists."""
    out = ["#EXTM3U", "#EXT-X-VERSION:3", f"#EXT-X-TARGETDURATION:{target}",
           f"#EXT-X-MEDIA-SEQUENCE:{media_sequence}"]
    if key_line:
        out.append(key_line)
    for uri, dur in frags:
        out.append(f"#EXTINF:{dur:.3f},")
        out.append(uri)
    if endlist:
        out.append("#EXT-X-ENDLIST")
    return "\n".join(out) + "\n"
