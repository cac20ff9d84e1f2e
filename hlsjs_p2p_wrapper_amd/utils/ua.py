"""Tiny user-agent parser for the bundle's capability gate (component C2).

The reference parses the UA once at module load with ua-parser-js
(``lib/hlsjs-p2p-bundle.js:7``) and refuses Safari and mobile/tablet/console devices
(``:49-60``).  A server-side MI355X peer has no browser, so the "user agent" is whatever
the embedding application declares: ``HLSJS_P2P_USER_AGENT`` in the environment, or
:func:`set_user_agent`.  The default describes this runtime (desktop Linux, a
Chrome-compatible engine), which is supported.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from typing import Optional

DEFAULT_UA = ("Mozilla/5.0 (X11; Linux x86_64) AppleWebKit/537.36 (KHTML, like Gecko) "
              "Chrome/120.0 Safari/537.36 hlsjs-p2p-wrapper-amd/MI355X")


@dataclass
class UAResult:
    ua: str
    browser: dict = field(default_factory=dict)
    os: dict = field(default_factory=dict)
    device: dict = field(default_factory=dict)


_BROWSERS = [
    ("Edge", re.compile(r"Edge?/([\d.]+)")),
    ("Opera", re.compile(r"OPR/([\d.]+)")),
    ("Firefox", re.compile(r"Firefox/([\d.]+)")),
    ("Chromium", re.compile(r"Chromium/([\d.]+)")),
    ("Chrome", re.compile(r"(?:Chrome|CriOS)/([\d.]+)")),
    ("Safari", re.compile(r"Version/([\d.]+).*Safari/")),
    ("IE", re.compile(r"(?:MSIE |Trident/.*rv:)([\d.]+)")),
]


def parse_user_agent(ua: str) -> UAResult:
    res = UAResult(ua=ua)
    for name, rx in _BROWSERS:
        m = rx.search(ua)
        if m:
            res.browser = {"name": name, "version": m.group(1)}
            break
    if re.search(r"Android", ua):
        res.os = {"name": "Android"}
    elif re.search(r"iPhone|iPad|iPod", ua):
        res.os = {"name": "iOS"}
    elif re.search(r"Mac OS X", ua):
        res.os = {"name": "Mac OS"}
    elif re.search(r"Windows", ua):
        res.os = {"name": "Windows"}
    elif re.search(r"Linux", ua):
        res.os = {"name": "Linux"}
    if re.search(r"iPad|Tablet", ua):
        res.device = {"type": "tablet"}
    elif re.search(r"Mobi|iPhone|iPod|Android.*Mobile", ua):
        res.device = {"type": "mobile"}
    elif re.search(r"PlayStation|Xbox|Nintendo", ua):
        res.device = {"type": "console"}
    return res


_override: Optional[str] = None


def set_user_agent(ua: Optional[str]) -> None:
    global _override
    _override = ua


def current_user_agent() -> UAResult:
    ua = _override or os.environ.get("HLSJS_P2P_USER_AGENT") or DEFAULT_UA
    return parse_user_agent(ua)


def is_safari(res: UAResult) -> bool:
    return res.browser.get("name") == "Safari"


def is_mobile(res: UAResult) -> bool:
    return (res.device.get("type") in ("mobile", "tablet", "console")
            or res.os.get("name") in ("Android", "iOS"))
