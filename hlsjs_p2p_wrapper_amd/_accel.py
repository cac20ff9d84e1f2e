"""Import guard for the Cython-compiled host modules (``ops/build.py: build_accel``).

CPython prefers an extension module over a same-named ``.py``.  A compiled module built
from an older source would therefore silently shadow edits.  This finder, installed
before any submodule is imported, checks each compiled module's recorded source SHA-1
(``_accel.json``).  For a changed source it loads the ``.py`` instead, so correctness
never depends on remembering to rebuild.  ``HLSJS_P2P_PURE=1`` forces pure Python for
all of them.
"""
from __future__ import annotations

import hashlib
import importlib.machinery
import importlib.util
import json
import os
import sys
from pathlib import Path

_PKG_DIR = Path(__file__).resolve().parent
_PKG = __name__.rsplit(".", 1)[0]


def _load_manifest() -> dict:
    try:
        return json.loads((_PKG_DIR / "_accel.json").read_text())
    except (OSError, ValueError):
        return {}


class _SourceFallbackFinder:
    """Route stale (or, with HLSJS_P2P_PURE=1, all) compiled modules to their source."""

    def __init__(self, pure: bool, manifest: dict) -> None:
        self.pure = pure
        self.manifest = manifest
        self.fallback: set = set()
        for rel, digest in manifest.items():
            src = _PKG_DIR / rel
            mod = f"{_PKG}." + rel[:-3].replace("/", ".")
            if pure:
                self.fallback.add(mod)
                continue
            try:
                if hashlib.sha1(src.read_bytes()).hexdigest() != digest:
                    self.fallback.add(mod)
            except OSError:
                pass

    def find_spec(self, fullname, path=None, target=None):
        if fullname not in self.fallback:
            return None
        rel = fullname[len(_PKG) + 1:].replace(".", "/") + ".py"
        src = _PKG_DIR / rel
        if not src.exists():
            return None
        loader = importlib.machinery.SourceFileLoader(fullname, str(src))
        return importlib.util.spec_from_file_location(fullname, str(src), loader=loader)


def install() -> _SourceFallbackFinder:
    finder = _SourceFallbackFinder(os.environ.get("HLSJS_P2P_PURE", "") not in ("", "0"), _load_manifest())
    if finder.fallback:
        sys.meta_path.insert(0, finder)
    return finder


def compiled_modules() -> list:
    """Names of host modules currently running compiled (for reports / tests)."""
    out = []
    for name, mod in list(sys.modules.items()):
        f = str(getattr(mod, "__file__", "") or "")
        if (name.startswith(_PKG + ".") and f.endswith(tuple(importlib.machinery.EXTENSION_SUFFIXES))
                and not name.endswith(("._C", "._runtime"))):
            out.append(name)
    return sorted(out)


FINDER = install()
