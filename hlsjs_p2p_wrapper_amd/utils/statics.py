"""Read-only static mirroring (component C12).

Parity: ``lib/utils.js:3-19`` — ``inheritStaticPropertiesReadOnly(target, source)`` gives
the bundle class read-only getters for every own static of the hls.js class
(``Hls.Events``, ``Hls.DefaultConfig``, ``Hls.ErrorTypes`` …) except ``prototype``,
``name``, ``length``, ``caller``, ``arguments`` and ``isSupported``.

Python classes have no per-property getters at class level, so the target class must use
:class:`StaticMirrorMeta` as its metaclass; this function registers the mirrored names on
it.  Reads are forwarded live to ``source`` (like the reference's getter) and writes raise
(strict-mode ES modules throw on assignment to a getter-only property).
"""
from __future__ import annotations

from typing import Any, Iterable

_EXCLUDED = frozenset({"prototype", "name", "length", "caller", "arguments", "isSupported"})


class StaticMirrorMeta(type):
    """Metaclass providing live, read-only class attributes mirrored from another class."""

    def __getattribute__(cls, name: str) -> Any:
        mirrors = type.__getattribute__(cls, "__dict__").get("_static_mirrors")
        if mirrors and name in mirrors:
            return getattr(mirrors[name], name)
        return type.__getattribute__(cls, name)

    def __setattr__(cls, name: str, value: Any) -> None:
        mirrors = type.__getattribute__(cls, "__dict__").get("_static_mirrors")
        if mirrors and name in mirrors:
            raise AttributeError(f"Cannot assign to read only static property '{name}'")
        type.__setattr__(cls, name, value)


def _own_statics(source: type) -> Iterable[str]:
    for name in vars(source):
        if name.startswith("__") and name.endswith("__"):
            continue
        if name.startswith("_"):
            continue
        yield name


def inheritStaticPropertiesReadOnly(target: type, source: type) -> None:
    if not isinstance(target, StaticMirrorMeta):
        raise TypeError("target class must use StaticMirrorMeta as its metaclass")
    mirrors = dict(type.__getattribute__(target, "__dict__").get("_static_mirrors") or {})
    for name in _own_statics(source):
        if name in _EXCLUDED:
            continue
        mirrors[name] = source
    type.__setattr__(target, "_static_mirrors", mirrors)


inherit_static_properties_read_only = inheritStaticPropertiesReadOnly
