"""Build-time version (the reference's ``_VERSION_`` global injected by uglify
``global_defs``, ``Gruntfile.js:27-29``; read by ``HlsjsP2PWrapperPrivate.version``).

``HLSJS_P2P_VERSION`` in the environment overrides it (the tests set it the way
``test/api.js`` sets ``global._VERSION_``)."""
import os

_BASE = "3.9.4+mi355x.1"


class _Version(str):
    pass


try:  # stamped by setup.py at build time (HLSJS_P2P_VERSION then)
    from ._build_info import VERSION as _STAMPED
except ImportError:
    _STAMPED = _BASE


def _current() -> str:
    return os.environ.get("HLSJS_P2P_VERSION", _STAMPED)


def __getattr__(name):  # module-level dynamic VERSION (PEP 562)
    if name == "VERSION":
        return _current()
    raise AttributeError(name)
