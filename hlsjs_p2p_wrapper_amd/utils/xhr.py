"""Sandboxed XHR mock and ``xhrSetup`` extraction (component C11).

Parity: ``lib/utils.js:27-48``.  hls.js lets an app customise every request through
``config.xhrSetup(xhr, url)``.  With the P2P engine the *agent*, not the player, issues
the real request, so the wrapper runs the user's ``xhrSetup`` against a mock that only
records ``setRequestHeader`` calls and ``withCredentials``; any other access is an error,
re-wrapped with the reference's exact message (``:41-45``).

``BaseXHR`` mirrors the xhr-shaper class the reference imports (``utils.js:1,30``): it is
constructed with an *implementation* dict; attributes present in the dict are allowed
(functions are callable, plain values are readable/writable), everything else raises.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional, Tuple

_FORBIDDEN_PREFIX = ("xhrSetup is trying to acces a forbidden property/method of XHR mock. "
                     "Please contact Streamroot support. Internal mock error: ")


class XHRMockError(Exception):
    pass


class BaseXHR:
    """A minimal XMLHttpRequest stand-in that forbids everything not implemented."""

    def __init__(self, impl: Optional[Dict[str, Any]] = None) -> None:
        object.__setattr__(self, "_impl", dict(impl or {}))

    def __getattr__(self, name: str) -> Any:
        impl = object.__getattribute__(self, "_impl")
        if name in impl:
            return impl[name]
        raise XHRMockError(f"XHR mock: access to '{name}' is not implemented")

    def __setattr__(self, name: str, value: Any) -> None:
        impl = object.__getattribute__(self, "_impl")
        if name in impl and not callable(impl[name]):
            impl[name] = value
            return
        raise XHRMockError(f"XHR mock: writing '{name}' is not allowed")

    def __delattr__(self, name: str) -> None:
        raise XHRMockError(f"XHR mock: deleting '{name}' is not allowed")


def extractInfoFromXhrSetup(xhrSetup: Optional[Callable[..., Any]], url: Any = None,
                            headersBase: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    """Run ``xhrSetup(xhr, url)`` against the mock; return ``{headers, withCredentials}``.

    ``headersBase`` is extended in place, as in the reference (``utils.js:28``).
    """
    headers: Dict[str, str] = headersBase if headersBase is not None else {}
    if not xhrSetup:  # nothing to run: skip building the sandbox (once per fragment request)
        return {"headers": headers, "withCredentials": False}

    def _set_request_header(header: str, value: Any) -> None:
        headers[header] = value

    xhr = BaseXHR({"setRequestHeader": _set_request_header, "withCredentials": False})
    try:
        if xhrSetup:
            xhrSetup(xhr, url)
    except Exception as e:  # noqa: BLE001 — the reference wraps everything
        raise Exception(_FORBIDDEN_PREFIX + str(e)) from e
    return {"headers": headers, "withCredentials": object.__getattribute__(xhr, "_impl")["withCredentials"]}


def extract_info_from_xhr_setup(xhr_setup, url=None, headers_base=None) -> Tuple[Dict[str, str], bool]:
    info = extractInfoFromXhrSetup(xhr_setup, url, headers_base)
    return info["headers"], info["withCredentials"]
