"""Minimal synchronous event emitters.

Two flavours are needed to reproduce the reference's contracts:

* :class:`EventEmitter` — Node ``events`` semantics (``on``/``emit``/``removeListener``)
  used by the player bridge (``lib/integration/player-interface.js:1,4``).
* :class:`Observer` — the hls.js observer semantics: listeners are called as
  ``fn(event, data)`` (``lib/hlsjs-p2p-wrapper-private.js:38,219``;
  ``lib/integration/player-interface.js:15,22``).

Both are deliberately tiny: they sit on the per-fragment hot path (``FRAG_LOADING``,
``FRAG_LOAD_PROGRESS``, ``FRAG_LOADED`` …) so dispatch is a list copy + loop.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List


class EventEmitter:
    """Node-style emitter: ``emit(name, *args)`` calls ``listener(*args)``."""

    __slots__ = ("_listeners",)

    def __init__(self) -> None:
        self._listeners: Dict[str, List[Callable[..., Any]]] = {}

    def on(self, name: str, listener: Callable[..., Any]) -> "EventEmitter":
        self._listeners.setdefault(name, []).append(listener)
        return self

    add_listener = on
    addListener = on

    def once(self, name: str, listener: Callable[..., Any]) -> "EventEmitter":
        def _wrapper(*args: Any) -> None:
            self.remove_listener(name, _wrapper)
            listener(*args)

        _wrapper.__wrapped__ = listener  # type: ignore[attr-defined]
        return self.on(name, _wrapper)

    def remove_listener(self, name: str, listener: Callable[..., Any]) -> "EventEmitter":
        lst = self._listeners.get(name)
        if not lst:
            return self
        for i in range(len(lst) - 1, -1, -1):
            fn = lst[i]
            if fn is listener or getattr(fn, "__wrapped__", None) is listener:
                del lst[i]
                break
        return self

    removeListener = remove_listener
    off = remove_listener

    def remove_all_listeners(self, name: str | None = None) -> "EventEmitter":
        if name is None:
            self._listeners.clear()
        else:
            self._listeners.pop(name, None)
        return self

    removeAllListeners = remove_all_listeners

    def listener_count(self, name: str) -> int:
        return len(self._listeners.get(name, ()))

    listenerCount = listener_count

    def emit(self, name: str, *args: Any) -> bool:
        lst = self._listeners.get(name)
        if not lst:
            return False
        for fn in tuple(lst):
            fn(*args)
        return True


class Observer:
    """hls.js-style observer: ``trigger(event, data)`` calls ``fn(event, data)``."""

    __slots__ = ("_listeners",)

    def __init__(self) -> None:
        self._listeners: Dict[str, List[Callable[[str, Any], Any]]] = {}

    def on(self, event: str, listener: Callable[[str, Any], Any]) -> None:
        self._listeners.setdefault(event, []).append(listener)

    def once(self, event: str, listener: Callable[[str, Any], Any]) -> None:
        def _wrapper(ev: str, data: Any) -> None:
            self.off(event, _wrapper)
            listener(ev, data)

        _wrapper.__wrapped__ = listener  # type: ignore[attr-defined]
        self.on(event, _wrapper)

    def off(self, event: str, listener: Callable[[str, Any], Any]) -> None:
        lst = self._listeners.get(event)
        if not lst:
            return
        for i in range(len(lst) - 1, -1, -1):
            fn = lst[i]
            if fn is listener or getattr(fn, "__wrapped__", None) is listener:
                del lst[i]
                return

    def remove_all_listeners(self, event: str | None = None) -> None:
        if event is None:
            self._listeners.clear()
        else:
            self._listeners.pop(event, None)

    removeAllListeners = remove_all_listeners

    def listener_count(self, event: str) -> int:
        return len(self._listeners.get(event, ()))

    def trigger(self, event: str, data: Any = None) -> None:
        lst = self._listeners.get(event)
        if not lst:
            return
        if len(lst) == 1:
            lst[0](event, data)
            return
        for fn in tuple(lst):
            fn(event, data)

    emit = trigger


class JsObject(dict):
    """Plain JS-object analog: a dict with attribute access (``undefined`` -> ``None``).

    Used for event payloads (``{currentTarget: {response}}``, ``{target: {status}}``) and
    loader stats (``{trequest, tfirst, tload, loaded, retry, aborted}``) so both
    ``stats.tload`` and ``stats["tload"]`` work, as they do in JavaScript.
    """

    __slots__ = ()

    def __getattr__(self, name: str) -> Any:
        try:
            return self[name]
        except KeyError:
            if name.startswith("__"):
                raise AttributeError(name)
            return None

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value

    def __delattr__(self, name: str) -> None:
        self.pop(name, None)
