"""L0 platform: event loop / timers, the in-process CDN origins and HTTP semantics."""
from .event_loop import EventLoop, get_event_loop, new_event_loop, set_event_loop, performance_now
from .http import HttpError, Response, Shaper, fetch, head, register_origin, unregister_origin, clear_origins

__all__ = [
    "EventLoop", "get_event_loop", "new_event_loop", "set_event_loop", "performance_now",
    "HttpError", "Response", "Shaper", "fetch", "head", "register_origin", "unregister_origin", "clear_origins",
]
