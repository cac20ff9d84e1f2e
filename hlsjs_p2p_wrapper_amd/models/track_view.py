"""TrackView — identity of one rendition track ``(level, urlId)``.

Parity: ``lib/integration/mapping/track-view.js:1-29`` (component C7 in SURVEY §2.1).

* constructed from any object/dict carrying ``level`` and ``urlId`` (``:3-6``);
* ``viewToString()`` → ``"L{level}U{urlId}"`` (``:11-13``);
* ``isEqual(other)`` compares level and urlId, ``False`` for a falsy argument (``:19-24``);
* ``type`` is always ``"video"`` (``:26-28``; required by the asynchronous peer agent,
  ``CHANGELOG.md:37``).

``urlId`` indexes a level's redundant (backup) URLs, which are separate tracks since
3.8.0 (``CHANGELOG.md:20-22``).
"""
from __future__ import annotations

from typing import Any, Optional, Tuple


def _field(obj: Any, name: str) -> Any:
    if obj is None:
        raise TypeError(f"Cannot read property '{name}' of undefined")
    if isinstance(obj, dict):
        return obj.get(name)
    return getattr(obj, name, None)


class TrackView:
    """One rendition track ``(level, urlId)``; built from any object or dict carrying both."""

    __slots__ = ("level", "urlId")

    def __init__(self, obj: Any = None, *, level: Any = None, urlId: Any = None) -> None:
        if obj is not None:
            level = _field(obj, "level")
            urlId = _field(obj, "urlId")
        self.level = level
        self.urlId = urlId

    # --- reference API -------------------------------------------------------
    def viewToString(self) -> str:
        """``"L{level}U{urlId}"``."""
        return f"L{_js_str(self.level)}U{_js_str(self.urlId)}"

    def isEqual(self, trackView: Optional["TrackView"]) -> bool:
        """Same level and urlId (``False`` for a falsy argument)."""
        if not trackView:
            return False
        return trackView.level == self.level and trackView.urlId == self.urlId

    @property
    def type(self) -> str:
        """Always ``"video"``."""
        return "video"

    # --- python conveniences -------------------------------------------------
    view_to_string = viewToString
    is_equal = isEqual

    @property
    def url_id(self) -> Any:
        """snake_case alias of ``urlId``."""
        return self.urlId

    def key(self) -> Tuple[Any, Any]:
        """``(level, urlId)``."""
        return (self.level, self.urlId)

    def to_dict(self) -> dict:
        """``{"level", "urlId"}`` (JSON form)."""
        return {"level": self.level, "urlId": self.urlId}

    toJSON = to_dict

    def __eq__(self, other: object) -> bool:  # deep (``should.eql``) equality
        return isinstance(other, TrackView) and self.level == other.level and self.urlId == other.urlId

    def __hash__(self) -> int:
        return hash((self.level, self.urlId))

    def __bool__(self) -> bool:
        return True

    def __repr__(self) -> str:
        return f"TrackView(level={self.level!r}, urlId={self.urlId!r})"


def _js_str(v: Any) -> str:
    """String conversion as a JS template literal would do it."""
    if v is None:
        return "undefined"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return str(v)
