"""Shared utilities: emitters, the xhrSetup sandbox, static mirroring, UA parsing."""
from .events import EventEmitter, JsObject, Observer
from .xhr import BaseXHR, extractInfoFromXhrSetup, extract_info_from_xhr_setup
from .statics import StaticMirrorMeta, inheritStaticPropertiesReadOnly

__all__ = [
    "EventEmitter", "JsObject", "Observer", "BaseXHR", "extractInfoFromXhrSetup",
    "extract_info_from_xhr_setup", "StaticMirrorMeta", "inheritStaticPropertiesReadOnly",
]
