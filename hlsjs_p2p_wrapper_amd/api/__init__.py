"""L4/L5 public API: the ``Hls`` bundle and the ``HlsjsP2PWrapper`` facade."""
from .bundle import Hls, StreamrootHlsjsBundle
from .wrapper import HlsjsP2PWrapper
from .wrapper_private import HlsjsP2PWrapperPrivate

__all__ = ["Hls", "StreamrootHlsjsBundle", "HlsjsP2PWrapper", "HlsjsP2PWrapperPrivate"]
