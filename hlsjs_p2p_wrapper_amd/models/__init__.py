"""L2 mapping / data model: segment identity and playlist view."""
from .track_view import TrackView
from .segment_view import SegmentView, KEY_BYTES
from .media_map import MediaMap

__all__ = ["TrackView", "SegmentView", "MediaMap", "KEY_BYTES"]
