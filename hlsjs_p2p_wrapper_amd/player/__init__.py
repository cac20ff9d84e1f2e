"""The hls.js-compatible media engine (the L1 player the reference wraps)."""
from .events import Events, ErrorTypes, ErrorDetails
from .config import HlsConfig, default_config
from .level import Fragment, Level, LevelDetails, DecryptData
from .media import MediaElement, HTMLVideoElement, TimeRanges
from .hls import Hls
from .loader import XhrLoader
from .abr import AbrController, EwmaBandWidthEstimator

__all__ = [
    "Events", "ErrorTypes", "ErrorDetails", "HlsConfig", "default_config", "Fragment", "Level",
    "LevelDetails", "DecryptData", "MediaElement", "HTMLVideoElement", "TimeRanges", "Hls", "XhrLoader",
    "AbrController", "EwmaBandWidthEstimator",
]
