"""hls.js event / error enumerations (the L1 player surface the wrapper consumes).

The wrapper subscribes to ``MANIFEST_LOADING`` (``lib/hlsjs-p2p-wrapper-private.js:38``),
``MEDIA_ATTACHING`` (``:178``), ``ERROR`` (``:219``), ``LEVEL_SWITCH`` and ``DESTROYING``
(``lib/integration/player-interface.js:15,22``); its tests drive ``FRAG_LOADING``,
``FRAG_LOADED``, ``FRAG_LOAD_PROGRESS`` (``test/html/p2p-loader-generator.js:63-78``) and
``MANIFEST_PARSED`` (``test/html/bundle.js:107``).  The string values follow hls.js 0.5/0.6
so application code that compares raw event names keeps working.
"""
from __future__ import annotations


class _Enum:
    """Attribute bag that is iterable like a JS enum object."""

    @classmethod
    def items(cls):
        return [(k, v) for k, v in vars(cls).items() if not k.startswith("_") and isinstance(v, str)]

    @classmethod
    def values(cls):
        return [v for _, v in cls.items()]


class Events(_Enum):
    MEDIA_ATTACHING = "hlsMediaAttaching"
    MEDIA_ATTACHED = "hlsMediaAttached"
    MEDIA_DETACHING = "hlsMediaDetaching"
    MEDIA_DETACHED = "hlsMediaDetached"
    BUFFER_RESET = "hlsBufferReset"
    BUFFER_CODECS = "hlsBufferCodecs"
    BUFFER_APPENDING = "hlsBufferAppending"
    BUFFER_APPENDED = "hlsBufferAppended"
    BUFFER_EOS = "hlsBufferEos"
    BUFFER_FLUSHING = "hlsBufferFlushing"
    BUFFER_FLUSHED = "hlsBufferFlushed"
    MANIFEST_LOADING = "hlsManifestLoading"
    MANIFEST_LOADED = "hlsManifestLoaded"
    MANIFEST_PARSED = "hlsManifestParsed"
    LEVEL_LOADING = "hlsLevelLoading"
    LEVEL_LOADED = "hlsLevelLoaded"
    LEVEL_UPDATED = "hlsLevelUpdated"
    LEVEL_PTS_UPDATED = "hlsLevelPtsUpdated"
    LEVEL_SWITCH = "hlsLevelSwitch"
    KEY_LOADING = "hlsKeyLoading"
    KEY_LOADED = "hlsKeyLoaded"
    FRAG_LOADING = "hlsFragLoading"
    FRAG_LOAD_PROGRESS = "hlsFragLoadProgress"
    FRAG_LOAD_EMERGENCY_ABORTED = "hlsFragLoadEmergencyAborted"
    FRAG_LOADED = "hlsFragLoaded"
    FRAG_DECRYPTED = "hlsFragDecrypted"
    FRAG_PARSING_INIT_SEGMENT = "hlsFragParsingInitSegment"
    FRAG_PARSING_USERDATA = "hlsFragParsingUserdata"
    FRAG_PARSING_METADATA = "hlsFragParsingMetadata"
    FRAG_PARSING_DATA = "hlsFragParsingData"
    FRAG_PARSED = "hlsFragParsed"
    FRAG_BUFFERED = "hlsFragBuffered"
    FRAG_CHANGED = "hlsFragChanged"
    FPS_DROP = "hlsFpsDrop"
    ERROR = "hlsError"
    DESTROYING = "hlsDestroying"


class ErrorTypes(_Enum):
    NETWORK_ERROR = "networkError"
    MEDIA_ERROR = "mediaError"
    OTHER_ERROR = "otherError"


class ErrorDetails(_Enum):
    MANIFEST_LOAD_ERROR = "manifestLoadError"
    MANIFEST_LOAD_TIMEOUT = "manifestLoadTimeOut"
    MANIFEST_PARSING_ERROR = "manifestParsingError"
    MANIFEST_INCOMPATIBLE_CODECS_ERROR = "manifestIncompatibleCodecsError"
    LEVEL_LOAD_ERROR = "levelLoadError"
    LEVEL_LOAD_TIMEOUT = "levelLoadTimeOut"
    LEVEL_SWITCH_ERROR = "levelSwitchError"
    FRAG_LOAD_ERROR = "fragLoadError"
    FRAG_LOOP_LOADING_ERROR = "fragLoopLoadingError"
    FRAG_LOAD_TIMEOUT = "fragLoadTimeOut"
    FRAG_DECRYPT_ERROR = "fragDecryptError"
    FRAG_PARSING_ERROR = "fragParsingError"
    FRAG_INTEGRITY_ERROR = "fragIntegrityError"
    KEY_LOAD_ERROR = "keyLoadError"
    KEY_LOAD_TIMEOUT = "keyLoadTimeOut"
    BUFFER_APPEND_ERROR = "bufferAppendError"
    BUFFER_APPENDING_ERROR = "bufferAppendingError"
    BUFFER_STALLED_ERROR = "bufferStalledError"
    BUFFER_FULL_ERROR = "bufferFullError"
    BUFFER_SEEK_OVER_HOLE = "bufferSeekOverHole"
    INTERNAL_EXCEPTION = "internalException"
