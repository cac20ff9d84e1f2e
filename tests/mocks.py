"""Test doubles mirroring the reference's mocks (``test/mocks/*.js``).

* :class:`HlsMock` — ``test/mocks/hls.js:3-59``: fake ``levels`` (``None`` when
  ``levelNumber == 0``), each with 2 redundant URLs; only ``definedLevel`` gets
  ``details{live, fragments}`` with sn 25..199 and ``start = 10*sn``; ``config`` is the
  engine's DefaultConfig; ``on``/``trigger`` are no-ops.
* :class:`PeerAgentMock` — ``test/mocks/peer-agent.js``: a CDN-only agent that fetches
  with the default (shaped) loader path and reports progress as ``cdnDownloaded``.
* :class:`HlsjsWrapperMock` — ``test/mocks/wrapper.js``: just ``peerAgentModule``.
"""
from types import SimpleNamespace

from hlsjs_p2p_wrapper_amd.net import http
from hlsjs_p2p_wrapper_amd.player.config import default_config
from hlsjs_p2p_wrapper_amd.player.loader import XhrLoader
from hlsjs_p2p_wrapper_amd.utils.events import JsObject


class HlsMock:
    def __init__(self, levelNumber, live, definedLevel=0, emptyLevel=True):
        self._levels = [] if levelNumber > 0 else None
        fragments = [SimpleNamespace(sn=f, start=f * 10, duration=10) for f in range(25, 200)]
        for i in range(levelNumber):
            url = [f"http://foo.bar/{i}/0/playlist.m3u8", f"http://foo.bar/{i}/1/playlist.m3u8"]
            if emptyLevel:
                level = SimpleNamespace(url=url, details=None, urlId=0)
            else:
                level = SimpleNamespace(details=SimpleNamespace(totalduration=120), audioCodec="fooCodec", url=url,
                                        urlId=0, bitrate=100000 * (i + 1))
            if live is not None and i == definedLevel:
                level.details = SimpleNamespace(live=live, fragments=fragments)
            self._levels.append(level)
        self._config = default_config()

    @property
    def levels(self):
        return self._levels

    @property
    def config(self):
        return self._config

    def on(self, *a):
        pass

    def trigger(self, *a):
        pass


class _Handle:
    def __init__(self, loader):
        self.loader = loader

    def abort(self):
        self.loader.abort()


class PeerAgentMock:
    """CDN-only agent: plain (shaped) HTTP fetch, progress reported as cdnDownloaded."""

    StreamTypes = JsObject(HLS="hls")

    def __init__(self, *args, **kwargs):
        self.requests = []
        self.stats = JsObject(cdn=0, p2p=0, upload=0, peers=0)
        self.p2pDownloadOn = True
        self.p2pUploadOn = True
        self.media = None
        self.disposed = False

    def getSegment(self, reqInfo, callbacks, segmentView):
        self.requests.append((reqInfo, segmentView))
        loader = XhrLoader(None)

        def ok(event, stats):
            self.stats.cdn += stats.loaded
            callbacks["onSuccess"](event.currentTarget.response)

        def err(event):
            callbacks["onError"](http.HttpError(event.target.status, reqInfo["url"]))

        def progress(event, stats):
            callbacks["onProgress"](JsObject(cdnDownloaded=event.loaded))

        loader.load(reqInfo["url"], "arraybuffer", ok, err, lambda e, s: None, 1e9, 0, 0, progress,
                    _FragShim(reqInfo))
        return _Handle(loader)

    def setMediaElement(self, media):
        self.media = media

    def dispose(self):
        self.disposed = True


class _FragShim:
    def __init__(self, reqInfo):
        rng = (reqInfo.get("headers") or {}).get("Range")
        if rng:
            s, e = rng[len("bytes="):].split("-")
            self.byteRangeStartOffset, self.byteRangeEndOffset = int(s), int(e) + 1
        else:
            self.byteRangeStartOffset = self.byteRangeEndOffset = None


class HlsjsWrapperMock:
    def __init__(self, Hls=None):
        self.peerAgentModule = PeerAgentMock()
        self.hls = None
