"""Ports of ``test/track-view.js`` and ``test/segment-view.js`` (one assertion each)."""
import json

import numpy as np

from hlsjs_p2p_wrapper_amd.models import SegmentView, TrackView
from hlsjs_p2p_wrapper_amd.ops import segment


# --- test/track-view.js:3-42 ------------------------------------------------------------
def test_trackview_equal():
    assert TrackView({"level": 0, "urlId": 1}).isEqual(TrackView({"level": 0, "urlId": 1}))


def test_trackview_not_equal_level():
    assert not TrackView({"level": 0, "urlId": 1}).isEqual(TrackView({"level": 1, "urlId": 1}))


def test_trackview_not_equal_urlid():
    assert not TrackView({"level": 0, "urlId": 1}).isEqual(TrackView({"level": 0, "urlId": 0}))


def test_trackview_falsy_arg():
    assert TrackView({"level": 0, "urlId": 1}).isEqual(None) is False


def test_trackview_strings():
    a, b = TrackView({"level": 0, "urlId": 1}), TrackView({"level": 0, "urlId": 1})
    assert a.viewToString() == b.viewToString() == "L0U1"
    assert a.viewToString() != TrackView({"level": 1, "urlId": 1}).viewToString()
    assert a.viewToString() != TrackView({"level": 0, "urlId": 0}).viewToString()
    assert a.type == "video"


# --- test/segment-view.js ------------------------------------------------------------------
def test_segmentview_json_roundtrip():
    # legacy field names: sn is undefined on both sides, equality passes trivially (:5-11)
    sv = SegmentView({"timestamp": 25, "trackView": {"adaptationId": 1, "representationId": 0}})
    transferred = SegmentView(json.loads(json.dumps(sv.to_dict())))
    assert transferred.isEqual(sv)


def test_segmentview_to_array_buffer_type_and_roundtrip():
    sv = SegmentView({"sn": 25, "trackView": {"level": 1, "urlId": 1}})
    buf = sv.toArrayBuffer()
    assert isinstance(buf, bytes) and len(buf) == 12
    assert SegmentView.fromArrayBuffer(buf).isEqual(sv)
    assert np.frombuffer(buf, dtype="<u4").tolist() == [1, 1, 25]


def test_segmentview_binary_key_matches_packed_tensor_rows():
    keys = segment.pack_keys([1, 5], [1, 0], [25, 1560], swarm=9)
    a = SegmentView({"sn": 25, "trackView": {"level": 1, "urlId": 1}})
    b = SegmentView({"sn": 1560, "trackView": {"level": 5, "urlId": 0}})
    assert segment.wire_keys(keys) == a.toArrayBuffer() + b.toArrayBuffer()


def test_segmentview_is_in_track():
    tv = TrackView({"level": 0, "urlId": 1})
    assert SegmentView({"sn": 25, "trackView": {"level": 0, "urlId": 1}}).isInTrack(tv)
    assert not SegmentView({"sn": 25, "trackView": {"level": 1, "urlId": 1}}).isInTrack(tv)
    assert not SegmentView({"sn": 25, "trackView": {"level": 0, "urlId": 0}}).isInTrack(tv)


def test_segmentview_is_equal():
    a = SegmentView({"sn": 25, "trackView": {"level": 1, "urlId": 1}})
    assert a.isEqual(SegmentView({"sn": 25, "trackView": {"level": 1, "urlId": 1}}))
    assert not a.isEqual(SegmentView({"sn": 1560, "trackView": {"level": 1, "urlId": 1}}))
    assert not a.isEqual(SegmentView({"sn": 25, "trackView": {"level": 5, "urlId": 1}}))
    assert not a.isEqual(SegmentView({"sn": 25, "trackView": {"level": 1, "urlId": 0}}))
    assert not a.isEqual(None)


def test_segmentview_string_and_id():
    sv = SegmentView(sn=7, trackView=TrackView(level=2, urlId=1), time=28.0)
    assert sv.viewToString() == "L2U1S7"
    assert sv.getId() == 7
    # the binary form drops time (segment-view.js:59-61)
    assert SegmentView.fromArrayBuffer(sv.toArrayBuffer()).time is None


def test_segmentview_deep_copies_track():
    tv = TrackView(level=1, urlId=0)
    sv = SegmentView(sn=1, trackView=tv)
    tv.level = 9
    assert sv.trackView.level == 1
