"""Port of ``test/media-map.js`` plus the batched ``getSegmentLists`` agreement with single queries."""
import pytest

from hlsjs_p2p_wrapper_amd.models import MediaMap, SegmentView, TrackView
from mocks import HlsMock


def _mm(*a):
    return MediaMap(HlsMock(*a))


def test_get_segment_time():
    tv = TrackView(level=1, urlId=1)
    assert _mm(3, False, 1).getSegmentTime(SegmentView(sn=56, trackView=tv, time=560)) == 560
    assert _mm(3, False, 1).getSegmentTime(SegmentView(sn=24, trackView=tv, time=240)) == 240
    assert _mm(3, False, 0).getSegmentTime(SegmentView(sn=56, trackView=tv, time=560)) == 560
    with pytest.raises(Exception, match="getSegmentTime: segmentView.time is undefined"):
        _mm(3, False, 0).getSegmentTime(SegmentView(sn=56, trackView=tv))


def _svs(tv, sns):
    return [SegmentView(sn=s, trackView=tv, time=s * 10) for s in sns]


@pytest.mark.parametrize("begin,dur,sns", [
    (365, 33, range(37, 40)),      # timerange included in index
    (10, 275, range(25, 29)),      # left intersection
    (1975, 3000, range(198, 200)),  # right intersection
    (240, 2100, range(25, 200)),   # timerange includes the index
    (2100, 3000, []),              # disjoint
])
def test_get_segment_list(begin, dur, sns):
    tv = TrackView(level=1, urlId=1)
    assert _mm(3, False, 1).getSegmentList(tv, begin, dur) == _svs(tv, sns)


def test_get_segment_list_unparsed_level_is_empty():
    assert _mm(3, False, 0).getSegmentList(TrackView(level=1, urlId=1), 2100, 3000) == []


def test_get_segment_list_missing_level_throws():
    with pytest.raises(Exception, match="getSegmentList: level doesn't exist"):
        _mm(3, False, 0).getSegmentList(TrackView(level=4, urlId=1), 2100, 3000)


def test_get_segment_list_closed_interval_edges():
    tv = TrackView(level=1, urlId=0)
    got = _mm(3, False, 1).getSegmentList(tv, 370, 20)  # starts 370, 380, 390 (both ends inclusive)
    assert [s.sn for s in got] == [37, 38, 39]


def test_get_track_list():
    assert _mm(0, False, 0).getTrackList() == []
    tracks = _mm(3, False, 1).getTrackList()
    assert len(tracks) == 6  # 3 levels x 2 urlIds
    assert [t.viewToString() for t in tracks[:3]] == ["L0U0", "L0U1", "L1U0"]


def test_get_segment_duration_is_first_fragment_duration():
    mm = _mm(3, False, 1)
    assert mm.getSegmentDuration(SegmentView(sn=100, trackView=TrackView(level=1, urlId=0))) == 10


_QUERIES = [(365, 33), (10, 275), (1975, 3000), (240, 2100), (2100, 3000), (0, 0), (250, 0), (-50, 60)]


def test_batched_segment_lists_match_single_queries():
    mm = _mm(3, False, 1)
    tv = TrackView(level=1, urlId=1)
    qs = [(tv, b, d) for b, d in _QUERIES]
    assert mm.getSegmentLists(qs) == [mm.getSegmentList(tv, b, d) for b, d in _QUERIES]
    with pytest.raises(Exception, match="level doesn't exist"):
        mm.getSegmentLists([(TrackView(level=7, urlId=0), 0, 10)])


def test_fragment_lookup():
    mm = _mm(3, False, 1)
    tv = TrackView(level=1, urlId=0)
    f = mm.fragment(SegmentView(sn=42, trackView=tv, time=420))
    assert f is not None and f.sn == 42
    assert mm.fragment(SegmentView(sn=100000, trackView=tv, time=0)) is None


def test_start_index_cache_follows_fragment_mutations():
    """The start-time cache must not outlive the playlist it was built from: an in-place
    ``frag.start`` rewrite (hls.js PTS realignment), a fragment object swapped in without a
    start assignment, and a re-sorted list each answer from the new starts."""
    from types import SimpleNamespace

    from hlsjs_p2p_wrapper_amd.player.level import Fragment, LevelDetails

    frags = [Fragment(url=f"s{i}.ts", sn=i, start=10.0 * i, duration=10.0) for i in range(10)]
    level = SimpleNamespace(url=["l0.m3u8"], details=LevelDetails(url="l0.m3u8", fragments=frags))
    mm = MediaMap(SimpleNamespace(levels=[level]))
    tv = TrackView(level=0, urlId=0)
    assert [s.sn for s in mm.getSegmentList(tv, 30, 20)] == [3, 4, 5]
    for f in frags:  # realignment shifts every start by +5 s in place (same list, same length)
        f.start += 5.0
    assert [s.sn for s in mm.getSegmentList(tv, 30, 20)] == [3, 4]      # starts 35, 45
    assert [s.time for s in mm.getSegmentList(tv, 30, 20)] == [35.0, 45.0]
    # a fragment object replaced without touching `start` on the list's own objects
    swapped = Fragment(url="x.ts", sn=99, start=1000.0, duration=10.0)
    object.__setattr__(swapped, "start", 1000.0)
    frags[-1] = swapped
    assert [s.sn for s in mm.getSegmentList(tv, 990, 20)] == [99]
    # a list re-sorted in place after a start rewrite falls back to / rebuilds the index
    frags[0].start = 500.0
    assert 0 in [s.sn for s in mm.getSegmentList(tv, 495, 10)]


def test_fragment_construction_keeps_other_levels_indexes():
    """Building fragments (a playlist parse or live reload of one level) does not bump the
    start generation, so other levels' cached start indexes stay valid; only a start
    REWRITE of an existing fragment does."""
    from hlsjs_p2p_wrapper_amd.player.level import Fragment, fragment_generation

    g0 = fragment_generation()
    frags = [Fragment(url=f"s{i}.ts", sn=i, start=4.0 * i, duration=4.0) for i in range(1000)]
    frags[3].loaded = 10  # other field writes: no hook at all
    assert fragment_generation() == g0
    frags[3].start = 13.0
    assert fragment_generation() == g0 + 1 and frags[3].start == 13.0 and frags[3].end == 17.0
