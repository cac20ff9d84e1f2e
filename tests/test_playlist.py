"""M3U8 media-playlist parsing: segment URL resolution (memoized per directory) must equal
urllib's urljoin for every URI shape a playlist can carry."""
from urllib.parse import urljoin

import pytest

from hlsjs_p2p_wrapper_amd.player.playlist import _resolver, parse_media, write_media_playlist


@pytest.mark.parametrize("base", ["http://cdn.x/live/a/r0/index.m3u8?tok=1", "https://h/p.m3u8", "http://h/a/b/"])
def test_segment_url_resolution_matches_urljoin(base):
    r = _resolver(base)
    for uri in ["../../r0/seg12.ts", "seg1.ts", "/abs/seg.ts", "http://o.y/z/seg.ts", "sub/dir/s.ts",
                "s.ts?x=a/b", "./s.ts", "../s.ts", "seg1.ts", "d/s.ts#frag"]:
        assert r(uri) == urljoin(base, uri), uri


def test_parse_media_resolves_every_segment():
    text = write_media_playlist([(f"../v/seg{i}.ts", 4.0) for i in range(50)] + [("other/x.ts", 2.0)], 4,
                                media_sequence=7)
    d = parse_media(text, "http://cdn/p/q/index.m3u8", 0)
    assert [f.sn for f in d.fragments][:2] == [7, 8] and d.fragments[-1].sn == 57
    assert d.fragments[3].url == "http://cdn/p/v/seg3.ts" and d.fragments[-1].url == "http://cdn/p/q/other/x.ts"
    assert d.totalduration == pytest.approx(202.0) and not d.live
