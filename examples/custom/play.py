"""Custom integration — inject your own engine constructor into the wrapper (reference
``example/custom/index.html:39-43``).

``HlsjsP2PWrapper(Hls)`` builds a P2P-configured player with ``createPlayer``; without
P2P support the application falls back to the plain engine.

    python examples/custom/play.py --peers 2
    python examples/custom/play.py --no-p2p          # plain engine fallback
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import config  # noqa: E402

from hlsjs_p2p_wrapper_amd import HlsjsP2PWrapper  # noqa: E402
from hlsjs_p2p_wrapper_amd.player.hls import Hls  # noqa: E402  (the plain engine)


def play(cfg, media, p2p_enabled):
    if not Hls.isSupported():
        raise RuntimeError("Your environment is not supported.")
    if p2p_enabled:
        wrapper = HlsjsP2PWrapper(Hls)  # DI of the engine constructor
        hls = wrapper.createPlayer(cfg["hlsjsConfig"], cfg["p2pConfig"])
    else:
        hls = Hls(cfg["hlsjsConfig"])  # fall back on the default engine
    hls.loadSource(cfg["contentUrl"])
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda event, data: media.play())
    return hls


if __name__ == "__main__":
    config.main(play, __doc__)
