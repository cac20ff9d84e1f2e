"""Legacy (v2) integration — plain wrapper without DI (reference
``example/legacy/index.html:40-51``).

The application builds the engine itself with ``fLoader: wrapper.P2PLoader`` and starts
the P2P module on ``MANIFEST_LOADING`` with the deprecated ``createSRModule``.

    python examples/legacy/play.py --peers 2
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import config  # noqa: E402

from hlsjs_p2p_wrapper_amd import HlsjsP2PWrapper  # noqa: E402
from hlsjs_p2p_wrapper_amd.player.hls import Hls  # noqa: E402


def play(cfg, media, p2p_enabled):
    if not Hls.isSupported():
        raise RuntimeError("Your environment is not supported.")
    if p2p_enabled:
        wrapper = HlsjsP2PWrapper()  # no engine constructor injected
        hls = Hls({"fLoader": wrapper.P2PLoader})  # add your custom config here
        hls.on(Hls.Events.MANIFEST_LOADING,
               lambda event, data: wrapper.createSRModule(cfg["p2pConfig"], hls, Hls.Events, cfg["p2pConfig"].get(
                   "contentId")))
    else:
        hls = Hls(cfg["hlsjsConfig"])
    hls.loadSource(cfg["contentUrl"])
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda event, data: media.play())
    return hls


if __name__ == "__main__":
    config.main(play, __doc__)
