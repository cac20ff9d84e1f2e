"""Bundle integration — the preferred way (reference ``example/bundle/index.html:45``).

The bundle's ``Hls`` shims the engine constructor: create the player exactly as usual
and pass the P2P config as a second argument.  Nothing else changes in the application.

    python examples/bundle/play.py --peers 4
    torchrun --nproc-per-node 8 examples/bundle/play.py        # one peer per MI355X
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import config  # noqa: E402

from hlsjs_p2p_wrapper_amd import Hls  # noqa: E402  (the bundle: hlsjs-p2p-bundle analog)


def play(cfg, media, p2p_enabled):
    if not p2p_enabled:
        raise RuntimeError("This process cannot join a swarm: the bundle requires P2P support.")
    if not Hls.isSupported():
        raise RuntimeError("Your environment is not supported.")
    hls = Hls(cfg["hlsjsConfig"], cfg["p2pConfig"])
    hls.loadSource(cfg["contentUrl"])
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda event, data: media.play())
    return hls


if __name__ == "__main__":
    config.main(play, __doc__)
