"""Stock demo of the plain media engine (no P2P) — the input of tools/update_demo.py,
which derives ``p2p_demo.py`` from it (the reference patches the upstream hls.js demo page
the same way, ``update_demo.rb:13-43``).

Plays a synthetic stream and prints a once-per-media-second status line (level, buffer,
bandwidth estimate), like the hls.js demo page's stats panel.

    python examples/demo/engine_demo.py --seconds 12
"""
import argparse
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from hlsjs_p2p_wrapper_amd.net import new_event_loop  # noqa: E402
from hlsjs_p2p_wrapper_amd.net.origin import PRESET_ABR5, SyntheticHlsOrigin  # noqa: E402
from hlsjs_p2p_wrapper_amd.player import MediaElement  # noqa: E402
from hlsjs_p2p_wrapper_amd.player.hls import Hls  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=12.0)
    args = ap.parse_args()
    loop = new_event_loop("virtual")
    origin = SyntheticHlsOrigin("http://cdn.demo/abr/", renditions=PRESET_ABR5, num_segments=20, encrypted=True,
                                pool_size=4, pin_memory=False)
    hlsjsConfig = {"debug": False}
    hls = Hls(hlsjsConfig)
    media = MediaElement()
    hls.loadSource(origin.master_url())
    hls.attachMedia(media)
    hls.on(Hls.Events.MANIFEST_PARSED, lambda event, data: media.play())
    shown = [-1]

    def status():
        t = int(media.currentTime)
        if t != shown[0]:
            shown[0] = t
            ahead = media._buffer_ahead(media.currentTime)
            bw = hls.abrController.bwEstimator.getEstimate() / 1e6
            print(f"t={media.currentTime:5.1f}s level={hls.currentLevel} buffered={ahead:5.1f}s "
                  f"bw={bw:7.2f} Mb/s", flush=True)
        return media.currentTime >= args.seconds

    ok = loop.run_until(status, timeout_ms=600_000)
    print("DEMO-OK" if ok else "DEMO-TIMEOUT", flush=True)
    hls.destroy()


if __name__ == "__main__":
    main()
