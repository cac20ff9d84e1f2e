"""hlsjs-p2p-wrapper-amd — an MI355X-native P2P HLS segment-delivery engine.

Same public API as ``hlsjs-p2p-wrapper`` (``Hls(hlsjsConfig, p2pConfig)``,
``HlsjsP2PWrapper(Hls).createPlayer / createSRModule / P2PLoader / stats /
p2pDownloadOn / p2pUploadOn / version``), with the swarm re-designed for the hardware:
one MI355X = one peer, segment cache in HBM, exchange over RCCL/xGMI, and the hot path
(decrypt, demux, integrity, cache/range ops) in hand-written CDNA4 HIP kernels.

Layout:
  api/          bundle ``Hls`` + wrapper facade + session orchestrator     (L4-L5)
  integration/  P2PLoader (hls.js fLoader) + PlayerInterface bridge        (L3)
  models/       TrackView / SegmentView (12-byte key) / MediaMap            (L2)
  player/       hls.js-compatible media engine (playlists, ABR, buffer)    (L1)
  agent/        PeerAgent contract + SwarmNode (HBM cache, exchange rounds) (L1)
  parallel/     swarm comm backends: thread hub, torch.distributed (RCCL)
  ops/          native: gfx950 kernels (_C) + host runtime (_runtime)
  net/          event loop / timers, CDN origins, HTTP semantics           (L0)
"""
from . import _accel  # noqa: F401  (first: stale compiled modules fall back to source)
from .version import _STAMPED as __version__
from .utils import log as _log
from .models import MediaMap, SegmentView, TrackView
from .api import Hls, HlsjsP2PWrapper, HlsjsP2PWrapperPrivate, StreamrootHlsjsBundle
from .agent import PeerAgent, SwarmNode
from .integration import PlayerInterface, p2p_loader_generator

_log.configure()

__all__ = [
    "Hls", "HlsjsP2PWrapper", "HlsjsP2PWrapperPrivate", "StreamrootHlsjsBundle", "PeerAgent", "SwarmNode",
    "PlayerInterface", "p2p_loader_generator", "MediaMap", "SegmentView", "TrackView", "__version__",
]
