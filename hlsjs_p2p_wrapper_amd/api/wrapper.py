"""HlsjsP2PWrapper — the public wrapper facade (component C3).

Parity: ``lib/hlsjs-p2p-wrapper.js:8-41``.  Builds the private orchestrator with the real
peer agent injected, binds ``createPlayer`` / ``createSRModule``, snapshots ``P2PLoader``
once, and exposes:

* ``stats`` → the agent's ``{cdn, p2p, upload, peers}`` (raises before a session exists,
  like the reference's ``wrapper.peerAgentModule.stats`` on ``undefined``);
* ``p2pDownloadOn`` / ``p2pUploadOn`` read/write, forwarded to the agent;
* static ``HlsjsP2PWrapper.version``.
"""
from __future__ import annotations

from typing import Any

from ..agent.peer_agent import PeerAgent
from .wrapper_private import HlsjsP2PWrapperPrivate


class _Version:
    def __get__(self, obj, owner):
        return HlsjsP2PWrapperPrivate.version


class HlsjsP2PWrapper:
    """Wrapper around a media-engine constructor: ``createPlayer(hlsjsConfig, p2pConfig)`` builds an
    engine with a P2P session attached once its manifest starts loading; ``P2PLoader`` is the
    fragment-loader class for engines built by hand."""

    version = _Version()

    def __init__(self, hlsjsConstructor: Any = None, peerAgentConstructor: Any = PeerAgent) -> None:
        wrapper = HlsjsP2PWrapperPrivate(hlsjsConstructor, peerAgentConstructor)
        self._wrapper = wrapper
        self.createPlayer = wrapper.createPlayer
        self.createSRModule = wrapper.createSRModule
        self.P2PLoader = wrapper.P2PLoader

    @property
    def stats(self):
        """The session's ``{cdn, p2p, upload, peers}`` byte / peer counters (raises before a session)."""
        agent = self._wrapper.peerAgentModule
        if agent is None:
            raise TypeError("Cannot read property 'stats' of undefined (no P2P session)")
        return agent.stats

    @property
    def p2pDownloadOn(self) -> bool:
        """Read / write: fetch fragments from peers (``False`` = CDN only)."""
        return self._require().p2pDownloadOn

    @p2pDownloadOn.setter
    def p2pDownloadOn(self, on: bool) -> None:
        self._require().p2pDownloadOn = on

    @property
    def p2pUploadOn(self) -> bool:
        """Read / write: serve cached fragments to peers."""
        return self._require().p2pUploadOn

    @p2pUploadOn.setter
    def p2pUploadOn(self, on: bool) -> None:
        self._require().p2pUploadOn = on

    def _require(self):
        agent = self._wrapper.peerAgentModule
        if agent is None:
            raise TypeError("Cannot read property of undefined (no P2P session)")
        return agent

    # python conveniences
    create_player = property(lambda self: self.createPlayer, doc="snake_case alias of ``createPlayer``")
    create_sr_module = property(lambda self: self.createSRModule, doc="snake_case alias of ``createSRModule``")
