"""L3 integration adapters: the P2P fragment loader and the player bridge."""
from .p2p_loader import p2p_loader_generator, P2PLoaderGenerator
from .player_interface import PlayerInterface

__all__ = ["p2p_loader_generator", "P2PLoaderGenerator", "PlayerInterface"]
