"""The peer agent (``streamroot-p2p`` contract) and its MI355X swarm node."""
from .node import SwarmNode, current_node, node_for_config, set_current_node, swarm_id_for
from .peer_agent import PeerAgent

__all__ = ["PeerAgent", "SwarmNode", "current_node", "set_current_node", "node_for_config", "swarm_id_for"]
