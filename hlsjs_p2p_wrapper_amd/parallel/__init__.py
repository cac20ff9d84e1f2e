"""Swarm parallelism: one MI355X = one peer; RCCL over xGMI between peers."""
from .comm import DistComm, LocalComm, SwarmComm, ThreadComm, ThreadHub

__all__ = ["SwarmComm", "LocalComm", "ThreadHub", "ThreadComm", "DistComm"]
