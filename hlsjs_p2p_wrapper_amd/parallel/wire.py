"""Which wire the native RCCL data plane actually runs on.

``data_transport == "rccl-native"`` only says that the node's own RCCL communicator opened.
RCCL then picks a transport per peer pair when the first send/recv connects it: on one
MI355X node that is ``P2P/IPC`` (or ``P2P/direct pointer``) over xGMI, but a box without
the P2P path (no ``iommu=pt``, a container without the peers' devices, NUMA policy...) falls
back to ``NET/Socket`` and still "works", at a fraction of the rate.  A multi-GPU record must
say which one it measured.

Two independent sources:

* **RCCL's own connection log.**  Before the first RCCL call of the process,
  :func:`configure_rccl_log` points RCCL's INFO output for the INIT / P2P / NET subsystems at
  a per-rank file (``NCCL_DEBUG=INFO``, ``NCCL_DEBUG_SUBSYS``, ``NCCL_DEBUG_FILE``; no per-op
  logging: those lines are in the COLL subsystem, which stays off).  Every connection RCCL
  sets up is one line ``Channel cc/k : a[..] -> b[..] [send|receive] via <TRANSPORT>``
  (format strings of librccl: ``via P2P/IPC``, ``via P2P/direct pointer``,
  ``via P2P/CUMEM``, ``via NET/Socket/0``, ``via SHM/direct/direct``); the init line
  ``comm .. rank r nRanks n nNodes m localRanks l ..`` gives how many hosts RCCL believes the
  group spans.  :func:`parse_rccl_log` turns the file into ``{peer: [transports]}``.
* **HIP's link table.**  ``hipExtGetLinkTypeAndHopCount`` between this rank's device and
  each peer's (``link_types``): ``XGMI`` on an MI355X node, ``PCIE`` otherwise.

``summarize`` classifies the result: ``p2p`` (every peer over RCCL's P2P transport), ``net``
(some peer over a network transport: degraded on one node), ``self`` (a world of one: sends to
self are local copies, RCCL connects nothing), ``unknown`` (no log: the user configured RCCL's
debug output, or the plane never connected).
"""
from __future__ import annotations

import os
import re
import tempfile
from typing import Dict, List, Optional

# "Channel 00/1 : 0[0] -> 1[1] via P2P/IPC comm 0x.. nRanks 02"
# "Channel 00/1 : 0[c1000] -> 1[c1000] [send] via NET/Socket/0 comm 0x.. nRanks 02"
# "Channel 00 : 0[0] -> 1[1] via SHM/direct/direct comm 0x.. nRanks 02"
_CHANNEL = re.compile(r"Channel\s+\d+(?:/\d+)?\s*:\s*(\d+)\[[0-9a-fA-Fx]*\]\s*->\s*(\d+)\[[0-9a-fA-Fx]*\]\s*"
                      r"(?:\[(send|receive)\]\s*)?via\s+(\S+(?: pointer)?)")
_INIT = re.compile(r"rank\s+(\d+)\s+nRanks\s+(\d+)\s+nNodes\s+(\d+)\s+localRanks\s+(\d+)")

LINK_TYPES = {0: "HYPERTRANSPORT", 1: "QPI", 2: "PCIE", 3: "INFINIBAND", 4: "XGMI"}

# One MI355X xGMI link, per direction: 153.6 GB/s is the bidirectional figure of a link (7 links,
# ~1.07 TB/s per GPU in aggregate), so a receiver's roofline is 76.8 GB/s per source link and
# 7 x 76.8 = 537.6 GB/s from all seven peers of an 8-GPU node.
XGMI_LINK_GBPS_PER_DIR = 76.8
XGMI_LINKS = 7


def configure_rccl_log(rank: int, directory: Optional[str] = None) -> Optional[str]:
    """Point RCCL's connection log at a per-rank file; returns its path, or None with
    ``HLSP2P_RCCL_WIRE_LOG=0`` or when the user asked for RCCL's INFO output on the console
    (``NCCL_DEBUG=INFO`` without a file: kept as is).  A user's INFO / TRACE file is read back
    where it is; a lower level (``VERSION`` / ``WARN``, as the GPU pool's environment sets) is
    raised to INFO into the file, whose warnings :func:`read_rccl_log` forwards to the log.
    Must run before the process's first RCCL call: RCCL reads these variables once."""
    if os.environ.get("HLSP2P_RCCL_WIRE_LOG", "1") == "0":
        return None
    level = os.environ.get("NCCL_DEBUG", "").upper()
    if level in ("INFO", "TRACE"):
        f = os.environ.get("NCCL_DEBUG_FILE")
        if f:
            return f.replace("%h", os.uname().nodename).replace("%p", str(os.getpid()))
        return None
    d = directory or os.environ.get("HLSP2P_RCCL_LOG_DIR") or tempfile.gettempdir()
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"hlsp2p-rccl.{os.getpid()}.rank{rank}.log")
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,P2P,NET")
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


def parse_rccl_log(text: str, me: Optional[int] = None) -> Dict[str, object]:
    """``{"peers": {peer: sorted transports}, "n_ranks", "n_nodes", "local_ranks",
    "connections"}`` from RCCL's log of one rank (``me``: that rank; a line is counted when it
    has ``me`` on one side and another rank on the other).  Transports are RCCL's labels
    without the channel detail: ``P2P/IPC``, ``P2P/direct pointer``, ``NET/Socket``, ..."""
    peers: Dict[int, set] = {}
    n = 0
    init = None
    for ln in text.splitlines():
        m = _CHANNEL.search(ln)
        if m is not None:
            a, b, _, via = int(m.group(1)), int(m.group(2)), m.group(3), m.group(4)
            if me is not None and me not in (a, b):
                continue
            other = b if (me is None or a == me) else a
            if me is not None and other == me:
                continue
            peers.setdefault(other, set()).add(_label(via))
            n += 1
            continue
        m = _INIT.search(ln)
        if m is not None and (me is None or int(m.group(1)) == me):
            init = (int(m.group(2)), int(m.group(3)), int(m.group(4)))
    return {"peers": {str(p): sorted(v) for p, v in sorted(peers.items())},
            "n_ranks": init[0] if init else None, "n_nodes": init[1] if init else None,
            "local_ranks": init[2] if init else None, "connections": n}


def _label(via: str) -> str:
    """``NET/Socket/0`` -> ``NET/Socket``; ``P2P/IPC/read`` -> ``P2P/IPC``; ``SHM/direct/direct``
    -> ``SHM/direct``: the transport and its mechanism, not the device / channel suffix."""
    parts = via.split("/")
    return "/".join(parts[:2])


def read_rccl_log(path: Optional[str], me: int) -> Optional[Dict[str, object]]:
    if not path:
        return None
    try:
        with open(path, errors="replace") as f:
            text = f.read()
    except OSError:
        return None
    out = parse_rccl_log(text, me)
    out["log"] = path
    out["log_bytes"] = len(text)
    warns = [ln for ln in text.splitlines() if " NCCL WARN " in ln]
    out["warnings"] = len(warns)
    if warns:
        import logging

        lg = logging.getLogger("hlsjs_p2p_wrapper_amd.rccl")
        seen = []
        for ln in warns:  # RCCL's own warnings went to the file: surface the distinct ones
            w = ln.split(" NCCL WARN ", 1)[1]
            if w not in seen:
                seen.append(w)
        for w in seen[:8]:
            lg.warning("rank %d RCCL: %s", me, w)
    return out


def summarize(report: Optional[Dict[str, object]], world: int) -> str:
    """``p2p`` / ``net`` / ``shm`` / ``self`` / ``unknown`` for one rank's parsed log."""
    if report is None:
        return "unknown"
    peers = report.get("peers") or {}
    if not peers:
        return "self" if world == 1 and report.get("n_ranks") == 1 else "unknown"
    kinds = {t.split("/")[0] for ts in peers.values() for t in ts}
    if "NET" in kinds or "COLLNET" in kinds:
        return "net"
    if kinds == {"P2P"}:
        return "p2p" if len(peers) >= world - 1 else "p2p-partial"
    if kinds <= {"P2P", "SHM"}:
        return "shm"
    return "unknown"


def link_types(device: int, peers: Dict[int, int]) -> Dict[str, object]:
    """HIP's link type and hop count from ``device`` to each peer rank's device index
    (``{rank: device}``; same visible-device numbering on every rank of one host)."""
    from ..ops._native import device as _dev

    d = _dev()
    out: Dict[str, object] = {}
    for r, pd in sorted(peers.items()):
        if pd == device:
            out[str(r)] = "same-device"
            continue
        try:
            t, hops = d.link_type(int(device), int(pd))
            out[str(r)] = f"{LINK_TYPES.get(int(t), str(t))}/{int(hops)}"
        except Exception as e:  # noqa: BLE001 - reported, not fatal
            out[str(r)] = f"error: {e}"
    return out


def degraded(plane: str, distinct_devices: Optional[bool], rehearsal: Optional[str],
             wires: List[str]) -> bool:
    """A run on the native RCCL plane with one GPU per rank must use RCCL's P2P transport
    (xGMI); any rank whose peers connected over a network transport, or through host shared
    memory (P2P access refused between the GPUs), is degraded."""
    return bool(plane.startswith("rccl") and distinct_devices and not rehearsal
                and ("net" in wires or "shm" in wires))


def link_kinds(ranks: List[dict]) -> List[str]:
    """The distinct HIP link types (``XGMI``, ``PCIE``, ...) between the ranks' devices, from
    every rank's ``comm.wire.links`` (one GPU per rank on one host)."""
    kinds = set()
    for r in ranks:
        links = (r.get("comm") or {}).get("wire", {}).get("links")
        if isinstance(links, dict):
            for v in links.values():
                if isinstance(v, str) and "/" in v:
                    kinds.add(v.split("/")[0])
    return sorted(kinds)
