"""Metrics / observability export.

The reference exposes cumulative byte counters through ``wrapper.stats`` =
``{cdn, p2p, upload, peers}`` (``wrapper.js:14-18``) and leaves plotting to external
demo widgets (``example/bundle/index.html:13-14``: ``p2pGraph.js`` / ``peerStat.js``).
Here the same counters — plus what only a GPU swarm node has: swarm-wide totals from the
round header, the offload ratio ``p2p / (p2p + cdn)``, HBM cache occupancy, CRC
failures, per-phase host time and per-request latency quantiles — are rendered in the
Prometheus text exposition format, so a serving fleet scrapes every rank the same way.

* :func:`node_metrics` — one snapshot ``[(name, type, help, [(labels, value)])]``.
* :func:`render` — the text format (``# HELP`` / ``# TYPE`` / samples).
* :class:`MetricsServer` — ``GET /metrics`` on a daemon thread (stdlib ``http.server``;
  nothing GPU-side runs on that thread, it reads host counters only), and ``GET /healthz``
  (:func:`health`: ``ok`` / ``starting`` / ``failed`` with the reason -- a divergence, a lost
  peer, a failed or stalled round -- as JSON, HTTP 503 once failed) for a serving fleet's
  liveness probe.

No dependency on ``prometheus_client``: the format is small and a registry would copy
counters the node already keeps.
"""
from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, Iterable, List, Optional, Sequence, Tuple

Sample = Tuple[Dict[str, str], float]
Family = Tuple[str, str, str, List[Sample]]

PREFIX = "hlsp2p_"

# node.stats key -> (metric suffix, help); all cumulative since the node started
_NODE_COUNTERS = (
    ("cdn", "cdn_bytes_total", "Bytes this rank fetched from the origin (CDN fallback)."),
    ("p2p", "p2p_bytes_total",
     "Bytes this rank received from peers and delivered after their CRC check passed (or pending it)."),
    ("p2p_wire", "p2p_wire_bytes_total", "Bytes this rank received from peers over the data plane (checked or not)."),
    ("p2p_rejected", "p2p_rejected_bytes_total", "Peer bytes whose CRC check failed (re-fetched from the CDN)."),
    ("upload", "upload_bytes_total", "Bytes this rank sent to peers."),
    ("cache", "cache_hit_bytes_total", "Bytes served from this rank's HBM cache."),
    ("segments", "segments_total", "Segments delivered by this rank."),
    ("cdn_segments", "cdn_segments_total", "Segments this rank fetched from the origin."),
    ("p2p_segments", "p2p_segments_total", "Segments this rank received from peers."),
    ("prefetched", "prefetched_total", "Prefetch requests accepted by this rank."),
    ("rounds", "rounds_total", "Swarm rounds completed."),
    ("crc_failures", "crc_failures_total", "Received segments whose CRC did not match (re-fetched)."),
    ("deferred", "deferred_total", "Wants deferred to a later round by cache backpressure."),
    ("cache_segments", "cache_hit_segments_total", "Segments served from this rank's HBM cache."),
)


def _esc(v: str) -> str:
    return v.replace("\\", "\\\\").replace("\n", "\\n").replace('"', '\\"')


def _fmt(v: float) -> str:
    if v != v:  # NaN
        return "NaN"
    if float(v).is_integer() and abs(v) < 1e15:
        return str(int(v))
    return repr(float(v))


def render(families: Iterable[Family]) -> str:
    """Prometheus text exposition format 0.0.4.  Families with the same name (one per
    agent, say) are merged so each name gets a single ``# HELP`` / ``# TYPE`` block."""
    merged: Dict[str, Family] = {}
    for name, kind, help_, samples in families:
        if name in merged:
            merged[name][3].extend(samples)
        else:
            merged[name] = (name, kind, help_, list(samples))
    out: List[str] = []
    for name, kind, help_, samples in merged.values():
        out.append(f"# HELP {name} {help_}")
        out.append(f"# TYPE {name} {kind}")
        for labels, value in samples:
            # a summary's _sum / _count series ride in the family with a "__suffix" pseudo-label
            suffix = labels.get("__suffix", "")
            lab = ",".join(f'{k}="{_esc(str(v))}"' for k, v in labels.items() if k != "__suffix")
            out.append(f"{name}{suffix}{{{lab}}} {_fmt(value)}" if lab else f"{name}{suffix} {_fmt(value)}")
    return "\n".join(out) + "\n"


def node_metrics(node: Any, quantiles: Sequence[float] = (0.5, 0.9, 0.99)) -> List[Family]:
    """Snapshot of one :class:`~hlsjs_p2p_wrapper_amd.agent.node.SwarmNode`."""
    base = {"rank": str(node.rank)}
    fams: List[Family] = []
    st = node.stats
    for key, suffix, help_ in _NODE_COUNTERS:
        fams.append((PREFIX + suffix, "counter", help_, [(dict(base), float(st.get(key, 0)))]))
    sw = node.swarm_stats
    fams.append((PREFIX + "swarm_bytes_total", "counter",
                 "Swarm-wide bytes by source, summed over ranks (round header).",
                 [(dict(base, source=s), float(sw.get(s, 0))) for s in ("cdn", "p2p", "upload")]))
    fams.append((PREFIX + "swarm_offload_ratio", "gauge", "Swarm-wide p2p / (p2p + cdn).",
                 [(dict(base), float(node.swarm_offload_ratio()))]))
    mine = st.get("cdn", 0) + st.get("p2p", 0)
    fams.append((PREFIX + "offload_ratio", "gauge", "This rank's p2p / (p2p + cdn).",
                 [(dict(base), st.get("p2p", 0) / mine if mine else 0.0)]))
    online = getattr(node, "peer_online", None)
    peers = int(online.sum()) - 1 if (online is not None and getattr(node, "online", True)) else 0
    fams.append((PREFIX + "peers", "gauge", "Peers online in the swarm (excluding this rank).",
                 [(dict(base), float(max(0, peers)))]))
    fams.append((PREFIX + "world_size", "gauge", "Ranks in the swarm.", [(dict(base), float(node.world))]))
    fams.append((PREFIX + "node_failed", "gauge",
                 "1 once this rank saw a divergence, a lost peer or a failed round (GET /healthz says which).",
                 [(dict(base), 1.0 if getattr(node, "failed", None) else 0.0)]))
    last = getattr(node, "last_complete", None)
    if last is not None:
        fams.append((PREFIX + "seconds_since_last_round", "gauge", "Seconds since this rank's last round completed.",
                     [(dict(base), max(0.0, time.monotonic() - last))]))
    store = node.store
    fams.append((PREFIX + "cache_capacity_bytes", "gauge", "HBM segment-cache arena size.",
                 [(dict(base), float(store.capacity))]))
    fams.append((PREFIX + "cache_used_bytes", "gauge", "HBM segment-cache bytes in use.",
                 [(dict(base), float(store.used_bytes))]))
    fams.append((PREFIX + "cache_entries", "gauge", "Segments resident in the HBM cache.",
                 [(dict(base), float(store.num_entries))]))
    fams.append((PREFIX + "cache_evictions_total", "counter", "Segments evicted from the HBM cache.",
                 [(dict(base), float(store.evictions))]))
    fams.append((PREFIX + "cache_unpin_underflows_total", "counter",
                 "Unpins of live cache entries that held no pin (a holder gave up a pin it did not own; "
                 "0 when the bookkeeping is sound, see agent/audit.py).",
                 [(dict(base), float(getattr(store, "unpin_underflows", 0)))]))
    timer = node.timer
    totals, counts = dict(timer.total), dict(timer.count)  # C-level copies: the round loop keeps adding
    fams.append((PREFIX + "phase_seconds_total", "counter", "Host wall time per round phase.",
                 [(dict(base, phase=k), float(v)) for k, v in sorted(totals.items())]))
    fams.append((PREFIX + "phase_calls_total", "counter", "Round phase executions.",
                 [(dict(base, phase=k), float(v)) for k, v in sorted(counts.items())]))
    trace = getattr(node, "trace", None)
    if trace is not None and len(trace):
        # one snapshot, grouped by source in one pass, each group sorted once
        samples: List[Sample] = []
        for src, (n, sum_ms, qs) in sorted(trace.latency_summary(quantiles).items()):
            for q, ms in qs:
                samples.append((dict(base, source=src, quantile=str(q)), ms / 1e3))
            samples.append(({**base, "source": src, "__suffix": "_sum"}, sum_ms / 1e3))
            samples.append(({**base, "source": src, "__suffix": "_count"}, float(n)))
        fams.append((PREFIX + "request_latency_seconds", "summary",
                     "Request latency (submit -> delivered) by source over the retained trace log (the "
                     "last gpuSwarm.trace records, lifetime rather than a time window); the unit follows "
                     "the event-loop clock (virtual time under the virtual loop).", samples))
    return fams


def agent_metrics(agent: Any, index: int = 0, rank: Optional[int] = None) -> List[Family]:
    """The reference ``stats`` object (``{cdn, p2p, upload, peers}``) of one peer agent.

    Labelled by ``rank`` and ``agent`` (the attach index on its node) besides ``content``:
    two players on one node watching the same stream would otherwise emit identical label
    sets (``contentId`` defaults to ``contentUrl``)."""
    s = agent.stats
    if rank is None:
        node = getattr(agent, "node", None)
        rank = getattr(node, "rank", 0) if node is not None else 0
    lab = {"rank": str(rank), "agent": str(index), "content": str(getattr(agent, "contentId", "") or "")}
    return [
        (PREFIX + "agent_bytes_total", "counter", "Per-session bytes (wrapper.stats).",
         [(dict(lab, source=k), float(s[k])) for k in ("cdn", "p2p", "upload")]),
        (PREFIX + "agent_peers", "gauge", "Peers (wrapper.stats.peers).", [(dict(lab), float(s["peers"]))]),
    ]


def health(node: Any, stall_s: Optional[float] = None) -> Dict[str, Any]:
    """Liveness of one node for ``GET /healthz``: ``ok`` (rounds completing), ``starting`` (no
    round completed yet), or ``failed`` -- the node saw a divergence, a lost peer or a failed
    round (``reason``), is closed, or its last round completed longer ago than ``stall_s``
    (default: the node's round deadline, ``gpuSwarm.roundTimeoutMs``)."""
    last = getattr(node, "last_complete", None)
    since = None if last is None else max(0.0, time.monotonic() - last)
    if stall_s is None:
        deadline = getattr(node, "round_deadline_s", None)
        stall_s = float(deadline()) if callable(deadline) else 60.0
    out: Dict[str, Any] = {"rank": int(getattr(node, "rank", 0)), "world": int(getattr(node, "world", 1)),
                           "round": int(getattr(node, "round", 0)), "seconds_since_last_round": since}
    reason = getattr(node, "failed", None)
    if reason is None and getattr(node, "closed", False):
        reason = "node closed"
    if reason is None and since is not None and getattr(node, "auto_tick", False) and since > stall_s:
        reason = f"no round completed for {since:.1f} s (> {stall_s:g} s)"
    out["status"] = "failed" if reason else ("starting" if since is None else "ok")
    if reason:
        out["reason"] = reason
    return out


class MetricsServer:
    """``GET /metrics`` for one node (and optionally its agents) on a daemon thread, and
    ``GET /healthz`` (:func:`health` as JSON; HTTP 503 once the node failed).

    ``port=0`` binds an ephemeral port (``.port`` reports it).  Binds 127.0.0.1 unless told
    otherwise: the counters are not secret, but exposure is the operator's choice."""

    def __init__(self, node: Any, port: int = 0, host: str = "127.0.0.1", agents: Optional[List[Any]] = None) -> None:
        self.node = node
        self.agents = agents
        outer = self

        class _Handler(BaseHTTPRequestHandler):
            def do_GET(self) -> None:  # noqa: N802 - http.server API
                path = self.path.split("?")[0]
                if path == "/healthz":
                    h = health(outer.node)
                    body = json.dumps(h).encode()
                    self.send_response(503 if h["status"] == "failed" else 200)
                    self.send_header("Content-Type", "application/json")
                    self.send_header("Content-Length", str(len(body)))
                    self.end_headers()
                    self.wfile.write(body)
                    return
                if path != "/metrics":
                    self.send_error(404)
                    return
                body = outer.text().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4; charset=utf-8")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *args: Any) -> None:  # scrapes are not log lines
                pass

        self._srv = ThreadingHTTPServer((host, port), _Handler)
        self._srv.daemon_threads = True
        self.port = self._srv.server_address[1]
        self._thread = threading.Thread(target=self._srv.serve_forever, name="hlsp2p-metrics", daemon=True)
        self._thread.start()

    def text(self) -> str:
        """Current exposition text (node families, then one set per agent)."""
        fams = node_metrics(self.node)
        agents = self.agents if self.agents is not None else getattr(self.node, "_agents", [])
        for i, a in enumerate(list(agents)):
            fams.extend(agent_metrics(a, i, getattr(self.node, "rank", 0)))
        return render(fams)

    def close(self) -> None:
        """Stop serving and release the port."""
        self._srv.shutdown()
        self._srv.server_close()
        self._thread.join(timeout=5)
