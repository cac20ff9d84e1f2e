"""Tracing / profiling helpers.

* :class:`PhaseTimer` — cheap host-side accumulation of named phase durations
  (``with timer("cdn"): ...``) used by the swarm node, the media pipeline and the bench
  to attribute wall time per round.
* :class:`RequestTrace` — per-request record ``{key, trequest, tfirst, tload, source,
  bytes, peer}`` kept (bounded) by the node when tracing is enabled.
* Device time comes from HIP events (node) and ``rocprofv3 --kernel-trace --stats``.
"""
from __future__ import annotations

import time
from collections import defaultdict, deque, namedtuple
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Deque, Dict, Iterator, List, Optional, Sequence, Tuple


class PhaseTimer:
    __slots__ = ("enabled", "total", "count")

    def __init__(self, enabled: bool = True) -> None:
        self.enabled = enabled
        self.total: Dict[str, float] = defaultdict(float)
        self.count: Dict[str, int] = defaultdict(int)

    @contextmanager
    def __call__(self, name: str) -> Iterator[None]:
        if not self.enabled:
            yield
            return
        t = time.perf_counter()
        try:
            yield
        finally:
            self.total[name] += time.perf_counter() - t
            self.count[name] += 1

    def add(self, name: str, seconds: float) -> None:
        if self.enabled:
            self.total[name] += seconds
            self.count[name] += 1

    def reset(self) -> None:
        self.total.clear()
        self.count.clear()

    def summary_ms(self, per: Optional[int] = None) -> Dict[str, float]:
        div = per or 1
        return {k: round(v * 1e3 / div, 4) for k, v in sorted(self.total.items(), key=lambda kv: -kv[1])}


@dataclass
class RequestTrace:
    """One delivered request.  Times are event-loop milliseconds (``performance.now``
    analog): ``trequest`` = submitted to the node, ``tfirst`` = device transfer start
    (``tload`` minus the HIP-event-timed H2D / RCCL duration of its round), ``tload`` =
    delivered.  ``peer`` = rank the bytes came from (own rank for CDN / cache)."""

    key: Tuple[int, int, int, int]
    trequest: float
    tfirst: float
    tload: float
    source: str
    bytes: int
    peer: int
    round: int


# count, sum of latencies (ms), [(quantile, latency ms)]
LatencySummary = namedtuple("LatencySummary", ["count", "sum_ms", "quantiles_ms"])


class TraceLog:
    def __init__(self, maxlen: int = 100_000) -> None:
        self.records: Deque[RequestTrace] = deque(maxlen=maxlen)

    def add(self, rec: RequestTrace) -> None:
        self.records.append(rec)

    def __len__(self) -> int:
        return len(self.records)

    def by_source(self) -> Dict[str, Tuple[int, int]]:
        """``{source: (requests, bytes)}``."""
        out: Dict[str, Tuple[int, int]] = {}
        for r in list(self.records):
            n, b = out.get(r.source, (0, 0))
            out[r.source] = (n + 1, b + r.bytes)
        return out

    def latency_ms(self, q: float = 0.5, source: Optional[str] = None) -> float:
        """``q``-quantile of ``tload - trequest``."""
        xs = sorted(r.tload - r.trequest for r in list(self.records) if source is None or r.source == source)
        if not xs:
            return 0.0
        return xs[min(len(xs) - 1, int(q * len(xs)))]

    def latency_summary(self, quantiles: Sequence[float] = (0.5, 0.9, 0.99)
                        ) -> Dict[str, Tuple[int, float, List[Tuple[float, float]]]]:
        """Per-source latency summary of the whole retained log in ONE pass.

        Safe to call from another thread while the round loop appends: ``list(deque)`` is a
        single C-level copy under the GIL, so the snapshot never sees a mutation mid-loop.
        Each source's latencies are sorted once and every quantile is read from that sort.
        Values are event-loop milliseconds (virtual time under the ``virtual`` loop) over
        the retained records (the last ``maxlen`` requests), not a sliding time window."""
        groups: Dict[str, List[float]] = {}
        for r in list(self.records):
            groups.setdefault(r.source, []).append(r.tload - r.trequest)
        out: Dict[str, Tuple[int, float, List[Tuple[float, float]]]] = {}
        for src, xs in groups.items():
            xs.sort()
            n = len(xs)
            out[src] = LatencySummary(n, float(sum(xs)), [(q, xs[min(n - 1, int(q * n))]) for q in quantiles])
        return out

    def to_dicts(self):
        return [{"key": list(r.key), "trequest": r.trequest, "tfirst": r.tfirst, "tload": r.tload,
                 "source": r.source, "bytes": r.bytes, "peer": r.peer, "round": r.round} for r in self.records]
