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
from collections import defaultdict, deque
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Deque, Dict, Iterator, Optional, Tuple


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
        for r in self.records:
            n, b = out.get(r.source, (0, 0))
            out[r.source] = (n + 1, b + r.bytes)
        return out

    def latency_ms(self, q: float = 0.5, source: Optional[str] = None) -> float:
        """``q``-quantile of ``tload - trequest``."""
        xs = sorted(r.tload - r.trequest for r in self.records if source is None or r.source == source)
        if not xs:
            return 0.0
        return xs[min(len(xs) - 1, int(q * len(xs)))]

    def to_dicts(self):
        return [{"key": list(r.key), "trequest": r.trequest, "tfirst": r.tfirst, "tload": r.tload,
                 "source": r.source, "bytes": r.bytes, "peer": r.peer, "round": r.round} for r in self.records]
