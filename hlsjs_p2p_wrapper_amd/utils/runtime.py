"""Process-level runtime tuning for long-running peers.

Python's cyclic GC periodically re-traverses every long-lived container object: the
parsed playlists (thousands of ``Fragment`` objects per level), the engine, the swarm
node.  A full (gen-2) pass over a 5-rendition ladder's state costs tens of milliseconds
and lands in the middle of a swarm round.  After start-up, :func:`tune_gc` moves
everything alive into the permanent generation (``gc.freeze``) and raises the gen-0
threshold, so collections only look at young objects.  The per-fragment churn (loader
stats, event payloads, closures) is mostly freed by reference counting anyway.  GC stays
enabled: new cycles are still collected.
"""
from __future__ import annotations

import gc
from typing import Tuple


def tune_gc(gen0_threshold: int = 50_000) -> Tuple[int, int, int]:
    """Collect once, freeze the surviving heap, raise the gen-0 threshold.

    Call it after the player / node / origin are set up (``bench.py`` does).  Returns the
    previous thresholds."""
    prev = gc.get_threshold()
    gc.collect()
    gc.freeze()
    gc.set_threshold(gen0_threshold, prev[1], prev[2])
    return prev
