"""Randomized swarm scenarios (``tests/swarm_chaos.py``) at fixed seeds: 2-4 in-process peers
with random caches (3-12 segments), start delays, in-flight windows, seeks, level switches,
offline periods, P2P download toggles, corrupted peer copies and deferred verification --
every peer plays to the end with no exception and no fatal media error.  A wider sweep:
``python tests/swarm_chaos.py 0 200``.

Seed 80 found a stream-loop livelock: after a seek to just before a buffered range, with
fragments in flight, the loop re-loaded the already-buffered fragments past the in-flight
run; each reload completed at once from the cache and re-kicked the loop, so (on the
virtual clock) time never advanced and the fragment under the playhead never arrived.
The loop now skips fragments already in the buffer.  Seed 119: that skip must not treat a
fragment as buffered when back-buffer eviction cut the range just past its start (a hole
the playhead stalls at).  Seed 153: a round's several ring reservations (CDN run, one run
per source peer) overlapped their own earlier runs when the total wrapped the ring; the
rank failed with "cannot make room" (a round now wraps before its first run: ``wrap_for``).
Seed 271: a seek that lands 0.2 s before a buffered range never completed -- the stream loop
counts the playhead as inside a range that starts within ``maxBufferHole`` and loads nothing,
the media has no data at the playhead; the loop now jumps such holes as hls.js does
(``BUFFER_SEEK_OVER_HOLE``)."""
import pytest

from swarm_chaos import check, scenario


@pytest.mark.parametrize("seed", [2, 9, 26, 29, 80, 119, 153, 208, 271])
def test_chaos_scenario(seed):
    check(scenario(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [80, 153, 271])
def test_chaos_scenario_on_the_gpu(cuda, seed):
    """The same scenarios with every peer's cache and transmux on the MI355X (streams, events
    and asynchronous copies under seeks, aborts, evictions and corrupted copies)."""
    check(scenario(seed, device="cuda:0"))
