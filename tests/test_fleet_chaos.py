"""Fleet chaos at fixed seeds (``tests/fleet_chaos.py``): player threads on pipes to the
node-side loop of one or more ranks, with random caches, in-flight windows, payload modes,
byte read-back and scripted seeks / pauses / level switches / restarts.

* Seeds 4 and 5 (one rank) caught an on-demand player's ``RemoteSegment.data()`` returning
  nothing: the delivered entries lost their in-flight pins when the next round launched,
  before the answer batch went out, and a small cache overwrote them before the player read
  them.  Delivered entries now stay pinned from ``FleetServer.deliver`` until the player
  handled the batch.
* Seeds 1, 4 and 32 (two ranks) caught it again another way: a second request for a segment
  whose peer copy was delivered and still awaited its deferred check fetched the segment
  again, and the new copy took the index slot -- pending, so the first player's fetch found
  nothing.  The request now waits for the check (``SwarmNode._park_on_pending``), and a fetch
  reads the exact copy the player was answered with while its batch holds it.
* Seed 8 (three ranks) looked like a player stalled on an unanswered fragment (about 1 run in
  7): the harness had stopped the scenario once every player was at the end, before a
  scripted seek sent one back.  Scenarios now end only after every script ran.
* Live (``live=True``): a switched-to level's first playlist off the playback timeline and a
  seek behind the sliding window stalled players (see ``test_fleet_chaos_live``)."""
import pytest

import fleet_chaos


@pytest.mark.parametrize("seed,ranks", [(0, 1), (4, 1), (5, 1), (11, 1), (1, 2), (4, 2), (32, 2), (8, 3)])
def test_fleet_chaos_seed(seed, ranks):
    fleet_chaos.check(fleet_chaos.scenario(seed, ranks=ranks))


@pytest.mark.parametrize("seed", [3, 15])
def test_fleet_chaos_with_faults(seed):
    """Three ranks that corrupt received rounds and go offline at random times (the two seeds
    hit CRC failures with requests parked on copies awaiting their check)."""
    res = fleet_chaos.scenario(seed, ranks=3, faults=True)
    fleet_chaos.check(res)
    assert any(f for f in res["faults"])


@pytest.mark.parametrize("seed,ranks", [(10, 1), (3, 2), (8, 2), (18, 2)])
def test_fleet_chaos_live(seed, ranks):
    """A live channel (sliding window, live-window eviction, seeks back into the window).  Seed 10
    stalled on a switched-to level's unaligned first playlist, seeds 8 and 18 on a seek behind
    the window (two ranks, with faults)."""
    fleet_chaos.check(fleet_chaos.scenario(seed, ranks=ranks, faults=ranks > 1, live=True))


@pytest.mark.parametrize("seed,ranks", [(1, 1), (2, 1), (5, 2)])
def test_fleet_chaos_payload_ring(seed, ranks):
    """Every player on payloads through a ring that starts at 1 MiB and grows (a first batch
    bigger than the configured ring raised inside the rank: seeds 1 and 2)."""
    fleet_chaos.check(fleet_chaos.scenario(seed, ranks=ranks, faults=ranks > 1, ring=True))


@pytest.mark.gpu
@pytest.mark.parametrize("seed,ranks,live,faults", [(4, 1, False, False), (5, 1, False, False),
                                                    (11, 1, False, False), (4, 2, False, False),
                                                    (32, 2, False, False), (3, 2, True, False),
                                                    (7, 2, False, True)])
def test_fleet_chaos_seed_gpu(seed, ranks, live, faults):
    """The nodes' caches are HBM rings and the transmux runs on the GPU: the on-demand bytes a
    player reads back come off the device (two ranks: both on the one GPU; with faults, the GPU
    decrypt / demux rejects corrupted CDN copies and the players invalidate them)."""
    fleet_chaos.check(fleet_chaos.scenario(seed, device="cuda:0", ranks=ranks, live=live, faults=faults))
