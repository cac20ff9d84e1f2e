"""Fleet chaos at fixed seeds (``tests/fleet_chaos.py``): player threads on pipes to one
node-side loop, with random caches, in-flight windows, payload modes, byte read-back and
scripted seeks / pauses / level switches / restarts.

Seeds 4 and 5 caught an on-demand player's ``RemoteSegment.data()`` returning nothing: the
delivered entries lost their in-flight pins when the next round launched, before the answer
batch went out, and a small cache overwrote them before the player read them.  Delivered
entries now stay pinned from ``FleetServer.deliver`` until the player handled the batch."""
import pytest

import fleet_chaos


@pytest.mark.parametrize("seed", [0, 4, 5, 11])
def test_fleet_chaos_seed(seed):
    fleet_chaos.check(fleet_chaos.scenario(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5, 11])
def test_fleet_chaos_seed_gpu(seed):
    """The node's cache is the HBM ring and the transmux runs on the GPU: the on-demand
    bytes a player reads back come off the device."""
    fleet_chaos.check(fleet_chaos.scenario(seed, device="cuda:0"))
