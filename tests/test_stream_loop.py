"""The stream loop's in-flight run end (``StreamController._run_end``): the O(1) chain path
must give exactly what one pass over every fragment in flight gives, through loads,
in-order and out-of-order completions, aborts, re-inserted keys and start rewrites."""
import numpy as np

from hlsjs_p2p_wrapper_amd.player.controllers import StreamController, _Inflight
from hlsjs_p2p_wrapper_amd.player.level import Fragment


def _reference(inflight, nxt):
    for f in inflight.values():
        if f.start + f.duration > nxt and f.start <= nxt + 0.5:
            nxt = f.start + f.duration
    return nxt


def _controller():
    sc = StreamController.__new__(StreamController)
    sc.inflight = _Inflight()
    sc._chain_gen = -1
    sc.run_scans = 0
    return sc


def test_run_end_matches_the_full_pass_under_random_operations():
    rng = np.random.default_rng(5)
    for trial in range(40):
        sc = _controller()
        frags = [Fragment(f"s{i}.ts", i, 4.0 * i, 4.0) for i in range(400)]
        nxt_sn = 0
        buf_end = 0.0
        calls = 0
        for step in range(300):
            op = rng.random()
            if op < 0.45 and nxt_sn < len(frags):  # load the next fragment(s) in order
                for _ in range(int(rng.integers(1, 4))):
                    if nxt_sn < len(frags):
                        f = frags[nxt_sn]
                        sc.inflight[(0, f.sn)] = f
                        nxt_sn += 1
            elif op < 0.75 and sc.inflight:  # the oldest completes: the buffer grows over it
                k = next(iter(sc.inflight))
                f = sc.inflight.pop(k)
                buf_end = max(buf_end, f.start + f.duration)
            elif op < 0.83 and sc.inflight:  # one in the middle completes or is aborted
                keys = list(sc.inflight)
                sc.inflight.pop(keys[int(rng.integers(0, len(keys)))], None)
            elif op < 0.87 and sc.inflight:  # a key loaded again (a retry of a fragment in flight)
                k = list(sc.inflight)[int(rng.integers(0, len(sc.inflight)))]
                sc.inflight[k] = sc.inflight[k]
            elif op < 0.90:  # a live playlist refresh moves a fragment's start
                f = frags[int(rng.integers(0, len(frags)))]
                f.start = f.start + float(rng.choice([-0.3, 0.0, 0.7]))
            elif op < 0.93:  # a seek: the buffer ends elsewhere
                buf_end = float(rng.integers(0, 1600))
            elif op < 0.95:
                sc.inflight.clear()
            want = _reference(sc.inflight, buf_end)
            calls += bool(sc.inflight)
            got = sc._run_end(buf_end)
            assert got == want, (trial, step)
        assert sc.run_scans < calls  # the O(1) path was taken


def test_run_end_of_an_in_order_chain_is_the_newest_end_without_a_scan():
    sc = _controller()
    frags = [Fragment(f"s{i}.ts", i, 4.0 * i, 4.0) for i in range(256)]
    for f in frags:
        sc.inflight[(0, f.sn)] = f
    assert sc._run_end(0.0) == 1024.0 and sc.run_scans == 1  # first call scans (generation unknown)
    sc.inflight.pop((0, 0))
    sc.inflight[(0, 256)] = Fragment("s256.ts", 256, 1024.0, 4.0)
    assert sc.inflight.chain_ok and sc._run_end(4.0) == 1028.0 and sc.run_scans == 1
    sc.inflight.pop((0, 100))  # a gap: the next call scans and stops at it
    assert not sc.inflight.chain_ok and sc._run_end(4.0) == 400.0 and sc.run_scans == 2
