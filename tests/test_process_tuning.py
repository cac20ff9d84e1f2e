"""Process-level tuning (``utils/runtime.py``): GC freeze and NUMA placement."""
import gc
import os

import pytest

from hlsjs_p2p_wrapper_amd.utils import runtime as rt


def test_tune_gc_freezes_and_raises_gen0():
    prev = gc.get_threshold()
    rt._freeze_after_full.full_passes = 0  # (the thawing pass is every 4th: not the one below)
    try:
        out = rt.tune_gc(12345)
        assert out == prev and gc.get_threshold()[0] == 12345 and gc.get_freeze_count() > 0
        # survivors of every later full collection are frozen too (long runs stay flat)
        kept = [[i] for i in range(1000)]
        before = gc.get_freeze_count()
        gc.collect(2)
        assert gc.get_freeze_count() >= before + len(kept)
        # cyclic garbage is still collected
        a = []
        a.append(a)
        del a
        assert gc.collect(0) >= 1
    finally:
        if rt._freeze_after_full in gc.callbacks:
            gc.callbacks.remove(rt._freeze_after_full)
        gc.unfreeze()
        gc.set_threshold(*prev)


def test_frozen_objects_that_become_cyclic_garbage_are_reclaimed():
    """an object alive at a freeze (e.g. a request in flight when a full pass
    ran) that later becomes part of a garbage cycle must not leak: every ``thaw_every``-th
    full pass thaws the permanent generation first and reclaims it."""
    import weakref

    class Node:
        pass

    prev = gc.get_threshold()
    holder = []
    try:
        a, b = Node(), Node()
        a.peer, b.peer = b, a  # a cycle, kept alive from outside for now
        holder.append(a)
        ref = weakref.ref(a)
        del a, b
        rt.tune_gc(12345, thaw_every=3)
        assert gc.get_freeze_count() > 0
        holder.clear()  # now cyclic garbage, inside the frozen generation
        passes = rt._freeze_after_full.full_passes
        while rt._freeze_after_full.full_passes < passes + 3 and ref() is not None:
            gc.collect(2)
        assert ref() is None
        assert rt._freeze_after_full.thaws >= 1
        assert gc.get_freeze_count() > 0  # the survivors are frozen again after the pass
    finally:
        if rt._freeze_after_full in gc.callbacks:
            gc.callbacks.remove(rt._freeze_after_full)
        gc.unfreeze()
        gc.set_threshold(*prev)


def test_parse_cpulist():
    assert rt._parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert rt._parse_cpulist("") == []


def test_bind_only_narrows_and_needs_enough_cpus(monkeypatch):
    allowed = os.sched_getaffinity(0)
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append(set(cpus)))
    # GPU unknown: nothing happens
    monkeypatch.setattr(rt, "gpu_local_cpus", lambda d: (None, []))
    assert rt.bind_to_gpu_numa(0) is None and not calls
    # too few allowed local CPUs: left alone
    few = sorted(allowed)[:2]
    monkeypatch.setattr(rt, "gpu_local_cpus", lambda d: (1, few + [10_000]))
    assert rt.bind_to_gpu_numa(0, min_cpus=8) is None and not calls
    # every allowed CPU is local: nothing to narrow, the node is reported
    monkeypatch.setattr(rt, "gpu_local_cpus", lambda d: (0, sorted(allowed) + [10_000]))
    assert rt.bind_to_gpu_numa(0, min_cpus=1) == 0 and not calls
    if len(allowed) < 2:
        pytest.skip("needs 2+ CPUs to narrow")
    half = sorted(allowed)[:len(allowed) // 2]
    monkeypatch.setattr(rt, "gpu_local_cpus", lambda d: (1, half + [10_000]))
    assert rt.bind_to_gpu_numa(0, min_cpus=1) == 1 and calls == [set(half)]  # the intersection only


def test_place_processes_modes(monkeypatch):
    # 4 physical cores with two SMT threads each: cpu c and c + 4 are siblings
    sib = {c: [c % 4, c % 4 + 4] for c in range(8)}
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8)))
    monkeypatch.setattr(rt, "physical_cores", lambda cpus: [sorted(sib[c]) for c in range(4)])
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append((pid, sorted(cpus))))
    assert rt.place_processes([10, 11], "shared") is None and not calls
    # one thread per core, shared by every process
    assert rt.place_processes([10, 11], "nosmt") == [[0, 1, 2, 3]] * 2
    assert calls == [(10, [0, 1, 2, 3]), (11, [0, 1, 2, 3])]
    calls.clear()
    # a core each; the second rank on the node takes the next cores
    assert rt.place_processes([10, 11], "cores", slot=1) == [[2, 6], [3, 7]]
    assert calls == [(10, [2, 6]), (11, [3, 7])]
    calls.clear()
    # not enough cores: left alone
    assert rt.place_processes([10, 11, 12], "cores", slot=1) is None and not calls
    with pytest.raises(ValueError):
        rt.place_processes([10], "bogus")


def test_physical_cores_groups_siblings(tmp_path, monkeypatch):
    import builtins

    real_open = builtins.open

    def fake_open(path, *a, **k):
        p = str(path)
        if p.startswith("/sys/devices/system/cpu/cpu") and p.endswith("thread_siblings_list"):
            c = int(p.split("/cpu/cpu")[1].split("/")[0])
            return io.StringIO(f"{c % 2},{c % 2 + 2}\n")
        return real_open(path, *a, **k)

    import io

    monkeypatch.setattr(builtins, "open", fake_open)
    assert rt.physical_cores({0, 1, 2, 3}) == [[0, 2], [1, 3]]
    assert rt.physical_cores({0, 1, 3}) == [[0], [1, 3]]
