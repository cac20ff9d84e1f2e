"""Process-level tuning (``utils/runtime.py``): GC freeze and NUMA placement."""
import gc
import os

import pytest

from hlsjs_p2p_wrapper_amd.utils import runtime as rt


def test_tune_gc_freezes_and_raises_gen0():
    prev = gc.get_threshold()
    try:
        out = rt.tune_gc(12345)
        assert out == prev and gc.get_threshold()[0] == 12345 and gc.get_freeze_count() > 0
    finally:
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
