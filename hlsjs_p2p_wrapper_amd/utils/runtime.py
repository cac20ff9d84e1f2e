"""Process-level runtime tuning for long-running peers.

Python's cyclic GC periodically re-traverses every long-lived container object: the
parsed playlists (thousands of ``Fragment`` objects per level), the engine, the swarm
node.  A full (gen-2) pass over a 5-rendition ladder's state costs tens of milliseconds
and lands in the middle of a swarm round.  After start-up, :func:`tune_gc` moves
everything alive into the permanent generation (``gc.freeze``) and raises the gen-0
threshold, so collections only look at young objects.  The per-fragment churn (loader
stats, event payloads, closures) is mostly freed by reference counting anyway.  GC stays
enabled: new cycles are still collected, and every few full passes one of them traverses the
whole (thawed) heap, so a cycle that formed among frozen objects is reclaimed too.

:func:`bind_to_gpu_numa` keeps a peer's host side on the NUMA node its GPU hangs off: the
CPUs it runs on (the host path is one Python thread per GPU) and, through first touch, the
pinned host buffers the CDN DMAs read, so those transfers do not cross the socket link.
"""
from __future__ import annotations

import gc
import os
import time
from typing import List, Optional, Tuple


def tune_gc(gen0_threshold: int = 50_000, thaw_every: int = 4) -> Tuple[int, int, int]:
    """Collect once, freeze the surviving heap, raise the gen-0 threshold.

    Call it after the player / node / origin are set up (``bench.py`` does).  Every
    ``thaw_every``-th full collection first thaws the frozen heap, so objects that were alive
    at a freeze and became cyclic garbage since (a request, a loader context or a round handle
    in flight when a full pass ran) are reclaimed instead of leaking.  Returns the previous
    thresholds."""
    prev = gc.get_threshold()
    gc.collect()
    gc.freeze()
    # full collections re-traverse every survivor since start-up; the hot paths leave almost
    # no cyclic garbage (host peak is the same with the GC off over 3000 steps,
    # profiles/r2_soak), so run them 10x less often than the default
    gc.set_threshold(gen0_threshold, prev[1], max(prev[2], 100))
    # State that builds up while a peer runs (buffered fragments, delivered-segment records)
    # would make every later full pass longer: over 3,000 HBM-origin bench steps the step time
    # drifted +16 % with the GC on and stayed flat with it off (profiles/r4_gc).  Freezing what
    # survives each full pass keeps the next one proportional to what is new since.
    _freeze_after_full.thaw_every = max(1, int(thaw_every))
    if _freeze_after_full not in gc.callbacks:
        gc.callbacks.append(_freeze_after_full)
    if os.environ.get("HLSP2P_GC_DISABLE") == "1":  # diagnostic: no cyclic GC after start-up at all
        gc.disable()
    return prev


class _FullPassFreezer:
    """gc callback: move the survivors of a full (gen-2) collection to the permanent
    generation; every ``thaw_every``-th full pass starts by thawing it (``gc.unfreeze`` merges
    the permanent generation into gen 2 before the pass runs), so that pass traverses the
    whole heap once and frees cycles among formerly frozen objects."""

    def __init__(self) -> None:
        self.thaw_every = 4
        self.full_passes = 0
        self.thaws = 0

    def __call__(self, phase: str, info: dict) -> None:
        if info.get("generation") != 2:
            return
        if phase == "start":
            self.full_passes += 1
            if self.full_passes % self.thaw_every == 0:
                gc.unfreeze()
                self.thaws += 1
        elif phase == "stop":
            gc.freeze()


_freeze_after_full = _FullPassFreezer()


def cpu_calibration_us(n: int = 20_000, reps: int = 3) -> float:
    """Best-of-``reps`` time of a fixed pure-Python loop, in microseconds: a process's own
    measure of how fast its core runs right now (soak analysis: if this drifts with the rest
    of a process's phases, the slowdown is the machine's -- clocks, co-tenants -- not growing
    state in the process)."""
    best = float("inf")
    for _ in range(reps):
        t = time.perf_counter()
        x = 0
        for i in range(n):
            x += i & 7
        best = min(best, time.perf_counter() - t)
    return best * 1e6


def _parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


def gpu_local_cpus(device_index: int = 0) -> Tuple[Optional[int], List[int]]:
    """``(numa_node, cpus)`` of a GPU from sysfs (its PCI function's ``numa_node`` and
    ``local_cpulist``); ``(None, [])`` when unknown."""
    import torch

    try:
        p = torch.cuda.get_device_properties(device_index)
        addr = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}.0"
        base = f"/sys/bus/pci/devices/{addr}"
        with open(os.path.join(base, "local_cpulist")) as f:
            cpus = _parse_cpulist(f.read())
        with open(os.path.join(base, "numa_node")) as f:
            node = int(f.read().strip())
    except (AttributeError, OSError, ValueError, RuntimeError):
        return None, []
    return (node if node >= 0 else None), cpus


def physical_cores(cpus) -> List[List[int]]:
    """Group logical CPUs into physical cores (SMT siblings together, from sysfs
    ``thread_siblings_list``), in ascending order of each core's first CPU; CPUs whose
    topology is unreadable count as one-thread cores."""
    allowed = set(cpus)
    cores, seen = [], set()
    for c in sorted(allowed):
        if c in seen:
            continue
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                sib = [s for s in _parse_cpulist(f.read()) if s in allowed]
        except (OSError, ValueError):
            sib = [c]
        if c not in sib:
            sib.append(c)
        seen.update(sib)
        cores.append(sorted(sib))
    return cores


def place_processes(pids: List[int], mode: str, slot: int = 0) -> Optional[List[List[int]]]:
    """CPU placement of one GPU's host processes (the rank first, then its players), inside
    the affinity the caller already has (e.g. its GPU's NUMA node).

    * ``shared``: leave it (every process may run on every allowed CPU);
    * ``nosmt``: every process may run on one thread of each allowed physical core, so the
      scheduler can never put two of them on SMT siblings (two busy Python processes on one
      core run at ~0.55x each);
    * ``cores``: each process gets a physical core of its own (all its threads).  ``slot``
      offsets the cores by ``slot * len(pids)`` so several ranks on one NUMA node do not
      overlap.

    Returns the CPU lists applied (None: left alone, e.g. too few cores)."""
    if mode == "shared" or not pids:
        return None
    cores = physical_cores(os.sched_getaffinity(0))
    if mode == "nosmt":
        if len(cores) < len(pids):
            return None
        cpus = [c[0] for c in cores]
        sets = [cpus] * len(pids)
    elif mode == "cores":
        first = slot * len(pids)
        if first + len(pids) > len(cores):
            return None
        sets = [cores[first + i] for i in range(len(pids))]
    else:
        raise ValueError(f"unknown CPU placement {mode!r}")
    for pid, s in zip(pids, sets):
        try:
            os.sched_setaffinity(pid, s)
        except OSError:
            return None
    return sets


def bind_to_gpu_numa(device_index: int = 0, min_cpus: int = 8) -> Optional[int]:
    """Restrict this process to the CPUs local to its GPU (and so, by first touch, its later
    host allocations to that NUMA node).  Only narrows the current affinity, and only when
    at least ``min_cpus`` of the GPU's CPUs are allowed; returns the node, or None when it
    left the affinity alone.  Call it before allocating pinned buffers."""
    node, cpus = gpu_local_cpus(device_index)
    if node is None or not cpus:
        return None
    allowed = os.sched_getaffinity(0)
    local = allowed.intersection(cpus)
    if len(local) < min_cpus or local == allowed:
        return node if local == allowed else None
    os.sched_setaffinity(0, local)
    return node


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def kfd_gpus(topology: str = KFD_TOPOLOGY, dev_dir: str = "/dev/dri") -> List[dict]:
    """The GPU agents ROCr would enumerate, read from the KFD topology without any HIP / HSA
    call: the nodes whose ``properties`` report SIMDs (``simd_count > 0``; CPU nodes have
    none) in node order, each with its ``gpu_id``, ``drm_render_minor`` and whether this
    process can open its render node (ROCr skips a GPU whose render node it cannot open, e.g.
    one a container did not pass through).  Opening a DRM render node creates no HSA queue
    or KFD mapping."""
    out: List[dict] = []
    try:
        names = sorted(os.listdir(topology), key=lambda s: int(s) if s.isdigit() else 1 << 30)
    except OSError:
        return out
    for name in names:
        props: dict = {}
        try:
            with open(os.path.join(topology, name, "properties")) as f:
                for ln in f:
                    k, _, v = ln.strip().partition(" ")
                    if v.strip().lstrip("-").isdigit():
                        props[k] = int(v)
        except OSError:
            continue
        if props.get("simd_count", 0) <= 0:
            continue
        minor = props.get("drm_render_minor")
        usable = False
        if minor is not None and minor >= 0:
            try:
                fd = os.open(os.path.join(dev_dir, f"renderD{minor}"), os.O_RDWR | os.O_CLOEXEC)
                os.close(fd)
                usable = True
            except OSError:
                usable = False
        out.append({"node": int(name) if name.isdigit() else name, "gpu_id": props.get("gpu_id"),
                    "render_minor": minor, "usable": usable})
    return out


def _visible_filter(n: int, spec: Optional[str]) -> int:
    """How many of ``n`` devices a ``*_VISIBLE_DEVICES`` list keeps: its entries up to the first
    invalid one (the runtimes stop parsing there; ``-1`` hides every device).  UUID entries
    (``GPU-...``) count as one device each."""
    if spec is None:
        return n
    k = 0
    seen: set = set()
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok:
            break
        if tok.upper().startswith("GPU-"):
            k += 1
            continue
        try:
            i = int(tok)
        except ValueError:
            break
        if i < 0 or i >= n or i in seen:
            break
        seen.add(i)
        k += 1
    return min(k, n)


def visible_gpu_count(topology: str = KFD_TOPOLOGY, dev_dir: str = "/dev/dri") -> int:
    """Number of GPUs a HIP process started now would see, computed WITHOUT initialising HIP
    (``torch.cuda.device_count()`` may fall back to ``hipGetDeviceCount``, which starts the HIP
    runtime and maps ``/dev/kfd`` in the calling process): the usable KFD GPU agents
    (:func:`kfd_gpus`), narrowed by ``ROCR_VISIBLE_DEVICES`` and then by ``HIP_VISIBLE_DEVICES``
    (or ``CUDA_VISIBLE_DEVICES``), as ROCr and HIP apply them."""
    n = sum(1 for g in kfd_gpus(topology, dev_dir) if g["usable"])
    n = _visible_filter(n, os.environ.get("ROCR_VISIBLE_DEVICES"))
    hip = os.environ.get("HIP_VISIBLE_DEVICES")
    if hip is None:
        hip = os.environ.get("CUDA_VISIBLE_DEVICES")
    return _visible_filter(n, hip)


def gpu_touched() -> dict:
    """Has this process initialised the GPU?  ``torch_initialized``: torch's HIP context
    (``torch.cuda.is_initialized``, without importing torch if it is not loaded);
    ``kfd_mapped``: some ``/dev/kfd`` mapping in ``/proc/self/maps`` (the HSA runtime maps its
    doorbells and queues from it); ``kfd_open``: an open ``/dev/kfd`` descriptor.  A process
    for which any is true must not fork-and-exec or exec another program on this pool."""
    import sys

    torch_mod = sys.modules.get("torch")
    init = False
    if torch_mod is not None:
        try:
            init = bool(torch_mod.cuda.is_initialized())
        except Exception:  # noqa: BLE001 - a torch without the cuda module
            init = False
    mapped = False
    try:
        with open("/proc/self/maps") as f:
            mapped = any("/dev/kfd" in ln for ln in f)
    except OSError:
        pass
    opened = False
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                    opened = True
                    break
            except OSError:
                continue
    except OSError:
        pass
    return {"torch_initialized": init, "kfd_mapped": mapped, "kfd_open": opened}
