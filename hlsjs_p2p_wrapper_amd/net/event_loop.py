"""Single-threaded timer loop: the ``setTimeout`` / ``performance.now()`` platform (L0).

The reference is browser JavaScript: everything asynchronous — the per-attempt request
timeout (``lib/integration/p2p-loader-generator.js:163``), the exponential-backoff retry
(``:114-120``), the stream controller's tick, the peer agent's scheduler — hangs off the
browser's timer queue, and every loader timestamp comes from ``performance.now()``
(``:77,98,181``).  This module is that platform for the MI355X engine.

Two clocks:

* ``clock="real"``    — ``time.perf_counter`` in milliseconds; timers fire when due.  Used
  by ``bench.py`` and production players.  ``speed`` > 1 compresses time (the live bench
  plays a channel faster than real time) and ``epoch`` pins the origin of the clock to a
  wall-clock instant shared by processes.
* ``clock="virtual"`` — a discrete-event clock: when no callback is ready the loop *jumps*
  to the next timer.  Tests run minutes of playback (retries with 64 s back-off, live
  playlist refreshes) in milliseconds, deterministically.

One loop per thread (``get_event_loop()``), mirroring the one-timer-queue-per-tab model;
the in-process multi-peer swarm test runs one peer per thread.  Work done on other threads
(network fetches, :mod:`.network`) comes back through :meth:`EventLoop.call_soon_threadsafe`;
while such work is outstanding (:meth:`EventLoop.hold` / :meth:`EventLoop.release`) an idle
loop waits for it instead of sleeping to its next timer, and a virtual clock does not jump
past it.
"""
from __future__ import annotations

import collections
import heapq
import itertools
import threading
import time
from typing import Any, Callable, List, Optional, Tuple


class TimerHandle:
    __slots__ = ("when", "seq", "fn", "args", "cancelled", "interval")

    def __init__(self, when: float, seq: int, fn: Callable[..., Any], args: tuple,
                 interval: Optional[float] = None) -> None:
        self.when = when
        self.seq = seq
        self.fn = fn
        self.args = args
        self.cancelled = False
        self.interval = interval

    def cancel(self) -> None:
        self.cancelled = True


class EventLoop:
    """Timer queue with a real or virtual millisecond clock."""

    def __init__(self, clock: str = "real", speed: float = 1.0, epoch: Optional[float] = None) -> None:
        if clock not in ("real", "virtual"):
            raise ValueError("clock must be 'real' or 'virtual'")
        if speed <= 0:
            raise ValueError("speed must be positive")
        self.clock = clock
        # a real clock may run `speed` times faster than the wall (a time-compressed live
        # channel: playlist reloads, ticks and the origin's live edge all advance together);
        # with `epoch` (a time.time() value) every process's loop reads the same time
        self.speed = float(speed)
        self.epoch = epoch
        self._t0 = time.perf_counter()
        self._vnow = 0.0
        # heap of (when, seq, handle): tuple order compares in C (a handle __lt__ cost a
        # Python call per comparison, ~12 per push on a few thousand pending timers)
        self._heap: List[Tuple[float, int, TimerHandle]] = []
        self._ready: List[Tuple[Callable[..., Any], tuple]] = []
        self._seq = itertools.count()
        self._idle_hooks: List[Callable[[], bool]] = []
        self._compact_at = 4096
        # callbacks posted from other threads (deque append / popleft are atomic) and the
        # event that wakes an idle loop for them; _external counts outstanding foreign work
        self._threadsafe: collections.deque = collections.deque()
        self._wake = threading.Event()
        self._external = 0
        self._ext_lock = threading.Lock()

    # ------------------------------------------------------------------ clock
    def now(self) -> float:
        """``performance.now()``: milliseconds since loop creation."""
        if self.clock == "virtual":
            return self._vnow
        if self.epoch is not None:
            return (time.time() - self.epoch) * 1000.0 * self.speed
        return (time.perf_counter() - self._t0) * 1000.0 * self.speed

    performance_now = now

    def advance(self, ms: float) -> None:
        """Virtual clock only: move time forward without running callbacks."""
        if self.clock != "virtual":
            raise RuntimeError("advance() needs a virtual clock")
        self._vnow += max(0.0, float(ms))

    # ----------------------------------------------------------------- timers
    def set_timeout(self, fn: Callable[..., Any], delay_ms: float = 0.0, *args: Any) -> TimerHandle:
        delay = 0.0 if delay_ms is None else max(0.0, float(delay_ms))
        h = TimerHandle(self.now() + delay, next(self._seq), fn, args)
        heap = self._heap
        if len(heap) >= self._compact_at:
            # cancelled timers are dropped lazily when they reach the top; a long-running
            # peer cancels one fragment-timeout timer per fragment (tens of thousands per
            # second), so sweep them out whenever the heap doubles
            heap[:] = [e for e in heap if not e[2].cancelled]
            heapq.heapify(heap)
            self._compact_at = max(4096, 2 * len(heap))
        heapq.heappush(heap, (h.when, h.seq, h))
        return h

    setTimeout = set_timeout

    def set_interval(self, fn: Callable[..., Any], interval_ms: float, *args: Any) -> TimerHandle:
        interval = max(0.0, float(interval_ms))
        h = TimerHandle(self.now() + interval, next(self._seq), fn, args, interval)
        heapq.heappush(self._heap, (h.when, h.seq, h))
        return h

    setInterval = set_interval

    @staticmethod
    def clear_timeout(handle: Optional[TimerHandle]) -> None:
        if handle is not None:
            handle.cancel()

    clearTimeout = clear_timeout
    clear_interval = clear_timeout
    clearInterval = clear_timeout

    def call_soon(self, fn: Callable[..., Any], *args: Any) -> None:
        self._ready.append((fn, args))

    def call_soon_threadsafe(self, fn: Callable[..., Any], *args: Any) -> None:
        """Schedule ``fn(*args)`` on this loop from any thread (wakes an idle loop)."""
        self._threadsafe.append((fn, args))
        self._wake.set()

    def hold(self) -> None:
        """Another thread is doing work whose result comes back through
        :meth:`call_soon_threadsafe`: an idle loop waits for it (and a virtual clock does not
        skip ahead of it).  Pair with :meth:`release`, called on any thread."""
        with self._ext_lock:
            self._external += 1

    def release(self) -> None:
        with self._ext_lock:
            self._external = max(0, self._external - 1)
        self._wake.set()

    def _take_threadsafe(self) -> None:
        q = self._threadsafe
        while q:
            self._ready.append(q.popleft())

    def add_idle_hook(self, hook: Callable[[], bool]) -> None:
        """``hook()`` runs when the loop would otherwise sleep; returns True if it did work."""
        self._idle_hooks.append(hook)

    def remove_idle_hook(self, hook: Callable[[], bool]) -> None:
        try:
            self._idle_hooks.remove(hook)
        except ValueError:
            pass

    # ---------------------------------------------------------------- running
    def _pop_due(self, now: float) -> Optional[TimerHandle]:
        heap = self._heap
        while heap:
            when, _, h = heap[0]
            if h.cancelled:
                heapq.heappop(heap)
                continue
            if when <= now:
                heapq.heappop(heap)
                return h
            return None
        return None

    def _next_deadline(self) -> Optional[float]:
        heap = self._heap
        while heap and heap[0][2].cancelled:
            heapq.heappop(heap)
        return heap[0][0] if heap else None

    def _fire(self, h: TimerHandle) -> None:
        if h.interval is not None and not h.cancelled:
            h.when = max(h.when + h.interval, self.now()) if self.clock == "real" else h.when + h.interval
            h.seq = next(self._seq)
            heapq.heappush(self._heap, (h.when, h.seq, h))
        h.fn(*h.args)

    def run_once(self, block: bool = True, max_wait_ms: float = 50.0) -> bool:
        """Run ready callbacks and due timers.  Returns False when nothing is left."""
        did = False
        if self._threadsafe:
            self._take_threadsafe()
        if self._ready:
            ready, self._ready = self._ready, []
            for fn, args in ready:
                fn(*args)
            did = True
        now = self.now()
        h = self._pop_due(now)
        while h is not None:
            self._fire(h)
            did = True
            if self._ready:
                return True
            h = self._pop_due(self.now())
        if did:
            return True
        for hook in tuple(self._idle_hooks):
            if hook():
                did = True
        if did:
            return True
        deadline = self._next_deadline()
        if self._external:  # foreign work outstanding: wait for it (or the next timer)
            if not block:
                return True
            wait = max_wait_ms if deadline is None or self.clock == "virtual" else \
                min(max(0.0, deadline - self.now()) / self.speed, max_wait_ms)
            self._wake.wait(wait / 1000.0)
            self._wake.clear()
            return True
        if deadline is None:
            return bool(self._ready) or bool(self._threadsafe)
        if self.clock == "virtual":
            self._vnow = max(self._vnow, deadline)
            return True
        if block:  # (loop ms -> wall seconds)
            wait = min(max(0.0, deadline - self.now()) / self.speed, max_wait_ms) / 1000.0
            if wait > 0:
                self._wake.wait(wait)
                self._wake.clear()
        return True

    def run_until(self, predicate: Callable[[], bool], timeout_ms: float = 60_000.0) -> bool:
        """Run until ``predicate()`` is true or ``timeout_ms`` of loop time elapses."""
        end = self.now() + timeout_ms
        while not predicate():
            if self.now() >= end:
                return False
            if self.clock == "virtual":
                nd = self._next_deadline()
                if not self._ready and nd is not None and nd > end and not self._idle_hooks \
                        and not self._external and not self._threadsafe:
                    self._vnow = end
                    return predicate()
            if not self.run_once():
                return predicate()
        return True

    def run_for(self, duration_ms: float) -> None:
        end = self.now() + duration_ms
        self.run_until(lambda: self.now() >= end, timeout_ms=duration_ms + 1.0)

    def pending(self) -> int:
        return (len(self._ready) + len(self._threadsafe) + self._external
                + sum(1 for e in self._heap if not e[2].cancelled))


_local = threading.local()


def get_event_loop() -> EventLoop:
    """The calling thread's loop (created on first use with a real clock)."""
    loop = getattr(_local, "loop", None)
    if loop is None:
        loop = EventLoop("real")
        _local.loop = loop
    return loop


def set_event_loop(loop: Optional[EventLoop]) -> None:
    _local.loop = loop


def new_event_loop(clock: str = "real", speed: float = 1.0, epoch: Optional[float] = None) -> EventLoop:
    loop = EventLoop(clock, speed=speed, epoch=epoch)
    set_event_loop(loop)
    return loop


def performance_now() -> float:
    return get_event_loop().now()


def set_timeout(fn: Callable[..., Any], delay_ms: float = 0.0, *args: Any) -> TimerHandle:
    return get_event_loop().set_timeout(fn, delay_ms, *args)


def clear_timeout(handle: Optional[TimerHandle]) -> None:
    EventLoop.clear_timeout(handle)
