"""Executable replicated-state invariants of a swarm node (``HLSP2P_AUDIT=1`` /
``gpuSwarm.audit``; SURVEY §5.2: "keep these invariants as explicit state-machine
assertions").

The node keeps its state in a few native tables (``SegmentStore``: the HBM ring, its index,
FIFO and pins; ``WantTable``: wants and the tokens waiting on them; ``Directory``: who holds
what) and in Python ledgers that say *why* an entry is pinned or a token is waiting.  Round 5
fixed eleven bugs in that bookkeeping, found late by long rehearsals and randomized sweeps
(``docs/ROUND5.md``).  :func:`audit_node` checks, after every ``launch_round`` and
``complete_round``:

* **Store layout** (native ``SegmentStore.audit``): used bytes = the live allocations; the
  index names live entries under their own keys; every live entry is in the FIFO once and
  the FIFO lies around the ring in allocation order (one wrap at most, no overlap); no live
  entry was ever unpinned more often than pinned (``unpin_underflows``).
* **Pin ledger**: each entry's pin count equals the pins its holders account for -- the
  delayed-unpin list (``_pins``), the rounds in flight (reservations, in-flight receives,
  send pins), cache hits waiting to be answered, delayed deliveries, deferred checks (one
  pin per pending entry) and every registered holder (a fleet's undelivered, in-transmux and
  acknowledged-later batches, on-demand fetches).  A holder that keeps an entry it no longer
  pins (the round-5 early unpin) or a pin nobody accounts for (a leak) fails here.
* **Retired region** (``check_region``, inside ``launch_round``): after the round's
  ``retire_region`` + ``wrap_for``, the region its reservations will take fits (nothing
  pinned in it) and no indexed entry is left in it for a peer to plan a send from.
* **Wants** (native ``WantTable.audit`` + the rounds in flight): index, records, token map
  and waiter lists agree; a want is waiting, or in flight in exactly the round that
  admitted it; a token is in exactly one place (a want, a parked list, a pending cache hit,
  a delayed delivery); in-process requests are joined to a live want or a delayed delivery;
  the node's ``W_ON_DEV`` flag is set exactly on wants whose origin bytes are in device
  memory (the round-5 alias with the table's "held" bit broke that).
* **Deferred verification**: a pending entry (``_vflag``) is live, pending (never
  committed before its check) and holds the key it was delivered for; every parked token
  waits on a pending entry; a fleet row still carrying its expected CRC refers to a pending
  entry (or one old enough for the node's sweep).
* **Directory**: every key the peers will believe this rank holds after its next control
  message (its replica plus the pending adds, minus the pending removes, applied in
  ``ingest_control``'s order) maps to an indexed, committed local entry -- so no peer plans a
  send this rank cannot look up.

A violation raises :class:`AuditError` naming the round and the first inconsistencies.
Cost: O(entries + wants) per call -- a test and rehearsal mode, off in production runs.
"""
from __future__ import annotations

from collections import Counter
from typing import Any, Iterable, List

import numpy as np

_M32 = 0xFFFFFFFF


class AuditError(AssertionError):
    """The node's replicated state broke one of its invariants."""


def _ids(arrs: Iterable[Any]) -> Counter:
    c: Counter = Counter()
    for a in arrs:
        if a is None:
            continue
        a = np.asarray(a, dtype=np.int64).reshape(-1)
        a = a[a >= 0]
        if len(a):
            c.update(a.tolist())
    return c


def expected_pins(node: Any) -> Counter:
    """Pins per entry id, as the node's holders account for them."""
    exp: Counter = Counter()
    exp.update(_ids(ids for _, ids in node._pins))
    for h in node._inflight.values():
        exp.update(_ids(h.hold))
        exp.update(_ids([h.send_pins]))
    exp.update(_ids(e for _, e in node._bulk_hits))
    for e, n in node._local_hits.items():
        if n:
            exp[e] += n
    exp.update(_ids(ids for ids, _ in node._delayed.values()))
    if len(node._vflag):
        exp.update(np.flatnonzero(node._vflag).tolist())
    for holder in node.pin_holders:
        exp.update(_ids(holder()))
    return exp


def _key_set(rows: np.ndarray) -> set:
    rows = np.asarray(rows, dtype=np.int64)
    if rows.ndim != 2 or not len(rows):
        return set()
    return set(map(tuple, (rows[:, :4] & _M32).tolist()))


def audit_node(node: Any, where: str) -> None:
    """Check every invariant of the module docstring; raise :class:`AuditError` on the first
    round that breaks one."""
    errs: List[str] = []
    store, wt = node.store, node._wt
    errs += [f"store: {e}" for e in store.audit()]
    errs += [f"wants: {e}" for e in wt.audit()]
    errs += _audit_pins(node)
    errs += _audit_wants(node)
    errs += _audit_deferred(node)
    errs += _audit_directory(node)
    node.audits = getattr(node, "audits", 0) + 1
    if errs:
        more = f" (+{len(errs) - 12} more)" if len(errs) > 12 else ""
        raise AuditError(f"rank {node.rank} after {where} of round {node.round}: " + "; ".join(errs[:12]) + more)


def check_region(node: Any, need: int) -> None:
    """Inside ``launch_round``, after ``retire_region(need)`` + ``wrap_for(need)``: the
    round's reservations (``need`` bytes at the head) fit, and nothing in their region is
    still indexed (a peer could plan a send from it, and the send's pin would block the
    reservation)."""
    errs: List[str] = []
    store = node.store
    if need <= 0:
        return
    if not store.fits(need):
        errs.append(f"the round's {need} admitted bytes no longer fit at the ring's head "
                    "(a pinned entry in the region)")
    start = store.region_start(need)
    end = start + need
    live = store.live_entries()
    if len(live):
        off, alloc, indexed = live[:, 5], live[:, 6], live[:, 8]
        inside = (off < end) & (off + alloc > start) & (indexed == 1)
        for row in live[inside][:8].tolist():
            errs.append(f"entry {row[0]} key {tuple(row[1:5])} at [{row[5]}, {row[5] + row[6]}) is still indexed "
                        f"inside the retired region [{start}, {end})")
    if errs:
        raise AuditError(f"rank {node.rank} in launch_round of round {node.round}: " + "; ".join(errs))


def _audit_pins(node: Any) -> List[str]:
    errs: List[str] = []
    exp = expected_pins(node)
    ids, pins = node.store.pin_table()
    actual = dict(zip(ids.tolist(), pins.tolist()))
    live = node.store.live_entries()
    live_ids = set(live[:, 0].tolist()) if len(live) else set()
    for e, n in sorted(exp.items()):
        if e not in live_ids:
            errs.append(f"entry {e} is held by {n} pin holder(s) but is free")
        elif actual.get(e, 0) != n:
            errs.append(f"entry {e} holds {actual.get(e, 0)} pins, its holders account for {n}")
    for e, n in sorted(actual.items()):
        if e not in exp:
            errs.append(f"entry {e} holds {n} pins no holder accounts for")
    return errs


def _audit_wants(node: Any) -> List[str]:
    errs: List[str] = []
    wt = node._wt
    ids = wt.ids()
    info = wt.info(ids) if len(ids) else np.zeros((0, 10), dtype=np.int64)
    # in flight in exactly the round that admitted it
    adm: dict = {}
    for h in node._inflight.values():
        if h.ids is None:
            continue
        for w in np.asarray(h.ids).tolist():
            if w in adm:
                errs.append(f"want {w} admitted by rounds {adm[w]} and {h.round}")
            adm[w] = h.round
    for w, rnd in zip(ids.tolist(), info[:, 8].tolist()):
        if rnd >= 0 and adm.get(w) != rnd:
            errs.append(f"want {w} is in flight in round {rnd}, which is not a round in flight admitting it "
                        f"(in flight: {sorted(node._inflight)})")
    for w, rnd in adm.items():
        j = np.searchsorted(ids, w)
        if j < len(ids) and ids[j] == w and info[j, 8] != rnd:
            state = "waiting" if info[j, 8] < 0 else f"in round {info[j, 8]}"
            errs.append(f"want {w} admitted by round {rnd} is {state}")
    # the node's W_ON_DEV: exactly the wants whose origin bytes live in device memory
    from . import node as _node_mod

    on_dev_bit = _node_mod.W_ON_DEV
    if len(info):
        dev_bases = {b for b, t in node._loc_keep.items() if getattr(t, "is_cuda", False)}
        flagged = (info[:, 7] & on_dev_bit) != 0
        for w, base, f in zip(ids.tolist(), info[:, 6].tolist(), flagged.tolist()):
            if base and f != (base in dev_bases):
                errs.append(f"want {w}: W_ON_DEV is {'set' if f else 'clear'} but its origin bytes are in "
                            f"{'device' if base in dev_bases else 'host'} memory")
    # every token in exactly one place
    toks, _ = wt.token_map()
    where: Counter = Counter(toks.tolist())
    for lst in node._vwait.values():
        where.update(int(t) for t in lst)
    for tok, _ in node._bulk_hits:
        where.update(np.asarray(tok, dtype=np.int64).tolist())
    delayed_tok = set()
    for _, tok in node._delayed.values():
        t = np.asarray(tok, dtype=np.int64).tolist()
        where.update(t)
        delayed_tok.update(t)
    dup = [t for t, n in where.items() if n > 1]
    if dup:
        errs.append(f"tokens in more than one place: {sorted(dup)[:8]}")
    live_tok = set(toks.tolist())
    for t in node._tok_req:
        if t not in live_tok and t not in delayed_tok:
            errs.append(f"in-process request token {t} is joined to no want and no pending delivery")
    return errs


def _audit_deferred(node: Any) -> List[str]:
    errs: List[str] = []
    pend = np.flatnonzero(node._vflag) if len(node._vflag) else np.zeros(0, dtype=np.int64)
    if len(pend) or node._vwait:
        live = node.store.live_entries()
        by_id = {int(r[0]): r for r in live} if len(live) else {}
        for e in pend.tolist():
            r = by_id.get(e)
            if r is None:
                errs.append(f"entry {e} awaits its deferred check but is free")
                continue
            if r[7] != 1:  # kPending
                errs.append(f"entry {e} awaits its deferred check but was committed (state {r[7]})")
            want = tuple(int(v) & _M32 for v in node._vinfo[e][:4])
            if tuple(int(v) for v in r[1:5]) != want:
                errs.append(f"entry {e} awaits the check of {want} but holds {tuple(r[1:5])}")
        for e in node._vwait:
            if e >= len(node._vflag) or not node._vflag[e]:
                errs.append(f"tokens are parked on entry {e}, which awaits no check")
    stale = node.VERIFY_STALE_ROUNDS
    for holder in node.expect_holders:
        for e in np.asarray(holder(), dtype=np.int64).tolist():
            if e < 0:
                continue
            pending = e < len(node._vflag) and node._vflag[e]
            swept_window = e < len(node._vround) and node.round - node._vround[e] > stale
            if not pending and not swept_window:
                errs.append(f"a delivery still carries the expected CRC of entry {e}, which awaits no check")
    return errs


def _audit_directory(node: Any) -> List[str]:
    errs: List[str] = []
    if node.world < 2:
        return errs
    held = _key_set(node.directory.holder_keys(node.rank))
    add, rm = node.store.peek_delta()
    after = (held | _key_set(add)) - _key_set(rm)  # ingest_control applies adds, then removes
    live = node.store.live_entries()
    if len(live):
        ok = (live[:, 8] == 1) & (live[:, 7] == 2)  # indexed, resident
        resident = set(map(tuple, (live[ok][:, 1:5] & _M32).tolist()))
    else:
        resident = set()
    missing = after - resident
    if missing:
        errs.append(f"{len(missing)} key(s) peers will believe this rank holds have no committed local entry, "
                    f"e.g. {sorted(missing)[:4]}")
    node.under_announced = len(resident - after)  # held but not announced: only costs offload
    return errs
