"""Batched decrypt + demux stage between ``FRAG_LOADED`` and the buffer (hls.js's
decrypter + TS demuxer, moved onto the MI355X).

Every fragment loaded during one event-loop iteration — typically all fragments
completed by one swarm exchange round — is decrypted by ONE AES-CBC launch and demuxed
by ONE demux launch sequence, then a single small device->host copy of the per-segment
``info`` rows delivers timing/status to the players.  Payloads that are views of the
node's HBM arena are consumed in place (no copy); host payloads (default CDN loader) are
staged with one H2D copy.

The batching point is per (thread, device): the peer threads of an in-process swarm each
get their own pipeline.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np
import torch

from ..net.event_loop import get_event_loop
from ..ops import aes as _aes
from ..ops import tsdemux as _ts
from ..ops._native import device as _native_device
from ..ops._native import runtime as _rt
from ..utils.trace import PhaseTimer

ALIGN = 256


class TransmuxJob:
    """One fragment to transmux: ``payload`` (torch uint8 tensor on any device / numpy /
    bytes), the AES-128 ``key`` and ``iv`` (``None``: clear), ``callback(result)``.  A plain
    slotted class: one is built per fragment, and a dataclass ``__init__`` stays interpreted
    code inside the compiled module."""

    __slots__ = ("payload", "key", "iv", "callback", "frag", "verify")

    def __init__(self, payload: Any, key: Optional[bytes], iv: Optional[bytes],
                 callback: Callable[[Dict[str, Any]], None], frag: Any = None, verify: Any = None) -> None:
        self.payload = payload
        self.key = key
        self.iv = iv
        self.callback = callback
        self.frag = frag
        self.verify = verify
        # a received segment's pending CRC check (agent/node.py VerifyTicket: ``expect``,
        # ``report(ok)``): the batch verifies the bytes -- fused into the decrypt -- reports the
        # outcome, and a fragment that fails gets a ``verify_failed`` error result

    def __repr__(self) -> str:
        return f"TransmuxJob(key={'set' if self.key else None}, frag={self.frag!r})"


def _as_tensor(payload: Any) -> torch.Tensor:
    if isinstance(payload, torch.Tensor):
        return payload if payload.dim() == 1 else payload.reshape(-1)  # arena slices are 1-D already
    if isinstance(payload, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(payload.reshape(-1)).view(np.uint8))
    if isinstance(payload, (bytes, bytearray, memoryview)):
        return torch.frombuffer(bytearray(payload), dtype=torch.uint8)
    raise TypeError(f"unsupported payload type {type(payload)!r}")


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class MediaPipeline:
    def __init__(self, device: torch.device, loop=None) -> None:
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            # "cuda" != "cuda:0": an index-less device would fail the in-place staging check
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.loop = loop or get_event_loop()
        self._jobs: List[TransmuxJob] = []
        self._scheduled = False
        self.segments = 0
        self.bytes_in = 0
        self.batches = 0
        self.timer = PhaseTimer()
        self._free_events: List[Any] = []  # timing events (start / end of each batch on the device)
        # event-loop players flush at the end of the loop iteration; a throughput driver
        # sets auto_flush=False and overlaps launch() / complete() of consecutive batches
        self.auto_flush = True

    def submit(self, job: TransmuxJob) -> None:
        self._jobs.append(job)
        if self.auto_flush and not self._scheduled:
            self._scheduled = True
            self.loop.call_soon(self.flush)

    def flush(self) -> None:
        """Synchronous batch: launch the kernels for everything submitted, then complete."""
        self._scheduled = False
        self.complete(self.launch())

    def launch(self) -> Optional["_Batch"]:
        """Enqueue decrypt + demux for every submitted job; the host does not wait."""
        jobs, self._jobs = self._jobs, []
        if not jobs:
            return None
        try:
            return self._launch(jobs)
        except Exception as e:  # deliver the failure to every job of the batch
            return _Batch(jobs, error=e)

    def complete(self, batch: Optional["_Batch"]) -> None:
        """Wait for a launched batch and run the per-fragment callbacks."""
        if batch is None:
            return
        if batch.error is not None:
            for j in batch.jobs:  # (a pending receive check is left to the node's own sweep)
                j.callback({"error": batch.error})
            return
        results = self._complete(batch)
        if batch.expect_mask is not None:  # deferred receive checks: report, drop failed results
            ok = self._verified(batch, len(batch.jobs))
            for i in np.flatnonzero(batch.expect_mask).tolist():
                batch.jobs[i].verify.report(bool(ok[i]))
                if not ok[i]:
                    results[i] = {"error": ValueError("received segment failed its CRC check"), "status": -1,
                                  "verify_failed": True}
        t = time.perf_counter()
        for j, r in zip(batch.jobs, results):
            j.callback(r)
        self.timer.add("callbacks", time.perf_counter() - t)

    # ------------------------------------------------------------------ device events
    def _event(self):
        """A recorded timing event on the current stream (recycled: a fresh event costs
        ~5 us of host time)."""
        ev = self._free_events.pop() if self._free_events else torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def _wait(self, b: "_Batch") -> None:
        """Host wait for a batch's device work; its device time goes to ``dev_transmux``."""
        if b.event is None:
            return
        b.event.synchronize()
        if b.start is not None:
            self.timer.add("dev_transmux", b.start.elapsed_time(b.event) / 1e3)
            self._free_events.append(b.start)
            b.start = None
        self._free_events.append(b.event)
        b.event = None

    # ------------------------------------------------------------------ batch
    def _stage(self, tensors: List[torch.Tensor], sizes: List[int]) -> Tuple[torch.Tensor, List[int]]:
        """One source buffer + offsets: in place when every payload is a view of the same
        device storage (the HBM arena), otherwise one staging copy.  Same-storage check: one
        ``data_ptr()`` per payload, every view inside the first payload's allocation
        (allocations never overlap), instead of a storage object per payload."""
        dev = self.device
        t0 = tensors[0]
        if t0.device == dev:
            cuda = dev.type == "cuda"
            storage = t0.untyped_storage()
            base_ptr, cap = storage.data_ptr(), storage.nbytes()
            offs = [t.data_ptr() - base_ptr for t in tensors]
            if all(o >= 0 and o + n <= cap and o % 16 == 0 and t.is_cuda == cuda
                   for o, n, t in zip(offs, sizes, tensors)):
                base = torch.empty(0, dtype=torch.uint8, device=dev).set_(storage, 0, (cap,))
                return base, offs
        offs, pos = [], 0
        for t in tensors:
            offs.append(pos)
            pos += _align(t.numel())
        buf = torch.empty(pos + ALIGN, dtype=torch.uint8, device=dev)
        for o, t in zip(offs, tensors):
            buf[o:o + t.numel()].copy_(t, non_blocking=True)
        return buf, offs

    def _launch(self, jobs: List[TransmuxJob]) -> "_Batch":
        dev = self.device
        tensors = [_as_tensor(j.payload) for j in jobs]
        sizes = [t.numel() for t in tensors]
        self.segments += len(jobs)
        self.bytes_in += sum(sizes)
        self.batches += 1
        tm = self.timer
        t0 = time.perf_counter()
        src, src_offs = self._stage(tensors, sizes)
        t1 = time.perf_counter()
        tm.add("stage", t1 - t0)
        enc = [i for i, j in enumerate(jobs) if j.key is not None]
        clear = [i for i, j in enumerate(jobs) if j.key is None]
        results: List[Optional[Dict[str, Any]]] = [None] * len(jobs)
        groups = []
        if enc:
            bad = [i for i in enc if sizes[i] == 0 or sizes[i] % 16]
            for i in bad:
                results[i] = {"error": ValueError("encrypted payload is not a multiple of 16 bytes"), "status": -1}
            if bad:
                enc = [i for i in enc if i not in bad]
        vjobs = [i for i, j in enumerate(jobs) if j.verify is not None]
        if dev.type == "cuda":
            return self._launch_native(jobs, src, src_offs, sizes, enc, clear, results, t1, vjobs)
        host_verify = None
        if vjobs:  # CPU: a host CRC of the received bytes (the GPU fuses it into the decrypt)
            vi = np.asarray(vjobs, dtype=np.int64)
            got = _rt().crc32_batch(src.numpy(), np.asarray([src_offs[i] for i in vjobs], dtype=np.int64),
                                    np.asarray([sizes[i] for i in vjobs], dtype=np.int64))
            exp = np.asarray([jobs[i].verify.expect for i in vjobs], dtype=np.int64)
            host_verify = [(vi, (got.astype(np.int64) & 0xFFFFFFFF) == (exp & 0xFFFFFFFF))]
        if enc:
            dec_offs, pos = [], 0
            for i in enc:
                dec_offs.append(pos)
                pos += _align(sizes[i])
            dec = torch.empty(pos + ALIGN, dtype=torch.uint8, device=dev)
            out_len = _aes.cbc_decrypt_batch(src, [src_offs[i] for i in enc], [sizes[i] for i in enc],
                                             [jobs[i].key for i in enc], [jobs[i].iv for i in enc], dec, dec_offs)
            groups.append((enc, dec, dec_offs, out_len, [sizes[i] for i in enc]))
        if clear:
            groups.append((clear, src, [src_offs[i] for i in clear], [sizes[i] for i in clear],
                           [sizes[i] for i in clear]))
        t2 = time.perf_counter()
        tm.add("decrypt_launch", t2 - t1)
        infos = []
        for idx, buf, offs, lens, caps in groups:
            es_offs, pos = [], 0
            for c in caps:
                es_offs.append(pos)
                pos += _align(c)
            es = torch.empty(pos + ALIGN, dtype=torch.uint8, device=dev)
            res = _ts.demux_batch(buf, offs, lens, es, es_offs, caps=caps)
            infos.append((idx, res, es_offs, lens))
        # async D2H of the small per-segment info rows (+ plaintext lengths) into pinned
        # host memory, then one event: completing the batch is the stage's only sync
        host = []
        for _, r, _, lens in infos:
            if dev.type == "cpu":
                host.append((r.info.numpy(), lens.numpy() if isinstance(lens, torch.Tensor) else np.asarray(lens)))
                continue
            hi = torch.empty(r.info.shape, dtype=torch.int64, pin_memory=True)
            hi.copy_(r.info, non_blocking=True)
            if isinstance(lens, torch.Tensor):
                hl = torch.empty(lens.shape, dtype=torch.int64, pin_memory=True)
                hl.copy_(lens, non_blocking=True)
            else:
                hl = np.asarray(lens)
            host.append((hi, hl))
        ev = None
        if dev.type != "cpu":
            ev = self._event()
        tm.add("demux_launch", time.perf_counter() - t2)
        return _Batch(jobs, infos=infos, host=host, event=ev, results=results, verify=host_verify,
                      expect_mask=_mask(len(jobs), vjobs))

    def _launch_native(self, jobs, src, src_offs, sizes, enc, clear, results, t1, vjobs=()) -> "_Batch":
        """GPU batch in ONE native call (``kernels/transmux.cpp``): descriptor math, one
        staging H2D, AES-CBC decrypt (with the receive CRC of ``vjobs`` fused in), demux per
        group, D2H of the info rows.  Received segments the decrypt does not read (clear
        ones, rejected ones) are checked by the CRC kernel."""
        tm = self.timer
        idx = enc + clear
        n = len(idx)
        verify = []
        ex = cw = ctab = None
        if vjobs:
            in_dec = set(enc)
            side = [i for i in vjobs if i not in in_dec]
            if side:
                from ..ops import crc as _crc

                _, okd = _crc.crc32_batch(src, [src_offs[i] for i in side], [sizes[i] for i in side],
                                          expect=[jobs[i].verify.expect & 0xFFFFFFFF for i in side])
                okh = torch.empty(len(side), dtype=torch.uint8, pin_memory=True)
                okh.copy_(okd, non_blocking=True)
                verify.append((np.asarray(side, dtype=np.int64), okh))
            if len(side) < len(vjobs):
                from ..ops import crc as _crc

                ex = np.full(n, -1, dtype=np.int64)
                for r, i in enumerate(enc):
                    if jobs[i].verify is not None:
                        ex[r] = jobs[i].verify.expect & 0xFFFFFFFF
                cw, ctab = _crc.fused_consts(self.device)
        mask = _mask(len(jobs), vjobs)
        if n == 0:  # every job was rejected above
            return _Batch(jobs, infos=[], host=[], event=self._event() if verify else None, results=results,
                          verify=verify or None, expect_mask=mask)
        offs = np.fromiter((src_offs[i] for i in idx), dtype=np.int64, count=n)
        nb = np.fromiter((sizes[i] for i in idx), dtype=np.int64, count=n)
        flags = np.zeros(n, dtype=np.uint8)
        flags[:len(enc)] = 1
        drk = np.zeros((n, 44), dtype=np.uint32)
        iv = np.zeros((n, 16), dtype=np.uint8)
        if enc:
            k0 = jobs[enc[0]].key
            if all(jobs[i].key is k0 or jobs[i].key == k0 for i in enc):  # one key per stream
                drk[:len(enc)] = _aes.round_keys_le(bytes(k0))
            else:
                for r, i in enumerate(enc):
                    drk[r] = _aes.round_keys_le(bytes(jobs[i].key))
            iv[:len(enc)] = np.frombuffer(b"".join(bytes(jobs[i].iv) for i in enc), dtype=np.uint8).reshape(-1, 16)
        td0, isb = _aes.device_tables(self.device)
        t2 = time.perf_counter()
        tm.add("decrypt_launch", t2 - t1)
        ev0 = self._event()
        groups, dec, host_block, fused = _native_device().transmux_launch(src, offs, nb, flags, drk, iv, td0, isb,
                                                                          _ts.DEFAULT_MAX_PES, ex, cw, ctab)
        infos, host = [], []
        for gidx, info, pes, es, es_offs, hinfo, hlens in groups:
            batch_idx = [idx[k] for k in gidx.tolist()]
            infos.append((batch_idx, _ts.DemuxResult(info, pes, es, es_offs), es_offs, hlens))
            host.append((hinfo, hlens))
        if fused is not None:  # rows of the launch -> job indices
            verify.append((np.asarray(idx, dtype=np.int64)[fused[0]], fused[1]))
        ev = self._event()
        tm.add("demux_launch", time.perf_counter() - t2)
        return _Batch(jobs, infos=infos, host=host, event=ev, results=results, keep=(dec, host_block), start=ev0,
                      verify=verify or None, expect_mask=mask)

    # ------------------------------------------------------------------ columnar batch
    def launch_columns(self, src: torch.Tensor, offs: np.ndarray, nbytes: np.ndarray, enc: np.ndarray,
                       drk: np.ndarray, iv: np.ndarray, tag: Any = None, keys: Optional[np.ndarray] = None,
                       expect: Optional[np.ndarray] = None) -> Optional["_Batch"]:
        """A batch given as columns (a fleet rank: no job object per fragment).  Fragment
        ``i`` is ``src[offs[i] : offs[i] + nbytes[i]]`` (the node's HBM arena, 16-byte aligned
        offsets); ``enc[i]``: AES-128-CBC with round keys ``drk[i]`` (44 little-endian words,
        ``ops.aes.round_keys_le``) and ``iv[i]``; ``keys[i]`` (raw 16-byte keys) is only read
        by the CPU path.  ``expect[i] >= 0``: fragment i's bytes must have that CRC-32 (a
        peer's trailer, verified here instead of by the node): an encrypted fragment is
        checked by the decrypt itself (the CRC fused into ``aes_cbc.hip``), a clear one by the
        CRC kernel; :meth:`complete_columns` reports the outcome.  ``tag`` comes back from
        :meth:`complete_columns`."""
        n = len(offs)
        if n == 0:
            return None
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        nb = np.ascontiguousarray(nbytes, dtype=np.int64)
        enc = np.asarray(enc, dtype=bool)
        if expect is not None:
            expect = np.ascontiguousarray(expect, dtype=np.int64)
            if not (expect >= 0).any():
                expect = None
        self.segments += n
        self.bytes_in += int(nb.sum())
        self.batches += 1
        t1 = time.perf_counter()
        if self.device.type != "cuda":  # CPU mode: the job path (host kernels)
            jobs = []
            for i in range(n):
                o, k = int(offs[i]), int(nb[i])
                key = bytes(keys[i]) if (enc[i] and keys is not None) else None
                jobs.append(TransmuxJob(src[o:o + k], key, bytes(iv[i]) if key is not None else None, None))
            b = self.launch_jobs(jobs)
            b.tag = tag
            if expect is not None:  # host CRC of the same bytes
                vi = np.flatnonzero(expect >= 0)
                got = _rt().crc32_batch(src.numpy(), offs[vi], nb[vi])
                b.verify = [(vi, (got.astype(np.int64) & 0xFFFFFFFF) == (expect[vi] & 0xFFFFFFFF))]
                b.expect_mask = expect >= 0
            return b
        ok = ~(enc & ((nb <= 0) | (nb % 16 != 0)))  # encrypted payloads must be whole AES blocks
        idx_ok = np.flatnonzero(ok)
        verify = []
        ex = None
        if expect is not None:
            # bytes with an expected CRC that no decrypt pass reads -- clear fragments, and
            # encrypted ones rejected for their length -- go through the CRC kernel: every
            # fragment that asked for a check gets one (complete_columns reports the rest False)
            crc_v = np.flatnonzero((expect >= 0) & (~enc | ~ok))
            if len(crc_v):
                from ..ops import crc as _crc

                _, okd = _crc.crc32_batch(src, offs[crc_v], nb[crc_v], expect=(expect[crc_v] & 0xFFFFFFFF).tolist())
                okh = torch.empty(len(crc_v), dtype=torch.uint8, pin_memory=True)
                okh.copy_(okd, non_blocking=True)
                verify.append((crc_v, okh))
            ex = np.where(enc, expect, -1)[ok] if (expect[enc & ok] >= 0).any() else None
        if not len(idx_ok):  # nothing to decrypt or demux (the CRC checks above still run)
            return _Batch(None, infos=[], host=[], event=self._event() if verify else None, tag=tag, n=n,
                          verify=verify or None, expect_mask=None if expect is None else expect >= 0)
        if not ok.all():
            offs, nb, enc, drk, iv = offs[ok], nb[ok], enc[ok], drk[ok], iv[ok]
        td0, isb = _aes.device_tables(self.device)
        cw, ctab = (None, None)
        if ex is not None:
            from ..ops import crc as _crc

            cw, ctab = _crc.fused_consts(self.device)
        ev0 = self._event()
        groups, dec, host_block, fused = _native_device().transmux_launch(
            src, offs, nb, enc.astype(np.uint8), np.ascontiguousarray(drk, dtype=np.uint32),
            np.ascontiguousarray(iv, dtype=np.uint8), td0, isb, _ts.DEFAULT_MAX_PES, ex, cw, ctab)
        infos, host = [], []
        for gidx, info, pes, es, es_offs, hinfo, hlens in groups:
            infos.append((idx_ok[gidx], _ts.DemuxResult(info, pes, es, es_offs), es_offs, hlens))
            host.append((hinfo, hlens))
        if fused is not None:
            verify.append((idx_ok[fused[0]], fused[1]))
        ev = self._event()
        self.timer.add("launch_columns", time.perf_counter() - t1)
        return _Batch(None, infos=infos, host=host, event=ev, keep=(dec, host_block), tag=tag, n=n, start=ev0,
                      verify=verify or None, expect_mask=None if expect is None else expect >= 0)

    def launch_jobs(self, jobs: List[TransmuxJob]) -> "_Batch":
        """:meth:`launch` for an explicit job list (the pipeline's own queue untouched)."""
        try:
            return self._launch(jobs)
        except Exception as e:  # noqa: BLE001 - delivered to every job of the batch
            return _Batch(jobs, error=e)

    def complete_columns(self, batch: "_Batch"):
        """Wait for a :meth:`launch_columns` batch: ``(tag, rows int64[n, INFO_WORDS], plain
        int64[n], has_row bool[n], verified bool[n])`` aligned with the launch columns
        (``verified[i]`` False: fragment i failed its ``expect`` CRC)."""
        if batch.jobs is not None:  # CPU job path
            _, rows, plain, has = self.complete_arrays(batch)
            return batch.tag, rows, plain, has, self._verified(batch, len(batch.jobs))
        n = batch.n
        rows = np.zeros((n, _ts.INFO_WORDS), dtype=np.int64)
        plain = np.full(n, -1, dtype=np.int64)
        has = np.zeros(n, dtype=bool)
        t3 = time.perf_counter()
        self._wait(batch)
        self.timer.add("wait_device", time.perf_counter() - t3)
        for (idx, _res, _es_offs, _lens), (hinfo, hlens) in zip(batch.infos, batch.host):
            k = len(idx)
            rows[idx] = (hinfo.numpy() if isinstance(hinfo, torch.Tensor) else np.asarray(hinfo))[:k]
            plain[idx] = (hlens.numpy() if isinstance(hlens, torch.Tensor) else np.asarray(hlens))[:k]
            has[idx] = True
        return batch.tag, rows, plain, has, self._verified(batch, n)

    @staticmethod
    def _verified(batch: "_Batch", n: int) -> np.ndarray:
        """Per fragment: passed its CRC check (True where none was asked); call after the wait.
        A fragment that asked for a check is True only if a check actually ran and passed."""
        out = np.ones(n, dtype=bool)
        if batch.expect_mask is not None:
            out[batch.expect_mask] = False
        for idx, ok in batch.verify or ():
            out[idx] = (ok.numpy() if isinstance(ok, torch.Tensor) else np.asarray(ok)).astype(bool)
        return out

    def complete_rows(self, batch: Optional["_Batch"]) -> List[Tuple["TransmuxJob", Optional[list], int]]:
        """Wait for a launched batch and return ``(job, info row, plaintext length)`` per job
        without building the per-fragment result dicts or running callbacks (a fleet node
        ships the rows to its player processes; ``row`` is None for a rejected job)."""
        if batch is None:
            return []
        if batch.error is not None:
            return [(j, None, -1) for j in batch.jobs]
        t3 = time.perf_counter()
        self._wait(batch)
        self.timer.add("wait_device", time.perf_counter() - t3)
        out: List[Any] = [None] * len(batch.jobs)
        for (idx, _res, _es_offs, _lens), (hinfo, hlens) in zip(batch.infos, batch.host):
            rows = (hinfo.numpy() if isinstance(hinfo, torch.Tensor) else hinfo).tolist()
            plain = (hlens.numpy() if isinstance(hlens, torch.Tensor) else np.asarray(hlens)).tolist()
            for k, i in enumerate(idx):
                out[i] = (batch.jobs[i], rows[k], int(plain[k]))
        for i, o in enumerate(out):
            if o is None:  # rejected before launch (e.g. not a multiple of 16 bytes)
                out[i] = (batch.jobs[i], None, -1)
        return out

    def complete_arrays(self, batch: Optional["_Batch"]):
        """Wait for a launched batch; return ``(jobs, rows, plain, has_row)``: the info rows as
        one int64 array ``[n, INFO_WORDS]`` aligned with ``jobs``, the plaintext lengths, and
        whether each job has a row (False: rejected before launch; its ``plain`` is -1).  The
        columnar form a fleet node ships to its players without a Python object per word."""
        if batch is None:
            return [], None, None, None
        n = len(batch.jobs)
        rows = np.zeros((n, _ts.INFO_WORDS), dtype=np.int64)
        plain = np.full(n, -1, dtype=np.int64)
        has = np.zeros(n, dtype=bool)
        if batch.error is not None:
            return batch.jobs, rows, plain, has
        t3 = time.perf_counter()
        self._wait(batch)
        self.timer.add("wait_device", time.perf_counter() - t3)
        for (idx, _res, _es_offs, _lens), (hinfo, hlens) in zip(batch.infos, batch.host):
            k = len(idx)
            rows[idx] = (hinfo.numpy() if isinstance(hinfo, torch.Tensor) else np.asarray(hinfo))[:k]
            plain[idx] = (hlens.numpy() if isinstance(hlens, torch.Tensor) else np.asarray(hlens))[:k]
            has[idx] = True
        return batch.jobs, rows, plain, has

    def _complete(self, b: "_Batch") -> List[Dict[str, Any]]:
        tm = self.timer
        t3 = time.perf_counter()
        self._wait(b)
        t4 = time.perf_counter()
        tm.add("wait_device", t4 - t3)
        results = b.results
        for (idx, res, es_offs, lens), (hinfo, hlens) in zip(b.infos, b.host):
            hinfo = hinfo.numpy() if isinstance(hinfo, torch.Tensor) else hinfo
            plain_lens = hlens.numpy() if isinstance(hlens, torch.Tensor) else hlens
            rows = hinfo.tolist()
            es = res.es
            for k, i in enumerate(idx):
                row = rows[k]
                # ES views (per class, at the row's offsets from es_offs[k]) are built on first access: the
                # buffer path only needs their byte counts, which the info row holds
                r = _Result(status=row[0], info=InfoRow(row), plain_bytes=int(plain_lens[k]), demux=res, index=k)
                r._es = (es, es_offs[k], row[_VB], row[_AB], row[_IB], row[_AO], row[_IO])
                if plain_lens[k] < 0:
                    r["error"] = ValueError("decryption failed (bad PKCS#7 padding)")
                results[i] = r
        tm.add("results", time.perf_counter() - t4)
        return results  # type: ignore[return-value]


def _mask(n: int, idx) -> Optional[np.ndarray]:
    """bool[n] with ``idx`` set (None when ``idx`` is empty)."""
    if not len(idx):
        return None
    m = np.zeros(n, dtype=bool)
    m[np.asarray(idx, dtype=np.int64)] = True
    return m


_VB, _AB, _IB = _ts.INFO["video_bytes"], _ts.INFO["audio_bytes"], _ts.INFO["id3_bytes"]
_AO, _IO = _ts.INFO["audio_es_offset"], _ts.INFO["id3_es_offset"]


class _Result(dict):
    """One fragment's transmux result: ``status``, ``info``, ``plain_bytes``, ``demux``,
    ``index`` (and ``error``) stored; ``video`` / ``audio`` / ``id3`` ES views of the batch's
    ES buffer made on first access."""

    __slots__ = ("_es",)

    def __missing__(self, key):
        if key not in ("video", "audio", "id3"):
            raise KeyError(key)
        es, base, vb, ab, ib, ao, io = self._es
        v = es.narrow(0, base, vb)
        a = es.narrow(0, base + ao, ab)
        i = es.narrow(0, base + io, ib)
        self["video"], self["audio"], self["id3"] = v, a, i
        return self[key]


class InfoRow:
    """Read-only ``{name: value}`` view of one demux ``info`` row (names of
    :data:`ops.tsdemux.INFO`), sharing one key->slot schema instead of a dict per fragment."""

    __slots__ = ("_row",)
    _SLOTS = _ts.INFO

    def __init__(self, row) -> None:
        self._row = row

    def __getitem__(self, name: str) -> int:
        return self._row[self._SLOTS[name]]

    def get(self, name: str, default=None):
        slot = self._SLOTS.get(name)
        return default if slot is None else self._row[slot]

    def keys(self):
        return self._SLOTS.keys()

    def items(self):
        return ((k, self._row[v]) for k, v in self._SLOTS.items())

    def __contains__(self, name: str) -> bool:
        return name in self._SLOTS

    def __iter__(self):
        return iter(self._SLOTS)

    def __len__(self) -> int:
        return len(self._SLOTS)

    def to_dict(self):
        return dict(self.items())

    def __repr__(self) -> str:
        return f"InfoRow({self.to_dict()})"


@dataclass(eq=False)
class _Batch:
    jobs: List[TransmuxJob]
    infos: Any = None
    host: Any = None
    event: Any = None
    results: Any = None
    error: Optional[BaseException] = None
    keep: Any = None  # device/pinned buffers the batch's in-flight work uses
    tag: Any = None  # launch_columns: the caller's columns, handed back by complete_columns
    n: int = 0  # launch_columns: fragments in the batch
    start: Any = None  # timing event recorded before the batch's first launch
    verify: Any = None  # [(fragment indices, ok flags (pinned uint8 / bool))] of expect-CRC checks
    expect_mask: Any = None  # bool[n]: fragments that asked for a CRC check (unchecked ones fail)


_local = threading.local()


def pipeline_for(device: torch.device, loop=None) -> MediaPipeline:
    """The calling thread's pipeline for ``device``."""
    cache = getattr(_local, "pipes", None)
    if cache is None:
        cache = {}
        _local.pipes = cache
    loop = loop or get_event_loop()
    key = (str(device), id(loop))
    p = cache.get(key)
    if p is None:
        p = MediaPipeline(device, loop)
        cache[key] = p
    return p


def default_transmux_device() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
