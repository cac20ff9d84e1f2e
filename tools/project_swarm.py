"""One rank of an N-rank swarm on ONE MI355X: the bench's own step, with synthetic peers.

The driver's N=8 run has never happened on this project's hardware pool.  This tool gives the
closest single-GPU stand-in: ``bench.py`` runs unchanged (fleet of player processes, CDN DMA
over PCIe from pinned host memory, the rank's node, the batched GPU transmux with the fused
CRC check) except that the swarm node's communicator is a fake with N-1 synthetic peers
(``tools/round_replay.py:FakePeers``: every peer wants what this rank wants, holds what it
was sent the round before) and its data plane is local:

* the plan is the real N-rank plan of the native planner: this rank seeds 1/N of the
  segments from the CDN and forwards each to the N-1 peers (sends: not executed) and receives
  the other (N-1)/N from the N-1 seeders;
* a receive moves the segment's bytes from an HBM copy of the origin pool into the rank's
  arena run (the HBM traffic of the real send + receive), with the seeder's keyed CRC trailer
  written beside it, so the consumer's fused decrypt CRC checks every received segment as in
  production.  ``--plane copy``: merged ``hipMemcpyAsync`` device-to-device copies on the node
  stream; ``--plane rccl`` (default): a ONE-rank RCCL communicator sends each contiguous span
  to itself in one ``ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd`` call per round on
  the node stream -- RCCL's own kernels move the bytes, holding CUs beside the decrypt grid as
  on the real node (the decrypt leaves the CU reserve free, calibratable with
  ``--cu-calibrate force``).

What it does NOT model: the xGMI links (a receive here is an HBM-to-HBM copy, faster than the
links).  The record therefore states the xGMI receive roofline
of the same bytes, ``(N-1) x 76.8 GB/s`` per direction, and ``projected_ms_per_step`` =
max(measured step, that roofline).

    PYTHONPATH=. python tools/project_swarm.py --peers 8 [bench.py options, e.g. --steps 40 --warmup 10]

Prints one JSON line (``"projection": ...``; never a bench record: ``n_gpus`` stays 1).
"""
from __future__ import annotations

import argparse
import contextlib
import ctypes
import io
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))

XGMI_GBPS_PER_DIR = 76.8  # parallel/wire.py:XGMI_LINK_GBPS_PER_DIR


def _spans(src: np.ndarray, dst: np.ndarray, lens: np.ndarray, max_gap: int, alloc=None):
    """Merge rows whose source and destination advance by the same delta with a gap below
    ``max_gap`` (the arena and the origin pools share the 256-byte alignment) -- and, given
    ``alloc``, whose sources lie in the same allocation -- into spans: (source pointers,
    destination pointers, bytes)."""
    if not len(src):
        z = np.zeros(0, dtype=np.int64)
        return z, z, z
    ds, ss = np.diff(dst), np.diff(src)
    brk = (ds != ss) | (ds < lens[:-1]) | (ds - lens[:-1] >= max_gap)
    if alloc is not None:  # never across two pool copies, even when they happen to be adjacent
        brk |= np.diff(alloc) != 0
    start = np.concatenate([[0], np.flatnonzero(brk) + 1])
    end = np.concatenate([start[1:], [len(src)]]) - 1
    return src[start].copy(), dst[start].copy(), (dst[end] + lens[end] - dst[start]).astype(np.int64)


class DevicePeers:
    """The fake peers' data plane: receives served from an HBM copy of the origin's pools."""

    def __init__(self, comm, node, origins, plane: str = "rccl", ring: int = 16) -> None:
        import torch

        from hlsjs_p2p_wrapper_amd.ops._native import device as _dev

        self.comm, self.node = comm, node
        self.plane = plane
        self.rccl = None
        self.rss = {"before_rccl": _rss_hwm()}
        if plane == "rccl":
            dev = _dev()
            self.rccl = dev.RcclComm(dev.rccl_unique_id(), 1, 0, node.device.index or 0)
            self.rss["after_rccl_init"] = _rss_hwm()
        self.dev = node.device
        # per pool of every synthetic origin: its host allocation base, an HBM copy, the
        # segments' offsets and plain CRC-32s (vectorized lookups: no per-row Python)
        pools = [p for o in origins for p in getattr(o, "pools", [])]
        pools.sort(key=lambda p: p.data.data_ptr())
        self.host_base = np.array([p.data.data_ptr() for p in pools], dtype=np.int64)
        self.dev_copy = [p.data.to(self.dev) for p in pools]
        self.dev_base = np.array([t.data_ptr() for t in self.dev_copy], dtype=np.int64)
        self.offsets = [np.asarray(p.offsets, dtype=np.int64) for p in pools]
        self.crcs = [np.asarray(p.crcs, dtype=np.int64).astype(np.uint32) for p in pools]
        self.ring = [torch.empty(1 << 16, dtype=torch.int32, pin_memory=True) for _ in range(ring)]
        self.ring_i = 0
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_void_p]
        self.hip.hipMemcpyAsync.restype = ctypes.c_int
        self.recv_rows = 0
        self.spans = 0

    def close(self) -> None:
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None

    def exchange_spans(self, sp, sb, sd, rp, rb, rs) -> None:
        import torch

        from hlsjs_p2p_wrapper_amd.agent.node import ALIGN
        from hlsjs_p2p_wrapper_amd.ops import crc as _crc
        from hlsjs_p2p_wrapper_amd.ops._native import device as _dev

        self.comm.exchanges += 1
        h = self.node._last_posted
        if h is None or h.recv is None or not len(rp):
            return
        wids, _, _, roff, lens, keys = h.recv
        info = self.node._wt.info(np.ascontiguousarray(wids))
        ptrs, bases = info[:, 5].copy(), info[:, 6].copy()
        for i in np.flatnonzero(bases == 0).tolist():  # live origins: the node resolves these in Python
            x = self.node._wx.get(int(wids[i]))
            if x is None or x.src is None:
                continue
            origin, path, rng = x.src
            data, off, _, _ = origin.resource(path)
            bases[i] = data.data_ptr()
            ptrs[i] = bases[i] + int(off) + (int(rng[0]) if rng is not None else 0)
        j = np.searchsorted(self.host_base, bases)
        jc = np.minimum(j, len(self.host_base) - 1)
        if ((j >= len(self.host_base)) | (self.host_base[jc] != bases)).any():
            raise RuntimeError("a received want has no synthetic-origin source")
        off = ptrs - bases
        dptr = self.dev_base[j] + off
        dbase = self.dev_base[j]
        plain = np.empty(len(wids), dtype=np.uint32)
        for k in np.unique(j).tolist():  # one lookup per pool
            m = j == k
            at = np.searchsorted(self.offsets[k], off[m])
            if (self.offsets[k][np.minimum(at, len(self.offsets[k]) - 1)] != off[m]).any():
                raise RuntimeError("a received want does not start at a pool segment")
            plain[m] = self.crcs[k][at]
        roff = np.ascontiguousarray(roff, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.int64)
        if self.rccl is None:  # the seeders' bytes: one merged D2D copy per contiguous run, on the node stream
            _dev().h2d_batch(self.node.arena, roff, dptr, lens, dbase, ALIGN, True)
        else:  # one RCCL group call: a send + receive to itself per contiguous span
            a0 = self.node.arena.data_ptr()
            s_ptr, r_ptr, nb = _spans(dptr, a0 + roff, lens, ALIGN, j)
            # host-side bounds of every span before RCCL's kernels touch them: receives inside
            # the arena, sends inside the pool copy they start in
            ends = self.dev_base + np.array([t.numel() for t in self.dev_copy], dtype=np.int64)
            order = np.argsort(self.dev_base)  # the pool copies' device addresses, ascending
            js = np.searchsorted(self.dev_base[order], s_ptr, side="right") - 1
            pool = order[np.maximum(js, 0)]
            if ((r_ptr < a0) | (r_ptr + nb > a0 + self.node.arena.numel()) | (js < 0) |
                    (s_ptr + nb > ends[pool])).any():
                raise RuntimeError("a receive span falls outside the arena or its source pool copy")
            peer = np.zeros(len(s_ptr), dtype=np.int64)
            self.rccl.exchange(s_ptr, nb, peer, r_ptr, nb.copy(), peer.copy(), torch.cuda.current_stream().cuda_stream)
            self.spans += len(s_ptr)
        # their trailers: keyed CRCs, as the seeders' ingest CRC tables hold them.  The
        # receive runs' trailer slices are back to back from row 0 (node._span_columns)
        keyed = plain.view(np.int32) ^ _crc.key_digest(keys)
        n = len(keyed)
        if n > self.ring[0].numel():
            raise RuntimeError("more received rows in one round than the trailer staging ring holds")
        # (a staging buffer is reused 16 rounds later: its H2D, queued on the node stream with
        # this round, completed rounds before -- the bench keeps at most lag + 1 in flight)
        stage = self.ring[self.ring_i]
        self.ring_i = (self.ring_i + 1) % len(self.ring)
        stage.numpy()[:n] = keyed
        stream = torch.cuda.current_stream().cuda_stream
        rc = self.hip.hipMemcpyAsync(ctypes.c_void_p(int(rp[1])), ctypes.c_void_p(stage.data_ptr()), 4 * n, 1,
                                     ctypes.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"hipMemcpyAsync of the trailers failed: {rc}")
        self.recv_rows += n
        if self.comm.exchanges in (1, 2, 10, 100, 1000):  # resident memory as the rounds go
            import torch as _t

            _t.cuda.current_stream().synchronize()
            self.rss[f"after_exchange_{self.comm.exchanges}"] = _rss_hwm()


def _status_mib() -> dict:
    """This process's resident memory by kind (``/proc/self/status``): RssAnon is heap and
    pinned host buffers, RssShmem shared / device-mapped pages, VmHWM the peak."""
    out = {}
    try:
        with open("/proc/self/status") as f:
            for ln in f:
                k = ln.split(":", 1)[0]
                if k in ("VmHWM", "VmRSS", "RssAnon", "RssFile", "RssShmem"):
                    out[k] = round(int(ln.split()[1]) / 1024, 1)
    except OSError:
        pass
    return out


def _rss_hwm() -> list:
    st = _status_mib()
    return [st.get("VmRSS"), st.get("VmHWM")]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--peers", type=int, default=8, help="the swarm size N this rank is one of")
    ap.add_argument("--plane", default="rccl", choices=["rccl", "copy"],
                    help="how received bytes move: a one-rank RCCL self-exchange, or merged D2D copies")
    args, bench_argv = ap.parse_known_args()
    if args.peers < 2:
        raise SystemExit("--peers must be >= 2")
    if os.environ.get("WORLD_SIZE", "1") != "1":
        raise SystemExit("project_swarm.py runs ONE process (rank 0 of the projected swarm)")
    import bench
    from hlsjs_p2p_wrapper_amd import agent
    from hlsjs_p2p_wrapper_amd.net import http as _http
    from round_replay import FakePeers

    churn = 0
    for i, a in enumerate(bench_argv):  # bench.py's --churn rotation, applied to the synthetic peers
        if a == "--churn" and i + 1 < len(bench_argv):
            churn = int(bench_argv[i + 1])
        elif a.startswith("--churn="):
            churn = int(a.split("=", 1)[1])
    comm = FakePeers(args.peers, churn=churn)
    comm.data_transport = f"projection: {args.peers - 1} synthetic peers, {args.plane} receives"
    orig = agent.node_for_config
    made = {}

    class _Hub:
        def comm(self, rank: int):
            return comm

    def node_for_config(p2p_config):
        cfg = dict((p2p_config or {}).get("gpuSwarm") or {})
        if cfg.get("backend", "auto") not in ("auto", "local"):
            return orig(p2p_config)
        cfg.update(backend="thread", hub=_Hub(), rank=0)
        node = orig({**p2p_config, "gpuSwarm": cfg})
        if not node.is_cuda:
            raise SystemExit("project_swarm.py needs the GPU")
        plane = DevicePeers(comm, node, list(_http._registry.values()), args.plane)
        if args.plane == "rccl":  # as DistComm does once its native RCCL plane is open
            from hlsjs_p2p_wrapper_amd.ops._native import device as _dev
            from hlsjs_p2p_wrapper_amd.parallel.comm import RCCL_CU_RESERVE

            _dev().set_cu_reserve(int(os.environ.get("HLSP2P_RCCL_CU_RESERVE", str(RCCL_CU_RESERVE))))
        comm.exchange_spans = plane.exchange_spans
        comm.node = node  # the peers' CDN counters follow what they seeded to this rank
        made["plane"] = plane
        return node

    agent.node_for_config = node_for_config
    if args.peers >= 8 and not any(a == "--inflight" or a.startswith("--inflight=") for a in bench_argv):
        bench_argv = ["--inflight", str(bench.INFLIGHT_N8), *bench_argv]  # bench.py's own default at N >= 8
    sys.argv = ["bench.py", "--cu-calibrate", "off", *bench_argv]
    out = io.StringIO()
    try:
        with contextlib.redirect_stdout(out):
            rc = bench.main()
    finally:
        if "plane" in made:
            made["plane"].rss["before_close"] = _rss_hwm()
            made["plane"].close()
            made["plane"].rss["after_close"] = _rss_hwm()
    lines = [ln for ln in out.getvalue().splitlines() if ln.startswith("{")]
    if rc or not lines:
        print(out.getvalue(), file=sys.stderr)
        return rc or 1
    rec = json.loads(lines[-1])
    from hlsjs_p2p_wrapper_amd.ops._native import device as _dev

    prof = getattr(_dev(), "transmux_launch_profile", None)
    tx = prof() if prof is not None else {}
    calls = max(1, int(tx.pop("calls", 0) or 1))
    tx_us = {k: round(v / calls, 1) for k, v in tx.items()}
    steps, ms = rec["steps"], rec["ms_per_step"]
    pr = (rec.get("per_rank") or [{}])[0]
    p2p_mb = float(pr.get("p2p_recv_MB", 0.0))  # received per round
    rounds_per_step = float(pr.get("rounds", steps)) / max(1, steps)
    roof_ms = p2p_mb * rounds_per_step / (XGMI_GBPS_PER_DIR * (args.peers - 1))  # MB / (GB/s) = ms
    step_ms = max(ms, roof_ms)
    per_rank = rec["value"] * ms / step_ms
    print(json.dumps({
        "projection": f"one rank of a {args.peers}-rank swarm on one MI355X (synthetic peers; receives are HBM "
                      f"copies by {'a one-rank RCCL self-exchange' if args.plane == 'rccl' else 'hipMemcpyAsync'}; "
                      "the xGMI links not modelled)", "plane": args.plane, "rccl_spans": made["plane"].spans,
        "peers": args.peers, "metric": rec["metric"], "unit": rec["unit"],
        "measured_ms_per_step": ms, "measured_per_rank_value": rec["value"],
        "xgmi_receive_roof_ms_per_step": round(roof_ms, 4),
        "projected_ms_per_step": round(step_ms, 4), "projected_per_rank_value": round(per_rank, 2),
        "projected_job_value": round(per_rank * args.peers, 2),
        "offload_ratio": rec.get("offload_ratio"), "received_rows": made["plane"].recv_rows,
        "transmux_launch_us_per_call": tx_us, "host_memory_MiB": _status_mib(),
        "rss_MiB_by_stage": made["plane"].rss,
        "bench_record": rec}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
