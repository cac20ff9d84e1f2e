"""Isolated timing of one transmux batch (decrypt + demux) on the MI355X: the fused kernel
(kernels/transmux_fused.hip) against the split sequence (aes_cbc.hip + ts_demux.hip) and the
scatter demux (ts_scatter.hip: no plaintext buffer), plus
the fused kernel's decomposition (HLSP2P_FUSED_DIAG=1: decrypt alone; =2: no payload
copy-out).  Batches of 1080p 6 Mb/s AES-128 segments (~3 MB), as a bench round delivers them.

    PYTHONPATH=. python tools/transmux_bench.py [--segs 256] [--iters 10]
"""
import argparse
import json
import os

import numpy as np
import torch

from hlsjs_p2p_wrapper_amd.net.origin import PRESET_1080P_6M, SyntheticHlsOrigin
from hlsjs_p2p_wrapper_amd.ops import aes, tsdemux
from hlsjs_p2p_wrapper_amd.ops._native import device


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segs", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--prof", action="store_true", help="also print the fused kernel's per-role timers")
    ap.add_argument("--pool", type=int, default=64,
                    help="distinct segments (the batch cycles through them): 64 x 3 MB fits the 256 MB "
                         "Infinity Cache (MALL), 256 does not -- as in the pipeline, where every segment is new")
    ap.add_argument("--modes", default="", help="comma list of modes to time (default: all)")
    ap.add_argument("--flags", default="0", help="HLSP2P_FUSED_FLAGS for the fused runs (A/B experiments)")
    args = ap.parse_args()
    cuda = torch.device("cuda", 0)
    dev = device()
    pool_n = min(args.segs, args.pool)
    origin = SyntheticHlsOrigin("http://cdn.tb/", renditions=PRESET_1080P_6M, num_segments=pool_n, encrypted=True,
                                pool_size=pool_n, pin_memory=True, seed=5, register=False)
    pool = origin.pools[0]
    src = pool.data.to(cuda)
    offs = np.array([pool.offsets[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    lens = np.array([pool.lengths[i % pool_n] for i in range(args.segs)], dtype=np.int64)
    enc = np.ones(args.segs, dtype=np.uint8)
    drk = np.tile(aes.round_keys_le(origin.key), (args.segs, 1)).astype(np.uint32)
    iv = np.tile(np.frombuffer(origin.iv, dtype=np.uint8), (args.segs, 1))
    td0, isb = aes.device_tables(cuda)
    total = int(lens.sum())
    out = {"segs": args.segs, "bytes": total}

    os.environ["HLSP2P_FUSED_FLAGS"] = args.flags

    def launch():
        return dev.transmux_launch(src, offs, lens, enc, drk, iv, td0, isb, tsdemux.DEFAULT_MAX_PES)

    ap_modes = (("split", "split", None), ("scatter", "scatter", None), ("split_onepass", "split1", None),
                ("fused", "fused", None), ("fused_decrypt_only", "fused", "1"), ("fused_no_copyout", "fused", "2"))
    for name, mode, diag in ap_modes:
        if args.modes and name not in args.modes.split(","):
            continue
        dev.set_transmux_mode("fused" if mode == "fused" else "split")
        dev.set_demux_mode({"split1": "onepass", "scatter": "scatter"}.get(mode, "fourpass"))
        if diag is None:
            os.environ.pop("HLSP2P_FUSED_DIAG", None)
        else:
            os.environ["HLSP2P_FUSED_DIAG"] = diag
        keep = [launch() for _ in range(2)]
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            keep.append(launch())
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / args.iters
        if mode == "fused":  # launches whose hand-off spins gave up (transmux.cpp: zw[z_tk] + 4 bytes)
            out[f"{name}_timeouts"] = sum(int(k[1][0][-2]) >> 32 != 0 for k in keep)
        out[f"{name}_us"] = round(us, 1)
        out[f"{name}_us_per_seg"] = round(us / args.segs, 3)
        out[f"{name}_GBps"] = round(total / (us * 1e-6) / 1e9, 1)
        del keep
    os.environ.pop("HLSP2P_FUSED_DIAG", None)
    dev.set_transmux_mode("split")
    dev.set_demux_mode("fourpass")
    print(json.dumps(out))
    if args.prof:  # HLSP2P_FUSED_PROF=1: [grid][16] shader-clock sums after the hand-off words
        os.environ["HLSP2P_FUSED_PROF"] = "1"
        launch()
        groups, keep, _ = launch()
        torch.cuda.synchronize()
        os.environ.pop("HLSP2P_FUSED_PROF", None)
        p = keep[0][-512 * 16:].view(512, 16).cpu().numpy().astype(np.float64)
        live = p[:, 7] > 0
        names = ["c_job", "c_plain", "c_parse", "c_lookback", "c_plan", "", "", "c_tiles",
                 "d_next", "d_stage", "d_decrypt", "d_tiles", "s_ring", "s_stage", "x_wait", "x_copy"]
        per_tile = {n: round(float(p[live, k].sum() / max(p[live, 7].sum(), 1)), 1) for k, n in enumerate(names)
                    if n and not n.endswith("tiles")}
        print(json.dumps({"workgroups": int(live.sum()), "tiles": int(p[live, 7].sum()),
                          "cycles_per_tile": per_tile}))


if __name__ == "__main__":
    main()
