"""Root-cause probe for the IPC-event failure of the single-GPU rehearsal plane
(parallel/comm.py:_IpcOutbox, HLSP2P_IPC_EVENTS=1): `hipStreamWaitEvent` on a peer's
interprocess event returned `invalid argument` after a few hundred rounds of a 4-rank soak.

N ranks on ONE MI355X (torchrun --nproc-per-node N, gloo), the outbox protocol stripped to
its event traffic: each round a rank runs a small kernel and records its interprocess event
(only on rounds where it "has sends", --send-prob), host barrier, then its stream waits on
the event of every peer that recorded this round, runs a kernel, host barrier.  Prints the
first failing round per rank with the record / wait counts at that point.

  --mode wait      : the protocol (events opened once)
  --mode reopen    : re-open the peers' handles every --every rounds
  --mode query     : hipEventQuery on the peers' events instead of stream waits
  --mode sync      : hipEventSynchronize (host) on the peers' events instead of stream waits
  --mode renew     : the fix — a ring of --ring events per rank, the whole set re-created and
                     re-shared before any event reaches 32 records (previous set kept alive
                     one generation)

Finding (gpurun, ROCm 7.2, MI355X): an interprocess event survives exactly 32 records —
the stream wait after a peer's 33rd record fails with `invalid argument`, for 2 and 4 ranks,
dense or sparse recording, re-opened handles or not; hipEventQuery never fails.
"""
import argparse
import os
import random
import sys
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="wait", choices=["wait", "reopen", "query", "sync", "renew"])
    ap.add_argument("--ring", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2000)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--send-prob", type=float, default=1.0, help="probability a rank records in a round")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream()
    x = torch.zeros(1 << 16, device=dev)
    K = args.ring if args.mode == "renew" else 1
    per_gen = 30 * K  # rounds per event generation: each event recorded <= 30 times

    def make_set():
        evs = [torch.cuda.Event(interprocess=True) for _ in range(K)]
        for e in evs:
            e.record(s)
        torch.cuda.synchronize()
        hs = [None] * world
        dist.all_gather_object(hs, [e.ipc_handle() for e in evs])
        peer = [None if r == rank else [torch.cuda.Event.from_ipc_handle(dev, h) for h in hs[r]]
                for r in range(world)]
        return evs, peer

    own, peers = make_set()
    old = None
    rng = random.Random(1234)  # identical on every rank: everyone knows who recorded
    records = waits = 0
    failed, err = -1, ""
    t0 = time.perf_counter()
    for r in range(args.rounds):
        if args.mode == "renew" and r and r % per_gen == 0:
            old = (own, peers)  # kept alive one generation: queued waits may still reference it
            own, peers = make_set()
        k = r % K
        rec = [rng.random() < args.send_prob for _ in range(world)]
        if failed < 0 and rec[rank]:
            with torch.cuda.stream(s):
                x.add_(1.0)
            own[k].record(s)
            records += 1
        dist.barrier()
        if args.mode == "reopen" and r and r % args.every == 0:  # collective: every rank, failed or not
            hs = [None] * world
            dist.all_gather_object(hs, [e.ipc_handle() for e in own])
            peers = [None if q == rank else [torch.cuda.Event.from_ipc_handle(dev, h) for h in hs[q]]
                     for q in range(world)]
        if failed < 0:
            try:
                for src in range(world):
                    if src == rank or not rec[src]:
                        continue
                    if args.mode in ("wait", "reopen", "renew"):
                        s.wait_event(peers[src][k])
                    elif args.mode == "query":
                        peers[src][k].query()
                    else:
                        peers[src][k].synchronize()
                    waits += 1
                with torch.cuda.stream(s):
                    x.add_(1.0)
            except Exception as e:  # noqa: BLE001 - the failure being probed
                failed, err = r, f"{type(e).__name__}: {str(e).splitlines()[0]}"
        if r % 50 == 0:
            torch.cuda.synchronize()
        dist.barrier()
    del old
    torch.cuda.synchronize()
    out = [None] * world
    dist.all_gather_object(out, (failed, records, waits, err))
    if rank == 0:
        print(f"mode={args.mode} world={world} rounds={args.rounds} send_prob={args.send_prob} every={args.every} "
              f"({time.perf_counter() - t0:.1f} s)", flush=True)
        for k, (f, rc, w, e) in enumerate(out):
            print(f"  rank {k}: first failure round {f} records {rc} waits {w} {e}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
