"""Root-cause probe for the IPC-event failure of the single-GPU rehearsal plane
(parallel/comm.py:_IpcOutbox, HLSP2P_IPC_EVENTS=1): `hipStreamWaitEvent` on a peer's
interprocess event returned `invalid argument` after a few hundred rounds of a 4-rank soak.

Two ranks on ONE MI355X (torchrun --nproc-per-node 2, gloo): rank 0 records its
interprocess event once per round after a small kernel (as a rank does after packing its
outbox), rank 1 waits on it once per round on its own stream, with the protocol's
host barriers around.  Counts the rounds until the first failure.

  --mode wait      : rank 1 waits every round on the event opened once (the protocol)
  --mode reopen    : rank 1 re-opens the handle every --every rounds
  --mode nowait    : rank 1 never waits (does recording alone fail?)
  --mode query     : rank 1 only queries the event (hipEventQuery) every round
  --waits N        : stream waits per round (a 4-rank round waits on 3 peers)
"""
import argparse
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="wait", choices=["wait", "reopen", "nowait", "query"])
    ap.add_argument("--rounds", type=int, default=3000)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--waits", type=int, default=1)
    args = ap.parse_args()
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = torch.cuda.Stream()
    x = torch.zeros(1 << 16, device=dev)
    if rank == 0:
        ev = torch.cuda.Event(interprocess=True)
        ev.record(s)
        torch.cuda.synchronize()
        h = [ev.ipc_handle()]
    else:
        h = [None]
    dist.broadcast_object_list(h, src=0)
    if rank == 1:
        ev = torch.cuda.Event.from_ipc_handle(dev, h[0])
    t0 = time.perf_counter()
    failed = -1
    err = ""
    for r in range(args.rounds):
        if rank == 0:
            with torch.cuda.stream(s):
                x.add_(1.0)
            ev.record(s)
        dist.barrier()
        if rank == 1 and failed < 0:
            try:
                if args.mode == "reopen" and r and r % args.every == 0:
                    ev = torch.cuda.Event.from_ipc_handle(dev, h[0])
                if args.mode in ("wait", "reopen"):
                    for _ in range(args.waits):
                        s.wait_event(ev)
                    with torch.cuda.stream(s):
                        x.add_(1.0)
                elif args.mode == "query":
                    ev.query()
            except Exception as e:  # noqa: BLE001 - the failure being probed
                failed, err = r, f"{type(e).__name__}: {str(e).splitlines()[0]}"
        if r % 100 == 0:
            torch.cuda.synchronize()
        dist.barrier()
    torch.cuda.synchronize()
    out = [None, None]
    dist.all_gather_object(out, (failed, err))
    if rank == 0:
        print(f"mode={args.mode} waits/round={args.waits} rounds={args.rounds} every={args.every} "
              f"first failure round={out[1][0]} ({out[1][1]}) in {time.perf_counter() - t0:.1f} s", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
