"""Feasibility probe: CUDA-IPC memory + interprocess events between two processes on ONE
MI355X (dmabuf IPC).  Rank 0 exports a buffer and an event, rank 1 opens both, waits on
the event on its stream and copies the bytes.  Prints timings; exits non-zero on mismatch."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = 64 << 20
    if rank == 0:
        buf = torch.empty(n, dtype=torch.uint8, device=dev)
        buf.copy_(torch.arange(n, dtype=torch.int64, device=dev).to(torch.uint8))
        ev = torch.cuda.Event(interprocess=True)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.cuda._sleep(50_000_000)  # the event completes well after rank 1 starts waiting
            buf.add_(1)
            ev.record(s)
        storage = buf.untyped_storage()
        handle = storage._share_cuda_()
        objs = [handle, ev.ipc_handle()]
    else:
        objs = [None, None]
    dist.broadcast_object_list(objs, src=0)
    if rank == 1:
        handle, evh = objs
        t0 = time.perf_counter()
        st = torch.UntypedStorage._new_shared_cuda(*handle)
        peer = torch.empty(0, dtype=torch.uint8, device=dev).set_(st, 0, (st.nbytes(),))
        ev = torch.cuda.Event.from_ipc_handle(dev, evh)
        t1 = time.perf_counter()
        out = torch.empty(n, dtype=torch.uint8, device=dev)
        s = torch.cuda.Stream()
        s.wait_event(ev)
        t2 = time.perf_counter()
        with torch.cuda.stream(s):
            out.copy_(peer[:n], non_blocking=True)
        s.synchronize()
        t3 = time.perf_counter()
        ref = (torch.arange(n, dtype=torch.int64, device=dev).to(torch.uint8) + 1)
        ok = torch.equal(out, ref)
        print(f"rank1 open {1e3 * (t1 - t0):.1f} ms, wait enqueue {1e3 * (t2 - t1):.2f} ms, "
              f"copy+wait {1e3 * (t3 - t2):.1f} ms, equal={ok}", flush=True)
        # bandwidth of a same-device peer copy
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            out.copy_(peer[:n], non_blocking=True)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 10
        print(f"rank1 ipc D2D copy {n / ms / 1e6:.0f} GB/s", flush=True)
        if not ok:
            sys.exit(3)
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
