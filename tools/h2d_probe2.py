"""Can the CDN ingest beat one DMA engine?  192 MB pinned -> HBM as one copy, and the same
bytes split over 2 / 3 / 4 streams (separate copy engines).  Run it also under
HSA_ENABLE_SDMA=0 (blit kernels instead of SDMA engines).  Prints GB/s."""
import time

import torch



def timeit(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    total = 192 << 20
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    host.random_(0, 255)
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    res = {"one_copy": total / timeit(lambda: dev.copy_(host, non_blocking=True)) / 1e9}
    for ns in (2, 3, 4):
        streams = [torch.cuda.Stream() for _ in range(ns)]
        part = total // ns

        def run():
            cur = torch.cuda.current_stream()
            for i, s in enumerate(streams):
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    dev[i * part:(i + 1) * part].copy_(host[i * part:(i + 1) * part], non_blocking=True)
            for s in streams:
                cur.wait_stream(s)

        res[f"split_{ns}_streams"] = total / timeit(run) / 1e9
    for k, v in res.items():
        print(f"{k:20s} {v:8.2f} GB/s")


if __name__ == "__main__":
    main()
