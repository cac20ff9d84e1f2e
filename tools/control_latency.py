"""Control-plane all-gather latency: DistComm over the shared-memory transport vs gloo.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/control_latency.py
(HLSP2P_CONTROL=gloo forces gloo.)  Message: 800 int64 words per rank (~ a 64-want round).
"""
import json
import os
import time

import numpy as np
import torch.distributed as dist

from hlsjs_p2p_wrapper_amd.parallel.comm import DistComm


def main():
    dist.init_process_group("gloo")
    comm = DistComm()
    msg = np.arange(800, dtype=np.int64)
    for _ in range(50):
        comm.allgather_control(msg)
    n = int(os.environ.get("ITERS", "500"))
    t = time.perf_counter()
    for _ in range(n):
        comm.allgather_control(msg)
    us = (time.perf_counter() - t) / n * 1e6
    if comm.rank == 0:
        print(json.dumps({"world": comm.world_size, "transport": comm.control_transport, "allgather_us": round(us, 1)}))
    comm.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
