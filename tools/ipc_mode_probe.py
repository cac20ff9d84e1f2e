"""Which HIP IPC exports work under each HSA IPC mode (one process, no peers).

    HSA_ENABLE_IPC_MODE_LEGACY=0 python tools/ipc_mode_probe.py
    HSA_ENABLE_IPC_MODE_LEGACY=1 python tools/ipc_mode_probe.py

Exports what a multi-rank run exports: a device buffer's IPC handle (``hipIpcGetMemHandle``:
RCCL's intra-node P2P transport maps peer buffers this way, and so do the HIP-IPC rehearsal
outboxes) and an interprocess event handle (``hipIpcGetEventHandle``).  Prints one JSON line.
"""
import json
import os

import torch


def main():
    out = {"HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}
    buf = torch.empty(1 << 20, dtype=torch.uint8, device="cuda:0")
    try:
        buf.untyped_storage()._share_cuda_()
        out["hipIpcGetMemHandle"] = "ok"
    except Exception as e:  # noqa: BLE001 - the probe reports the failure
        out["hipIpcGetMemHandle"] = f"{type(e).__name__}: {e}".splitlines()[0][:200]
    try:
        ev = torch.cuda.Event(interprocess=True)
        ev.record()
        ev.ipc_handle()
        out["hipIpcGetEventHandle"] = "ok"
    except Exception as e:  # noqa: BLE001
        out["hipIpcGetEventHandle"] = f"{type(e).__name__}: {e}".splitlines()[0][:200]
    torch.cuda.synchronize()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
