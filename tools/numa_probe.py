#!/usr/bin/env python3
"""Where does this process run relative to its GPU?  PCI address, the GPU's NUMA node and
local CPUs (sysfs), the CPUs this process may use, and the host NUMA layout."""
import glob
import json
import os

import torch

out = {"allowed_cpus": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
p = torch.cuda.get_device_properties(0)
out["props"] = {k: getattr(p, k) for k in dir(p) if k.startswith("pci") or k in ("name", "gcnArchName")}
nodes = {}
for d in sorted(glob.glob("/sys/devices/system/node/node*/cpulist")):
    nodes[d.split("/")[-2]] = open(d).read().strip()
out["numa_nodes"] = nodes
bus = getattr(p, "pci_bus_id", None)
dom = getattr(p, "pci_domain_id", 0)
dev = getattr(p, "pci_device_id", 0)
if bus is not None:
    addr = f"{dom:04x}:{bus:02x}:{dev:02x}.0"
    base = f"/sys/bus/pci/devices/{addr}"
    out["pci_addr"] = addr
    for f in ("numa_node", "local_cpulist"):
        try:
            out[f] = open(os.path.join(base, f)).read().strip()
        except OSError as e:
            out[f] = f"error: {e}"
out["self_numa_hint"] = open("/proc/self/status").read().split("Cpus_allowed_list:")[1].split("\n")[0].strip()
print(json.dumps(out, indent=1, default=str))
