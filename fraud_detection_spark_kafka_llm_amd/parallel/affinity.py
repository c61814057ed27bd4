"""NUMA placement for one-process-per-GPU runs.

Each MI355X hangs off one socket's PCIe root complex; a rank whose pinned ring (or any page-locked
staging buffer) sits in the other socket's memory pays the socket interconnect on every H2D copy.
``bind_to_gpu`` restricts the calling process to the CPUs local to its GPU (sysfs
``/sys/bus/pci/devices/<bdf>/local_cpulist``, intersected with the CPUs the process may use) so
that first-touch allocations of later pinned buffers land on the GPU's NUMA node. It is a no-op
when the topology is not visible (containers, CPU-only). ``FDX_NUMA_BIND=0`` disables it.
"""
from __future__ import annotations

import os
from typing import Optional


def parse_cpulist(text: str) -> list:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def gpu_pci_address(index: int) -> Optional[str]:
    import torch

    if not torch.cuda.is_available():
        return None
    p = torch.cuda.get_device_properties(index)
    return f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"


def gpu_local_cpus(index: int, sysfs: str = "/sys/bus/pci/devices") -> Optional[list]:
    bdf = gpu_pci_address(index)
    if bdf is None:
        return None
    try:
        with open(os.path.join(sysfs, bdf, "local_cpulist")) as fh:
            return parse_cpulist(fh.read())
    except OSError:
        return None


def bind_to_gpu(index: int) -> dict:
    """Pin this process to the CPUs local to GPU ``index``; returns what was done."""
    if os.environ.get("FDX_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return {"bound": False, "reason": "disabled"}
    local = gpu_local_cpus(index)
    if not local:
        return {"bound": False, "reason": "topology not visible"}
    allowed = os.sched_getaffinity(0)
    cpus = sorted(set(local) & allowed)
    if not cpus or len(cpus) == len(allowed):
        return {"bound": False, "reason": "no narrower local set", "local": len(local), "allowed": len(allowed)}
    os.sched_setaffinity(0, cpus)
    return {"bound": True, "cpus": len(cpus), "allowed": len(allowed), "pci": gpu_pci_address(index)}
