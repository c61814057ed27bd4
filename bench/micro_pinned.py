"""CPU read cost of D2H destination buffers: torch pinned vs registered pageable vs plain memory."""
import json
import time

import numpy as np
import torch


def cpu_read_ms(arr: np.ndarray, reps: int = 20) -> float:
    t0 = time.perf_counter()
    s = 0.0
    for _ in range(reps):
        s += float(np.exp(-arr[:, 0]).sum())
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    n = 65536
    dev = torch.device("cuda:0")
    src = torch.randn((n, 1), dtype=torch.float64, device=dev)
    out = {}
    pinned = torch.empty((n, 1), dtype=torch.float64).pin_memory()
    pinned.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    out["torch_pinned_read_ms"] = cpu_read_ms(pinned.numpy())
    plain = torch.empty((n, 1), dtype=torch.float64)
    plain.copy_(src)
    out["plain_read_ms"] = cpu_read_ms(plain.numpy())
    reg = torch.empty((n, 1), dtype=torch.float64)
    rt = torch.cuda.cudart()
    rc = rt.cudaHostRegister(reg.data_ptr(), reg.numel() * 8, 0)
    out["register_rc"] = int(rc) if not isinstance(rc, tuple) else int(rc[0])
    reg.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    out["registered_read_ms"] = cpu_read_ms(reg.numpy())
    # D2H time into each
    for name, dst in (("pinned", pinned), ("plain", plain), ("registered", reg)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        out[f"d2h_{name}_ms"] = (time.perf_counter() - t0) / 20 * 1e3
    print(json.dumps(out))


if __name__ == "__main__":
    main()
