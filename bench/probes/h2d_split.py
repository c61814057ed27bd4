"""Probe: H2D bandwidth of one 126 MB pinned copy (one streaming micro-batch of text) vs the same
bytes split into k chunks on k streams (several SDMA engines in flight)."""
import json

import torch

dev = torch.device("cuda:0")
nbytes = 65536 * 1930
src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
src.fill_(7)
dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
streams = [torch.cuda.Stream(dev) for _ in range(8)]
out = {}
for k in (1, 2, 4, 8):
    chunk = (nbytes + k - 1) // k
    for rep in range(2):          # first pass warms up
        main = torch.cuda.current_stream(dev)
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record(main)
        iters = 20
        for _ in range(iters):
            ev = main.record_event()
            for i in range(k):
                s = streams[i]
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    dst[i * chunk:(i + 1) * chunk].copy_(src[i * chunk:(i + 1) * chunk], non_blocking=True)
            for i in range(k):
                main.wait_stream(streams[i])
        t1.record(main)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / iters
    out[f"chunks_{k}"] = {"ms_per_batch": round(ms, 3), "GB_per_s": round(nbytes / ms / 1e6, 2)}
print(json.dumps(out))
