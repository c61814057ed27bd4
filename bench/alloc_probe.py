import torch, time
d = torch.device("cuda:0")
torch.zeros(1, device=d); torch.cuda.synchronize()
for n in (1 << 30, 4 << 30, 4 << 30):
    t = time.perf_counter(); x = torch.empty(n, dtype=torch.uint8, device=d); torch.cuda.synchronize(); a = time.perf_counter() - t
    t = time.perf_counter(); x.zero_(); torch.cuda.synchronize(); b = time.perf_counter() - t
    print(f"empty {n>>20} MB: {a*1e3:.2f} ms, first zero_ {b*1e3:.2f} ms")
    t = time.perf_counter(); x.zero_(); torch.cuda.synchronize(); print(f"  second zero_ {(time.perf_counter()-t)*1e3:.2f} ms")
    del x
import numpy as np
a = np.arange(300000, dtype=np.int64)
for i in range(3):
    t = time.perf_counter(); x = torch.from_numpy(a).to(d); torch.cuda.synchronize(); print(f"pageable H2D 2.4MB: {(time.perf_counter()-t)*1e3:.2f} ms")
b = np.arange(1000, dtype=np.int32)
for i in range(3):
    t = time.perf_counter(); x = torch.from_numpy(b).to(d); torch.cuda.synchronize(); print(f"pageable H2D 4KB: {(time.perf_counter()-t)*1e3:.2f} ms")
y = torch.zeros(1200000, dtype=torch.int64, device=d)
for i in range(3):
    t = time.perf_counter(); z = y.cpu(); print(f"pageable D2H 9.6MB: {(time.perf_counter()-t)*1e3:.2f} ms")
