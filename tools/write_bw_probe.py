"""Probe: raw device write / copy bandwidth for an obs-sized (142.6 MB) buffer
(torch fill_/copy_), the ceiling for the step kernel's observation stream."""
import torch, time
n = 142606336 // 4
x = torch.empty(n, dtype=torch.float32, device="cuda")
y = torch.empty(n, dtype=torch.float32, device="cuda")
def t(f, k=50):
    for _ in range(5): f()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(k): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / k * 1e3
us = t(lambda: x.fill_(1.0)); print("fill 142.6MB us", us, "TB/s", 142.6e6/us/1e6)
us = t(lambda: y.copy_(x)); print("copy us", us, "TB/s (r+w)", 2*142.6e6/us/1e6)
big = torch.empty(8*n, dtype=torch.float32, device="cuda")
us = t(lambda: big.fill_(1.0), 20); print("fill 1.14GB us", us, "TB/s", 8*142.6e6/us/1e6)
