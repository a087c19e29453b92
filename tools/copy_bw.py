"""Device copy bandwidth reference point (torch copy_, same bytes as an N=1024 x count u64 NTT pass)."""
import sys
import torch
count = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
x = torch.empty(count * 1024, dtype=torch.int64, device="cuda")
y = torch.empty_like(x)
for _ in range(5):
    y.copy_(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    y.copy_(x)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 200 * 1e3
print(f"copy count={count}: {us:.2f} us  {2 * x.numel() * 8 / us / 1e3:.1f} GB/s")
