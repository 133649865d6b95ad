"""Write-only HBM bandwidth reference: fill / zero / copy of a 4.1 GB buffer (the size of one
10^6-command log window), timed with HIP events."""
import torch

n = 4_100_000_000
x = torch.empty(n, dtype=torch.uint8, device="cuda")
y = torch.empty(n // 2, dtype=torch.uint8, device="cuda")
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for name, f, b in [("fill_", lambda: x.fill_(7), n), ("zero_", lambda: x.zero_(), n),
                   ("copy 2.05 GB", lambda: y.copy_(x[: n // 2]), n)]:
    f()
    torch.cuda.synchronize()
    s.record()
    for _ in range(5):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 5
    print(f"{name}: {ms:.3f} ms  {b / ms / 1e9:.2f} TB/s (bytes moved {b / 1e9:.2f} GB)")
