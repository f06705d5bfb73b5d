#!/usr/bin/env python3
"""Per-launch kernel time over a few seconds of back-to-back launches (DVFS / power steady state)."""
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from extio_sddc_amd import R2iq, output_samples
d = int(sys.argv[1]) if len(sys.argv) > 1 else 0
nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
secs = float(sys.argv[3]) if len(sys.argv) > 3 else 3.0
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(1)
src = sys.argv[4] if len(sys.argv) > 4 else "uniform"
if src == "mix":
    import bench
    x = bench.make_input(torch, nblk, 0x5DDC, dev)
elif src == "zeros":
    x = torch.zeros(4096 + nblk * 65536, dtype=torch.int16, device=dev)
else:
    x = torch.randint(-30000, 30000, (4096 + nblk * 65536,), dtype=torch.int16, device=dev, generator=g)
y = torch.empty(output_samples(d, nblk) * 2, dtype=torch.float32, device=dev)
r = R2iq(1.0); r.setDecimate(d); r.setTuneBin(1024)
evs = []
t0 = time.time()
while time.time() - t0 < secs:
    batch = []
    for _ in range(20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); r.process_device(x, nblk, y); e1.record(); batch.append((e0, e1))
    torch.cuda.synchronize()
    evs += [a.elapsed_time(b) for a, b in batch]
n = len(evs)
q = [evs[int(i * n / 10)] for i in range(10)]
print(json.dumps({"src": src, "d": d, "nblk": nblk, "launches": n, "first5_ms": evs[:5], "decile_ms": q,
                  "last20_median_ms": sorted(evs[-20:])[10],
                  "GSps_last20": nblk * 65536 / (sorted(evs[-20:])[10] * 1e-3) / 1e9}))
