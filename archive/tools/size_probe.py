#!/usr/bin/env python3
"""tools/size_probe.py -- does the encode rate depend on the launch size or on the value
size?  One process, library encode (PERM), back-to-back launches, events around 10.
Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

k, m = 3, 2
mat = ec.coding_matrix(k, m)
s = torch.cuda.current_stream()
MAXB = 1 << 30
g = torch.Generator(device="cuda").manual_seed(3)
data = [torch.randint(0, 256, (MAXB,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
parity = [torch.empty(MAXB, dtype=torch.uint8, device="cuda") for _ in range(m)]


def timed(fn, iters=10):
    fn()
    a, b = ec.Event(), ec.Event()
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    return a.elapsed_ms(b) / iters


cases = []
for per_shard in (64 << 20, 256 << 20, 1 << 30):
    for n in (4096, 65536, 1 << 20):
        B = per_shard // n
        cases.append((per_shard, n, ec.Plan([(i * n, 0, n, 0) for i in range(B)])))
for rnd in range(2):
    for per_shard, n, plan in cases:
        t = timed(lambda: ec.encode(k, m, mat, data, parity, plan, s))
        print(f"round {rnd}: {per_shard >> 20:5d} MiB/shard  value {n:8d} B  {t:.4f} ms  "
              f"{5 * per_shard / t / 1e6:.0f} GB/s", flush=True)
    for per_shard in (64 << 20, 256 << 20, 1 << 30):
        t = timed(lambda: ec.encode_region(k, m, mat, data, parity, per_shard, s))
        print(f"round {rnd}: {per_shard >> 20:5d} MiB/shard  region          {t:.4f} ms  "
              f"{5 * per_shard / t / 1e6:.0f} GB/s", flush=True)
