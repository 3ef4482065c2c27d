#!/usr/bin/env python3
"""tools/encode_gap.py -- where do the last percent of the RS(3,2) 4 KiB encode go?
One process, the bench's arenas, interleaved rounds (not product):
  plan      cec_encode over the 65,536-extent plan (the bench's kernel)
  region    cec_encode_region: the same bytes as one implicit range (no tile list)
  xor       cec_encode_region with both parity rows all ones (no GF multiply)
  plan_xor  the plan with the all-ones matrix
ENCODE_GAP_STRIPES=b: b stripes instead of 65,536 (the strong-scaling shares: is the
small launch's fixed cost in the tile list, the GF multiply or neither?)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

k, m, n = 3, 2, 4096
B = int(os.environ.get("ENCODE_GAP_STRIPES", "65536"))
L = n * B
mat = ec.coding_matrix(k, m)
ones = mat[:k * k] + [1] * (m * k)
s = torch.cuda.current_stream()
ar = ec.arena_tensors(k + m, L)
for t in ar[:k]:
    t.random_(0, 256)
data, par = ar[:k], ar[k:]
plan = ec.Plan([(i * n, 0, n, 0) for i in range(B)])
runs = {
    "plan": lambda: ec.encode(k, m, mat, data, par, plan, s),
    "region": lambda: ec.encode_region(k, m, mat, data, par, L, s),
    "xor": lambda: ec.encode_region(k, m, ones, data, par, L, s),
    "plan_xor": lambda: ec.encode(k, m, ones, data, par, plan, s),
}
res = {x: [] for x in runs}
a, b = ec.Event(), ec.Event()
for rnd in range(8):
    for name, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        a.record(s)
        for _ in range(10):
            fn()
        b.record(s)
        res[name].append(a.elapsed_ms(b) / 10)
print(f"stripes {B}")
for name, v in res.items():
    v.sort()
    print(f"{name:9s} median {v[len(v) // 2] * 1e3:7.1f} us  {5 * L / (v[len(v) // 2] * 1e-3) / 1e9:6.0f} GB/s  "
          f"best {5 * L / (v[0] * 1e-3) / 1e9:6.0f}")
