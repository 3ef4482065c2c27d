#!/usr/bin/env python3
"""tools/placement_probe.py -- how much of the encode / decode rate is arena placement?
One process: BASELINE configs[1] arenas (5 x 256 MiB + 3 out) re-allocated several times
as separate tensors, and carved out of one allocation at several strides.  Not product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

k, m, n, B = 3, 2, 4096, 65536
L = n * B
mat = ec.coding_matrix(k, m)
s = torch.cuda.current_stream()
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
ep = ec.Plan([(i * n, 0, n, 0) for i in range(B)])
dp = ec.Plan([(i * n, 0, n, i % 6) for i in range(B)])


def timed(fn, iters=10):
    fn()
    a, b = ec.Event(), ec.Event()
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    return a.elapsed_ms(b) / iters


def measure(arenas, label):
    data, parity, out = arenas[:k], arenas[k:k + m], arenas[k + m:]
    for t in data:
        t.random_(0, 256)
    te = timed(lambda: ec.encode(k, m, mat, data, parity, ep, s))
    td = timed(lambda: ec.decode(k, m, mat, masks, data + parity, out, dp, s))
    print(f"{label:40s} encode {5 * L / te / 1e6:6.0f} GB/s  decode {4 * L / td / 1e6:6.0f} GB/s  "
          f"step {te + td:.4f} ms", flush=True)


for trial in range(4):
    arenas = [torch.empty(L, dtype=torch.uint8, device="cuda") for _ in range(k + m + k)]
    measure(arenas, f"separate allocations #{trial}")
    del arenas
    torch.cuda.empty_cache()
extras = [int(x) for x in os.environ.get("PROBE_EXTRAS", "0,4096,65536,2097152,12544").split(",")]
for trial in range(int(os.environ.get("PROBE_TRIALS", "1"))):
    for extra in extras:
        stride = L + extra
        big = torch.empty(stride * (k + m + k), dtype=torch.uint8, device="cuda")
        arenas = [big[i * stride:i * stride + L] for i in range(k + m + k)]
        measure(arenas, f"one allocation, stride L+{extra} #{trial}")
        del arenas, big
        torch.cuda.empty_cache()
