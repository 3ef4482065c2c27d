#!/usr/bin/env python3
"""tools/isolate.py -- where does the encode kernel lose time inside bench.py?

One process, BASELINE configs[1] buffers: library encode back-to-back, decode
back-to-back, and the bench's alternating encode/decode, each timed with one event pair
around 20 launches (no events between kernels).  Not part of the product.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

k, m, n, B = 3, 2, 4096, 65536
mat = ec.coding_matrix(k, m)
g = torch.Generator(device="cuda").manual_seed(1)
data = [torch.randint(0, 256, (B * n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
parity = [torch.empty(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
ep = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
dp = ec.Plan([(s * n, 0, n, s % 6) for s in range(B)])
s = torch.cuda.current_stream()


def enc():
    ec.encode(k, m, mat, data, parity, ep, s)


def dec():
    ec.decode(k, m, mat, masks, data + parity, out, dp, s)


def enc_region():
    ec.encode_region(k, m, mat, data, parity, B * n)


def timed(fn, iters=20):
    fn()
    a, b = ec.Event(), ec.Event()
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(iters):
        fn()
    b.record(s)
    return a.elapsed_ms(b) / iters


for rnd in range(3):
    te = timed(enc)
    tr = timed(enc_region)
    td = timed(dec)
    ta = timed(lambda: (enc(), dec()))
    print(f"round {rnd}: encode-only {5 * B * n / te / 1e6:.0f} GB/s ({te:.4f} ms)  "
          f"encode_region {5 * B * n / tr / 1e6:.0f}  decode-only {4 * B * n / td / 1e6:.0f} GB/s ({td:.4f} ms)  "
          f"alternating step {ta:.4f} ms (sum of singles {te + td:.4f})", flush=True)

# ---- HIP graph replay of the encode + decode step vs eager launches
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    s2 = torch.cuda.current_stream()
    ec.encode(k, m, mat, data, parity, ep, s2)
    ec.decode(k, m, mat, masks, data + parity, out, dp, s2)
for rnd in range(3):
    tg = timed(lambda: g.replay())
    ta = timed(lambda: (enc(), dec()))
    print(f"round {rnd}: graph step {tg:.4f} ms  eager step {ta:.4f} ms", flush=True)
