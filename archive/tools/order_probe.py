#!/usr/bin/env python3
"""tools/order_probe.py WORKLOAD -- does the order of a rotating-erasure decode's tiles
matter?  (tools probe, not product.)  One process, bench.py's arenas and masks (lost
shard and leader rotating per stripe), the same tiles in different orders, interleaved
rounds, median of 10 back-to-back launches each:
  stripe      stripe order (bench.py)
  group       all stripes of mask 0, then mask 1, ...
  win<W>      windows of W consecutive stripes, each window's stripes grouped by mask
Every order rebuilds the same bytes; the probe checks that they equal the originals.
WORKLOAD: rs42_64k (default) or rs32_4k."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

W_ = sys.argv[1] if len(sys.argv) > 1 else "rs42_64k"
k, m, n, B = {"rs42_64k": (4, 2, 65536, 16384), "rs32_4k": (3, 2, 4096, 65536)}[W_]
L = n * B
mat = ec.coding_matrix(k, m)
s = torch.cuda.current_stream()
ar = ec.arena_tensors(k + m + k, L)
for t in ar[:k]:
    t.random_(0, 256)
data, par, out = ar[:k], ar[k:k + m], ar[k + m:]
ec.encode_region(k, m, mat, data, par, L, s)
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
nm = len(masks)


def order(win):
    """Stripe indices: windows of `win` stripes, each grouped by mask (win=1: stripe order)."""
    idx = []
    for w0 in range(0, B, win):
        ws = range(w0, min(B, w0 + win))
        idx += sorted(ws, key=lambda x: (x % nm, x))
    return idx


variants = {"stripe": order(1), "group": order(B)}
for w in (nm * 4, nm * 16, nm * 64, nm * 256):
    variants[f"win{w}"] = order(w)
plans = {name: ec.Plan([(i * n, 0, n, i % nm) for i in idx]) for name, idx in variants.items()}
res = {x: [] for x in plans}
a, b = ec.Event(), ec.Event()
for rnd in range(7):
    for name, plan in plans.items():
        for o in out:
            o.zero_()
        ec.decode(k, m, mat, masks, data + par, out, plan, s)
        torch.cuda.synchronize()
        if rnd == 0:  # every stripe's lost shard rebuilt, whatever the order
            lost = torch.tensor([[j for j in range(k) if not (mk >> j) & 1][0] for mk in masks])[
                torch.arange(B) % nm]
            for j in range(k):
                sel = (lost == j).repeat_interleave(n).cuda()
                assert torch.equal(out[j][sel], data[j][sel]), (name, j)
        a.record(s)
        for _ in range(10):
            ec.decode(k, m, mat, masks, data + par, out, plan, s)
        b.record(s)
        res[name].append(a.elapsed_ms(b) / 10)
for name, v in res.items():
    v.sort()
    med = v[len(v) // 2]
    print(f"{W_} {name:9s} median {med * 1e3:7.1f} us  {(k + 1) * L / (med * 1e-3) / 1e9:6.0f} GB/s  "
          f"best {(k + 1) * L / (v[0] * 1e-3) / 1e9:6.0f}", flush=True)
