#!/usr/bin/env python3
"""tools/decode_probe.py -- decode under rotating erasures: what the 6 % below the 3:1
stream is (not product).  One process, bench arenas, interleaved rounds:
  rotate      masks rotate per stripe over all 6 (lost, leader) pairs, out[lost] (bench)
  rotate_one  the same, every lost shard's bytes into ONE out arena at the stripe offset
  lost_only   the lost shard rotates, leader fixed P0
  leader_only the leader rotates, lost shard fixed D0
  single      one mask (D0 lost, leader P0)"""
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
ar = ec.arena_tensors(k + m + k, L)
for t in ar[:k]:
    t.random_(0, 256)
data, par, out = ar[:k], ar[k:k + m], ar[k + m:]
ec.encode_region(k, m, mat, data, par, L, s)


def mask(lost, leader):
    return ec.recovery_mask(k, m, k + leader, [int(i != lost) for i in range(k + m)])


all6 = [mask(j, p) for p in range(m) for j in range(k)]
plans = {
    "rotate": (all6, ec.Plan([(i * n, 0, n, i % 6) for i in range(B)]), out),
    "rotate_one": (all6, ec.Plan([(i * n, 0, n, i % 6) for i in range(B)]), [out[0]] * k),
    "lost_only": ([mask(j, 0) for j in range(k)], ec.Plan([(i * n, 0, n, i % 3) for i in range(B)]), out),
    "leader_only": ([mask(0, p) for p in range(m)], ec.Plan([(i * n, 0, n, i % 2) for i in range(B)]), out),
    "single": ([mask(0, 0)], ec.Plan([(i * n, 0, n, 0) for i in range(B)]), out),
}
res = {x: [] for x in plans}
a, b = ec.Event(), ec.Event()
for rnd in range(8):
    for name, (masks, plan, o) in plans.items():
        fn = lambda: ec.decode(k, m, mat, masks, data + par, o, plan, s)  # noqa: E731
        fn()
        torch.cuda.synchronize()
        a.record(s)
        for _ in range(10):
            fn()
        b.record(s)
        res[name].append(a.elapsed_ms(b) / 10)
for name, v in res.items():
    v.sort()
    print(f"{name:12s} median {v[len(v) // 2] * 1e3:7.1f} us  {4 * L / (v[len(v) // 2] * 1e-3) / 1e9:6.0f} GB/s  "
          f"best {4 * L / (v[0] * 1e-3) / 1e9:6.0f}")
