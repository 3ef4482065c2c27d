#!/usr/bin/env python3
"""tools/event_cost.py -- what bench.py's per-launch HIP events cost its step (not
product).  One process, the metric's workload, interleaved rounds of 20 steps:
  none   encode, decode; wall clock only
  three  an event before encode, between, after decode (bench.py before this probe)
  two    one event between consecutive launches (each event ends one and starts the next)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
import bench  # noqa: E402
from cocytus_amd import ec  # noqa: E402

k, m, n, _, _ = bench.WORKLOADS["rs32_4k"]
stripes, arena = bench.layout("rs32_4k")
mat = ec.coding_matrix(k, m)
ar = ec.arena_tensors(2 * k + m, arena)
for t in ar[:k]:
    t.random_(0, 256)
data, par, out = ar[:k], ar[k:k + m], ar[k + m:]
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
ep = ec.Plan([(o, 0, ln, 0) for o, ln in stripes])
dp = ec.Plan([(o, 0, ln, s % len(masks)) for s, (o, ln) in enumerate(stripes)])
s = torch.cuda.current_stream()
S = 20
evs = [ec.Event() for _ in range(3 * S + 1)]


def run(mode):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e = 0
    for _ in range(S):
        if mode == "three":
            evs[e].record(s); e += 1
        elif mode == "two" and e == 0:
            evs[e].record(s); e += 1
        ec.encode(k, m, mat, data, par, ep, s)
        if mode != "none":
            evs[e].record(s); e += 1
        ec.decode(k, m, mat, masks, data + par, out, dp, s)
        if mode != "none":
            evs[e].record(s); e += 1
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / S


for mode in ("none", "three", "two"):
    run(mode)
res = {x: [] for x in ("none", "three", "two")}
for _ in range(int(os.environ.get("ROUNDS", "15"))):
    for mode in res:
        res[mode].append(run(mode))
for mode, v in res.items():
    v.sort()
    print(f"{mode:6s} median step {v[len(v) // 2] * 1e6:7.1f} us  best {v[0] * 1e6:7.1f} us")
