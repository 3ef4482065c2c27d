"""Launch gaps of the bench step: direct launches vs HIP-graph replay (tools probe, not
product).  One process, the metric's RS(3,2) 4 KiB arenas; per variant the median over
rounds of the wall time of 50 steps (synchronised), and rocprof-free gap estimate =
step - (encode + decode kernel time from events around a single-step graph)."""
from __future__ import annotations

import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

k, m, n, B = 3, 2, 4096, 65536
mat = ec.coding_matrix(k, m)
ar = ec.arena_tensors(k + m + k, n * B)
data, parity, out = ar[:k], ar[k:k + m], ar[k + m:]
for t in data:
    t.random_(0, 256)
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
ep = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
dp = ec.Plan([(s * n, 0, n, s % 6) for s in range(B)])
side = torch.cuda.Stream()


def step(s):
    ec.encode(k, m, mat, data, parity, ep, s)
    ec.decode(k, m, mat, masks, data + parity, out, dp, s)


with torch.cuda.stream(side):
    step(side)
torch.cuda.synchronize()
g1 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g1, stream=side):
    step(side)
g10 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g10, stream=side):
    for _ in range(10):
        step(side)
torch.cuda.synchronize()
S = 50
res = {"direct": [], "graph_1step": [], "graph_10steps": []}
for rnd in range(7):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        for _ in range(S):
            step(side)
    torch.cuda.synchronize()
    res["direct"].append((time.perf_counter() - t0) / S)
    t0 = time.perf_counter()
    for _ in range(S):
        g1.replay()
    torch.cuda.synchronize()
    res["graph_1step"].append((time.perf_counter() - t0) / S)
    t0 = time.perf_counter()
    for _ in range(S // 10):
        g10.replay()
    torch.cuda.synchronize()
    res["graph_10steps"].append((time.perf_counter() - t0) / S)
payload = (k + 1) * n * B
print(json.dumps({v: {"ms_per_step": round(statistics.median(x) * 1e3, 4),
                      "GiBps": round(payload / statistics.median(x) / 2**30, 1)} for v, x in res.items()}, indent=1))
