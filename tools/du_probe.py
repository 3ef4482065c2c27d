"""Where the fused diff-update's time goes (tools probe, not product).

One process, one MI355X: cec_diff_update over 65,536 x 4 KiB SETs (256 MiB per arena)
with different source-shard patterns and options, median of HIP-event launch times:
  random j (the bench), j fixed, j rotating per SET, install on / off, XOR-only matrix.
The algorithmic bytes are (2 + 2M) n per SET, + n with install.
"""
from __future__ import annotations

import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
torch.cuda.set_device(0)
torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

k, m, n, B = 3, 2, 4096, 65536
T = n * B
ar = ec.arena_tensors(k + m + 2, T)
data, parity, stage = ar[:k], ar[k:k + m], ar[k + m:]
g = torch.Generator(device="cuda").manual_seed(1)
for t in ar:
    t.random_(0, 256, generator=g)
s = torch.cuda.current_stream()
rnd = torch.randint(0, k, (B,), generator=torch.Generator().manual_seed(2)).tolist()
mat = ec.coding_matrix(k, m)
ones = [1] * ((k + m) * k)
for i in range(k):
    for j in range(k):
        ones[i * k + j] = int(i == j)
variants = {
    "random_j": ([(i * n, i * n, n, rnd[i]) for i in range(B)], mat, True),
    "fixed_j0": ([(i * n, i * n, n, 0) for i in range(B)], mat, True),
    "rotating_j": ([(i * n, i * n, n, i % k) for i in range(B)], mat, True),
    "random_j_no_install": ([(i * n, i * n, n, rnd[i]) for i in range(B)], mat, False),
    "fixed_j0_no_install": ([(i * n, i * n, n, 0) for i in range(B)], mat, False),
    "random_j_xor_only": ([(i * n, i * n, n, rnd[i]) for i in range(B)], ones, True),
}
plans = {name: ec.Plan(v[0]) for name, v in variants.items()}
res = {name: [] for name in variants}
for rnd_i in range(5):
    for name, (ext, mt, inst) in variants.items():
        pl = plans[name]
        for w in range(2):
            ec.diff_update(k, m, mt, data, stage[w % 2], parity, inst, pl, s)
        evs = [ec.Event() for _ in range(21)]
        evs[0].record(s)
        for i in range(20):
            ec.diff_update(k, m, mt, data, stage[i % 2], parity, inst, pl, s)
            evs[i + 1].record(s)
        torch.cuda.synchronize()
        res[name] += [evs[i].elapsed_ms(evs[i + 1]) for i in range(20)]
out = {}
for name, (ext, mt, inst) in variants.items():
    ms = statistics.median(res[name])
    nbytes = (2 + 2 * m + (1 if inst else 0)) * T
    out[name] = {"us": round(ms * 1e3, 1), "TBps": round(nbytes / ms / 1e9, 3), "frac": round(nbytes / ms / 1e9 / 8.0, 4)}
print(json.dumps(out, indent=1))
