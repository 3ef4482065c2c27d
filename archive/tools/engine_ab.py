#!/usr/bin/env python3
"""tools/engine_ab.py -- PERM vs LDS engine in one process, interleaved rounds, on the
bench's RS(3,2) 4 KiB arenas (encode, rotating-mask decode, diff-update) (not product)."""
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
ar = ec.arena_tensors(k + m + k + 1, L)
for t in ar:
    t.random_(0, 256)
data, par, out, stage = ar[:k], ar[k:k + m], ar[k + m:k + m + k], ar[-1]
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
ep = ec.Plan([(i * n, 0, n, 0) for i in range(B)])
dp = ec.Plan([(i * n, 0, n, i % 6) for i in range(B)])
up = ec.Plan([(i * n, i * n, n, i % 3) for i in range(B)])
ops = {
    "encode": (5 * L, lambda: ec.encode(k, m, mat, data, par, ep, s)),
    "decode": (4 * L, lambda: ec.decode(k, m, mat, masks, data + par, out, dp, s)),
    "diff_update": (7 * L, lambda: ec.diff_update(k, m, mat, data, stage, par, True, up, s)),
}
engines = {"perm": ec.CEC_ENGINE_PERM, "lds": ec.CEC_ENGINE_LDS}
res = {(e, o): [] for e in engines for o in ops}
a, b = ec.Event(), ec.Event()
for rnd in range(8):
    for e, code in engines.items():
        ec.set_engine(code)
        for o, (nb, fn) in ops.items():
            fn()
            torch.cuda.synchronize()
            a.record(s)
            for _ in range(10):
                fn()
            b.record(s)
            res[(e, o)].append(a.elapsed_ms(b) / 10)
for o, (nb, _) in ops.items():
    line = []
    for e in engines:
        v = sorted(res[(e, o)])
        line.append(f"{e} {v[4] * 1e3:7.1f} us ({nb / (v[4] * 1e-3) / 1e9:5.0f} GB/s)")
    print(f"{o:12s} " + "   ".join(line))
