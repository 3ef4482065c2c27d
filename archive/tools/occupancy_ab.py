#!/usr/bin/env python3
"""tools/occupancy_ab.py WORKLOAD CAP... -- encode / rotating-mask decode of a bench.py
workload under cec_set_waves_per_cu caps, interleaved in one process (not product).
Prints one line per cap: median launch us and algorithmic TB/s of encode and decode.
ALT=1: bench.py's step instead (encode, decode alternating, an event around each)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

torch.cuda.set_device(0)
torch.empty(1, device="cuda")
import bench  # noqa: E402
from cocytus_amd import ec  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "rs32_4k"
caps = [int(x) for x in sys.argv[2:]] or [0, 8, 12, 16, 24]
k, m, n, _, _ = bench.WORKLOADS[w]
stripes, arena = bench.layout(w)
mat = ec.coding_matrix(k, m)
ar = ec.arena_tensors(2 * k + m, arena)
for t in ar[:k]:
    t.random_(0, 256)
data, par, out = ar[:k], ar[k:k + m], ar[k + m:]
masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)]) for p in range(m) for j in range(k)]
ep = ec.Plan([(o, 0, ln, 0) for o, ln in stripes])
dp = ec.Plan([(o, 0, ln, s % len(masks)) for s, (o, ln) in enumerate(stripes)])
s = torch.cuda.current_stream()
total = sum(ln for _, ln in stripes)
ops = {
    "encode": (lambda: ec.encode(k, m, mat, data, par, ep, s), (k + m) * total),
    "decode": (lambda: ec.decode(k, m, mat, masks, data + par, out, dp, s), (k + 1) * total),
}
res = {(c, o): [] for c in caps for o in ops}
if os.environ.get("ALT"):  # bench.py's step: encode, decode alternating, an event around each
    ev = [ec.Event() for _ in range(3 * 10)]
    for rnd in range(int(os.environ.get("ROUNDS", "7"))):
        for c in caps:
            ec.set_waves_per_cu(c)
            for i in range(10):
                ev[3 * i].record(s)
                ops["encode"][0]()
                ev[3 * i + 1].record(s)
                ops["decode"][0]()
                ev[3 * i + 2].record(s)
            torch.cuda.synchronize()
            res[(c, "encode")].append(sum(ev[3 * i].elapsed_ms(ev[3 * i + 1]) for i in range(10)) / 10)
            res[(c, "decode")].append(sum(ev[3 * i + 1].elapsed_ms(ev[3 * i + 2]) for i in range(10)) / 10)
    ops_loop = 0
else:
    ops_loop = 1
a, b = ec.Event(), ec.Event()
for rnd in range(int(os.environ.get("ROUNDS", "7")) * ops_loop):
    for c in caps:
        ec.set_waves_per_cu(c)
        for o, (fn, _) in ops.items():
            fn()
            a.record(s)
            for _ in range(10):
                fn()
            b.record(s)
            res[(c, o)].append(a.elapsed_ms(b) / 10)
ec.set_waves_per_cu(0)
print(f"{w}: {len(stripes)} values, {total} B per shard")
for c in caps:
    line = [f"waves/CU {c:3d}"]
    for o, (_, nb) in ops.items():
        v = sorted(res[(c, o)])
        med = v[len(v) // 2]
        line.append(f"{o} {med * 1e3:7.1f} us {nb / (med * 1e-3) / 1e12:5.2f} TB/s (best {nb / (v[0] * 1e-3) / 1e12:5.2f})")
    print("  ".join(line), flush=True)
