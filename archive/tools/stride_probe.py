"""tools/stride_probe.py -- does the distance between arena bases set the rate of the
rotating RS(4,2) 64 KiB decode (BASELINE configs[3], 1 GiB per shard)?

DESIGN.md §4: the same rotating shape ran 4 % faster with 256 MiB arenas than with the
bench's 1 GiB ones, in the XOR stream as in the library.  The arenas come from one slab
at cec_arena_stride (an odd number of 4 KiB pages).  Here the library's encode and
decode run on slabs laid out with other strides, in one process, interleaved over
rounds, with the bench's stripes, masks and plans; bytes of every rebuilt shard are
checked once per layout.  Prints one JSON line per layout and round.

usage: python tools/stride_probe.py [rounds] [steps]
"""
from __future__ import annotations

import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402

K, M, N, B = 4, 2, 65536, 16384
ARENA = N * B
PAGE = 4096


def layouts():
    """name -> list of the 10 arena offsets inside one slab."""
    base = ec.arena_stride(ARENA)  # 1 GiB + 4 KiB
    out = {"lib (1 GiB + 4 KiB)": [i * base for i in range(K + M + K)]}
    for extra in (3, 5, 9, 17, 33, 513):  # odd page counts past the arena
        s = ARENA + extra * PAGE
        out[f"1 GiB + {extra} x 4 KiB"] = [i * s for i in range(K + M + K)]
    s = ARENA + (2 << 20) + PAGE
    out["1 GiB + 2 MiB + 4 KiB"] = [i * s for i in range(K + M + K)]
    # skew growing with the index: arena i starts i*(1 GiB) + i*i*4 KiB
    out["quadratic skew"] = [i * ARENA + i * i * PAGE for i in range(K + M + K)]
    # data / parity / out groups each in their own 1 GiB-aligned region, skewed within
    out["group skew 64 KiB"] = [i * (ARENA + 16 * PAGE) for i in range(K + M + K)]
    return out


def run(name, offs, steps, check):
    need = max(offs) + ARENA
    slab = torch.empty(need, dtype=torch.uint8, device="cuda")
    ar = [slab[o:o + ARENA] for o in offs]
    data, parity, out = ar[:K], ar[K:K + M], ar[K + M:]
    g = torch.Generator(device="cuda").manual_seed(7)
    for t in data:
        t.random_(0, 256, generator=g)
    mat = ec.coding_matrix(K, M)
    masks = [ec.recovery_mask(K, M, K + p, [int(i != j) for i in range(K + M)]) for p in range(M) for j in range(K)]
    stripes = [(s * N, N) for s in range(B)]
    enc = ec.Plan([(o, 0, ln, 0) for o, ln in stripes])
    dec = ec.Plan([(o, 0, ln, s % len(masks)) for s, (o, ln) in enumerate(stripes)])
    st = torch.cuda.current_stream()
    for _ in range(2):
        ec.encode(K, M, mat, data, parity, enc, st)
        ec.decode(K, M, mat, masks, data + parity, out, dec, st)
    torch.cuda.synchronize()
    evs = [ec.Event() for _ in range(2 * steps + 1)]
    evs[0].record(st)
    for s in range(steps):
        ec.encode(K, M, mat, data, parity, enc, st)
        evs[2 * s + 1].record(st)
        ec.decode(K, M, mat, masks, data + parity, out, dec, st)
        evs[2 * s + 2].record(st)
    torch.cuda.synchronize()
    e = statistics.median(evs[2 * s].elapsed_ms(evs[2 * s + 1]) for s in range(steps))
    d = statistics.median(evs[2 * s + 1].elapsed_ms(evs[2 * s + 2]) for s in range(steps))
    ok = None
    if check:
        ok = True
        lost = [[x for x in range(K) if not (mk >> x) & 1][0] for mk in masks]
        for s in range(0, B, 97):  # a sample of stripes, every mask
            j = lost[s % len(masks)]
            ok &= bool(torch.equal(out[j][s * N:(s + 1) * N], data[j][s * N:(s + 1) * N]))
    enc.destroy()
    dec.destroy()
    del ar, data, parity, out, slab
    torch.cuda.empty_cache()
    return {"layout": name, "encode_ms": round(e, 4), "decode_ms": round(d, 4),
            "encode_TBps": round((K + M) * ARENA / e / 1e9, 3), "decode_TBps": round((K + 1) * ARENA / d / 1e9, 3),
            "verified": ok}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    lays = layouts()
    # optional: only these layouts, in this order (comma-separated name prefixes), and a
    # throwaway allocation of PREALLOC GiB made and freed before the first one
    if os.environ.get("ORDER"):
        lays = {n: lays[n] for p in os.environ["ORDER"].split(",") for n in lays if n.startswith(p)}
    pre = float(os.environ.get("PREALLOC", "0"))
    if pre:
        x = torch.empty(int(pre * 2**30), dtype=torch.uint8, device="cuda")
        x.fill_(1)
        torch.cuda.synchronize()
        del x
        torch.cuda.empty_cache()
    for r in range(rounds):
        for name, offs in lays.items():
            row = run(name, offs, steps, check=(r == 0))
            row["round"] = r
            row["prealloc_GiB"] = pre
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
