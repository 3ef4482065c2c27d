"""tools/mapped_probe.py -- what the host reads back from the drop-in's zero-copy path
when a call spans more than one 4 KiB page of its mapped staging.

Prints, for a few sizes, the positions that differ from the oracle and, at those
positions, the bytes the call returned, the destination's original bytes, the source
bytes and the expected bytes.  `--torch` imports torch first, so that the library runs
on torch's HIP runtime, as under pytest.  (Round 2: without a system-scope release
before the completion signal, the second tile of a 4098-byte call came back stale on
some boxes)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if "--torch" in sys.argv:  # torch first: the library then runs on torch's HIP runtime
    import torch  # noqa: E402

    torch.empty(1, device="cuda")
from cocytus_amd import ec  # noqa: E402
from oracle import pyoracle as oracle  # noqa: E402


def case(tag, n, c, add):
    rng = np.random.default_rng(n * 7 + c)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    b0 = b.copy()
    exp = b.copy() if add else np.zeros(n, np.uint8)
    oracle.region_multiply(a, c, exp, 1)
    ec.galois_w08_region_multiply(a, c, n, b, add)
    bad = np.flatnonzero(b != exp)
    row = {"tag": tag, "n": n, "c": c, "add": add, "bad": int(bad.size)}
    if bad.size:
        i = bad[:6]
        row.update(first=bad[:6].tolist(), last=bad[-4:].tolist(), got=b[i].tolist(), dst0=b0[i].tolist(),
                   src=a[i].tolist(), exp=exp[i].tolist())
    print(json.dumps(row), flush=True)


def main():
    for n in (1, 2, 4095):  # (the parity test's first calls)
        case("pageable", n, 245, 1)
    for n in (4096, 4097, 4098, 4112, 8192, 8194, 12000, 40000):
        for c, add in ((1, 1), (2, 1), (245, 0)):
            case("pageable", n, c, add)


if __name__ == "__main__":
    main()
