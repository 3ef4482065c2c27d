#!/usr/bin/env python3
"""tools/dispatch_cap_probe.py -- what a region multiply of one stream above 64 GiB does
with a given library build (tools probe, not product).  Above 2^24 tiles a launch with
one workgroup per (quarter) tile exceeds one dispatch's 2^32 - 1 work items; the
round-2 library caps its grid there and walks the rest grid-stride.  Run with
CEC_LIB_PATH=<build> to compare builds; prints one JSON line (error text, or whether
the head / tail / tile-2^24 windows equal the expected bytes)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    torch.cuda.set_device(0)
    torch.empty(1, device="cuda")
    from cocytus_amd import ec

    n = (1 << 36) + 3 * 4096 + 77
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    src.random_(0, 256, generator=torch.Generator(device="cuda").manual_seed(7))
    dst = torch.full((n,), 0xFF, dtype=torch.uint8, device="cuda")
    out = {"lib": os.environ.get("CEC_LIB_PATH", "in-tree"), "bytes": n}
    try:
        ec.region_multiply(src, 1, n, dst, 0)  # c = 1: dst must equal src
        torch.cuda.synchronize()
        W = 1 << 20
        out["windows_equal"] = {str(o): bool(torch.equal(dst[o:o + W], src[o:o + W]))
                                for o in (0, (1 << 36) - W + 8192, n - W)}
        out["all_equal"] = bool(torch.equal(dst, src))
    except Exception as e:  # noqa: BLE001 -- report what the build does
        out["error"] = str(e)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
