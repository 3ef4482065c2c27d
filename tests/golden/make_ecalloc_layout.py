#!/usr/bin/env python3
"""Freeze a SET batch laid out by the reference's own allocator (oracle/ecalloc_ref.py,
/root/reference/ecalloc.c run here) into tests/golden/ecalloc_layout.npz.

Data only: per SET its source shard j, arena address and nbytes (vlen + 2).  Run here
(needs /root/reference and `make -C oracle ref`); the GPU tests read the npz."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import ecalloc_ref  # noqa: E402

SEED, K = 0xC0C7_0A10, 3


def main():
    t = ecalloc_ref.set_trace(SEED, K)
    arr = np.array(t, dtype=np.uint64)
    np.savez_compressed(os.path.join(HERE, "ecalloc_layout.npz"), sets=arr,
                        seed=np.uint64(SEED), k=np.uint64(K))
    print(f"{len(t)} SETs, max end {int((arr[:, 1] + arr[:, 2]).max())}")


if __name__ == "__main__":
    main()
