#!/bin/bash
# tools/galois_tp_compare.sh -- the reference's own micro-benchmark (microbenchmarks/galois_tp.c,
# built unmodified on the shim by `make -C oracle ref`) vs the restated GF-Complete kernel
# (oracle, AVX2, 1 thread) on the same call: one 512 MiB region multiply-XOR by 2 from
# malloc'd memory.  Run ON the GPU box.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for i in 1 2 3; do
  echo "galois_tp on the shim (GPU, pageable 512 MiB, staged): $(timeout -k 10 120 "$R/oracle/_ref/galois_tp")"
done
timeout -k 10 120 python3 - <<'PY'
import os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from oracle import pyoracle
n = 512 << 20
i = np.arange(n, dtype=np.int64) % 20
src = i.astype(np.uint8)
r2 = src.copy()
for _ in range(3):
    t = time.perf_counter()
    pyoracle.region_multiply_simd(src, 2, r2)
    dt = time.perf_counter() - t
    print(f"restated GF-Complete SPLIT(8,4) AVX2, 1 thread, same call: {dt * 1e3:.1f} ms ({n / dt / 1e9:.2f} GB/s of region)")
PY
