#!/usr/bin/env python3
"""cec_region_multiply_batch against the per-call drop-in and the restated CPU path, on the
recovery shapes the server glue runs (integration/cocytus_recovery.c):

  range   recovery_recover_units over one 1 MiB range (256 units, recovery.c:61-96): each
          unit its own malloc'd-style 4 KiB host buffer, scattered; first peer = first
          touch (unit = parity unit ^ c * peer), second peer folded in place;
  idle    the idle recoverer's 85 single-unit requests in flight (memcached.c:5712-5734,
          const.h:27), two data peers' replies each: 170 unit folds per flush.

One JSON line per shape: the batch (one call), the drop-in loop (one synchronous
galois_w08_region_multiply per unit, as the unchanged server), and the restated CPU
region multiply (oracle, SIMD, one thread) -- bytes checked equal.

    python tools/hostbatch_bench.py [reps]
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

U = 4096


def main(reps=20):
    import torch

    torch.cuda.set_device(0)
    torch.empty(1, device="cuda")
    from cocytus_amd import ec
    from oracle import pyoracle as orc

    L = ec.lib()
    rng = np.random.default_rng(1)
    out = []
    for shape, nunits, peers in (("range_1MiB", 256, 2), ("idle_85", 85, 2)):
        heap = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
        base = heap.ctypes.data
        arena = 0
        peer_off = [(8 << 20) + p * (nunits * U) for p in range(peers)]
        unit_off = [(32 << 20) + int(i) * (U + 64) for i in rng.permutation(nunits)]
        arena_off = [arena + int(x) * U for x in rng.permutation(4096)[:nunits]] if shape == "idle_85" else \
            [arena + i * U for i in range(nunits)]
        coefs = [245, 244]

        def jobs_for(p):
            arr = (ec.RegionJob * nunits)()
            for i in range(nunits):
                arr[i] = ec.RegionJob(base + peer_off[p] + i * U, base + unit_off[i],
                                      base + arena_off[i] if p == 0 else None, U, coefs[p], 1)
            return arr

        batches = [jobs_for(p) for p in range(peers)]
        snap = heap.copy()

        def run_batch():
            for arr in batches:
                assert L.cec_region_multiply_batch(arr, nunits, None) == 0, L.cec_last_error()

        def run_dropin():
            for p in range(peers):
                for i in range(nunits):
                    if p == 0:  # recovery.c:79-82: malloc + memcpy of the parity unit
                        ctypes.memmove(base + unit_off[i], base + arena_off[i], U)
                    L.galois_w08_region_multiply(base + peer_off[p] + i * U, coefs[p], U, base + unit_off[i], 1)

        def run_cpu():
            for p in range(peers):
                for i in range(nunits):
                    if p == 0:
                        ctypes.memmove(base + unit_off[i], base + arena_off[i], U)
                    orc.lib().ref_region_multiply_simd(base + peer_off[p] + i * U, coefs[p], U, base + unit_off[i])

        res = {"shape": shape, "units": nunits, "peers": peers, "payload_bytes": nunits * U * peers}
        results = {}
        for name, fn in (("batch", run_batch), ("dropin_loop", run_dropin), ("cpu_simd_1thread", run_cpu)):
            heap[:] = snap
            fn()  # warm-up (and the result to compare)
            results[name] = heap[32 << 20:(32 << 20) + nunits * (U + 64)].copy()
            ts = []
            for _ in range(reps if name != "dropin_loop" else max(3, reps // 4)):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            med = ts[len(ts) // 2]
            res[name + "_us"] = round(1e6 * med, 1)
            res[name + "_GiBps"] = round(res["payload_bytes"] / med / 2**30, 3)
        heap[:] = snap
        run_batch()
        res["batch_last_call"] = {k: round(v, 1) for k, v in ec.batch_stats().items()}
        res["same_bytes"] = bool(all(np.array_equal(results["batch"], v) for v in results.values()))
        res["batch_vs_dropin"] = round(res["dropin_loop_us"] / res["batch_us"], 1)
        res["batch_vs_cpu"] = round(res["cpu_simd_1thread_us"] / res["batch_us"], 2)
        print(json.dumps(res), flush=True)
        out.append(res)
    return out


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
