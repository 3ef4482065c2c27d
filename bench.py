#!/usr/bin/env python3
"""bench.py -- device-resident RS(K,M) encode + decode throughput of libcocytus_ec.so.

Metric (BASELINE.json): GiB/s device-resident RS(3,2) encode+decode, 4 KiB values.
One step = one batch of the workload on each GPU, inputs already resident in HBM:
  1. cec_encode  over B stripes  (parity[p] = sum_j MATRIX(K+p, j) * D_j, per 4 KiB value)
  2. cec_decode  over the same B stripes, one lost data shard per stripe, the lost shard
     and the recovery leader rotating over all K x M (lost shard, leader parity) pairs
     (masks as start_recovery builds them, memcached.c:8136-8151).
value = payload GiB/s over all ranks = (K*n encoded + n rebuilt) * B * N * steps / max-rank
time / 2^30.  roofline = the encode kernel's algorithmic HBM bytes ((K+M)*n per stripe)
per launch / its HIP-event launch time, against 8 TB/s.  cpu_baseline = the oracle's
restated Jerasure/GF-Complete path (AVX2 split-nibble) on the host, same chaining.

Multi-GPU: `torch.distributed.run --nproc-per-node N bench.py --gpus N`; each rank
encodes/decodes its own batch (independent stripes, no collective on the data path);
barrier + synchronize around the timed steps, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak, MI355X_MICROARCH.md

WORKLOADS = {
    # name: (k, m, value bytes, stripes per GPU)
    "rs32_4k": (3, 2, 4096, 65536),        # BASELINE configs[1] (+ decode: the metric)
    "rs32_1m": (3, 2, 1 << 20, 1024),      # configs[4] sizes
    "rs42_64k": (4, 2, 65536, 16384),      # configs[3] per GPU
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="rs32_4k", choices=sorted(WORKLOADS))
    ap.add_argument("--engine", default="perm", choices=["perm", "lds"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU work budget (thread-seconds)")
    ap.add_argument("--quiet", action="store_true")
    return ap.parse_args()


def cpu_baseline(k, m, n, budget_s):
    """Oracle (restated Jerasure/GF-Complete, AVX2) on the host cores, bounded sample."""
    from oracle import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    stripes = 16384  # 64 MiB per shard at 4 KiB: larger than the host LLC
    if n * stripes > (256 << 20):
        stripes = max(threads, (256 << 20) // n)
    t1 = pyoracle.bench_encode_decode(k, m, n, stripes, threads, 1, True)
    reps = max(1, int(budget_s / max(t1 * threads, 1e-6)))
    reps = min(reps, 50)
    t = pyoracle.bench_encode_decode(k, m, n, stripes, threads, reps, True)
    payload = (k + 1) * n * stripes * reps
    return {
        "value": round(payload / t / 2**30, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"RS({k},{m}) encode+decode of {stripes} x {n} B stripes x {reps} passes, "
                  f"{threads} threads, {t:.2f} s wall; restated GF-Complete SPLIT(8,4) "
                  f"split-nibble ({'AVX2' if pyoracle.simd_available() else 'scalar'}), "
                  "chained like memcached.c/recovery.c (Jerasure not available)",
    }


def load_traffic(workload):
    """HBM bytes per encode launch from the committed rocprofv3 --pmc summary."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        e = d.get(workload, {})
        return e.get("encode_hbm_bytes_per_launch"), e.get("decode_hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None, None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.empty(1, device="cuda")

    from cocytus_amd import ec

    ec.lib()
    if ec.device_check() != ec.CEC_OK:
        raise SystemExit("libcocytus_ec: " + ec.lib().cec_last_error().decode())
    ec.set_engine(ec.CEC_ENGINE_LDS if args.engine == "lds" else ec.CEC_ENGINE_PERM)

    k, m, n, B = WORKLOADS[args.workload]
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70002 + rank)
    data = [torch.randint(0, 256, (B * n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    enc_plan = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
    dec_plan = ec.Plan([(s * n, 0, n, s % len(masks)) for s in range(B)])
    stream = torch.cuda.current_stream()

    def step():
        ec.encode(k, m, mat, data, parity, enc_plan, stream)
        ec.decode(k, m, mat, masks, data + parity, out, dec_plan, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # verify once (device-side): every rebuilt shard equals the original
    ok = True
    for q, mk in enumerate(masks):
        j = [x for x in range(k) if not (mk >> x) & 1][0]
        sel = torch.arange(q, B, len(masks), device="cuda")
        ok &= bool(torch.equal(out[j].view(B, n)[sel], data[j].view(B, n)[sel]))

    evs = [[ec.Event() for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        evs[s][0].record(stream)
        ec.encode(k, m, mat, data, parity, enc_plan, stream)
        evs[s][1].record(stream)
        ec.decode(k, m, mat, masks, data + parity, out, dec_plan, stream)
        evs[s][2].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    enc_ms = sum(e[0].elapsed_ms(e[1]) for e in evs) / args.steps
    dec_ms = sum(e[1].elapsed_ms(e[2]) for e in evs) / args.steps

    t = torch.tensor([elapsed, enc_ms, dec_ms, 0.0 if ok else 1.0], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, enc_ms_max, dec_ms_max, bad = [float(x) for x in t.tolist()]

    payload = (k * n + n) * B * world * args.steps
    value = payload / elapsed / 2**30
    enc_bytes = (k + m) * n * B          # algorithmic HBM bytes per encode launch
    dec_bytes = (k + 1) * n * B          # per decode launch (read K survivors, write 1)
    enc_gbps = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbps = dec_bytes / (dec_ms * 1e-3) / 1e9
    enc_traffic, dec_traffic = load_traffic(args.workload)

    if rank == 0:
        res = {
            "metric": "GiB/s device-resident RS(3,2) encode+decode, 4 KiB values",
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes, torch.Generator seeded per rank)",
            "config": {
                "workload": f"RS({k},{m}) encode + single-shard decode, {n} B values, "
                            f"{B} stripes per GPU (BASELINE configs[1] + decode)",
                "k": k, "m": m, "value_bytes": n, "stripes_per_gpu": B,
                "parallelism": f"{world} independent shards of stripes, no collective",
                "engine": args.engine,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(enc_gbps, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(enc_gbps / HBM_PEAK_GBPS, 4),
                "traffic": enc_traffic,
                "kernel": "combine_kernel<3,2,PermEngine,kAccNone,exact> (cec_encode)",
                "algorithmic_bytes_per_launch": enc_bytes,
                "launch_ms": round(enc_ms, 4),
            },
            "decode_roofline": {
                "achieved": round(dec_gbps, 1), "frac": round(dec_gbps / HBM_PEAK_GBPS, 4),
                "algorithmic_bytes_per_launch": dec_bytes, "launch_ms": round(dec_ms, 4),
                "traffic": dec_traffic,
            },
            "verified": ok and bad == 0.0,
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(k, m, n, args.cpu_seconds)
        print(json.dumps(res), flush=True)
    enc_plan.destroy()
    dec_plan.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
