#!/usr/bin/env python3
"""bench.py -- device-resident RS(K,M) encode + decode throughput of libcocytus_ec.so.

Metric (BASELINE.json): GiB/s device-resident RS(3,2) encode+decode, 4 KiB values.
One step = one batch of the workload on each GPU, inputs already resident in HBM:
  1. cec_encode  over B stripes  (parity[p] = sum_j MATRIX(K+p, j) * D_j, per value)
  2. cec_decode  over the same B stripes, one lost data shard per stripe; the lost shard
     and the recovery leader rotate over all K x M (lost shard, leader parity) pairs
     (masks as start_recovery builds them, /root/reference/memcached.c:8136-8151).
value = payload GiB/s over all ranks = (K*n encoded + n rebuilt) per stripe * stripes *
ranks * steps / max-over-ranks wall time / 2^30.  roofline = the encode kernel's
algorithmic HBM bytes ((K+M)*n per stripe) per launch / its HIP-event launch time vs
8 TB/s; traffic = HBM bytes per launch from the committed rocprofv3 --pmc summary.
cpu_baseline = the oracle's restated Jerasure/GF-Complete path (AVX2 split-nibble), on
the host cores, same chaining as the reference's call sites.

Multi-GPU: `bench.py --gpus N` starts N rank processes itself (torch.distributed.run as
a child, before anything touches the GPU), or runs as one rank of an outer
`torch.distributed.run --nproc-per-node N bench.py --gpus N`: every rank
encodes/decodes its own batch (independent stripes, no collective on the data path);
barrier + synchronize around the timed steps, max over ranks (weak scaling: `value`).
`strong`: the metric's one batch split contiguously over the ranks, whole
payload / max over ranks; at N = 1 it times the shares a fixed batch gives at N = 2, 4,
8 on the one GPU instead and reports the implied factor.
other_workloads also carries the fused per-SET diff-update (the north star's first op)
and the pinned-host end-to-end path, each with its own roofline / PCIe fraction.

--e2e: values start and end in pinned host memory (client sockets / recovery peers):
H2D -> kernel -> D2H pipelined over --e2e-streams HIP streams; printed as its own JSON
line.  --e2e-zero-copy: the kernels read and write the pinned host buffers directly.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
METRIC = "GiB/s device-resident RS(3,2) encode+decode, 4 KiB values"

WORKLOADS = {
    # name: (k, m, value bytes (0 = mixed), stripes per GPU, what)
    "rs32_4k": (3, 2, 4096, 65536, "BASELINE configs[1] (+ decode): the metric"),
    "rs32_mixed": (3, 2, 0, 0, "BASELINE configs[2]: log-uniform 256 B - 1 MiB values, ~1 GiB"),
    "rs42_64k": (4, 2, 65536, 16384, "BASELINE configs[3], per GPU"),
    "rs32_1m": (3, 2, 1 << 20, 1024, "BASELINE configs[4] sizes"),
}
# Other north-star paths measured beside the encode + decode workloads (--also).
EXTRA_WORKLOADS = {
    "rs32_diff_update": "per-SET diff-update fused with install (SURVEY §8a a4: memcached.c:2664-2710 "
                        "data side + 7739-7798 parity side), 65,536 x 4 KiB SETs, device-resident",
    "rs32_e2e": "RS(3,2) 4 KiB encode + decode, values from and back to pinned host memory "
                "(H2D -> kernels -> D2H pipelined over HIP streams)",
    "rs32_4k_lds": "the metric's workload with the LDS engine: GF(2^8) products from 256-entry "
                   "log/antilog product rows staged in LDS (the north star's named kernel form)",
    "rs32_diff_update_lds": "the per-SET diff-update + install with the LDS engine (AUTO runs it with "
                            "PERM: the comparison, DESIGN.md §4)",
    "rs32_1m_recovery": "BASELINE configs[4] as stated: online recovery decode of ONE lost data shard "
                        "(every stripe the same), 1,024 x 1 MiB values, device-resident; D0 led by P0 "
                        "(inverse 1) and D1 led by P1 (inverse 1/245), SURVEY §8d",
    # The server placements: the state where the
    # unchanged server keeps it -- host memory, the arena registered once -- through the
    # library API only, each beside the reference's 1-thread CPU loop (restated).
    "drain_host_ecmem": "parity drain (memcached.c:4350 -> 7739-7767): 65,536 pageable 4098-B diffs at "
                        "shuffled slots of a host ecmem registered with cec_host_register, one "
                        "cec_drainer_apply per step",
    "recovery_pool_host": "recovery into a cec_recovery_pool over a registered host ecmem "
                          "(recovery.c:61-96 + memcached.c:7842-7922; idle recoverer memcached.c:5712-5734): "
                          "one 1 MiB range and an 85-request idle pass, replies received into the pool's "
                          "staging, ONE add_peers + flush_solve_host per pass, rebuilt bytes read in place",
    "set_diffs_host": "data-side SET diffs (memcached.c:2676-2681): 65,536 SETs of 4098 B, pageable values, "
                      "shuffled addresses of a registered host ecmem, one cec_region_multiply_batch per step",
}
SERVER_WORKLOADS = ("drain_host_ecmem", "recovery_pool_host", "set_diffs_host")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="rs32_4k", choices=sorted(WORKLOADS))
    ap.add_argument("--engine", default="auto", choices=["auto", "perm", "lds"],
                    help="GF(2^8) engine (cec_set_engine); auto = the library default: LDS for "
                         "decodes of values of 64 KiB and more, PERM for every other op "
                         "(cocytus_ec.h)")
    ap.add_argument("--e2e", action="store_true", help="pinned host -> HBM -> host pipeline")
    ap.add_argument("--e2e-streams", type=int, default=6)  # best of a 3..16 sweep
    ap.add_argument("--drain", action="store_true", help="batched parity drain from host diffs")
    ap.add_argument("--recovery", action="store_true", help="online recovery session, host survivors")
    ap.add_argument("--ops", action="store_true",
                    help="device-resident roofline of every SURVEY §8a op (a1-a7 + fused decode)")
    ap.add_argument("--e2e-chunk", type=int, default=4096, help="stripes per pipelined chunk")
    ap.add_argument("--e2e-zero-copy", action="store_true",
                    help="--e2e with the kernels reading / writing pinned host memory directly")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the fixed-batch (strong scaling) record of the metric's workload")
    ap.add_argument("--harness-check", action="store_true",
                    help="run only the multi-rank harness (gloo, no GPU): launcher, shards, "
                         "barriers, max over ranks")
    ap.add_argument("--also", default="rs32_4k_lds,rs32_mixed,rs32_1m,rs42_64k,rs32_1m_recovery,"
                                      "rs32_diff_update,rs32_diff_update_lds,rs32_e2e,"
                                      "drain_host_ecmem,recovery_pool_host,set_diffs_host",
                    help="other workloads measured after the main one, reported under "
                         "other_workloads ('' = none)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="wall-clock budget of the CPU-baseline thread sweep (seconds)")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend for the barrier / max-over-ranks (nccl = RCCL; "
                         "auto = nccl, or gloo when CEC_BENCH_DEVICE pins every rank to one card)")
    args = ap.parse_args(argv)
    if args.dist_backend == "auto":
        args.dist_backend = "gloo" if os.environ.get("CEC_BENCH_DEVICE") else "nccl"
    bad = [w for w in args.also.split(",") if w and w not in WORKLOADS and w not in EXTRA_WORKLOADS]
    if bad:
        ap.error(f"--also: unknown workload(s) {bad}; choose from "
                 f"{sorted(WORKLOADS) + sorted(EXTRA_WORKLOADS)}")
    return args


def layout(workload, seed=0xC0C70003):
    """[(arena offset, length)] of every stripe; starts 16-B aligned (ecalloc.c:176)."""
    k, m, n, B, _ = WORKLOADS[workload]
    if n:
        return [(s * n, n) for s in range(B)], B * n
    import random

    rng = random.Random(seed)
    out, off, total = [], 0, 0
    lo, hi = math.log(256), math.log(1 << 20)
    while total < (1 << 30):
        ln = int(math.exp(rng.uniform(lo, hi)))
        out.append((off, ln))
        total += ln
        off = (off + ln + 15) & ~15
    return out, off


def shard_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous split of `total` units over `world` ranks."""
    return total * rank // world, total * (rank + 1) // world


def shard_stripes(stripes, rank: int, world: int) -> tuple[int, int]:
    """The stripes [lo, hi) of rank `rank` in a contiguous split of a batch over `world`
    GPUs: by count when every value has one size, by byte count for mixed
    sizes (each rank's share holds about total / world bytes)."""
    if len({ln for _, ln in stripes}) <= 1:
        return shard_range(len(stripes), rank, world)
    ends, acc = [], 0
    for _, ln in stripes:
        acc += ln
        ends.append(acc)

    def cut(r):  # first stripe whose bytes start at or past r * total / world
        target = acc * r // world
        lo, hi = 0, len(ends)
        while lo < hi:
            mid = (lo + hi) // 2
            if ends[mid] <= target:
                lo = mid + 1
            else:
                hi = mid
        return lo if r else 0

    return (cut(rank), cut(rank + 1) if rank + 1 < world else len(stripes))


def dist_on(dist) -> bool:
    """A process group is up (world size > 1, or CEC_BENCH_PG=1 at world size 1): the
    barriers and the max over ranks then run as collectives."""
    return dist is not None and dist.is_available() and dist.is_initialized()


def max_over_ranks(values, dist):
    """Element-wise max of a list of floats over all ranks (identity without a process
    group; a real all_reduce with one, even of one rank)."""
    import torch

    if not dist_on(dist):
        return [float(x) for x in values]
    device = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.tolist()]


def host_cpu() -> dict:
    """The host the CPU baseline ran on (model, visible CPUs)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = None
    return {"model": model, "nproc": os.cpu_count(), "affinity": allowed, "cpu_quota": cpu_quota()}


def cpu_quota():
    """CPUs this process's cgroup may use (cpu.max / cfs quota), None if unlimited.  A
    shared GPU box grants one GPU's share of the host: more threads than that only
    time-slice."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(float(q) / float(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = float(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_thread_counts(allowed: int) -> list[int]:
    """SURVEY §8d sweep: 1 (the reference's own configuration: one worker thread per
    server process, memcached.c:6990), 16, 64 and every CPU this process may run on."""
    return sorted({t for t in (1, 16, 64, allowed) if 1 <= t <= allowed})


CPU_SAMPLES = 5  # timed passes per thread count, after one warm-up pass


def cpu_allowed(h=None) -> int:
    """CPUs this process may run threads on: its affinity, capped at the cgroup quota
    (threads beyond the quota only time-slice)."""
    h = h or host_cpu()
    allowed = h["affinity"] or os.cpu_count() or 1
    if h["cpu_quota"]:
        allowed = max(1, min(allowed, math.ceil(h["cpu_quota"])))
    return allowed


CPU_OTHER_S = 3.0  # CPU-baseline budget per other workload (top thread count only)


def cpu_baseline(k, m, n, wall_s, threads_list=None, samples=CPU_SAMPLES, sizes=None):
    """Oracle (restated Jerasure/GF-Complete, AVX2) on the host cores, bounded samples.

    One pthread per CPU on disjoint stripes, swept over cpu_thread_counts(); at each
    point the batch is filled once, one pass warms up, then `samples` timed passes of
    about wall_s / len(sweep) / (samples + 1) seconds each: median, min and max.
    `value` / `cores` is the median of the all-CPU point (the host's ceiling);
    `reference_config` is the 1-thread point (the reference's configuration).
    sizes: the value lengths of a mixed batch (the whole batch, instead of 256 MiB of
    n-byte stripes per shard); n is then ignored."""
    from oracle import pyoracle

    h = host_cpu()
    counts = threads_list or cpu_thread_counts(cpu_allowed(h))
    per_point = max(0.2, wall_s / len(counts))
    if sizes is None:
        stripes = (256 << 20) // n  # 256 MiB per shard, 1.25 GiB for RS(3,2): above any LLC
        payload = (k + 1) * n * stripes  # K*n encoded + n rebuilt per stripe, as the GPU metric

        def run(T, reps, count):
            return pyoracle.bench_encode_decode_samples(k, m, n, stripes, T, reps, count, True)
    else:
        stripes = len(sizes)
        payload = (k + 1) * sum(sizes)

        def run(T, reps, count):
            return pyoracle.bench_encode_decode_sizes(k, m, sizes, T, reps, count, True)
    simd = "AVX2" if pyoracle.simd_available() else "scalar"
    sweep = []
    for T in counts:
        # calibrate: one pass after a warm-up pass (fill untimed)
        t1 = run(T, 1, 2)[1]
        reps = max(1, min(1000, int(per_point / (samples + 1) / max(t1, 1e-6))))
        ts = run(T, reps, samples + 1)[1:]
        vals = sorted(round(payload * reps / t / 2**30, 3) for t in ts)
        sweep.append({"threads": T, "value": statistics.median(vals), "median": statistics.median(vals),
                      "min": vals[0], "max": vals[-1], "samples": vals, "passes_per_sample": reps,
                      "wall_s": round(sum(ts), 2)})
    top = sweep[-1]
    from oracle import jerasure_probe

    ref_lib, where = jerasure_probe.load()  # probe for the real library
    return {
        "value": top["median"],
        "unit": "GiB/s",
        "cores": top["threads"],
        "host": h,
        "kind": "port",
        "label": "restated CPU baseline",  # Jerasure / GF-Complete absent
        "median": top["median"], "min": top["min"], "max": top["max"], "samples": top["samples"],
        "sample": f"RS({k},{m}) encode+decode of {stripes} x "
                  f"{'%d B' % n if sizes is None else 'mixed 256 B - 1 MiB (the GPU batch)'} stripes on "
                  f"{top['threads']} threads: "
                  f"median of {samples} timed passes ({top['passes_per_sample']} repetitions each) after "
                  f"one warm-up pass; every CPU this process may use (affinity {h['affinity']}, cgroup "
                  f"quota {h['cpu_quota']}), the host's ceiling for it; restated GF-Complete SPLIT(8,4) "
                  f"split-nibble ({simd}), chained like memcached.c/recovery.c",
        "reference_config": dict(sweep[0], note="1 thread: the reference's configuration, one worker "
                                                "thread per server process (memcached.c:6990)"),
        "sweep": sweep,
        "reference_probe": f"system libJerasure found at {where} (pins the oracle: tests/test_oracle.py)"
                           if ref_lib is not None else where,
    }


_CODE_ID = []


def this_code_id():
    """ec.kernel_code_id() of the in-tree library, computed once per process (~2 s)."""
    if not _CODE_ID:
        from cocytus_amd import ec

        _CODE_ID.append(ec.kernel_code_id())
    return _CODE_ID[0]


def load_traffic(workload, ops=("encode", "decode"), engine="perm", code_id=None):
    """HBM bytes per launch of each op from the committed rocprofv3 --pmc summary of the
    engine that ran it (profiles/pmc_traffic.json: PERM, pmc_traffic_lds.json: LDS;
    written by tools/profile_round.sh + tools/pmc_summary.py), and whether it is stale.

    The summary records the device code it measured (`_build.kernel_code_id`: a hash of
    the library's disassembled gfx950 kernels, ec.kernel_code_id).  When that differs
    from the library this run loads (`code_id`, default: the in-tree build), or is
    missing, the bytes describe other kernels: every value is None and stale is True.
    Returns (values tuple, stale)."""
    name = "pmc_traffic.json" if engine == "perm" else f"pmc_traffic_{engine}.json"
    none = tuple(None for _ in ops)
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return none, True
    if code_id is None:
        code_id = this_code_id()
    if not code_id or doc.get("_build", {}).get("kernel_code_id") != code_id:
        return none, True
    e = doc.get(workload, {})
    return tuple(e.get(f"{op}_hbm_bytes_per_launch") for op in ops), False


def device_identity(torch, dev) -> dict:
    """Which physical GPU this rank ran on: ordinal, name, PCI address and UUID (the
    N > 1 line must show on its own that N distinct GPUs ran)."""
    p = torch.cuda.get_device_properties(dev)
    return {"device": dev, "name": p.name, "arch": p.gcnArchName.split(":")[0],
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "uuid": str(p.uuid)}


def gather_ranks(dist, mine: dict) -> list:
    """Every rank's entry, in rank order, on every rank (one all_gather_object, outside
    every timed region; identity when alone)."""
    if not dist_on(dist):
        return [mine]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, mine)
    return out


def ranks_summary(entries: list, backend: str) -> dict:
    """The N > 1 line's evidence: per rank its device identity and its own
    step times (before the max over ranks), whether the ranks ran on distinct devices
    (by UUID and PCI address), and which rank was slowest in each record."""
    ids = {(e["identity"].get("uuid"), e["identity"].get("pci")) for e in entries}
    out = {"world_size": len(entries), "backend": backend, "distinct_devices": len(ids) == len(entries),
           "per_rank": entries}
    for rec in ("weak", "strong"):
        ts = [(e[rec]["ms_per_step"], e["rank"]) for e in entries if e.get(rec)]
        if ts:
            out[f"slowest_rank_{rec}"] = max(ts)[1]
    return out


def setup(backend="nccl"):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CEC_BENCH_DEVICE pins every rank to one device: a gloo rehearsal of the
    # multi-rank path on a one-GPU box (never used for reported numbers).
    dev = int(os.environ.get("CEC_BENCH_DEVICE", local))
    torch.cuda.set_device(dev)
    # CEC_BENCH_PG=1 brings the process group up at world size 1 as well (a one-rank RCCL
    # communicator): the N > 1 line's collectives -- barriers, the all_reduce MAX, the
    # per-rank all_gather -- then run on a one-GPU box (tests/test_gpu_parity.py).
    if world > 1 or os.environ.get("CEC_BENCH_PG") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
    torch.empty(1, device="cuda")  # torch owns the HIP runtime before the library loads
    from cocytus_amd import ec

    ec.lib()
    if ec.device_check() != ec.CEC_OK:
        raise SystemExit("libcocytus_ec: " + ec.lib().cec_last_error().decode())
    return torch, dist, ec, world, rank


ENGINES = {"auto": 2, "perm": 0, "lds": 1}  # cec_engine


def set_engine(ec, name):
    ec.set_engine(ENGINES[name])


def engine_ran(ec):
    """The engine the calling thread's last op ran with, as the library reports it
    (cec_last_engine: AUTO resolved per op)."""
    e = ec.last_engine()
    if e < 0:
        raise RuntimeError("cec_last_engine: no op has run on this thread")
    return "lds" if e == ec.CEC_ENGINE_LDS else "perm"


def share_layout(stripes, lo, hi):
    """Stripes [lo, hi) of a batch, re-based to offset 0 (one GPU's own arenas hold its
    share of a fixed batch: SURVEY §8e), and the arena bytes they need."""
    sub = stripes[lo:hi]
    if not sub:
        return [], 0
    base = sub[0][0]
    out = [(o - base, ln) for o, ln in sub]
    return out, (out[-1][0] + out[-1][1] + 15) & ~15


def measure_device(torch, dist, ec, world, rank, workload, args, share=None):
    """Encode + rotating single-shard decode of `workload`, timed over args.steps.

    share = (lo, hi): this rank runs only stripes [lo, hi) of the workload's batch (the
    fixed-batch split of SURVEY §8e); `value` then counts the whole batch's payload once
    over all ranks (strong scaling).  Otherwise every rank runs the whole batch (weak).
    Returns the rank-0 result fields (every rank returns them; only rank 0 prints)."""
    k, m, n, _, what = WORKLOADS[workload]
    stripes, arena = layout(workload)
    full_bytes = sum(ln for _, ln in stripes)
    full_arena = arena
    if share is not None:
        stripes, arena = share_layout(stripes, *share)
        # A GPU's arenas keep the whole batch's size and its share fills their start: a
        # Cocytus server's arenas are MEMSIZE whatever number of values its key shard
        # receives (const.h:25, memcached.c:380-381), so only the values per GPU change
        # with N.  (Share-sized arenas, CEC_BENCH_SHARE_ARENA=share, put the streams
        # 32 MiB apart at 8,192 stripes: encode 28.3-28.7 against 27.6-28.1 us,
        # profiles/r03_evidence/share_arena_ab/.)
        if os.environ.get("CEC_BENCH_SHARE_ARENA") != "share":
            arena = full_arena
    B = len(stripes)
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70002 + rank)
    # the K data, M parity and K rebuilt arenas, carved from one allocation at the
    # odd-4 KiB stride of cec_arenas_alloc (HBM channel layout)
    arenas = ec.arena_tensors(k + m + k, arena)
    data, parity, out = arenas[:k], arenas[k:k + m], arenas[k + m:]
    for t in data:
        t.random_(0, 256, generator=g)
    for t in out:
        t.zero_()
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    enc_plan = ec.Plan([(o, 0, ln, 0) for o, ln in stripes])
    dec_ext = [(o, 0, ln, s % len(masks)) for s, (o, ln) in enumerate(stripes)]
    dec_plan = ec.Plan(dec_ext)
    stream = torch.cuda.current_stream()
    bytes_total = sum(ln for _, ln in stripes)

    eng = {}
    for _ in range(max(1, args.warmup)):
        ec.encode(k, m, mat, data, parity, enc_plan, stream)
        eng["encode"] = engine_ran(ec)
        ec.decode(k, m, mat, masks, data + parity, out, dec_plan, stream)
        eng["decode"] = engine_ran(ec)
    torch.cuda.synchronize()

    # One event between consecutive launches: event 2s..2s+1 brackets step s's encode and
    # 2s+1..2s+2 its decode.  (An event before and after every launch cost 1.4 % of the
    # step, two per step 0.4 %: tools/event_cost.py)
    evs = [ec.Event() for _ in range(2 * args.steps + 1)]
    host = [0.0, 0.0]  # host time spent enqueueing the encodes / the decodes
    pc = time.perf_counter
    if dist_on(dist):
        dist.barrier()
    torch.cuda.synchronize()
    t0 = pc()
    evs[0].record(stream)
    for s in range(args.steps):
        h0 = pc()
        ec.encode(k, m, mat, data, parity, enc_plan, stream)
        h1 = pc()
        evs[2 * s + 1].record(stream)
        h2 = pc()
        ec.decode(k, m, mat, masks, data + parity, out, dec_plan, stream)
        h3 = pc()
        evs[2 * s + 2].record(stream)
        host[0] += h1 - h0
        host[1] += h3 - h2
    t_enq = pc() - t0  # the host is this far ahead of the GPU when the loop ends
    torch.cuda.synchronize()
    elapsed = pc() - t0  # this rank's K steps; the max over ranks is taken below
    if dist_on(dist):
        dist.barrier()
    own_elapsed = elapsed
    enc_t = [evs[2 * s].elapsed_ms(evs[2 * s + 1]) for s in range(args.steps)]
    dec_t = [evs[2 * s + 1].elapsed_ms(evs[2 * s + 2]) for s in range(args.steps)]
    enc_ms, dec_ms = sum(enc_t) / args.steps, sum(dec_t) / args.steps  # = rocprof's average
    import numpy as np

    ok = True  # every shard the timed steps rebuilt equals the original (on the device)
    lost_of = [[x for x in range(k) if not (mk >> x) & 1][0] for mk in masks]
    for j in range(k):
        sel = np.zeros(arena, dtype=bool)
        for s, (o, ln) in enumerate(stripes):
            if lost_of[s % len(masks)] == j:
                sel[o:o + ln] = True
        sel_d = torch.from_numpy(sel).cuda()
        # elementwise (no boolean indexing: its nonzero() allocates index tensors of the
        # arena's size and synchronises; four ranks sharing one card stalled in it)
        ok &= not bool(((out[j] != data[j]) & sel_d).any())
    elapsed, bad = max_over_ranks([elapsed, 0.0 if ok else 1.0], dist)
    enc_plan.destroy()
    dec_plan.destroy()
    del arenas, data, parity, out

    # weak: every rank ran the whole batch; strong: the ranks' shares add up to one batch
    payload = (k + 1) * (full_bytes if share is not None else bytes_total * world) * args.steps
    enc_bytes = (k + m) * bytes_total  # algorithmic HBM bytes per encode launch
    dec_bytes = (k + 1) * bytes_total  # per decode launch (read K survivors, write 1)
    enc_gbps = enc_bytes / (enc_ms * 1e-3) / 1e9
    dec_gbps = dec_bytes / (dec_ms * 1e-3) / 1e9
    # traffic from the committed PMC summary of the engine each op ran with (the library's
    # own report, cec_last_engine), if it measured this build's kernels
    (enc_traffic, _), enc_stale = load_traffic(workload, engine=eng["encode"])
    (_, dec_traffic), dec_stale = load_traffic(workload, engine=eng["decode"])
    return {
        "k": k, "m": m, "n": n, "B": B, "what": what, "bytes_total": bytes_total, "engine": eng,
        "value": payload / elapsed / 2**30,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "verified": ok and bad == 0.0,
        "rank": {"ms_per_step": round(own_elapsed * 1e3 / args.steps, 4), "encode_ms": round(enc_ms, 4),
                 "decode_ms": round(dec_ms, 4), "verified": bool(ok)},
        "kernel_ms_per_step": enc_ms + dec_ms,
        "host_enqueue_us": {"encode": round(host[0] / args.steps * 1e6, 2),
                            "decode": round(host[1] / args.steps * 1e6, 2),
                            "step_loop": round(t_enq / args.steps * 1e6, 2)},
        "roofline": {
            "bound": "hbm",
            "achieved": round(enc_gbps, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(enc_gbps / HBM_PEAK_GBPS, 4),
            "traffic": enc_traffic,
            "traffic_stale": enc_stale,
            "kernel_code_id": this_code_id(),
            "kernel": f"combine_kernel<{k},{m},{'LdsEngine' if eng['encode'] == 'lds' else 'PermEngine'},"
                      "kAccNone,exact> (cec_encode)",
            "algorithmic_bytes_per_launch": enc_bytes,
            "launch_ms": round(enc_ms, 4),
            "launch_ms_median": round(statistics.median(enc_t), 4),
        },
        "decode_roofline": {
            "achieved": round(dec_gbps, 1), "frac": round(dec_gbps / HBM_PEAK_GBPS, 4),
            "algorithmic_bytes_per_launch": dec_bytes, "launch_ms": round(dec_ms, 4),
            "launch_ms_median": round(statistics.median(dec_t), 4), "traffic": dec_traffic,
            "traffic_stale": dec_stale,
        },
    }


STRONG_PREDICT_N = (2, 4, 8)


def measure_strong(torch, dist, ec, world, rank, args, whole):
    """Fixed-batch (strong) scaling of the metric's workload, SURVEY §8e: the batch's
    65,536 stripes split contiguously over the ranks with shard_range, each GPU holding
    only its share; aggregate = whole-batch payload / max over ranks of the step time.

    At N = 1 the shares a fixed batch gives at N = 2, 4, 8 are timed on the one GPU
    instead (32,768, 16,384, 8,192 stripes): GPUs share nothing on this path (no
    collective, no host or PCIe traffic in the timed region), so the N-GPU step takes
    what one GPU takes for its share, and the predicted factor is t(batch) / t(share).
    `whole` is the weak (whole-batch) result of this rank, the N = 1 point."""
    stripes = layout(args.workload)[0]
    B = len(stripes)

    def point(r, stripes, n_gpus):
        return {"n_gpus": n_gpus, "stripes_per_gpu": stripes, "ms_per_step": round(r["ms_per_step"], 4),
                "kernel_ms_per_step": round(r["kernel_ms_per_step"], 4),
                "encode_ms": r["roofline"]["launch_ms"], "decode_ms": r["decode_roofline"]["launch_ms"],
                "gap_ms_per_step": round(r["ms_per_step"] - r["kernel_ms_per_step"], 4),
                "host_enqueue_us": r["host_enqueue_us"], "verified": r["verified"]}

    if world > 1:
        lo, hi = shard_stripes(stripes, rank, world)
        r = measure_device(torch, dist, ec, world, rank, args.workload, args, share=(lo, hi))
        out = point(r, hi - lo, world)
        out.update(value=round(r["value"], 2), unit="GiB/s", rank=dict(r["rank"], stripes=[lo, hi]),
                   split=f"contiguous split of the {B} stripes over {world} GPUs (shard_stripes: by "
                         "count, by bytes for mixed sizes), max over ranks")
        return out
    t1 = whole["ms_per_step"]
    pts = [dict(point(whole, B, 1), speedup=1.0, efficiency=1.0, value=round(whole["value"], 2))]
    for N in STRONG_PREDICT_N:
        torch.cuda.empty_cache()
        lo, hi = shard_stripes(stripes, 0, N)
        r = measure_device(torch, dist, ec, 1, 0, args.workload, args, share=(lo, hi))
        sp = t1 / r["ms_per_step"]
        pts.append(dict(point(r, hi - lo, N), speedup=round(sp, 3), efficiency=round(sp / N, 4),
                        value=round(whole["value"] * sp, 2)))
    return {"n_gpus": 1, "value": round(whole["value"], 2), "unit": "GiB/s",
            "predicted": pts,
            "method": "per-GPU shares of the fixed batch timed on this GPU; predicted value at N = "
                      "whole-batch payload / the share's step time (no cross-GPU traffic)"}


def measure_diff_update(torch, dist, ec, world, rank, args):
    """The north star's first op on device-resident arenas: 65,536 SETs of 4 KiB per GPU,
    source shard j uniform in {0,1,2}, one cec_diff_update launch per step
    (d = new ^ old; P_p ^= MATRIX(K+p, j) * d for both parities; old := new).  Steps
    alternate between two staging batches so every step changes every value.  Check
    (size-independent): afterwards parity == encode(data), on the device."""
    k, m, n, B = 3, 2, 4096, 65536
    T = n * B
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70006 + rank)
    ar = ec.arena_tensors(k + m + 2, T)
    data, parity, stage = ar[:k], ar[k:k + m], ar[k + m:]
    for t in data + stage:
        t.random_(0, 256, generator=g)
    src = torch.randint(0, k, (B,), generator=torch.Generator().manual_seed(0xC0C70006 + rank)).tolist()
    plan = ec.Plan([(s * n, s * n, n, src[s]) for s in range(B)])
    stream = torch.cuda.current_stream()
    ec.encode_region(k, m, mat, data, parity, T, stream)
    warm = max(1, args.warmup)
    for w in range(warm):
        ec.diff_update(k, m, mat, data, stage[w % 2], parity, True, plan, stream)
    eng = engine_ran(ec)  # the library's own report of the engine the op ran with
    evs = [ec.Event() for _ in range(args.steps + 1)]
    torch.cuda.synchronize()
    if dist_on(dist):
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record(stream)
    for s in range(args.steps):
        ec.diff_update(k, m, mat, data, stage[(warm + s) % 2], parity, True, plan, stream)
        evs[s + 1].record(stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist_on(dist):
        dist.barrier()
    du_t = [evs[s].elapsed_ms(evs[s + 1]) for s in range(args.steps)]
    ms = sum(du_t) / args.steps
    lds = eng == "lds"
    own_elapsed = elapsed
    chk = [torch.empty(T, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, chk, T, stream)
    torch.cuda.synchronize()
    ok = all(torch.equal(chk[p], parity[p]) for p in range(m))
    elapsed, bad = max_over_ranks([elapsed, 0.0 if ok else 1.0], dist)
    plan.destroy()
    del ar, data, parity, stage, chk
    nbytes = (2 + 2 * m + 1) * T  # read old, new, M parities; write M parities + install
    gbps = nbytes / (ms * 1e-3) / 1e9
    traffic, stale = load_traffic("rs32_diff_update", ("diff_update",), eng)
    return {
        "value": round(T * world * args.steps / elapsed / 2**30, 2), "unit": "GiB/s",
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "workload": f"RS(3,2) {EXTRA_WORKLOADS['rs32_diff_update']}; value = SET payload (n per SET)",
        "roofline": {"bound": "hbm", "achieved": round(gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(gbps / HBM_PEAK_GBPS, 4), "algorithmic_bytes_per_launch": nbytes,
                     "launch_ms": round(ms, 4), "launch_ms_median": round(statistics.median(du_t), 4),
                     "kernel": f"combine_kernel<2,3,{'LdsEngine' if lds else 'PermEngine'},kAccAllButLast,exact> "
                               "(cec_diff_update, install)",
                     "traffic": traffic[0], "traffic_stale": stale},
        "engine": eng,
        "verified": bool(ok and bad == 0.0),
        "rank": {"ms_per_step": round(own_elapsed * 1e3 / args.steps, 4), "launch_ms": round(ms, 4),
                 "verified": bool(ok)},
    }


def measure_recovery_decode(torch, dist, ec, world, rank, args):
    """BASELINE configs[4] as SURVEY §8d states it: RS(3,2) decode of one lost data shard,
    1,024 x 1 MiB values, one fixed mask for the whole batch (a recovering server rebuilds
    one lid, memcached.c:7842-7922): D0 led by P0 (inverse 1) and D1 led by P1 (inverse
    1/245), each timed as args.steps back-to-back cec_decode launches of the whole batch.
    value = rebuilt GiB/s (n per stripe), per case; check: the rebuilt shard == the data."""
    k, m, n, B = 3, 2, 1 << 20, 1024
    T = n * B
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70005 + rank)
    ar = ec.arena_tensors(k + m + 1, T)
    data, parity, out = ar[:k], ar[k:k + m], ar[k + m]
    for t in data:
        t.random_(0, 256, generator=g)
    stream = torch.cuda.current_stream()
    ec.encode_region(k, m, mat, data, parity, T, stream)
    plan = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
    cases = {}
    for name, lost, leader in (("D0_leader_P0", 0, k), ("D1_leader_P1", 1, k + 1)):
        mask = ec.recovery_mask(k, m, leader, [int(i != lost) for i in range(k + m)])
        outs = [out if j == lost else None for j in range(k)]
        out.zero_()
        for _ in range(max(1, args.warmup)):
            ec.decode(k, m, mat, [mask], data + parity, outs, plan, stream)
        eng = engine_ran(ec)
        evs = [ec.Event() for _ in range(args.steps + 1)]
        torch.cuda.synchronize()
        if dist_on(dist):
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evs[0].record(stream)
        for s in range(args.steps):
            ec.decode(k, m, mat, [mask], data + parity, outs, plan, stream)
            evs[s + 1].record(stream)
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        if dist_on(dist):
            dist.barrier()
        ts = [evs[s].elapsed_ms(evs[s + 1]) for s in range(args.steps)]
        ms = sum(ts) / args.steps
        ok = bool(torch.equal(out, data[lost]))
        own_elapsed = elapsed
        elapsed, bad = max_over_ranks([elapsed, 0.0 if ok else 1.0], dist)
        dec_bytes = (k + 1) * T  # read K survivors, write the rebuilt shard
        gbps = dec_bytes / (ms * 1e-3) / 1e9
        cases[name] = {
            "value": round(n * B * world * args.steps / elapsed / 2**30, 2), "unit": "GiB/s rebuilt",
            "mask": mask, "launch_ms": round(ms, 4), "launch_ms_median": round(statistics.median(ts), 4),
            "decode_frac": round(gbps / HBM_PEAK_GBPS, 4), "achieved_GBps": round(gbps, 1),
            "algorithmic_bytes_per_launch": dec_bytes, "verified": ok and bad == 0.0, "engine": eng,
            "rank": {"ms_per_step": round(own_elapsed * 1e3 / args.steps, 4), "launch_ms": round(ms, 4),
                     "verified": ok},
        }
    plan.destroy()
    del ar, data, parity, out
    return {"workload": EXTRA_WORKLOADS["rs32_1m_recovery"], "cases": cases, "engine": eng,
            "value": min(c["value"] for c in cases.values()), "unit": "GiB/s rebuilt (slower case)",
            "decode_frac": min(c["decode_frac"] for c in cases.values()),
            "verified": all(c["verified"] for c in cases.values())}


_PCIE = {}


def pcie_floor(torch, h2d_bytes, d2h_bytes):
    """The PCIe floor of a step that moves h2d_bytes host -> device and d2h_bytes back
    (the two directions overlap): max over directions of bytes / this link's raw pinned
    copy rate (measured once per process, outside every timed region).  Seconds, and the
    rates."""
    if not _PCIE:
        _PCIE["h2d"], _PCIE["d2h"] = pcie_raw(torch)
    return (max(h2d_bytes / (_PCIE["h2d"] * 1e9), d2h_bytes / (_PCIE["d2h"] * 1e9)),
            {x: round(v, 1) for x, v in _PCIE.items()})


def pcie_raw(torch, nbytes=256 << 20, reps=4):
    """Raw pinned H2D / D2H copy rates of this GPU's link (GB/s)."""
    x = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    y = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    y.copy_(x, non_blocking=True)
    torch.cuda.synchronize()
    rates = []
    for a, b in ((y, x), (x, y)):
        t1 = time.perf_counter()
        for _ in range(reps):
            a.copy_(b, non_blocking=True)
        torch.cuda.synchronize()
        rates.append(reps * nbytes / (time.perf_counter() - t1) / 1e9)
    return rates[0], rates[1]


class E2E:
    """RS(3,2) 4 KiB encode + decode with the values in pinned host memory.

    Staged (default): per chunk of stripes, H2D of the K data shards -> encode -> D2H of
    the M parities, and H2D of the K survivors (D1..D_{K-1}, P0) -> decode of D0 -> D2H
    of the rebuilt shard; chunks round-robin over HIP streams.  Zero-copy: the kernels
    read and write the pinned host buffers over PCIe, one launch per op."""

    def __init__(self, torch, ec, args, zero_copy=False):
        self.torch, self.ec = torch, ec
        self.k, self.m, self.n, self.B, _ = WORKLOADS["rs32_4k"]
        k, m, n, B = self.k, self.m, self.n, self.B
        self.mat = ec.coding_matrix(k, m)
        self.chunk = args.e2e_chunk  # stripes per chunk (4096: 16 MiB per shard)
        self.ns = args.e2e_streams
        self.zero_copy = zero_copy
        clen = self.chunk * n
        pin = dict(dtype=torch.uint8, pin_memory=True)
        self.data_h = [torch.randint(0, 256, (B * n,), dtype=torch.uint8).pin_memory() for _ in range(k)]
        self.par_h = [torch.empty(B * n, **pin) for _ in range(m)]
        self.out_h = torch.empty(B * n, **pin)
        self.streams = [torch.cuda.Stream() for _ in range(self.ns)]
        self.slots = [{"d": [torch.empty(clen, dtype=torch.uint8, device="cuda") for _ in range(k)],
                       "p": [torch.empty(clen, dtype=torch.uint8, device="cuda") for _ in range(m)],
                       "o": torch.empty(clen, dtype=torch.uint8, device="cuda")} for _ in self.streams]
        self.mask = ec.recovery_mask(k, m, k, [0] + [1] * (k + m - 1))  # D0 lost, leader P0
        self.plan = ec.Plan([(s * n, 0, n, 0) for s in range(self.chunk)])
        self.zc_plan = ec.Plan([(s * n, 0, n, 0) for s in range(B)]) if zero_copy else None
        self.h2d_bytes = 2 * k * n * B  # per step: K data shards, then K survivors
        self.d2h_bytes = (m + 1) * n * B  # M parities + the rebuilt shard
        self.payload = (k + 1) * n * B  # K*n encoded + n rebuilt per stripe (the metric's)

    def step(self):
        torch, ec, k, m = self.torch, self.ec, self.k, self.m
        if self.zero_copy:
            s = torch.cuda.current_stream()
            ec.encode(k, m, self.mat, self.data_h, self.par_h, self.zc_plan, s)
            ec.decode(k, m, self.mat, [self.mask], self.data_h + self.par_h, [self.out_h, None, None],
                      self.zc_plan, s)
            return
        clen = self.chunk * self.n
        for c in range(self.B // self.chunk):
            st, sl = self.streams[c % self.ns], self.slots[c % self.ns]
            lo, hi = c * clen, (c + 1) * clen
            with torch.cuda.stream(st):
                for j in range(k):
                    sl["d"][j].copy_(self.data_h[j][lo:hi], non_blocking=True)
                ec.encode(k, m, self.mat, sl["d"], sl["p"], self.plan, st)
                for p in range(m):
                    self.par_h[p][lo:hi].copy_(sl["p"][p], non_blocking=True)
                for j in range(1, k):  # survivors arrive again from the peers
                    sl["d"][j].copy_(self.data_h[j][lo:hi], non_blocking=True)
                sl["p"][0].copy_(self.par_h[0][lo:hi], non_blocking=True)
                ec.decode(k, m, self.mat, [self.mask], sl["d"] + sl["p"], [sl["o"], None, None],
                          self.plan, st)
                self.out_h[lo:hi].copy_(sl["o"], non_blocking=True)

    def verified(self):
        return bool(self.torch.equal(self.out_h, self.data_h[0]))

    def close(self):
        self.plan.destroy()
        if self.zc_plan is not None:
            self.zc_plan.destroy()


def measure_e2e(torch, dist, ec, world, rank, args):
    """E2E (staged) beside the device-resident workloads, barrier + max over ranks (each
    GPU has its own PCIe link: weak scaling).  pcie_bound_frac = the step's PCIe floor
    max(H2D bytes / raw H2D, D2H bytes / raw D2H) over the measured step time."""
    e = E2E(torch, ec, args)
    for _ in range(max(1, args.warmup)):
        e.step()
    torch.cuda.synchronize()
    ok = e.verified()
    steps = max(1, min(args.steps, 10))
    if dist_on(dist):
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        e.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist_on(dist):
        dist.barrier()
    floor_s, raw = pcie_floor(torch, e.h2d_bytes, e.d2h_bytes)
    h2d, d2h = raw["h2d"], raw["d2h"]
    own = el
    el, bad = max_over_ranks([el, 0.0 if ok else 1.0], dist)
    out = {
        "value": round(e.payload * world * steps / el / 2**30, 2), "unit": "GiB/s",
        "ms_per_step": round(el * 1e3 / steps, 3), "steps": steps,
        "workload": f"{EXTRA_WORKLOADS['rs32_e2e']}; 65,536 stripes per GPU, {e.chunk}-stripe chunks "
                    f"over {e.ns} streams",
        "pcie_bound_frac": round(floor_s / (el / steps), 4),
        "pcie_GBps_raw": {"h2d": round(h2d, 1), "d2h": round(d2h, 1)},
        "h2d_bytes_per_step": e.h2d_bytes, "d2h_bytes_per_step": e.d2h_bytes,
        "verified": bool(ok and bad == 0.0),
        "rank": {"ms_per_step": round(own * 1e3 / steps, 3), "verified": bool(ok)},
    }
    e.close()
    return out


def host_array(nbytes: int, fill_seed=None):
    """A page-aligned uint8 numpy array of nbytes in ordinary (pageable) host memory, filled
    with seeded random bytes when fill_seed is given (the server's malloc / mmap memory)."""
    import numpy as np

    raw = np.empty(nbytes + 4096, np.uint8)
    off = (-raw.ctypes.data) % 4096
    a = raw[off:off + nbytes]
    if fill_seed is not None:
        rng = np.random.default_rng(fill_seed)
        step = 64 << 20
        for o in range(0, nbytes, step):
            n = min(step, nbytes - o)
            a[o:o + n] = np.frombuffer(rng.bytes(n), np.uint8)
    return a


def _cpu_entry(gib, ts, sample):
    """cpu_baseline block of a server-placement entry: the 1-thread restated loop, median of
    the timed passes."""
    t = statistics.median(ts)
    return {"value": round(gib / t, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "label": "restated CPU baseline", "median_ms": round(t * 1e3, 3),
            "samples_ms": [round(x * 1e3, 3) for x in ts], "host": host_cpu(), "sample": sample}


def measure_drain_host(torch, dist, ec, world, rank, args):
    """SURVEY §8f rank 1, as the unchanged server would run it: the
    parity P1 drains 65,536 pending 4098-B diffs -- each in pageable host memory at its own
    shuffled slot, as malloc'd e->vbuf are -- into its host ecmem at shuffled 16-B aligned
    addresses, the arena registered once (cec_host_register).  One cec_drainer_apply per
    step (synchronous).  CPU beside it: the reference's loop, one region multiply per diff,
    one thread (memcached.c:4350 -> process_rep_command :7764), the restated GF-Complete
    kernel -- and its result is the check: after the timed steps the arena has taken the
    window an odd number of times, so it must equal one oracle application."""
    import numpy as np
    from oracle import pyoracle

    k, m, N, size = 3, 2, 65536, 4098
    stride = (size + 15) & ~15
    lid_self = k + 1
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0xC0C70007 + rank)
    arena = host_array(N * stride, 0xC0C70008 + rank)
    initial = arena.copy()
    diffs = host_array(N * stride, 0xC0C70009 + rank)
    dslot = rng.permutation(N).astype(np.uint64)
    addrs = rng.permutation(N).astype(np.uint64) * np.uint64(stride)
    src = rng.integers(0, k, N)
    base = diffs.ctypes.data
    upd = ec.host_updates([(base + int(dslot[i]) * stride, int(addrs[i]), int(src[i]), size) for i in range(N)])
    stream = torch.cuda.current_stream()
    alias = ec.host_register(arena)
    try:
        with ec.Drainer(k, m, mat, lid_self, staging_bytes=64 << 20) as d:
            warm = max(1, args.warmup)
            for _ in range(warm):
                d.apply(upd, alias, stream)
            if dist_on(dist):
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                launches = d.apply(upd, alias, stream)  # synchronous: applied on return
            el = time.perf_counter() - t0
            if dist_on(dist):
                dist.barrier()
            applied = warm + args.steps
            if applied % 2 == 0:  # (an odd count: the arena holds ONE application)
                d.apply(upd, alias, stream)
    finally:
        ec.host_unregister(arena)
    cpu = initial
    coefs = [mat[lid_self * k + int(j)] for j in src]
    lens = np.full(N, size, np.uint32)
    ts = [pyoracle.bench_apply(diffs, dslot * np.uint64(stride), addrs, lens, coefs, cpu) for _ in range(3)]
    ok = bool(np.array_equal(arena, cpu))  # 3 oracle passes: one application as well
    own = el
    el, bad = max_over_ranks([el, 0.0 if ok else 1.0], dist)
    gib = N * size / 2**30
    # PCIe per step: the diffs up, the arena's bytes read and written back (read-modify-write
    # of the registered host ecmem by the kernel)
    floor, raw = pcie_floor(torch, 2 * N * size, N * size)
    out = {"value": round(gib * world * args.steps / el, 2), "unit": "GiB/s of diffs",
           "ms_per_step": round(el * 1e3 / args.steps, 3), "us_per_diff": round(el * 1e6 / args.steps / N, 4),
           "pcie_bound_frac": round(floor / (own / args.steps), 4), "pcie_GBps_raw": raw,
           "pcie_bytes_per_step": {"h2d": 2 * N * size, "d2h": N * size},
           "workload": EXTRA_WORKLOADS["drain_host_ecmem"], "launches_per_apply": launches,
           "verified": ok and bad == 0.0,
           "rank": {"ms_per_step": round(own * 1e3 / args.steps, 3), "verified": ok}}
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_entry(gib, ts, "the reference's drain loop over the same 65,536 diffs "
                                                  "(pageable, same slots and addresses), one region multiply "
                                                  "per diff, 1 thread, median of 3 passes")
        out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
    return out


def measure_recovery_pool_host(torch, dist, ec, world, rank, args):
    """SURVEY §8f rank 2 in the pool placement: RS(3,2), this parity
    P1 leads the recovery of lost D1 (mask D0 + D2 + P1, start_recovery's), its ecmem in
    host memory registered once.  Two passes: one 1 MiB range (256 units) and the idle
    recoverer's 85 single-unit requests in flight (const.h:27).  Per pass: the requests
    begun and both data peers' replies received into the pool's staging (the recv, untimed
    as every path's recv into c->vbuf), then -- timed -- ONE cec_recovery_pool_add_peers
    and ONE cec_recovery_pool_flush_solve_host (fold + first-touch copy + leader solve in
    one launch), after which the rebuilt bytes are read in place.  Every rep recovers other
    units, 32 MiB further into a host arena, so the parity units are read cold.  CPU
    beside it: the reference's per-unit chain (malloc'd units, recovery.c:72-94, then the
    bottom half) on one thread over the same units and replies; its outputs check every
    rep's rebuilt bytes."""
    import numpy as np
    from oracle import pyoracle

    k, m, U, SELF, lost, peers = 3, 2, 4096, 4, 1, (0, 2)
    mat = ec.coding_matrix(k, m)
    mask = ec.recovery_mask(k, m, SELF, [int(i != lost) for i in range(k + m)])
    inv = ec.galois_single_divide(1, mat[SELF * k + lost])
    coefs = [mat[SELF * k + p] for p in peers]
    reps = max(3, min(args.steps, 15))
    walk = 8192  # units (32 MiB) between consecutive reps' ranges
    nunits = walk * (reps + 2)
    ecmem = host_array(nunits * U, 0xC0C7000A + rank)
    rng = np.random.default_rng(0xC0C7000B + rank)
    starts85 = (512 + rng.choice(walk - 512, 85, replace=False)).tolist()
    alias = ec.host_register(ecmem)
    shapes, ok = {}, True
    try:
        for name, units, starts in (("range_1MiB", 256, [100]), ("idle_85", 1, starts85)):
            nreq = len(starts)
            replies = [host_array(units * U, 0xC0C70100 + 7 * rank + x) for x in range(2 * nreq)]
            gpu_t, cpu_t, add_t = [], [], []
            with ec.RecoveryPool(k, m, mat, SELF, alias, capacity_units=nreq * units) as pool:
                for rep in range(reps + 1):  # rep 0: warm-up
                    first = [s + rep * walk for s in starts]
                    rids = [pool.begin(mask, u0, u0 + units - 1) for u0 in first]
                    ids, lids, stg = [], [], []
                    for q, rid in enumerate(rids):
                        for p, peer in enumerate(peers):
                            addr, view = pool.staging(rid, peer)
                            view[:] = replies[2 * q + p]  # the recv into c->ritem (untimed)
                            ids.append(rid)
                            lids.append(peer)
                            stg.append(addr)
                    arrs = ec.pool_replies(ids, lids, stg)
                    if dist_on(dist):
                        dist.barrier()
                    t0 = time.perf_counter()
                    pool.add_peers(arrs)
                    tm = time.perf_counter()
                    solved = pool.flush_solve_host()
                    t1 = time.perf_counter()
                    got = [pool.output(rid) for rid in rids]  # fill_completed_recovered_data
                    got = [None if g is None else g.copy() for g in got]  # (None: not solved)
                    for rid in rids:
                        pool.end(rid)
                    tc, exp = pyoracle.bench_recover_requests(ecmem, first, units, replies, 2, coefs, inv)
                    ok &= solved == nreq and all(g is not None and np.array_equal(g, e) for g, e in zip(got, exp))
                    if rep:
                        gpu_t.append(t1 - t0)
                        add_t.append(tm - t0)
                        cpu_t.append(tc)
            g_med, c_med = statistics.median(gpu_t), statistics.median(cpu_t)
            g_max = max_over_ranks([g_med], dist)[0]
            gib = 3 * nreq * units * U / 2**30  # two replies folded + the bytes rebuilt
            # PCIe per pass: the parity units and both replies read in place, the rebuilt bytes
            # written to the mapped output
            floor, _ = pcie_floor(torch, 3 * nreq * units * U, nreq * units * U)
            shapes[name] = {"requests": nreq, "units_per_request": units, "reps": reps,
                            "us": round(g_max * 1e6, 1), "value": round(gib * world / g_max, 3),
                            "unit": "GiB/s (replies folded + bytes rebuilt)",
                            "pcie_floor_us": round(floor * 1e6, 1), "pcie_bound_frac": round(floor / g_med, 4),
                            "add_peers_us": round(statistics.median(add_t) * 1e6, 1),  # the rest: the flush
                            "rank_us": round(g_med * 1e6, 1)}
            if world == 1 and not args.no_cpu_baseline:
                shapes[name]["cpu_baseline"] = _cpu_entry(
                    gib, cpu_t, f"the reference's chain for the same {nreq} request(s) x {units} unit(s): "
                                "per reply and unit malloc + parity copy + region multiply, then the bottom "
                                "half, 1 thread, cold parity units, median of the reps")
                shapes[name]["cpu_us"] = round(c_med * 1e6, 1)
                shapes[name]["gpu_over_cpu"] = round(c_med / g_max, 2)
    finally:
        ec.host_unregister(ecmem)
    ok, = [x == 0.0 for x in max_over_ranks([0.0 if ok else 1.0], dist)]
    out = {"value": shapes["range_1MiB"]["value"], "unit": shapes["range_1MiB"]["unit"] + ", 1 MiB range",
           "workload": EXTRA_WORKLOADS["recovery_pool_host"], "mask": mask, "shapes": shapes,
           "pcie_GBps_raw": {x: round(v, 1) for x, v in _PCIE.items()},
           "verified": bool(ok),
           "rank": {n: {"us": v["rank_us"]} for n, v in shapes.items()}}
    for v in shapes.values():
        v.pop("rank_us")
    return out


def measure_set_diffs_host(torch, dist, ec, world, rank, args):
    """The data side: the diffs of 65,536 SETs of 4098 B
    (complete_nread, memcached.c:2676-2681: diff = new ^ ecmem[addr]), values pageable at
    shuffled slots, old bytes at shuffled 16-B aligned addresses of a host ecmem registered
    once (read in place by the kernel), one cec_region_multiply_batch (a prepared job list)
    per step.  CPU beside it: memcpy + XOR per SET, 1 thread; its diffs check the batch's."""
    import numpy as np
    from oracle import pyoracle

    N, size = 65536, 4098
    stride = (size + 15) & ~15
    rng = np.random.default_rng(0xC0C7000C + rank)
    ecmem = host_array(N * stride, 0xC0C7000D + rank)
    values = host_array(N * stride, 0xC0C7000E + rank)
    diffs = host_array(N * stride)
    diffs[:] = 0
    vslot = rng.permutation(N).astype(np.uint64) * np.uint64(stride)
    addrs = rng.permutation(N).astype(np.uint64) * np.uint64(stride)
    doffs = np.arange(N, dtype=np.uint64) * np.uint64(stride)
    vb, db, eb = values.ctypes.data, diffs.ctypes.data, ecmem.ctypes.data
    jobs = ec.region_jobs([(vb + int(vslot[i]), db + int(doffs[i]), eb + int(addrs[i]), size, 1, 1)
                           for i in range(N)])
    ec.host_register(ecmem)
    try:
        for _ in range(max(1, args.warmup)):
            ec.region_multiply_batch(jobs)
        if dist_on(dist):
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            launches, rounds = ec.region_multiply_batch(jobs)  # synchronous
        el = time.perf_counter() - t0
        stats = ec.batch_stats()
        if dist_on(dist):
            dist.barrier()
    finally:
        ec.host_unregister(ecmem)
    cpu = host_array(N * stride)
    cpu[:] = 0
    lens = np.full(N, size, np.uint32)
    ts = [pyoracle.bench_set_diffs(values, vslot, ecmem, addrs, lens, cpu, doffs) for _ in range(3)]
    ok = bool(np.array_equal(diffs, cpu))
    own = el
    el, bad = max_over_ranks([el, 0.0 if ok else 1.0], dist)
    gib = N * size / 2**30
    # PCIe per step: the values up (staged) and the old bytes read in place; the diffs back
    floor, raw = pcie_floor(torch, 2 * N * size, N * size)
    out = {"value": round(gib * world * args.steps / el, 2), "unit": "GiB/s of values",
           "ms_per_step": round(el * 1e3 / args.steps, 3), "us_per_set": round(el * 1e6 / args.steps / N, 4),
           "pcie_bound_frac": round(floor / (own / args.steps), 4), "pcie_GBps_raw": raw,
           "pcie_bytes_per_step": {"h2d": 2 * N * size, "d2h": N * size},
           "workload": EXTRA_WORKLOADS["set_diffs_host"],
           "last_batch": {"launches": launches, "rounds": rounds, "in_place_launches": stats["in_place_launches"],
                          "plan_us": round(stats["plan_us"]), "pack_us": round(stats["pack_us"]),
                          "gpu_wait_us": round(stats["gpu_us"]), "unpack_us": round(stats["unpack_us"])},
           "verified": ok and bad == 0.0,
           "rank": {"ms_per_step": round(own * 1e3 / args.steps, 3), "verified": ok}}
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = _cpu_entry(gib, ts, "the reference's SET-diff code over the same 65,536 SETs "
                                                  "(memcpy, then XOR with the old bytes), 1 thread, median of 3")
        out["gpu_over_cpu"] = round(out["value"] / out["cpu_baseline"]["value"], 2)
    return out


SERVER_MEASURE = {"drain_host_ecmem": measure_drain_host, "recovery_pool_host": measure_recovery_pool_host,
                  "set_diffs_host": measure_set_diffs_host}


def run_device(args):
    torch, dist, ec, world, rank = setup(args.dist_backend)

    set_engine(ec, args.engine)
    r = measure_device(torch, dist, ec, world, rank, args.workload, args)
    strong = None
    if not args.no_strong:
        torch.cuda.empty_cache()
        strong = measure_strong(torch, dist, ec, world, rank, args, r)
    # The other device-resident BASELINE configs at the same N, on the same ranks, so the
    # 1/2/4/8-GPU scaling run also covers configs[3] (RS(4,2) 64 KiB, an 8-GPU config)
    # and the north star's 1 MiB values.  `value` stays the metric's workload.
    also = {}
    for w in [x for x in args.also.split(",") if x and x != args.workload]:
        torch.cuda.empty_cache()
        if w in ("rs32_diff_update", "rs32_diff_update_lds"):
            if w == "rs32_diff_update_lds":
                ec.set_engine(ec.CEC_ENGINE_LDS)
            try:
                also[w] = measure_diff_update(torch, dist, ec, world, rank, args)
            finally:
                set_engine(ec, args.engine)
            continue
        if w == "rs32_e2e":
            also[w] = measure_e2e(torch, dist, ec, world, rank, args)
            continue
        if w == "rs32_1m_recovery":
            also[w] = measure_recovery_decode(torch, dist, ec, world, rank, args)
            continue
        if w in SERVER_MEASURE:
            also[w] = SERVER_MEASURE[w](torch, dist, ec, world, rank, args)
            continue
        if w == "rs32_4k_lds":
            ec.set_engine(ec.CEC_ENGINE_LDS)
        try:
            o = measure_device(torch, dist, ec, world, rank, "rs32_4k" if w == "rs32_4k_lds" else w, args)
        finally:
            set_engine(ec, args.engine)
        also[w] = {
            "value": round(o["value"], 2), "unit": "GiB/s",
            "ms_per_step": round(o["ms_per_step"], 4),
            "workload": f"RS({o['k']},{o['m']}) encode + single-shard decode, "
                        f"{'%d B' % o['n'] if o['n'] else 'mixed 256 B-1 MiB'} values, "
                        f"{o['B']} stripes per GPU ({o['what']})",
            "engine": o["engine"],
            "encode_frac": o["roofline"]["frac"], "decode_frac": o["decode_roofline"]["frac"],
            "encode_ms": o["roofline"]["launch_ms"], "decode_ms": o["decode_roofline"]["launch_ms"],
            "verified": o["verified"], "rank": o["rank"],
        }
        if w == "rs32_4k_lds":
            also[w]["kernel"] = o["roofline"]["kernel"]
        elif world == 1 and not args.no_cpu_baseline:
            # BASELINE.md §2's other CPU-baseline configs, beside the GPU number: the same
            # restated path on every CPU this process may use, over the same value sizes
            # (the mixed batch itself; 256 MiB per shard of n-byte values otherwise)
            cb = cpu_baseline(o["k"], o["m"], o["n"] or 4096, CPU_OTHER_S, threads_list=[cpu_allowed()],
                              sizes=None if o["n"] else [ln for _, ln in layout(w)[0]])
            also[w]["cpu_baseline"] = {x: cb[x] for x in ("value", "unit", "cores", "kind", "label", "median",
                                                          "min", "max", "sample")}
            also[w]["gpu_over_cpu"] = round(o["value"] / cb["value"], 1)
    # per-rank evidence, outside every timed region: device identity and own times
    mine = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "identity": device_identity(torch, torch.cuda.current_device()),
            "weak": r["rank"], "strong": strong.pop("rank", None) if strong else None,
            "other_workloads": {w: v.pop("rank", None) or  # the recovery cases carry theirs per case
                                {n: c.pop("rank", None) for n, c in v.get("cases", {}).items()}
                                for w, v in also.items()}}
    ranks = ranks_summary(gather_ranks(dist, mine), dist.get_backend() if dist_on(dist) else "none")
    if rank == 0:
        k, m, n, B = r["k"], r["m"], r["n"], r["B"]
        res = {
            "metric": METRIC if args.workload == "rs32_4k" else f"GiB/s device-resident {args.workload}",
            "value": round(r["value"], 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_run": max(1, args.warmup),  # warmups actually run (at least one per measurement)
            "ms_per_step": round(r["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (uniform random bytes, torch.Generator seeded per rank)",
            "config": {
                "workload": f"RS({k},{m}) encode + single-shard decode, "
                            f"{'%d B' % n if n else 'mixed 256 B-1 MiB'} values, {B} stripes per GPU ({r['what']})",
                "k": k, "m": m, "value_bytes": n or "mixed", "stripes_per_gpu": B,
                "bytes_per_shard_per_gpu": r["bytes_total"],
                "parallelism": f"{world} x independent stripe batches, no collective",
                "engine": (args.engine if args.engine != "auto" else "auto") +
                          f" (ran: encode {r['engine']['encode'].upper()}, decode {r['engine']['decode'].upper()}, "
                          "as cec_last_engine reports; AUTO = LDS for decodes of values of 64 KiB and more, "
                          "PERM for every other op)",
            },
            "roofline": r["roofline"],
            "decode_roofline": r["decode_roofline"],
            "verified": r["verified"] and all(v["verified"] for v in also.values()),
            "ranks": ranks,
        }
        if strong is not None:
            res["strong"] = strong
            res["verified"] = res["verified"] and all(
                p["verified"] for p in strong.get("predicted", [strong]))
        if also:
            res["other_workloads"] = also
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(k, m, n or 4096, args.cpu_seconds)
        print(json.dumps(res), flush=True)


def run_e2e(args):
    """--e2e: the E2E pipeline alone, printed as its own JSON line (1 GPU)."""
    torch, dist, ec, world, rank = setup(args.dist_backend)
    e = E2E(torch, ec, args, zero_copy=args.e2e_zero_copy)
    for _ in range(max(1, args.warmup)):
        e.step()
    torch.cuda.synchronize()
    ok = e.verified()
    steps = max(1, min(args.steps, 10))
    t0 = time.perf_counter()
    for _ in range(steps):
        e.step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    h2d, d2h = pcie_raw(torch)  # raw copy rates for context
    floor_s = max(e.h2d_bytes / (h2d * 1e9), e.d2h_bytes / (d2h * 1e9))
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s end-to-end (pinned host -> HBM -> host) RS(3,2) encode+decode, 4 KiB values",
            "value": round(e.payload * steps / el / 2**30, 2), "unit": "GiB/s", "n_gpus": 1, "steps": steps,
            "ms_per_step": round(el * 1e3 / steps, 3), "verified": ok,
            "h2d_bytes_per_stripe": 2 * e.k * e.n, "d2h_bytes_per_stripe": (e.m + 1) * e.n,
            "pcie_h2d_GBps_raw": round(h2d, 1), "pcie_d2h_GBps_raw": round(d2h, 1),
            "pcie_bound_frac": round(floor_s / (el / steps), 4),
            "config": ({"path": "zero-copy: kernels read / write pinned host memory over PCIe",
                        "stripes": e.B} if args.e2e_zero_copy else
                       {"path": "staged: hipMemcpyAsync H2D -> kernel -> D2H",
                        "chunk_stripes": e.chunk, "streams": e.ns, "stripes": e.B}),
        }), flush=True)
    e.close()


def run_drain(args):
    """a parity process drains 65,536 pending 4 KiB diffs that sit
    in (pageable) host memory, as shipped by the data servers, into its parity arena
    in HBM.  GPU: one cec_drainer_apply (pack -> one H2D -> fold kernel).  CPU: the
    reference's loop (one galois_w08_region_multiply per diff, one thread:
    memcached.c:4350 -> 7764), restated GF-Complete kernel from the oracle."""
    import numpy as np

    torch, dist, ec, world, rank = setup(args.dist_backend)
    from oracle import pyoracle

    k, m, n, N = 3, 2, 4096, 65536
    mat = ec.coding_matrix(k, m)
    lid_self = k + 1
    rng = np.random.default_rng(0xC0C70001)
    diffs = rng.integers(0, 256, N * n, dtype=np.uint8)
    src = rng.integers(0, k, N)
    addrs = np.arange(N, dtype=np.uint64) * n
    arr = ec.host_updates([(diffs.ctypes.data + i * n, int(addrs[i]), int(src[i]), n) for i in range(N)])
    parity = torch.zeros(N * n, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()
    with ec.Drainer(k, m, mat, lid_self, staging_bytes=N * n) as d:
        for _ in range(max(1, args.warmup)):
            d.apply(arr, parity, stream)
        torch.cuda.synchronize()
        steps = max(1, args.steps)
        t0 = time.perf_counter()
        for _ in range(steps):
            d.apply(arr, parity, stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # the same diffs received straight into the drainer's pinned staging (recv into
        # e->vbuf carved from it): no pack copy; applied steps more times
        base, view = d.staging()
        view[:N * n] = diffs
        arr_ip = ec.host_updates([(base + i * n, int(addrs[i]), int(src[i]), n) for i in range(N)])
        d.apply(arr_ip, parity, stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            d.apply(arr_ip, parity, stream)
        torch.cuda.synchronize()
        el_ip = time.perf_counter() - t0
    # check: (warmup + steps) applications of the same diffs
    reps = max(1, args.warmup) + steps + 1 + steps  # XOR: odd count == applied once
    exp = np.zeros(N * n, np.uint8)
    coefs = [mat[lid_self * k + int(j)] for j in src]
    if reps % 2:
        pyoracle.bench_apply(diffs, addrs, addrs, np.full(N, n), coefs, exp)
    ok = np.array_equal(parity.cpu().numpy(), exp)
    cpu = np.zeros(N * n, np.uint8)
    t_cpu = pyoracle.bench_apply(diffs, addrs, addrs, np.full(N, n), coefs, cpu)
    gib = N * n / 2**30
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s parity drain: 65,536 pending 4 KiB diffs, host memory -> HBM parity arena",
            "value": round(gib * steps / el_ip, 2), "unit": "GiB/s", "n_gpus": 1, "steps": steps,
            "ms_per_step": round(el_ip * 1e3 / steps, 3), "verified": bool(ok),
            "includes": "diffs received into the drainer's pinned staging: one H2D + fold kernel + "
                        "synchronize",
            "pack_path": {"value": round(gib * steps / el, 2), "ms_per_step": round(el * 1e3 / steps, 3),
                          "includes": "diffs in pageable malloc'd buffers: threaded pack into pinned "
                                      "staging overlapped with H2D + fold"},
            "cpu_baseline": {"value": round(gib / t_cpu, 3), "unit": "GiB/s", "cores": 1, "kind": "port", "host": host_cpu(),
                             "sample": "the reference's drain loop (one region multiply per diff, "
                                       "one thread) over the same 65,536 diffs, restated GF-Complete AVX2"},
        }), flush=True)


def run_recovery(args):
    """the leader parity P0 recovers lost D0 over a 256 MiB range
    (65,536 units): survivors D1, D2 arrive as host bytes (recover_units_reply), the
    parity arena is in HBM, the rebuilt shard goes back to host memory.  GPU: one
    cec_recovery (add_peer, then finish = last peer + solve; the two-step chain
    add_peer x 2 + solve is timed beside it).  CPU: the reference's chain on one thread
    (per-unit residual, then the bottom half), restated GF-Complete kernel."""
    import numpy as np

    torch, dist, ec, world, rank = setup(args.dist_backend)
    from oracle import pyoracle

    k, m, U, nunits = 3, 2, 4096, 65536
    n = U * nunits
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70005)
    data = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, parity, n)
    torch.cuda.synchronize()
    host = [d.cpu().numpy() for d in data]
    mask = ec.recovery_mask(k, m, k, [0, 1, 1, 1, 1])  # D0 lost, leader P0
    out = np.zeros(n, np.uint8)
    steps = max(1, min(args.steps, 10))
    pin = [torch.from_numpy(h).pin_memory() for h in host[1:]]
    out_pin = torch.zeros(n, dtype=torch.uint8).pin_memory()

    def session(units, o, fused):
        t0 = time.perf_counter()  # session create / destroy (device residual) included
        with ec.Recovery(k, m, mat, k, mask, 0, nunits - 1, parity[0]) as rec:
            rec.add_peer(1, units[0])
            if fused:  # last peer + leader solve, pipelined (cec_recovery_finish)
                rec.finish(2, units[1], {}, {0: o})
            else:
                rec.add_peer(2, units[1])
                rec.solve({}, {0: o})
        return time.perf_counter() - t0

    variants = {}
    ok = True
    for name, units, o, fused in (("pageable", host[1:], out, True),
                                  ("pinned_finish", pin, out_pin, True),
                                  ("pinned_two_step", pin, out_pin, False)):
        session(units, o, fused)  # warm-up (allocations, first-use staging)
        o[:] = 0
        t = sum(session(units, o, fused) for _ in range(steps))
        got = o.numpy() if hasattr(o, "numpy") else o
        ok &= bool(np.array_equal(got, host[0]))
        variants[name] = {"value": round(n / 2**30 * steps / t, 2), "ms_per_step": round(t * 1e3 / steps, 3)}
    p0 = parity[0].cpu().numpy()
    t_cpu, cpu_out = pyoracle.bench_recover(p0, [host[1], host[2]], [mat[k * k + 1], mat[k * k + 2]],
                                            pyoracle.gf_div(1, mat[k * k + 0]))
    ok &= np.array_equal(cpu_out, host[0])
    gib = n / 2**30
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s online recovery of one lost data shard, 65,536 x 4 KiB units, host survivors -> host rebuilt",
            "value": variants["pageable"]["value"], "unit": "GiB/s", "n_gpus": 1, "steps": steps,
            "ms_per_step": variants["pageable"]["ms_per_step"], "verified": bool(ok),
            "variants": variants,
            "includes": "session create + destroy; survivors and the rebuilt shard in pageable host "
                        "memory: add_peer x 2 (pipelined pinned staging + fold) + solve + staged D2H. "
                        "pinned_finish: add_peer, then ONE pass for the last peer + solve, the kernel "
                        "reading and writing host memory over PCIe in both directions at once",
            "cpu_baseline": {"value": round(gib / t_cpu, 3), "unit": "GiB/s", "cores": 1, "kind": "port", "host": host_cpu(),
                             "sample": "the reference's recovery chain for the same range on one thread "
                                       "(recovery.c:72-94 per unit, memcached.c:7913-7922), restated GF-Complete AVX2"},
        }), flush=True)


def run_ops(args):
    """One JSON line: every op of SURVEY §8a on device-resident RS(3,2) arenas of
    65,536 x 4 KiB values (256 MiB per arena), its algorithmic HBM bytes per launch
     over its HIP-event launch time, against 8 TB/s.  Each op is first
    run once on fresh inputs and 32 sampled values are checked against the oracle."""
    import numpy as np

    torch, dist, ec, world, rank = setup(args.dist_backend)
    from oracle import pyoracle

    set_engine(ec, args.engine)
    k, m, n, B = 3, 2, 4096, 65536
    T = n * B
    mat = ec.coding_matrix(k, m)
    names = ["d0", "d1", "d2", "p0", "p1", "stage", "diff", "res", "o0", "o1", "o2"]
    ar = dict(zip(names, ec.arena_tensors(len(names), T)))
    g = torch.Generator(device="cuda").manual_seed(0xC0C70004)
    for x in names:
        ar[x].random_(0, 256, generator=g)
    data = [ar["d0"], ar["d1"], ar["d2"]]
    par = [ar["p0"], ar["p1"]]
    rng = np.random.default_rng(7)
    src_j = rng.integers(0, k, B)
    plain = ec.Plan([(s * n, s * n, n, 0) for s in range(B)])
    by_j = ec.Plan([(s * n, s * n, n, int(src_j[s])) for s in range(B)])
    lid = k  # P0: the recovery leader of a lost D0 (start_recovery, memcached.c:8136-8151)
    mask0 = ec.recovery_mask(k, m, lid, [0, 1, 1, 1, 1])
    mask1 = ec.recovery_mask(k, m, k + 1, [1, 0, 1, 1, 1])  # D1 lost, leader P1 (inverse != 1)
    sample = sorted(rng.choice(B, 32, replace=False).tolist())
    stream = torch.cuda.current_stream()

    def host(t, s):
        return t[s * n:(s + 1) * n].cpu().numpy()

    def snap(keys):
        return {x: [host(ar[x], s) for s in sample] for x in keys}

    res = {}

    def measure(name, row, nbytes, launch, check):
        before = snap(names)
        launch()
        torch.cuda.synchronize()
        after = snap(names)
        ok = all(check(before, after, i, s) for i, s in enumerate(sample))
        for _ in range(2):
            launch()
        evs = [(ec.Event(), ec.Event()) for _ in range(args.steps)]
        torch.cuda.synchronize()
        for a, b in evs:
            a.record(stream)
            launch()
            b.record(stream)
        torch.cuda.synchronize()
        ms = sum(a.elapsed_ms(b) for a, b in evs) / len(evs)
        gbps = nbytes / (ms * 1e-3) / 1e9
        res[name] = {"row": row, "algorithmic_bytes_per_launch": nbytes, "launch_ms": round(ms, 4),
                     "achieved_GBps": round(gbps, 1), "frac": round(gbps / HBM_PEAK_GBPS, 4),
                     "verified": bool(ok)}

    def eq(a, b):
        return bool(np.array_equal(a, b))

    def chk_rm(bf, af, i, s):
        exp = bf["p0"][i].copy()
        pyoracle.region_multiply(bf["d0"][i], 245, exp, 1)
        return eq(af["p0"][i], exp)

    measure("region_multiply", "a1 galois_w08_region_multiply(add=1), one 256 MiB region", 3 * T,
            lambda: ec.region_multiply(ar["d0"], 245, T, ar["p0"], 1, stream), chk_rm)

    def chk_sd(bf, af, i, s):
        return eq(af["diff"][i], pyoracle.set_diff(bf["d%d" % src_j[s]][i], bf["stage"][i]))

    measure("set_diff", "a2 diff = new ^ old (memcached.c:2664-2681)", 3 * T,
            lambda: ec.set_diff(k, data, ar["stage"], ar["diff"], by_j, stream), chk_sd)

    def chk_ap(bf, af, i, s):
        exp = bf["p1"][i].copy()
        pyoracle.parity_apply(mat, k, k + 1, int(src_j[s]), bf["diff"][i], exp)
        return eq(af["p1"][i], exp)

    measure("apply_diffs", "a3 parity ^= MATRIX(self, j) * diff (memcached.c:7739-7767)", 3 * T,
            lambda: ec.apply_diffs(k, m, mat, k + 1, ar["diff"], ar["p1"], by_j, stream), chk_ap)

    def chk_du(bf, af, i, s):
        j = int(src_j[s])
        pv = [bf["p0"][i].copy(), bf["p1"][i].copy()]
        pyoracle.diff_update(mat, k, m, j, bf["d%d" % j][i].copy(), bf["stage"][i], pv, True)
        return eq(af["p0"][i], pv[0]) and eq(af["p1"][i], pv[1]) and eq(af["d%d" % j][i], bf["stage"][i])

    measure("diff_update", "a4 fused per-SET diff-update + install (a2 + M x a3, memcached.c:5666)",
            (2 + 2 * m + 1) * T,
            lambda: ec.diff_update(k, m, mat, data, ar["stage"], par, True, by_j, stream), chk_du)

    def chk_en(bf, af, i, s):
        ps = pyoracle.encode(mat, k, m, [bf["d0"][i], bf["d1"][i], bf["d2"][i]])
        return eq(af["p0"][i], ps[0]) and eq(af["p1"][i], ps[1])

    measure("encode", "a5 full-stripe encode", (k + m) * T,
            lambda: ec.encode(k, m, mat, data, par, plain, stream), chk_en)

    arenas = data + par

    def chk_rs(bf, af, i, s):
        exp = bf["p0"][i].copy()
        for j in (1, 2):
            pyoracle.region_multiply(bf["d%d" % j][i], mat[lid * k + j], exp, 1)
        return eq(af["res"][i], exp)

    measure("residual", "a6 residual R = P ^ sum c*D (recovery.c:61-96)", (k + 1) * T,
            lambda: ec.residual(k, m, mat, lid, mask0, arenas, ar["res"], plain, stream), chk_rs)

    res_arenas = [None] * (k + m)
    res_arenas[k + 1] = ar["res"]
    outs = [ar["o0"], ar["o1"], ar["o2"]]

    def chk_sv(bf, af, i, s):
        exp = np.zeros(n, np.uint8)
        pyoracle.region_multiply(bf["res"][i], pyoracle.gf_div(1, mat[(k + 1) * k + 1]), exp, 1)
        return eq(af["o1"][i], exp)

    measure("solve", "a7 leader solve D = inv * R, inverse 1/245 (memcached.c:7842-7922)", 2 * T,
            lambda: ec.solve(k, m, mat, mask1, [ar["res"] if x == k + 1 else ar["res"] for x in range(k + m)],
                             outs, plain, stream), chk_sv)

    def chk_dc(bf, af, i, s):
        return eq(af["o1"][i], bf["d1"][i])

    ec.encode(k, m, mat, data, par, plain, stream)  # consistent stripes for the decode
    measure("decode", "a6 + a7 fused: rebuild D1 from D0, D2, P1 (leader P1)", (k + 1) * T,
            lambda: ec.decode(k, m, mat, [mask1], arenas, outs, plain, stream), chk_dc)
    if rank == 0:
        print(json.dumps({
            "metric": "device-resident roofline per SURVEY §8a op, RS(3,2), 65,536 x 4 KiB values",
            "unit": "GB/s", "n_gpus": 1, "steps": args.steps, "engine": args.engine,
            "peak_GBps": HBM_PEAK_GBPS, "ops": res,
            "verified": all(v["verified"] for v in res.values()),
        }), flush=True)
    for pl in (plain, by_j):
        pl.destroy()


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` (N > 1) started without a torch.distributed.run parent: start
    the N rank processes, one per GPU, and relay their output.  This process touches no
    GPU (nothing here initialises HIP) and does not exec: the ranks are children, and
    it exits with their launcher's code.  Rank 0 prints the JSON line."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts
    # stdout carries only the JSON line(s); the launcher's and the process groups' chatter
    # (gloo prints connection notes on stdout) goes to stderr, line by line as it comes.
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in p.stdout:
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return p.wait()


def run_harness_check(args):
    """--harness-check: the multi-rank harness without a GPU (gloo): each rank takes its
    contiguous shard of the metric's 65,536 stripes, barriers, times a CPU stand-in step
    and reports max-over-ranks exactly as the device path does.  For the CPU tests."""
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1 or os.environ.get("CEC_BENCH_PG") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group("gloo")
    lo, hi = shard_range(WORKLOADS["rs32_4k"][3] * world, rank, world)
    if dist_on(dist):
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (rank + 1))  # ranks finish at different times: the max must win
    elapsed = time.perf_counter() - t0
    if dist_on(dist):
        dist.barrier()
    mine = [float(elapsed), float(0.01 * (rank + 1)), float(rank)]
    got = max_over_ranks(mine, dist)
    spans = [None] * world
    if dist_on(dist):
        dist.all_gather_object(spans, (rank, lo, hi))
    else:
        spans = [(0, lo, hi)]
    # the per-rank evidence block of the device line, with a CPU stand-in for the device
    # identity: the process, or one shared "device" when CEC_BENCH_DEVICE pins every rank
    # to one (as it pins every GPU rank to one card)
    shared = os.environ.get("CEC_BENCH_DEVICE")
    ident = {"device": shared or f"cpu-process-{os.getpid()}", "name": "cpu stand-in", "arch": None,
             "pci": None, "uuid": f"cpu-{shared}" if shared else f"cpu-{os.getpid()}"}
    mine = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "identity": ident,
            "weak": {"ms_per_step": round(elapsed * 1e3, 4), "stripes": [lo, hi]}, "strong": None}
    ranks = ranks_summary(gather_ranks(dist, mine), dist.get_backend() if dist_on(dist) else "none")
    if rank == 0:
        print(json.dumps({"harness_check": True, "n_gpus": world, "gpus_arg": args.gpus,
                          "elapsed_max": got[0], "slowest_sleep": got[1], "max_rank": got[2],
                          "shards": spans, "local_rank_env": os.environ.get("LOCAL_RANK"),
                          "backend": "gloo", "ranks": ranks}), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    if args.gpus > 1 and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    if os.environ.get("CEC_BENCH_WATCHDOG"):  # diagnosis: every thread's stack after N s
        import faulthandler

        faulthandler.dump_traceback_later(float(os.environ["CEC_BENCH_WATCHDOG"]), repeat=True)
    if args.harness_check:
        run_harness_check(args)
    elif args.e2e:
        run_e2e(args)
    elif args.drain:
        run_drain(args)
    elif args.recovery:
        run_recovery(args)
    elif args.ops:
        run_ops(args)
    else:
        run_device(args)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
