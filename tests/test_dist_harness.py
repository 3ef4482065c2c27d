"""The multi-rank bench harness on CPU (gloo, world size 2): contiguous sharding of a
fixed batch, max-over-ranks timing, and the workload layouts."""
from __future__ import annotations

import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    lo, hi = bench.shard_range(65536, rank, world)
    # each rank's "elapsed" differs; the harness must report the slowest
    got = bench.max_over_ranks([0.5 + rank, 0.0 if rank else 1.0], dist)
    dist.barrier()
    q.put((rank, lo, hi, got))
    dist.destroy_process_group()


def test_gloo_world2_max_and_shards():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 32768), (32768, 65536)]
    for r in res:
        assert r[3] == [1.5, 1.0]  # max elapsed over ranks, any rank's failure flag


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_range_partitions(world):
    import bench

    total = 65537
    spans = [bench.shard_range(total, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for a, b in zip(spans, spans[1:]):
        assert a[1] == b[0]
    sizes = [hi - lo for lo, hi in spans]
    assert max(sizes) - min(sizes) <= 1


def test_layouts():
    import bench

    s, arena = bench.layout("rs32_4k")
    assert len(s) == 65536 and arena == 65536 * 4096 and s[1] == (4096, 4096)
    s, arena = bench.layout("rs32_mixed")
    assert sum(ln for _, ln in s) >= 1 << 30
    assert all(o % 16 == 0 for o, _ in s)  # ecalloc.c:176
    assert all(256 <= ln <= 1 << 20 for _, ln in s)
    assert all(a[0] + a[1] <= b[0] for a, b in zip(s, s[1:]))  # no overlap
    assert bench.layout("rs32_mixed") == (s, arena)  # seeded


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(args, env_extra=None, timeout=300):
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_self_launches_ranks(world):
    """`python bench.py --gpus N` with no torch.distributed.run parent (how the driver runs
    it) starts N ranks itself and prints exactly ONE JSON line on stdout (rank 0's), with
    n_gpus = N, contiguous shards and the max over ranks (gloo, no GPU)."""
    import json

    r = _run_bench(["--gpus", str(world), "--harness-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["gpus_arg"] == world
    per = 65536
    assert sorted(tuple(s) for s in out["shards"]) == [(q, q * per, (q + 1) * per) for q in range(world)]
    assert out["max_rank"] == world - 1  # the slowest rank's numbers are the ones reported
    assert out["slowest_sleep"] == pytest.approx(0.01 * world)
    assert out["elapsed_max"] >= 0.01 * world
    # the per-rank evidence block the device line carries (the N > 1 line shows
    # on its own which devices ran and which rank straggled)
    rk = out["ranks"]
    assert rk["world_size"] == world and rk["backend"] == "gloo"
    assert rk["distinct_devices"] is True
    assert [e["rank"] for e in rk["per_rank"]] == list(range(world))
    assert rk["slowest_rank_weak"] == world - 1
    assert [e["weak"]["stripes"] for e in rk["per_rank"]] == [[q * per, (q + 1) * per] for q in range(world)]
    assert max(e["weak"]["ms_per_step"] for e in rk["per_rank"]) == pytest.approx(out["elapsed_max"] * 1e3, rel=1e-3)


def test_bench_ranks_on_one_device_are_not_distinct():
    """CEC_BENCH_DEVICE pins every rank to one device (the one-card rehearsal): the line
    says so (distinct_devices false) instead of passing for an N-GPU run."""
    import json

    r = _run_bench(["--gpus", "2", "--harness-check"], env_extra={"CEC_BENCH_DEVICE": "0"})
    assert r.returncode == 0, r.stderr[-3000:]
    rk = json.loads(r.stdout.strip().splitlines()[-1])["ranks"]
    assert rk["world_size"] == 2 and rk["distinct_devices"] is False


def test_ranks_summary():
    import bench

    def e(rank, uuid, pci, weak, strong=None):
        return {"rank": rank, "identity": {"uuid": uuid, "pci": pci}, "weak": {"ms_per_step": weak},
                "strong": None if strong is None else {"ms_per_step": strong}}

    s = bench.ranks_summary([e(0, "u0", "0000:05:00", 1.0, 0.2), e(1, "u1", "0000:15:00", 1.2, 0.1)], "nccl")
    assert s["distinct_devices"] and s["slowest_rank_weak"] == 1 and s["slowest_rank_strong"] == 0
    s = bench.ranks_summary([e(0, "u0", "0000:05:00", 1.0), e(1, "u0", "0000:05:00", 0.5)], "gloo")
    assert not s["distinct_devices"] and s["slowest_rank_weak"] == 0 and "slowest_rank_strong" not in s
    assert bench.ranks_summary([e(0, "u0", "p", 1.0)], "none")["distinct_devices"]


def test_bench_single_rank_runs_in_process():
    import json

    r = _run_bench(["--harness-check"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n_gpus"] == 1 and out["shards"] == [[0, 0, 65536]]


def test_bench_process_group_at_world_one():
    """CEC_BENCH_PG=1: the process group comes up at world size 1 too, so the line's
    collectives (barrier, all_reduce MAX, all_gather of the per-rank evidence) run as
    real collectives on a one-device box (the GPU twin runs a one-rank RCCL group)."""
    import json

    r = _run_bench(["--harness-check"], env_extra={"CEC_BENCH_PG": "1"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ranks"]["backend"] == "gloo" and out["ranks"]["world_size"] == 1
    assert out["shards"] == [[0, 0, 65536]]


def test_bench_world_size_mismatch_refused():
    r = _run_bench(["--gpus", "2", "--harness-check"],
                   env_extra={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_bench_backend_auto():
    import bench

    old = os.environ.pop("CEC_BENCH_DEVICE", None)
    try:
        assert bench.parse([]).dist_backend == "nccl"
        os.environ["CEC_BENCH_DEVICE"] = "0"  # every rank on one card: RCCL refuses, gloo
        assert bench.parse([]).dist_backend == "gloo"
        assert bench.parse(["--dist-backend", "nccl"]).dist_backend == "nccl"
    finally:
        os.environ.pop("CEC_BENCH_DEVICE", None)
        if old is not None:
            os.environ["CEC_BENCH_DEVICE"] = old


def test_cpu_thread_sweep():
    import bench

    assert bench.cpu_thread_counts(256) == [1, 16, 64, 256]
    assert bench.cpu_thread_counts(8) == [1, 8]
    assert bench.cpu_thread_counts(1) == [1]
    assert bench.cpu_thread_counts(64) == [1, 16, 64]


def test_cpu_baseline_small():
    """The CPU-baseline leg (oracle, AVX2 restatement) on a short sweep: both the
    1-thread reference configuration and the all-thread ceiling, cores stated."""
    import bench

    cb = bench.cpu_baseline(3, 2, 4096, 0.4, threads_list=[1, 2])
    assert cb["cores"] == 2 and cb["kind"] == "port" and cb["value"] > 0
    assert cb["label"] == "restated CPU baseline"
    assert cb["reference_config"]["threads"] == 1 and cb["reference_config"]["value"] > 0
    assert [p["threads"] for p in cb["sweep"]] == [1, 2]
    for p in cb["sweep"]:  # median of >= 5 timed passes after a warm-up, at both points
        assert len(p["samples"]) == bench.CPU_SAMPLES >= 5
        assert p["min"] <= p["median"] <= p["max"] and p["value"] == p["median"]
    assert cb["value"] == cb["median"] == cb["sweep"][-1]["median"]


def test_cpu_baseline_mixed_sizes():
    """The CPU-baseline leg over a mixed batch's own value sizes (BASELINE.md §2 config
    (2)): the same restated path, payload = (K+1) x the batch's bytes, threads split by
    bytes; a uniform batch through the sizes form matches the uniform form's work."""
    import bench
    from oracle import pyoracle

    sizes = [ln for _, ln in bench.layout("rs32_mixed")[0]][:400]
    cb = bench.cpu_baseline(3, 2, 4096, 0.3, threads_list=[2], sizes=sizes)
    assert cb["value"] > 0 and cb["cores"] == 2 and "mixed" in cb["sample"]
    assert len(cb["samples"]) == bench.CPU_SAMPLES
    # every thread count, including more threads than stripes, runs and times the batch
    for T in (1, 3, 500):
        assert all(t > 0 for t in pyoracle.bench_encode_decode_sizes(3, 2, sizes[:7], T, 1, 2))


def test_cpu_baseline_split_under_asan(tmp_path):
    """The oracle's CPU-baseline workers (oracle/gf8_cpu_baseline.c) split stripes over
    threads by count or by bytes; under AddressSanitizer + UBSan, with more threads than
    stripes and mixed sizes, no access leaves the batch."""
    import subprocess

    exe = tmp_path / "bench_sizes"
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-std=gnu11", "-mavx2", "-o", str(exe),
                    os.path.join(ROOT, "tests", "oracle_c", "bench_sizes_main.c"),
                    os.path.join(ROOT, "oracle", "gf8_ref.c"), os.path.join(ROOT, "oracle", "gf8_cpu_baseline.c"),
                    "-lpthread"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stderr[-2000:]


def test_shard_stripes_by_count_and_by_bytes():
    """contiguous split by stripe count for one value size, by byte count for
    mixed sizes; the shares tile the batch exactly."""
    import bench

    s, _ = bench.layout("rs32_4k")
    assert [bench.shard_stripes(s, r, 8) for r in range(8)] == [bench.shard_range(65536, r, 8) for r in range(8)]
    s, _ = bench.layout("rs32_mixed")
    total = sum(ln for _, ln in s)
    for world in (2, 4, 8):
        spans = [bench.shard_stripes(s, r, world) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == len(s)
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        for lo, hi in spans:  # each share within one 1 MiB value of total / world
            got = sum(ln for _, ln in s[lo:hi])
            assert abs(got - total / world) <= (1 << 20), (world, got, total / world)


def test_share_layout_rebases_a_contiguous_split():
    """Each GPU's arenas hold only its share of the fixed batch."""
    import bench

    s, _ = bench.layout("rs32_4k")
    for world in (2, 4, 8):
        tot = 0
        for r in range(world):
            lo, hi = bench.shard_range(len(s), r, world)
            sub, arena = bench.share_layout(s, lo, hi)
            assert sub[0][0] == 0 and arena == (hi - lo) * 4096
            assert sub[1] == (4096, 4096)
            tot += sum(ln for _, ln in sub)
        assert tot == 65536 * 4096
    s, _ = bench.layout("rs32_mixed")
    sub, arena = bench.share_layout(s, 10, 20)
    assert sub[0][0] == 0 and arena % 16 == 0 and arena >= sub[-1][0] + sub[-1][1]
    assert [ln for _, ln in sub] == [ln for _, ln in s[10:20]]


def test_bench_arguments():
    """The driver's contract: no flags = N=1, the metric's workload, steps/warmup that
    finish in minutes; the other device-resident configs and the server placements (host
    ecmem) ride along (--also)."""
    import bench

    a = bench.parse([])
    assert (a.gpus, a.workload, a.engine) == (1, "rs32_4k", "auto")
    assert 1 <= a.steps <= 100 and a.warmup >= 1
    assert set(a.also.split(",")) == {"rs32_4k_lds", "rs32_mixed", "rs32_1m", "rs42_64k",
                                      "rs32_1m_recovery", "rs32_diff_update", "rs32_diff_update_lds",
                                      "rs32_e2e", "drain_host_ecmem", "recovery_pool_host", "set_diffs_host"}
    assert not a.no_strong
    assert bench.parse(["--also="]).also == ""
    with pytest.raises(SystemExit):
        bench.parse(["--also=rs99"])
    a = bench.parse(["--gpus", "8", "--steps", "7", "--warmup", "2"])
    assert (a.gpus, a.steps, a.warmup) == (8, 7, 2)
    h = bench.host_cpu()
    assert h["nproc"] >= 1 and isinstance(h["model"], str)
