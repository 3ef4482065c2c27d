"""GPU: the runtime around the kernels -- completion tracking, caches, capture.

* destroy of a plan / drainer / recovery session / recovery pool waits for that
  object's own work only, never for unrelated work on another stream;
* cec_recovery_solve / _finish are synchronous (cocytus_ec.h): a pinned output is
  complete when the call returns, with no device synchronisation by the caller;
* the coefficient-table cache is bounded (LRU) and the idle recoverer's pool does not
  mint new cache keys per flush: device memory stays flat over 10^5 random flushes;
* a graph capture works on a cold cache (tables never seen before), no warm-up call.
"""
from __future__ import annotations

import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def busy(gpu):
    """launch(): queue ~0.5 s of unrelated GPU work on a fresh stream; returns its event."""
    torch, _ = gpu
    t0 = time.perf_counter()
    torch.cuda._sleep(10_000_000)
    torch.cuda.synchronize()
    per_cycle = (time.perf_counter() - t0) / 10_000_000
    cycles = int(min(max(0.5 / max(per_cycle, 1e-12), 1e6), 5e10))

    def launch():
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.cuda._sleep(cycles)
        ev = torch.cuda.Event()
        ev.record(s)
        return ev

    return launch


def _rs32(torch, ec, B=256, n=4096):
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(11)
    data = [torch.randint(0, 256, (B * n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    return k, m, mat, data, parity


def test_plan_destroy_ignores_other_streams(gpu, busy):
    torch, ec = gpu
    k, m, mat, data, parity = _rs32(torch, ec)
    s = torch.cuda.Stream()
    plan = ec.Plan([(i * 4096, 0, 4096, 0) for i in range(256)], stream=s)
    ec.encode(k, m, mat, data, parity, plan, s)
    s.synchronize()  # the plan's own work is complete
    other = busy()
    t0 = time.perf_counter()
    plan.destroy()
    dt = time.perf_counter() - t0
    still_busy = not other.query()
    torch.cuda.synchronize()
    assert still_busy, f"plan destroy waited for another stream's work ({dt * 1e3:.1f} ms)"


def test_plan_destroy_waits_for_own_launch(gpu, busy):
    """The plan's tiles stay valid until its last launch completed, on any stream."""
    torch, ec = gpu
    k, m, mat, data, parity = _rs32(torch, ec)
    s = torch.cuda.Stream()
    ev = busy()
    s.wait_event(ev)  # the plan's launch is queued behind 0.5 s of work
    plan = ec.Plan([(i * 4096, 0, 4096, 0) for i in range(256)], stream=s)
    ec.encode(k, m, mat, data, parity, plan, s)
    plan.destroy()
    assert ev.query(), "destroy returned before the plan's own launch ran"
    torch.cuda.synchronize()
    from oracle import pyoracle

    host = [d[:4096].cpu().numpy() for d in data]
    exp = pyoracle.encode(mat, k, m, host)
    assert all(np.array_equal(parity[p][:4096].cpu().numpy(), exp[p]) for p in range(m))


def test_drainer_destroy_ignores_other_streams(gpu, busy):
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    parity = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    diffs = [np.full(4096, i + 1, np.uint8) for i in range(8)]
    d = ec.Drainer(k, m, mat, k, staging_bytes=1 << 20)
    d.apply([(diffs[i], i * 4096, i % k) for i in range(8)], parity)
    other = busy()
    d.destroy()
    still_busy = not other.query()
    torch.cuda.synchronize()
    assert still_busy, "drainer destroy waited for another stream's work"


def test_recovery_and_pool_destroy_ignore_other_streams(gpu, busy):
    torch, ec = gpu
    k, m, mat, data, parity = _rs32(torch, ec, B=16)
    ec.encode_region(k, m, mat, data, parity, 16 * 4096)
    torch.cuda.synchronize()
    mask = ec.recovery_mask(k, m, k, [0, 1, 1, 1, 1])
    r = ec.Recovery(k, m, mat, k, mask, 0, 15, parity[0])
    r.add_peer(1, data[1])
    pool = ec.RecoveryPool(k, m, mat, k, parity[0], capacity_units=64)
    rid = pool.begin(mask, 3, 3)
    pool.add_peer(rid, 1, data[1][3 * 4096:4 * 4096].cpu().numpy())
    pool.flush()
    other = busy()
    r.destroy()
    pool.destroy()
    still_busy = not other.query()
    torch.cuda.synchronize()
    assert still_busy, "session / pool destroy waited for another stream's work"


@pytest.mark.parametrize("fused", [True, False])
def test_recovery_solve_is_synchronous_on_pinned_output(gpu, oracle, fused):
    """with device survivors and a pinned output, the rebuilt bytes
    must be in the output when finish / solve return -- read with no device sync."""
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    n_units = 4096  # 16 MiB: long enough that an async return would be caught
    n = n_units * 4096
    g = torch.Generator(device="cuda").manual_seed(5)
    data = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, parity, n)
    want = data[0].cpu().numpy()
    mask = ec.recovery_mask(k, m, k, [0, 1, 1, 1, 1])  # D0 lost, leader P0
    s = torch.cuda.Stream()
    for attempt in range(3):
        out = torch.zeros(n, dtype=torch.uint8).pin_memory()
        torch.cuda.synchronize()
        with ec.Recovery(k, m, mat, k, mask, 0, n_units - 1, parity[0]) as rec:
            rec.add_peer(1, data[1], stream=s)
            if fused:
                rec.finish(2, data[2], {}, {0: out}, stream=s)
            else:
                rec.add_peer(2, data[2], stream=s)
                rec.solve({}, {0: out}, stream=s)
            got = out.numpy().copy()  # no synchronize: the call is synchronous
        assert np.array_equal(got, want), f"attempt {attempt}: output incomplete on return"


def test_pattern_cache_lru_bound(gpu, oracle):
    """More distinct coefficient sets than the limit: entries stay at the limit, evicted
    tables are re-uploaded on reuse, and every result stays bit-exact."""
    torch, ec = gpu
    n = 8192
    src = oracle.splitmix_bytes(3, n)
    ds = torch.from_numpy(src).cuda()
    ec.cache_set_pattern_limit(16)
    try:
        before = ec.cache_info()
        for rep in range(2):
            for c in range(2, 66):  # 64 distinct sets, 4x the limit
                dd = torch.zeros(n, dtype=torch.uint8, device="cuda")
                ec.region_multiply(ds, c, n, dd, 1)
                torch.cuda.synchronize()
                exp = np.zeros(n, np.uint8)
                oracle.region_multiply(src, c, exp, 1)
                assert np.array_equal(dd.cpu().numpy(), exp), (rep, c)
                assert ec.cache_info()["pattern_entries"] <= 16
        after = ec.cache_info()
        assert after["pattern_evictions"] - before["pattern_evictions"] >= 100
    finally:
        ec.cache_set_pattern_limit(4096)


@pytest.mark.parametrize("k,m,n_flushes", [(3, 2, 100_000), (6, 3, 20_000)])
def test_pool_flushes_keep_memory_flat(gpu, oracle, k, m, n_flushes):
    """Randomized idle-recoverer flushes (random peer order, partial replies, leader
    solve or not; 10^5 at RS(3,2), 2 x 10^4 at RS(6,3), whose 896 possible flush
    patterns used to mint one coefficient-cache key per table version): the flushes use
    the pool's own append-only table, so the coefficient-table cache gains no entry and
    evicts nothing, and device memory in use does not grow."""
    torch, ec = gpu
    mat = ec.coding_matrix(k, m)
    units = 512
    n = units * 4096
    g = torch.Generator(device="cuda").manual_seed(9)
    data = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, parity, n)
    hostd = [d.cpu().numpy() for d in data]
    out = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    rng = np.random.default_rng(1)
    masks = {j: ec.recovery_mask(k, m, k, [int(i != j) for i in range(k + m)]) for j in range(k)}
    pool = ec.RecoveryPool(k, m, mat, k, parity[0], capacity_units=128)
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    info0 = ec.cache_info()
    flushes = 0
    checked = 0
    while flushes < n_flushes:
        live = []
        for _ in range(int(rng.integers(1, 6))):
            lost = int(rng.integers(0, k))
            u = int(rng.integers(0, units))
            rid = pool.begin(masks[lost], u, u)
            peers = [j for j in range(k) if j != lost]
            rng.shuffle(peers)
            live.append((rid, lost, u, peers, int(rng.integers(1, k))))
        # replies arrive in random order, some requests get only one of two this flush
        for rid, lost, u, peers, first in live:
            for j in peers[:first]:
                pool.add_peer(rid, j, hostd[j][u * 4096:(u + 1) * 4096])
        if rng.integers(0, 2):
            pool.flush_solve(out)
        else:
            pool.flush()
        flushes += 1
        for rid, lost, u, peers, first in live:
            for j in peers[first:]:
                pool.add_peer(rid, j, hostd[j][u * 4096:(u + 1) * 4096])
        solved = pool.flush_solve(out)
        flushes += 1
        del solved
        if flushes % (n_flushes // 5) < 2:  # spot-check the rebuilt units against the originals
            torch.cuda.synchronize()
            for rid, lost, u, peers, first in live:
                got = out[lost][u * 4096:(u + 1) * 4096].cpu().numpy()
                assert np.array_equal(got, hostd[lost][u * 4096:(u + 1) * 4096]), (flushes, lost, u)
                checked += 1
        for rid, *_ in live:
            pool.end(rid)
    torch.cuda.synchronize()
    info1 = ec.cache_info()
    free1 = torch.cuda.mem_get_info()[0]
    pool.destroy()
    assert checked > 0
    # the flushes' patterns live in the pool, not in the LRU cache
    assert info1["pattern_entries"] == info0["pattern_entries"], (info0, info1)
    assert info1["pattern_evictions"] == info0["pattern_evictions"], (info0, info1)
    assert free0 - free1 < (64 << 20), f"device memory grew by {(free0 - free1) >> 20} MiB"


def test_plan_used_on_many_streams(gpu, oracle):
    """One plan used on 100 streams (one per connection, say): its destroy waits on every
    one of them and touches no stream handle before that (the tracker no
    longer queries noted streams past 64); every stream's result is bit-exact."""
    torch, ec = gpu
    k, m, mat, data, parity = _rs32(torch, ec, B=64)
    plan = ec.Plan([(i * 4096, 0, 4096, 0) for i in range(64)])
    streams = [torch.cuda.Stream() for _ in range(100)]
    torch.cuda.synchronize()
    outs = []
    for s in streams:
        par = [torch.zeros(64 * 4096, dtype=torch.uint8, device="cuda") for _ in range(m)]
        torch.cuda.current_stream().synchronize()
        ec.encode(k, m, mat, data, par, plan, s)
        outs.append(par)
    plan.destroy()  # waits for all 100 streams' launches
    host = [d.cpu().numpy() for d in data]
    exp = oracle.encode(mat, k, m, host)
    for i, par in enumerate(outs):
        assert all(np.array_equal(par[p].cpu().numpy(), exp[p]) for p in range(m)), i
    del streams
    torch.cuda.synchronize()


def test_graph_capture_cold_cache(gpu, oracle):
    """Capture an RS(5,3) encode + double-erasure decode whose coefficient tables were
    never used before (cold cache, no warm-up call), replay, compare with the oracle;
    then trim the caches: the captured tables survive, and the graph still replays."""
    torch, ec = gpu
    k, m, n, B = 5, 3, 4096, 64
    mat = ec.coding_matrix(k, m)
    host = [oracle.splitmix_bytes(0xC0C70010 + j, B * n) for j in range(k)]
    data = [torch.from_numpy(h).cuda() for h in host]
    parity = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    mask = sum(1 << x for x in (1, 2, 4, 5, 6))  # D0, D3 lost; parities P5, P6 (lids 5, 6)
    ep = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
    dp = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream()
        ec.encode(k, m, mat, data, parity, ep, s)
        ec.decode(k, m, mat, [mask], data + parity, out, dp, s)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, host)
    for p in range(m):
        assert np.array_equal(parity[p].cpu().numpy(), exp[p])
    assert torch.equal(out[0], data[0]) and torch.equal(out[3], data[3])
    ec.cache_trim()  # captured tables are kept: the graph still holds their address
    for t in parity + out:
        t.zero_()
    g.replay()
    torch.cuda.synchronize()
    for p in range(m):
        assert np.array_equal(parity[p].cpu().numpy(), exp[p])
    assert torch.equal(out[0], data[0]) and torch.equal(out[3], data[3])
    ep.destroy()
    dp.destroy()


def test_graph_capture_on_the_warm_stream(gpu, oracle):
    """The tables were first uploaded on stream s (their upload event recorded there) and
    the capture then runs on that same stream: no event call may touch it while it
    captures.  Replays are bit-exact; direct launches afterwards still work."""
    torch, ec = gpu
    k, m, n, B = 4, 3, 4096, 32  # a code no other test uses: a fresh upload on s
    mat = ec.coding_matrix(k, m)
    host = [oracle.splitmix_bytes(0xC0C70020 + j, B * n) for j in range(k)]
    data = [torch.from_numpy(h).cuda() for h in host]
    parity = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    side = torch.cuda.Stream()
    plan = ec.Plan([(i * n, 0, n, 0) for i in range(B)], stream=side)
    ec.encode(k, m, mat, data, parity, plan, side)  # upload queued on `side`, not waited for
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        ec.encode(k, m, mat, data, parity, plan, side)
    for t in parity:
        t.zero_()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, host)
    for p in range(m):
        assert np.array_equal(parity[p].cpu().numpy(), exp[p])
    for t in parity:
        t.zero_()
    ec.encode(k, m, mat, data, parity, plan, side)
    side.synchronize()
    for p in range(m):
        assert np.array_equal(parity[p].cpu().numpy(), exp[p])
    plan.destroy()


def test_caches_under_concurrent_threads(gpu, tmp_path):
    """8 host threads, a stream each, a different RS(k,m) per iteration with the table
    cache capped at 6 sets (evicting while other threads launch), a plan per batch,
    region multiplies, and cec_cache_trim() from one thread meanwhile: every rebuilt
    shard and every c * (1/c) round trip exact (tests/dropin/cache_threads.c)."""
    from tests.dropin import run_cache_threads

    out = run_cache_threads(tmp_path, threads=8, iters=60, limit=6)
    assert out["bad"] == 0 and out["errors"] == 0 and out["checks"] == 8 * 60 * 49
    assert out["evictions"] > 0


def test_engine_switch_under_concurrent_ops(gpu, oracle):
    """cec_set_engine is process-wide: another thread may switch it while an op runs.
    Each op reads the engine once, so its coefficient tables and its kernel always agree
    (PERM tables under the LDS kernel, or the reverse, would give wrong bytes).  One
    thread flips the engine as fast as it can while this one encodes, diff-updates and
    multiplies regions on its own stream; every result is checked."""
    import threading

    torch, ec = gpu
    k, m, n, B = 3, 2, 4096, 64
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0xE1)
    host = [rng.integers(0, 256, B * n, dtype=np.uint8) for _ in range(k)]
    exp_par = oracle.encode(mat, k, m, host)
    data = [torch.from_numpy(h).cuda() for h in host]
    parity = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    src = rng.integers(0, 256, 3 * n + 5, dtype=np.uint8)
    base = rng.integers(0, 256, 3 * n + 5, dtype=np.uint8)
    exp_rm = base.copy()
    oracle.region_multiply(src, 0x53, exp_rm, 1)
    dsrc = torch.from_numpy(src).cuda()
    default = ec.get_engine()
    stop = threading.Event()
    flips = [0]

    def flipper():
        e = 0
        while not stop.is_set():
            e ^= 1
            ec.set_engine(ec.CEC_ENGINE_LDS if e else ec.CEC_ENGINE_PERM)
            flips[0] += 1

    t = threading.Thread(target=flipper)
    s = torch.cuda.Stream()
    t.start()
    try:
        with ec.Plan([(i * n, 0, n, 0) for i in range(B)]) as plan, torch.cuda.stream(s):
            for it in range(150):
                for p in parity:
                    p.zero_()
                ec.encode(k, m, mat, data, parity, plan, s)
                dst = torch.from_numpy(base.copy()).cuda()
                ec.region_multiply(dsrc, 0x53, src.size, dst, 1, s)
                s.synchronize()
                for p in range(m):
                    assert np.array_equal(parity[p].cpu().numpy(), exp_par[p]), (it, p)
                assert np.array_equal(dst.cpu().numpy(), exp_rm), it
    finally:
        stop.set()
        t.join()
        ec.set_engine(default)
    assert flips[0] > 150


def test_auto_engine_choices(gpu):
    """AUTO's per-op rule (cocytus_ec.h), read back from the library itself
    (cec_last_engine, what bench.py reports): LDS only for cec_decode of values of 64 KiB
    and more (one mask or many); PERM for the 4 KiB encode and rotating decode (the
    metric), 4 KiB single-mask decodes, every encode, the diff-update, residual, solve,
    set diff, apply and region multiply.  A pinned engine is what every op then
    reports."""
    torch, ec = gpu
    P, L = ec.CEC_ENGINE_PERM, ec.CEC_ENGINE_LDS
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    import bench

    mixed = bench.layout("rs32_mixed")[0][:400]
    base = mixed[0][0]
    mixed = [(o - base, ln) for o, ln in mixed]
    size = max(4096 * 64, 65536 * 8, mixed[-1][0] + mixed[-1][1])
    ar = ec.arena_tensors(2 * k + m + 2, size)
    data, par, out, stage, res = ar[:k], ar[k:k + m], ar[k + m:2 * k + m], ar[-2], ar[-1]
    for t in ar:
        t.random_(0, 256)
    plans = {"4k": [(s * 4096, 0, 4096) for s in range(64)], "64k": [(s * 65536, 0, 65536) for s in range(8)],
             "mixed": [(o, 0, ln) for o, ln in mixed]}
    assert sum(ln for _, ln in mixed) >= (64 << 10) * len(mixed)  # the mixed batch's mean is >= 64 KiB

    def ran(fn):
        fn()
        return ec.last_engine()

    def choices():
        got = {}
        for name, ext in plans.items():
            with ec.Plan([(o, s, n, 0) for o, s, n in ext]) as one, \
                 ec.Plan([(o, s, n, q % 6) for q, (o, s, n) in enumerate(ext)]) as rot:
                got[f"encode_{name}"] = ran(lambda: ec.encode(k, m, mat, data, par, one))
                got[f"decode_rotating_{name}"] = ran(lambda: ec.decode(k, m, mat, masks, data + par, out, rot))
                got[f"decode_one_mask_{name}"] = ran(lambda: ec.decode(k, m, mat, [masks[4]], data + par, out, one))
        with ec.Plan([(s * 4096, s * 4096, 4096, s % k) for s in range(64)]) as byj, \
             ec.Plan([(s * 4096, 0, 4096, 0) for s in range(64)]) as one:
            got["diff_update"] = ran(lambda: ec.diff_update(k, m, mat, data, stage, par, True, byj))
            got["set_diff"] = ran(lambda: ec.set_diff(k, data, stage, res, byj))
            got["apply_diffs"] = ran(lambda: ec.apply_diffs(k, m, mat, k + 1, res, par[1], byj))
            got["residual"] = ran(lambda: ec.residual(k, m, mat, k, masks[0], data + par, res, one))
            got["solve"] = ran(lambda: ec.solve(k, m, mat, masks[4], [None] * (k + 1) + [res], out, one))
        got["encode_region"] = ran(lambda: ec.encode_region(k, m, mat, data, par, 65536 * 8))
        got["region_multiply"] = ran(lambda: ec.region_multiply(data[0], 245, 65536, par[0], 1))
        torch.cuda.synchronize()
        return got

    default = ec.get_engine()
    try:
        ec.set_engine(ec.CEC_ENGINE_AUTO)
        got = choices()
        lds = {"decode_one_mask_64k", "decode_one_mask_mixed", "decode_rotating_64k", "decode_rotating_mixed"}
        assert got == {op: (L if op in lds else P) for op in got}, got
        for pinned in (P, L):
            ec.set_engine(pinned)
            assert set(choices().values()) == {pinned}
    finally:
        ec.set_engine(default)


def _c_stream(ec):
    import ctypes

    s = ctypes.c_void_p()
    assert ec.lib().cec_stream_create(ctypes.byref(s)) == ec.CEC_OK
    return s.value


def test_release_stream_keeps_tracking_bounded(gpu, oracle):
    """A long-lived plan, drainer and recovery pool used on 40 short-lived streams (one per
    client connection), each released (cec_*_release_stream) and then destroyed: the plan
    tracks no dead stream (its list stays at the streams alive), every result is
    bit-exact, and the objects' destroys touch no destroyed handle."""
    torch, ec = gpu
    k, m, mat, data, parity = _rs32(torch, ec, B=64)
    torch.cuda.synchronize()
    plan = ec.Plan([(i * 4096, 0, 4096, 0) for i in range(64)])
    torch.cuda.synchronize()
    base = plan.tracked_streams  # the creation stream
    host = [d.cpu().numpy() for d in data]
    exp = oracle.encode(mat, k, m, host)
    n = 64 * 4096
    drained = torch.zeros(n, dtype=torch.uint8, device="cuda")
    diff = oracle.splitmix_bytes(77, 4096)
    want = np.zeros(n, np.uint8)
    pool_parity = parity[0].clone()
    with ec.Drainer(k, m, mat, k + 1, staging_bytes=1 << 20) as dr, \
         ec.RecoveryPool(k, m, mat, k, pool_parity, capacity_units=8) as pool:
        for i in range(40):
            s = _c_stream(ec)
            par = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(m)]
            torch.cuda.synchronize()
            ec.encode(k, m, mat, data, par, plan, s)
            dr.apply([(diff, (i % 64) * 4096, i % k)], drained, s)
            oracle.region_multiply(diff.copy(), mat[(k + 1) * k + i % k], want[(i % 64) * 4096:(i % 64 + 1) * 4096], 1)
            rid = pool.begin(ec.recovery_mask(k, m, k, [0, 1, 1, 1, 1]), i % 64, i % 64)
            pool.add_peer(rid, 1, host[1][(i % 64) * 4096:(i % 64 + 1) * 4096].copy())
            pool.flush(s)
            pool.end(rid)
            for obj in (plan, dr, pool):
                obj.release_stream(s)
            assert plan.tracked_streams == base
            assert ec.lib().cec_stream_destroy(ctypes_vp(s)) == ec.CEC_OK
            assert all(np.array_equal(par[p].cpu().numpy(), exp[p]) for p in range(m)), i
        assert np.array_equal(drained.cpu().numpy(), want)
    plan.release_stream(12345)  # a stream it never used: no-op
    plan.destroy()


def ctypes_vp(x):
    import ctypes

    return ctypes.c_void_p(x)


def test_release_stream_refused_while_capturing(gpu, oracle):
    """cec_plan_release_stream on a stream that is being captured into a graph cannot wait
    for it: refused (CEC_EHIP), the plan keeps the stream listed and the capture is
    unharmed; after the capture the release works."""
    torch, ec = gpu
    k, m, mat, data, parity = _rs32(torch, ec, B=16)
    s = torch.cuda.Stream()
    plan = ec.Plan([(i * 4096, 0, 4096, 0) for i in range(16)], stream=s)
    ec.encode(k, m, mat, data, parity, plan, s)  # tables cached, s listed
    s.synchronize()
    listed = plan.tracked_streams
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        with pytest.raises(ec.CecError) as ei:
            plan.release_stream(s)
        assert ei.value.code == ec.CEC_EHIP
        ec.encode(k, m, mat, data, parity, plan, s)
    assert plan.tracked_streams == listed
    for p in parity:
        p.zero_()
    g.replay()
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, [d.cpu().numpy() for d in data])
    assert all(np.array_equal(parity[p].cpu().numpy(), exp[p]) for p in range(m))
    plan.release_stream(s)
    assert plan.tracked_streams == listed - 1
    plan.destroy()


@pytest.mark.parametrize("path", ["drain_small", "drain_pack", "host_batch", "pool_fold_updates"])
def test_failed_later_wave_leaves_nothing_in_flight(gpu, oracle, path):
    """A launch that fails after earlier waves of the same call ran (fault injection:
    cec_internal_fail_launch(1) -- the second launch of the call fails as a HIP error
    would): the call returns CEC_EHIP only after the first wave has completed, so nothing of
    it still reads the object's staging when the next call overwrites it.  A
    window of distinct 4 KiB updates plus one exact duplicate of the first takes two waves:
    the first wave holds every distinct update once, whichever of the twin pair it took.
    Checked: the registered host arena holds exactly the first wave's bytes on return (read
    without a device sync), the host batch wrote no destination, the pool's residual holds
    the first wave's folds; then the whole window again gives the reference's bytes."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0xFA11 + len(path))
    n = 24 if path in ("drain_small", "pool_fold_updates") else 400  # 400 x 4 KiB: the pack path
    lid_self, src = k, 1
    c = mat[lid_self * k + src]
    ups = [(rng.integers(0, 256, U, dtype=np.uint8), 2 * i * U, src) for i in range(n)]
    ups.append((ups[0][0].copy(), ups[0][1], src))  # the twin: a second wave
    once = np.zeros(2 * n * U + U, np.uint8)  # c * every distinct update, once
    for buf, addr, _ in ups[:n]:
        oracle.region_multiply(buf, c, once[addr:addr + U], 1)
    try:
        if path.startswith("drain"):
            arena = rng.integers(0, 256, once.size, dtype=np.uint8)
            before = arena.copy()
            alias = ec.host_register(arena)
            try:
                with ec.Drainer(k, m, mat, lid_self, staging_bytes=8 << 20) as d:
                    ec.fail_launch(1)
                    with pytest.raises(ec.CecError) as e:
                        d.apply(ups, alias)
                    assert e.value.code == ec.CEC_EHIP
                    assert np.array_equal(arena, before ^ once)  # wave 0 complete on return
                    d.apply(ups, alias)  # the whole window again: every update twice
                    exp = before.copy()   # but the first (three times in all)
                    oracle.region_multiply(ups[0][0], c, exp[0:U], 1)
                    assert np.array_equal(arena, exp)
            finally:
                ec.host_unregister(arena)
        elif path == "host_batch":
            dst = rng.integers(0, 256, once.size, dtype=np.uint8)
            before = dst.copy()
            jobs = [(buf, dst.ctypes.data + addr, None, U, c, 1) for buf, addr, _ in ups]
            ec.fail_launch(1)
            with pytest.raises(ec.CecError) as e:
                ec.region_multiply_batch(jobs)
            assert e.value.code == ec.CEC_EHIP
            assert np.array_equal(dst, before)  # nothing unpacked: no destination written
            assert ec.region_multiply_batch(jobs)[0] == 2  # two waves
            exp = before ^ once
            oracle.region_multiply(ups[0][0], c, exp[0:U], 1)
            assert np.array_equal(dst, exp)
        else:
            data = [rng.integers(0, 256, once.size, dtype=np.uint8) for _ in range(k)]
            par = to_dev_np(torch, oracle.encode(mat, k, m, data)[0])
            nunits = once.size // U
            mask = (1 << lid_self) | 0b110  # D0 lost, leader P0; D1 has not replied yet
            with ec.RecoveryPool(k, m, mat, lid_self, par, capacity_units=nunits) as pool:
                rid = pool.begin(mask, 0, nunits - 1)
                pool.add_peer(rid, 2, data[2].copy())
                pool.flush()
                res0 = np.empty(once.size, np.uint8)
                pool.residual(rid, res0)
                ec.fail_launch(1)
                with pytest.raises(ec.CecError) as e:
                    pool.fold_updates(ups)
                assert e.value.code == ec.CEC_EHIP
                res1 = np.empty(once.size, np.uint8)
                pool.residual(rid, res1)
                assert np.array_equal(res1, res0 ^ once)
                pool.fold_updates(ups)
                res2 = np.empty(once.size, np.uint8)
                pool.residual(rid, res2)
                exp = res0 ^ once ^ once
                oracle.region_multiply(ups[0][0], c, exp[0:U], 1)
                assert np.array_equal(res2, exp)
    finally:
        ec.fail_launch(-1)


def to_dev_np(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()
