"""cec_region_multiply_batch: galois_w08_region_multiply (the drop-in symbol SURVEY §8a a1
names, called once per 4 KiB unit at recovery.c:91, 123 and memcached.c:7918) batched
over host memory.  The oracle runs the same calls one by one in job order (the
reference's own sequential chain); the batch must leave every byte identical.

Jobs are carved out of one host "heap" (numpy, pageable) so that destinations can
overlap each other the way the server's units and solve outputs do."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _model(oracle, heap, jobs):
    """The sequential chain: for each job in order, galois_w08_region_multiply(src, c,
    len, dst, add), with a base first copied into dst (recovery.c:79-82 then :91)."""
    h = heap.copy()
    for s, d, b, n, c, add in jobs:
        src = h[s:s + n].copy()
        dst = h[d:d + n]
        if b is not None:
            dst[:] = h[b:b + n]
        oracle.region_multiply(src, c, dst, add)
    return h


def _run(ec, heap, jobs, stream=None):
    base = heap.ctypes.data
    return ec.region_multiply_batch(
        [(base + s, base + d, None if b is None else base + b, n, c, add) for s, d, b, n, c, add in jobs], stream)


def _disjoint_jobs(rng, heap_len, count, max_len, kinds=("xor", "write", "base"), align=16):
    """count jobs whose dst ranges are disjoint; src / base ranges in the upper half."""
    half = heap_len // 2
    jobs, dcur = [], 0
    for _ in range(count):
        n = int(rng.integers(1, max_len + 1))
        dcur += 16 * int(rng.integers(0, 64)) if align == 16 else int(rng.integers(0, 1024))
        dcur = (dcur + align - 1) // align * align
        if dcur + n > half:
            break
        kind = kinds[int(rng.integers(0, len(kinds)))]
        s = half + int(rng.integers(0, half - n))
        b = half + int(rng.integers(0, half - n)) if kind == "base" else None
        c = int(rng.integers(0, 256))
        jobs.append((s, dcur, b, n, c, 0 if kind == "write" else 1))
        dcur += n
    return jobs


@pytest.mark.parametrize("align", [16, 1])
def test_batch_disjoint_matches_sequential(gpu, oracle, align):
    """Disjoint destinations, every kind (XOR, write, base), every coefficient including
    0 and 1, lengths 1 B - 20 KiB at 16-B-aligned and at arbitrary addresses."""
    torch, ec = gpu
    rng = np.random.default_rng(100 + align)
    heap = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    jobs = _disjoint_jobs(rng, heap.size, 600, 20 << 10, align=align)
    assert len(jobs) > 300
    want = _model(oracle, heap, jobs)
    launches, rounds = _run(ec, heap, jobs)
    assert np.array_equal(heap, want)
    assert launches == rounds  # disjoint destinations: one wave per staging round (pipelined rounds above 4 MiB)


def test_batch_recovery_units_shape(gpu, oracle):
    """recovery_recover_units for a 1 MiB range (256 units), the shape the glue runs: each
    unit its own 4 KiB malloc'd buffer (scattered in the heap), first touch = base (the
    parity arena's unit) ^ c * peer, then a second peer folded in place."""
    torch, ec = gpu
    rng = np.random.default_rng(7)
    U = 4096
    heap = rng.integers(0, 256, 32 << 20, dtype=np.uint8)
    arena, peer1, peer2 = 0, 2 << 20, 4 << 20   # parity arena, two peers' replies (1 MiB each)
    units = [(8 << 20) + i * (U + 48) for i in rng.permutation(256)]  # scattered unit buffers
    first = [(peer1 + i * U, units[i], arena + i * U, U, 245, 1) for i in range(256)]
    second = [(peer2 + i * U, units[i], None, U, 244, 1) for i in range(256)]
    want = _model(oracle, heap, first + second)
    _run(ec, heap, first)
    _run(ec, heap, second)
    assert np.array_equal(heap, want)


def test_batch_overlapping_xor_waves(gpu, oracle):
    """Drain-window folds (recovery_try_update_unit pieces of many SETs): XOR-only jobs whose
    destinations overlap each other arbitrarily -- separate launches, same bytes."""
    torch, ec = gpu
    rng = np.random.default_rng(21)
    heap = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    jobs = []
    for _ in range(2000):
        n = int(rng.integers(1, 6000))
        d = int(rng.integers(0, (256 << 10) - n))          # 256 KiB of destinations: dense overlap
        s = (2 << 20) + int(rng.integers(0, (2 << 20) - n))
        jobs.append((s, d, None, n, int(rng.integers(0, 256)), 1))
    want = _model(oracle, heap, jobs)
    launches, _ = _run(ec, heap, jobs)
    assert np.array_equal(heap, want)
    assert launches > 1


def test_batch_overlapping_writes_in_job_order(gpu, oracle):
    """The leader solve's shape (memcached.c:7913-7922): out[i] = calloc, then += inv[i][j]
    * C[j] -- a write followed by XORs onto the same destination, in job order; plus
    random mixes of writes, bases and XORs over overlapping destinations, whose result
    depends on the order."""
    torch, ec = gpu
    rng = np.random.default_rng(5)
    heap = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    nbuf = 64 << 10
    C = [(4 << 20) + j * nbuf for j in range(2)]
    out = [0, nbuf]
    inv = [[1, 245], [3, 7]]
    jobs = [(C[j], out[i], None, nbuf, inv[i][j], 0 if j == 0 else 1) for i in range(2) for j in range(2)]
    want = _model(oracle, heap, jobs)
    launches, _ = _run(ec, heap, jobs)
    assert np.array_equal(heap, want) and launches == 2
    # random order-dependent mixes
    heap = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    jobs = []
    for _ in range(700):
        n = int(rng.integers(1, 9000))
        d = int(rng.integers(0, (512 << 10) - n))
        s = (4 << 20) + int(rng.integers(0, (2 << 20) - n))
        kind = rng.choice(["xor", "xor", "write", "base"])
        b = (6 << 20) + int(rng.integers(0, (2 << 20) - n)) if kind == "base" else None
        jobs.append((s, d, b, n, int(rng.integers(0, 256)), 0 if kind == "write" else 1))
    want = _model(oracle, heap, jobs)
    _run(ec, heap, jobs)
    assert np.array_equal(heap, want)


def test_batch_many_rounds_and_large_jobs(gpu, oracle):
    """More than one staging round (the batch exceeds the per-thread staging) and jobs
    longer than a piece (1 MiB): 3 MiB + ragged lengths, 60 MiB in all."""
    torch, ec = gpu
    rng = np.random.default_rng(9)
    heap = rng.integers(0, 256, 160 << 20, dtype=np.uint8)
    jobs, d = [], 0
    for i in range(24):
        n = (3 << 20) - int(rng.integers(0, 4096)) if i % 3 == 0 else int(rng.integers(1, 2 << 20))
        s = (80 << 20) + int(rng.integers(0, (80 << 20) - n))
        add = 0 if i % 5 == 2 else 1
        b = (80 << 20) + int(rng.integers(0, (80 << 20) - n)) if i % 4 == 1 and add else None
        jobs.append((s, d, b, n, int(rng.integers(0, 256)), add))
        d += n + 16
    assert d < 80 << 20
    want = _model(oracle, heap, jobs)
    launches, rounds = _run(ec, heap, jobs)
    assert np.array_equal(heap, want)
    assert rounds >= 2


def test_batch_in_place_base_and_noops(gpu, oracle):
    """base == dst is the plain in-place add; multby 0 with add is a no-op (no launch);
    zero-length jobs are skipped; an empty batch returns at once."""
    torch, ec = gpu
    rng = np.random.default_rng(13)
    heap = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    jobs = [(512 << 10, 0, 0, 4096, 77, 1), (600 << 10, 8192, None, 4096, 0, 1),
            (700 << 10, 16384, None, 0, 5, 1), (800 << 10, 20480, None, 100, 0, 0)]
    want = _model(oracle, heap, jobs)
    _run(ec, heap, jobs)
    assert np.array_equal(heap, want)
    assert _run(ec, heap, []) == (0, 0)
    assert _run(ec, heap, [(600 << 10, 8192, None, 4096, 0, 1)]) == (0, 0)


def test_batch_refuses_reads_of_written_bytes(gpu, oracle):
    """A src or base that overlaps any job's dst would read bytes the batch changes (the
    sequential chain would see the earlier job's output): refused with CEC_EOVERLAP
    before anything runs; bad multby / add / base-with-write are CEC_EINVAL."""
    torch, ec = gpu
    heap = np.arange(1 << 16, dtype=np.uint32).view(np.uint8)[:1 << 16].copy()
    keep = heap.copy()
    for jobs in ([(0, 4096, None, 4096, 3, 1), (8192, 0, None, 100, 3, 1)],      # src meets dst of job 1
                 [(9000, 4096, 4000, 4096, 3, 1)]):                            # base meets its own dst
        with pytest.raises(ec.CecError) as e:
            _run(ec, heap, jobs)
        assert e.value.code == ec.CEC_EOVERLAP
    for bad in ([(0, 4096, None, 16, 256, 1)], [(0, 4096, None, 16, 3, 2)], [(0, 4096, 8192, 16, 3, 0)]):
        with pytest.raises(ec.CecError) as e:
            _run(ec, heap, bad)
        assert e.value.code == ec.CEC_EINVAL
    assert np.array_equal(heap, keep)


def test_batch_pinned_host_buffers(gpu, oracle):
    """Pinned (torch pin_memory) host buffers take the same path as pageable ones."""
    torch, ec = gpu
    rng = np.random.default_rng(17)
    t = torch.from_numpy(rng.integers(0, 256, 4 << 20, dtype=np.uint8)).pin_memory()
    heap = t.numpy()
    jobs = _disjoint_jobs(rng, heap.size, 200, 16 << 10)
    want = _model(oracle, heap, jobs)
    _run(ec, heap, jobs)
    assert np.array_equal(heap, want)


def test_batch_fuzz_small(gpu, oracle):
    """300 random small batches (1-60 jobs of 1 B - 12 KiB, every kind, dense or sparse
    overlap of destinations, unaligned everything, base == dst now and then): each equals
    the sequential chain."""
    torch, ec = gpu
    rng = np.random.default_rng(2024)
    heap = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    for it in range(300):
        span = int(rng.choice([16 << 10, 256 << 10, 2 << 20]))     # destination region: overlap density
        jobs = []
        for _ in range(int(rng.integers(1, 61))):
            n = int(rng.integers(1, 12 << 10))
            d = int(rng.integers(0, span - n)) if span > n else 0
            s = (2 << 20) + int(rng.integers(0, (2 << 20) - n))
            kind = rng.choice(["xor", "xor", "write", "base", "inplace"])
            b = (2 << 20) + int(rng.integers(0, (2 << 20) - n)) if kind == "base" else (d if kind == "inplace" else None)
            jobs.append((s, d, b, n, int(rng.integers(0, 256)), 0 if kind == "write" else 1))
        want = _model(oracle, heap, jobs)
        _run(ec, heap, jobs)
        assert np.array_equal(heap, want), f"iteration {it}"


def test_batch_refused_while_capturing(gpu, oracle):
    """The batch is synchronous (it waits for its own launches and then copies the results
    out): on a stream being captured into a graph it is refused (CEC_EINVAL) before
    anything is launched, and the capture is unharmed."""
    torch, ec = gpu
    heap = np.arange(1 << 16, dtype=np.uint32).view(np.uint8)[:1 << 18].copy()
    keep = heap.copy()
    s = torch.cuda.Stream()
    x = torch.zeros(16, device="cuda")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        with pytest.raises(ec.CecError) as e:
            _run(ec, heap, [(128 << 10, 0, None, 4096, 7, 1)], stream=s)
        assert e.value.code == ec.CEC_EINVAL
        x.add_(1)
    g.replay()
    torch.cuda.synchronize()
    assert float(x.sum()) == 16.0 and np.array_equal(heap, keep)


def test_batch_bases_in_place_from_a_registered_region(gpu, oracle):
    """Bases inside a region registered with cec_host_register (the server's ecmem) are read
    in place through its device alias -- recovery's first touch (unit = parity unit ^ c *
    peer) and SET diffs (diff = old ^ new) -- with the same bytes as the staged path; a
    round whose bases leave the region, or whose destinations overlap, is staged."""
    torch, ec = gpu
    rng = np.random.default_rng(31)
    heap = rng.integers(0, 256, 16 << 20, dtype=np.uint8)
    arena = heap[:4 << 20]                       # the registered "ecmem"
    ec.host_register(arena)
    try:
        U = 4096
        units = [(8 << 20) + int(i) * (U + 80) for i in rng.permutation(256)]
        jobs = [((5 << 20) + i * U, units[i], int(rng.integers(0, 1000)) * U + 16 * int(rng.integers(0, 4)),
                 U - 16 * int(rng.integers(0, 2)), 245, 1) for i in range(256)]
        want = _model(oracle, heap, jobs)
        _run(ec, heap, jobs)
        st = ec.batch_stats()
        assert np.array_equal(heap, want) and st["in_place_launches"] == st["launches"] >= 1
        # SET diffs: 600 values, old bytes in the registered arena, diffs elsewhere
        heap[:] = rng.integers(0, 256, heap.size, dtype=np.uint8)
        jobs, d = [], 9 << 20
        for _ in range(600):
            n = int(rng.integers(1, 9000))
            addr = 16 * int(rng.integers(0, ((4 << 20) - n) // 16))
            jobs.append(((6 << 20) + int(rng.integers(0, (2 << 20) - n)), d, addr, n, 1, 1))
            d += n + int(rng.integers(0, 64))
        want = _model(oracle, heap, jobs)
        _run(ec, heap, jobs)
        st = ec.batch_stats()
        assert np.array_equal(heap, want) and st["in_place_launches"] == st["launches"]
        # a base outside the region: staged (same bytes)
        jobs[7] = (jobs[7][0], jobs[7][1], (31 << 19), jobs[7][3], 1, 1)  # past every destination
        heap[:] = rng.integers(0, 256, heap.size, dtype=np.uint8)
        want = _model(oracle, heap, jobs)
        _run(ec, heap, jobs)
        assert np.array_equal(heap, want) and ec.batch_stats()["in_place_launches"] < ec.batch_stats()["launches"]
    finally:
        ec.host_unregister(arena)
    # unregistered again: staged
    _run(ec, heap, [((5 << 20), (8 << 20), 0, 4096, 3, 1)])
    assert ec.batch_stats()["in_place_launches"] == 0


def test_batch_pipelined_rounds_in_place_odd_sizes(gpu, oracle):
    """A batch above 4 MiB runs as double-buffered rounds; with 4098-B SETs the staging half's
    size is no multiple of 16 unless rounded: every round -- the odd ones in the
    second half included -- must read its bases in place and leave the sequential chain's
    bytes.  2,000 SET diffs (memcached.c:2676-2681: diff = old ^ 1 * value), old bytes in a
    registered arena at shuffled 16-B aligned addresses."""
    torch, ec = gpu
    rng = np.random.default_rng(4098)
    n_sets, size, stride = 2000, 4098, 4112
    heap = rng.integers(0, 256, 48 << 20, dtype=np.uint8)
    arena = heap[:n_sets * stride]                  # the registered ecmem
    vbase, dbase = 16 << 20, 32 << 20
    slots = rng.permutation(n_sets)
    jobs = [(vbase + i * stride, dbase + i * stride, int(slots[i]) * stride, size, 1, 1) for i in range(n_sets)]
    want = _model(oracle, heap, jobs)
    ec.host_register(arena)
    try:
        launches, rounds = _run(ec, heap, jobs)
        st = ec.batch_stats()
    finally:
        ec.host_unregister(arena)
    assert np.array_equal(heap, want)
    assert rounds >= 4 and st["in_place_launches"] == launches == rounds
