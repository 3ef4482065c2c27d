"""GPU parity: every op of libcocytus_ec.so (called through its C-ABI) against the
CPU restatement in oracle/ on the same seeded inputs.  Bit-exact (byte arithmetic).

Parity is "unpinned" (see oracle/gf8_ref.h): the reference's Jerasure/GF-Complete is
not available, so the oracle restates it; tests/test_oracle.py pins the oracle to the
independent known answers that exist.
"""
from __future__ import annotations

import itertools
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODES = [(3, 2), (4, 2), (6, 3), (10, 4), (16, 4), (2, 5)]
SENT = 0xA5


@pytest.fixture(params=["perm", "lds"])
def engine(request, gpu):
    torch, ec = gpu
    default = ec.get_engine()
    ec.set_engine(ec.CEC_ENGINE_PERM if request.param == "perm" else ec.CEC_ENGINE_LDS)
    yield request.param
    ec.set_engine(default)


def to_dev(torch, a: np.ndarray):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def to_host(t) -> np.ndarray:
    return t.cpu().numpy()


def make_extents(rng, lens, align=16, gap=48, unaligned_every=0):
    """Non-overlapping extents laid out like ecalloc (16-B aligned starts)."""
    ext, off, soff = [], 64, 32
    for i, n in enumerate(lens):
        o = off
        if unaligned_every and i % unaligned_every == unaligned_every - 1:
            o += 1 + int(rng.integers(0, 15))  # deliberately misaligned arena offset
        ext.append([o, soff, n, 0])
        off = ((o + n + gap + align - 1) // align) * align
        soff = ((soff + n + 16 + 15) // 16) * 16
    return ext, off, soff


MIXED = [0, 1, 15, 16, 17, 255, 256, 4095, 4096, 4097, 4098, 8195, 65536, 100003, 1 << 20]


# ------------------------------------------------------------------ region multiply (a1)
@pytest.mark.parametrize("c", [0, 1, 2, 0x80, 244, 245, 255, 0x53])
@pytest.mark.parametrize("add", [0, 1])
def test_region_multiply_device(gpu, oracle, engine, c, add):
    torch, ec = gpu
    rng = np.random.default_rng(c * 2 + add)
    for n in [1, 15, 16, 17, 4095, 4096, 4098, (1 << 20) + 3]:
        for so, do in [(0, 0), (16, 32), (3, 3), (1, 7)]:
            src = rng.integers(0, 256, n + 64, dtype=np.uint8)
            dst = rng.integers(0, 256, n + 64, dtype=np.uint8)
            exp = dst.copy()
            view = exp[do:do + n].copy()
            oracle.region_multiply(src[so:so + n].copy(), c, view, add)
            exp[do:do + n] = view
            ds, dd = to_dev(torch, src), to_dev(torch, dst)
            ec.region_multiply(ds.data_ptr() + so, c, n, dd.data_ptr() + do, add)
            torch.cuda.synchronize()
            got = to_host(dd)
            assert np.array_equal(got, exp), (c, add, n, so, do)


def test_region_multiply_in_place(gpu, oracle):
    torch, ec = gpu
    a = oracle.splitmix_bytes(7, 9000)
    exp = a.copy()
    oracle.region_multiply(exp, 0x1D, None, 0)
    d = to_dev(torch, a)
    ec.region_multiply(d, 0x1D, 9000, None, 0)
    torch.cuda.synchronize()
    assert np.array_equal(to_host(d), exp)


def test_region_multiply_past_one_dispatch(gpu, oracle, engine):
    """Maximum sizes: 64 GiB + 3 tiles + 77 B per stream is more than one dispatch's
    2^32 - 1 work items, so the grid is capped and workgroups walk the rest grid-stride
    (run_combine).  Windows at the head, the tail and across the first tiles past the
    cap (offset 2^36 = tile 2^24) are checked against the oracle; then x ^= c * src again
    must leave every byte 0 (size-independent: a tile skipped in either pass leaves the
    0xFF fill or c * src)."""
    torch, ec = gpu
    n = (1 << 36) + 3 * 4096 + 77
    torch.cuda.empty_cache()
    ec.cache_trim()
    if torch.cuda.mem_get_info()[0] < 2 * n + (4 << 30):
        pytest.skip("needs 2 x 64 GiB of free HBM")
    g = torch.Generator(device="cuda").manual_seed(0xC0C70007)
    src = torch.empty(n, dtype=torch.uint8, device="cuda")
    src.random_(0, 256, generator=g)
    dst = torch.full((n,), 0xFF, dtype=torch.uint8, device="cuda")
    c, W = 0x53, 1 << 20
    try:
        ec.region_multiply(src, c, n, dst, 0)
        torch.cuda.synchronize()
        rng = np.random.default_rng(7)
        for off in [0, n - W, (1 << 36) - W + 8192, *rng.integers(0, n - W, 4).tolist()]:
            exp = np.zeros(W, dtype=np.uint8)
            oracle.region_multiply(to_host(src[off:off + W]), c, exp, 0)
            assert np.array_equal(to_host(dst[off:off + W]), exp), off
        ec.region_multiply(src, c, n, dst, 1)
        torch.cuda.synchronize()
        assert not bool(dst.any())
    finally:
        del src, dst
        torch.cuda.empty_cache()


# ------------------------------------------------------------------ encode (a5)
@pytest.mark.parametrize("k,m", CODES)
def test_encode_plan(gpu, oracle, engine, k, m):
    torch, ec = gpu
    mat = ec.coding_matrix(k, m)
    assert mat == oracle.big_vandermonde(k + m, k)
    rng = np.random.default_rng(1000 * k + m)
    ext, arena_len, _ = make_extents(rng, MIXED, unaligned_every=5)
    data = [rng.integers(0, 256, arena_len, dtype=np.uint8) for _ in range(k)]
    par0 = np.full(arena_len, SENT, np.uint8)
    ddev = [to_dev(torch, d) for d in data]
    pdev = [to_dev(torch, par0) for _ in range(m)]
    with ec.Plan([tuple(e) for e in ext]) as plan:
        assert plan.num_extents == len(ext)
        assert plan.total_bytes == sum(MIXED)
        ec.encode(k, m, mat, ddev, pdev, plan)
        torch.cuda.synchronize()
    exp = [par0.copy() for _ in range(m)]
    for off, _, n, _ in ext:
        if n == 0:
            continue
        ps = oracle.encode(mat, k, m, [d[off:off + n].copy() for d in data])
        for p in range(m):
            exp[p][off:off + n] = ps[p]
    for p in range(m):
        assert np.array_equal(to_host(pdev[p]), exp[p]), f"parity {p}"


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (8, 4)])
def test_encode_region(gpu, oracle, engine, k, m):
    torch, ec = gpu
    mat = ec.coding_matrix(k, m)
    n = 3 * 4096 + 1234
    data = [oracle.splitmix_bytes(0xC0C70001 + j, n) for j in range(k)]
    pdev = [to_dev(torch, np.zeros(n, np.uint8)) for _ in range(m)]
    ec.encode_region(k, m, mat, [to_dev(torch, d) for d in data], pdev, n)
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, data)
    for p in range(m):
        assert np.array_equal(to_host(pdev[p]), exp[p])


def test_extent_pattern_validated(gpu, oracle):
    """cocytus_ec.h: every op checks its extents' pattern index before launching (the
    kernel indexes the op's pattern table with it): single-pattern ops require 0, the
    others an index below k / n_masks; anything else is CEC_EINVAL and nothing runs."""
    torch, ec = gpu
    k, m, n, B = 3, 2, 4096, 8
    mat = ec.coding_matrix(k, m)
    host = [oracle.splitmix_bytes(70 + j, B * n) for j in range(k)]
    data = [to_dev(torch, h) for h in host]
    parity = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ok = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
    ec.encode(k, m, mat, data, parity, ok)
    res = torch.zeros(B * n, dtype=torch.uint8, device="cuda")
    mask = ec.recovery_mask(k, m, k, [0, 1, 1, 1, 1])
    wild = ec.Plan([(s * n, 0, n, 1000 + 77 * s) for s in range(B)])
    for call in (lambda: ec.encode(k, m, mat, data, parity, wild),
                 lambda: ec.residual(k, m, mat, k, mask, data + parity, res, wild),
                 lambda: ec.solve(k, m, mat, mask, [None, None, None, res, res], [res, None, None], wild)):
        with pytest.raises(ec.CecError) as e:
            call()
        assert e.value.code == ec.CEC_EINVAL
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, host)
    for p in range(m):
        assert np.array_equal(to_host(parity[p]), exp[p]), p
    assert not to_host(res).any()  # nothing launched
    ok.destroy()
    stage = torch.zeros(B * n, dtype=torch.uint8, device="cuda")
    bad = ec.Plan([(s * n, s * n, n, k if s == B - 1 else s % k) for s in range(B)])
    with pytest.raises(ec.CecError) as e:
        ec.diff_update(k, m, mat, data, stage, parity, True, bad)
    assert e.value.code == ec.CEC_EINVAL
    with pytest.raises(ec.CecError) as e:
        ec.apply_diffs(k, m, mat, k, stage, parity[0], bad)
    assert e.value.code == ec.CEC_EINVAL
    with pytest.raises(ec.CecError) as e:
        ec.set_diff(k, data, stage, res, bad)
    assert e.value.code == ec.CEC_EINVAL
    with pytest.raises(ec.CecError) as e:
        ec.decode(k, m, mat, [mask], data + parity, [res, None, None], bad)
    assert e.value.code == ec.CEC_EINVAL
    torch.cuda.synchronize()
    assert all(np.array_equal(to_host(parity[p]), exp[p]) for p in range(m))  # nothing launched
    wild.destroy()
    bad.destroy()


def test_encode_lost_parity_not_written(gpu, oracle):
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    n = 8192
    data = [oracle.splitmix_bytes(j + 1, n) for j in range(k)]
    p0 = to_dev(torch, np.zeros(n, np.uint8))
    ec.encode_region(k, m, mat, [to_dev(torch, d) for d in data], [p0, None], n)
    torch.cuda.synchronize()
    assert np.array_equal(to_host(p0), oracle.encode(mat, k, m, data)[0])


# ------------------------------------------------------------------ diff-update (a2+a3)
@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3), (2, 5)])
@pytest.mark.parametrize("install", [False, True])
def test_diff_update(gpu, oracle, engine, k, m, install):
    torch, ec = gpu
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(77 + k * 10 + m + install)
    lens = [int(x) for x in rng.integers(1, 20000, 40)] + [4098, 4096, 16, 17]
    ext, arena_len, stage_len = make_extents(rng, lens, unaligned_every=7)
    for e in ext:
        e[3] = int(rng.integers(0, k))  # source data shard lid j
    data = [rng.integers(0, 256, arena_len, dtype=np.uint8) for _ in range(k)]
    parity = oracle.encode(mat, k, m, data)
    staging = rng.integers(0, 256, stage_len, dtype=np.uint8)
    ddev = [to_dev(torch, d) for d in data]
    pdev = [to_dev(torch, p) for p in parity]
    with ec.Plan([tuple(e) for e in ext]) as plan:
        ec.diff_update(k, m, mat, ddev, to_dev(torch, staging), pdev, install, plan)
        torch.cuda.synchronize()
    for off, soff, n, j in ext:  # the reference chain, SET by SET
        old = data[j][off:off + n].copy()
        pv = [p[off:off + n].copy() for p in parity]
        oracle.diff_update(mat, k, m, j, old, staging[soff:soff + n].copy(), pv, install)
        data[j][off:off + n] = old
        for p in range(m):
            parity[p][off:off + n] = pv[p]
    for j in range(k):
        assert np.array_equal(to_host(ddev[j]), data[j]), f"data {j}"
    for p in range(m):
        assert np.array_equal(to_host(pdev[p]), parity[p]), f"parity {p}"
    if install:  # parity is again the encode of the installed data
        enc = oracle.encode(mat, k, m, data)
        for p in range(m):
            assert np.array_equal(enc[p], parity[p])


@pytest.mark.parametrize("engine_name", ["auto", "perm", "lds"])
def test_diff_update_full_size(gpu, oracle, engine_name):
    """The north star's per-SET diff-update at the bench's size (65,536 SETs of
    4 KiB, source shard j uniform in {0,1,2}, RS(3,2), install), three rounds of new
    values: the parity arenas stay the encode of the installed data (a size-independent
    property), checked against the oracle's encode of the whole 256 MiB arenas; and, per
    round, every shard equals its value before the round outside the SETs of that shard and
    the round's staged values inside them (a kernel that installed a SET's value into
    another shard's range, or left a shard's own range stale, fails)."""
    torch, ec = gpu
    k, m, n, B = 3, 2, 4096, 65536
    T = n * B
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70006)
    data = [torch.randint(0, 256, (T,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(T, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, parity, T)
    src = np.random.default_rng(6).integers(0, k, B)
    default = ec.get_engine()
    ec.set_engine({"auto": ec.CEC_ENGINE_AUTO, "perm": ec.CEC_ENGINE_PERM, "lds": ec.CEC_ENGINE_LDS}[engine_name])
    sel = [torch.from_numpy(np.repeat(src == j, n)).cuda() for j in range(k)]  # shard j's SET bytes
    try:
        with ec.Plan([(s * n, s * n, n, int(src[s])) for s in range(B)]) as plan:
            for rnd in range(3):
                stage = torch.randint(0, 256, (T,), dtype=torch.uint8, device="cuda", generator=g)
                before = [d.clone() for d in data]
                ec.diff_update(k, m, mat, data, stage, parity, True, plan)
                ran = ec.last_engine()
                torch.cuda.synchronize()
                for j in range(k):  # each SET installed its value into its own shard only
                    assert torch.equal(data[j][sel[j]], stage[sel[j]]), f"round {rnd}: install into shard {j}"
                    assert torch.equal(data[j][~sel[j]], before[j][~sel[j]]), f"round {rnd}: shard {j} off its SETs"
                del before
    finally:
        ec.set_engine(default)
    if engine_name == "auto":
        assert ran == ec.CEC_ENGINE_PERM
    _assert_parity_matches_oracle(torch, oracle, mat, k, m, data, parity)


def test_diff_update_lost_parity_and_overlap(gpu, oracle):
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    n = 4096
    data = [oracle.splitmix_bytes(10 + j, 4 * n) for j in range(k)]
    parity = oracle.encode(mat, k, m, data)
    new = oracle.splitmix_bytes(99, n)
    ddev = [to_dev(torch, d) for d in data]
    p0 = to_dev(torch, parity[0])
    with ec.Plan([(n, 0, n, 1)]) as plan:
        ec.diff_update(k, m, mat, ddev, to_dev(torch, new), [p0, None], True, plan)
        torch.cuda.synchronize()
    old = data[1][n:2 * n].copy()
    pv = [parity[0][n:2 * n].copy(), np.zeros(n, np.uint8)]
    oracle.diff_update(mat, k, m, 1, old, new, pv, True)
    parity[0][n:2 * n] = pv[0]
    data[1][n:2 * n] = old
    assert np.array_equal(to_host(p0), parity[0])
    assert np.array_equal(to_host(ddev[1]), data[1])
    with ec.Plan([(0, 0, 4096, 0), (4000, 0, 200, 1)]) as plan:  # overlapping SETs
        with pytest.raises(ec.CecError) as ei:
            ec.diff_update(k, m, mat, ddev, to_dev(torch, new), [p0, None], True, plan)
        assert ei.value.code == ec.CEC_EOVERLAP


def test_set_diff_and_apply_diffs(gpu, oracle, engine):
    torch, ec = gpu
    k, m = 4, 2
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(5)
    lens = [int(x) for x in rng.integers(1, 9000, 30)]
    ext, arena_len, stage_len = make_extents(rng, lens, unaligned_every=6)
    for e in ext:
        e[3] = int(rng.integers(0, k))
    data = [rng.integers(0, 256, arena_len, dtype=np.uint8) for _ in range(k)]
    staging = rng.integers(0, 256, stage_len, dtype=np.uint8)
    diff_dev = to_dev(torch, np.zeros(stage_len, np.uint8))
    par = rng.integers(0, 256, arena_len, dtype=np.uint8)
    par_dev = to_dev(torch, par)
    with ec.Plan([tuple(e) for e in ext]) as plan:
        ec.set_diff(k, [to_dev(torch, d) for d in data], to_dev(torch, staging), diff_dev, plan)
        ec.apply_diffs(k, m, mat, k + 1, diff_dev, par_dev, plan)
        torch.cuda.synchronize()
    diffs = to_host(diff_dev)
    for off, soff, n, j in ext:
        d = oracle.set_diff(data[j][off:off + n].copy(), staging[soff:soff + n].copy())
        assert np.array_equal(diffs[soff:soff + n], d)
        pv = par[off:off + n].copy()
        oracle.parity_apply(mat, k, k + 1, j, d, pv)
        par[off:off + n] = pv
    assert np.array_equal(to_host(par_dev), par)


# ------------------------------------------------------------------ recovery (a6, a7)
def all_masks(k, m):
    for lids in itertools.combinations(range(k + m), k):
        mask = sum(1 << x for x in lids)
        if mask != (1 << k) - 1:
            yield mask


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3), (4, 4)])
def test_decode_every_mask(gpu, oracle, engine, k, m):
    torch, ec = gpu
    mat = ec.coding_matrix(k, m)
    masks = list(all_masks(k, m))
    rng = np.random.default_rng(31 * k + m)
    lens = [4096] * 8 + [1, 17, 4098, 65536 + 5, 300]
    ext, arena_len, _ = make_extents(rng, lens * 3, unaligned_every=9)
    for e in ext:
        e[3] = int(rng.integers(0, len(masks)))
    data = [rng.integers(0, 256, arena_len, dtype=np.uint8) for _ in range(k)]
    parity = oracle.encode(mat, k, m, data)
    arenas = data + parity
    adev = [to_dev(torch, a) for a in arenas]
    out0 = np.full(arena_len, SENT, np.uint8)
    odev = [to_dev(torch, out0) for _ in range(k)]
    with ec.Plan([tuple(e) for e in ext]) as plan:
        ec.decode(k, m, mat, masks, adev, odev, plan)
        torch.cuda.synchronize()
    exp = [out0.copy() for _ in range(k)]
    for off, _, n, q in ext:
        mask = masks[q]
        lost = [j for j in range(k) if not (mask >> j) & 1]
        ref = oracle.decode(mat, k, m, mask, [a[off:off + n].copy() if (mask >> i) & 1 else None
                                              for i, a in enumerate(arenas)])
        for x, j in enumerate(lost):
            assert np.array_equal(ref[x], data[j][off:off + n])  # oracle round trip
            exp[j][off:off + n] = ref[x]
    for j in range(k):
        assert np.array_equal(to_host(odev[j]), exp[j]), f"rebuilt shard {j}"


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3)])
def test_residual_then_solve(gpu, oracle, engine, k, m):
    torch, ec = gpu
    mat = ec.coding_matrix(k, m)
    n = 64 * 4096  # 64 recovery units
    data = [oracle.splitmix_bytes(0xC0C70005 + j, n) for j in range(k)]
    parity = oracle.encode(mat, k, m, data)
    arenas = data + parity
    adev = [to_dev(torch, a) for a in arenas]
    for mask in all_masks(k, m):
        pars = [p for p in range(k, k + m) if (mask >> p) & 1]
        lost = [j for j in range(k) if not (mask >> j) & 1]
        res = {p: to_dev(torch, np.zeros(n, np.uint8)) for p in pars}
        outs = {j: to_dev(torch, np.zeros(n, np.uint8)) for j in lost}
        with ec.Plan([(0, 0, n, 0)]) as plan:
            for p in pars:
                ec.residual(k, m, mat, p, mask, adev, res[p], plan)
            ec.solve(k, m, mat, mask, [res.get(i) for i in range(k + m)],
                     [outs.get(j) for j in range(k)], plan)
            torch.cuda.synchronize()
        C = []
        for p in pars:  # recovery_recover_units, survivor by survivor
            r = np.empty(n, np.uint8)
            touched = [0]
            for s in range(k):
                if (mask >> s) & 1:
                    oracle.recover_units(mat, k, p, s, parity[p - k], data[s], r, touched)
            if not touched[0]:
                r[:] = parity[p - k]
            assert np.array_equal(to_host(res[p]), r), (hex(mask), p)
            C.append(r)
        ref = oracle.bottom_half(mat, k, m, mask, C)
        for x, j in enumerate(lost):
            assert np.array_equal(ref[x], data[j])
            assert np.array_equal(to_host(outs[j]), data[j]), (hex(mask), j)


def test_recovery_mask_matches_reference(gpu, oracle):
    _, ec = gpu
    rng = np.random.default_rng(3)
    for _ in range(200):
        k, m = int(rng.integers(1, 9)), int(rng.integers(1, 5))
        conn = [int(x) for x in rng.integers(0, 2, k + m)]
        leader = int(rng.integers(k, k + m))
        assert ec.recovery_mask(k, m, leader, conn) == oracle.recovery_mask(k, m, leader, conn)


# ------------------------------------------------------------------ BASELINE full sizes
def test_cfg2_full_size_roundtrip(gpu, oracle):
    """BASELINE configs[1]: RS(3,2), 65,536 x 4 KiB stripes; encode, erase one data
    shard per stripe (leader rotates over both parities), decode; compare on device."""
    torch, ec = gpu
    k, m, n, B = 3, 2, 4096, 65536
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70002)
    data = [torch.randint(0, 256, (B * n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    # lost data shard j, leader parity k+p (start_recovery, memcached.c:8136-8151)
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    assert all(masks) and len(set(masks)) == k * m
    with ec.Plan([(s * n, 0, n, 0) for s in range(B)]) as enc_plan, \
         ec.Plan([(s * n, 0, n, s % len(masks)) for s in range(B)]) as dec_plan:
        ec.encode(k, m, mat, data, parity, enc_plan)
        ec.decode(k, m, mat, masks, data + parity, out, dec_plan)
        torch.cuda.synchronize()
    lost_of = [[j for j in range(k) if not (mk >> j) & 1][0] for mk in masks]
    for q, j in enumerate(lost_of):
        sel = torch.arange(q, B, len(masks), device="cuda")
        got = out[j].view(B, n)[sel]
        want = data[j].view(B, n)[sel]
        assert torch.equal(got, want), f"mask {q}"
    for s in [0, 1, 4097, B - 1]:  # spot-check parity against the oracle
        d = [to_host(x[s * n:(s + 1) * n]) for x in data]
        ps = oracle.encode(mat, k, m, d)
        for p in range(m):
            assert np.array_equal(to_host(parity[p][s * n:(s + 1) * n]), ps[p])


def test_cfg5_1mib_decode_d0_p0_and_d1_p1(gpu, oracle):
    """BASELINE configs[4]: RS(3,2) online recovery of one lost data shard, 1 MiB values
    x 1,024: D0 with leader P0 (inverse 1) and D1 with leader P1 (inverse 1/245); the
    encoded parity of the whole batch equals the oracle's, every rebuilt value equals the
    data, and one stripe equals the reference's two-step chain."""
    torch, ec = gpu
    k, m, n, B = 3, 2, 1 << 20, 1024
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70005)
    data = [torch.randint(0, 256, (B * n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, parity, B * n)
    m_d0 = ec.recovery_mask(k, m, 3, [0, 1, 1, 1, 1])  # D0 lost, leader P0
    m_d1 = ec.recovery_mask(k, m, 4, [1, 0, 1, 0, 1])  # D1 + P0 lost, leader P1
    assert (m_d0, m_d1) == (0b01110, 0b10101)
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    with ec.Plan([(s * n, 0, n, s & 1) for s in range(B)]) as plan:
        ec.decode(k, m, mat, [m_d0, m_d1], data + parity, out, plan)
        torch.cuda.synchronize()
    assert torch.equal(out[0].view(B, n)[0::2], data[0].view(B, n)[0::2])
    assert torch.equal(out[1].view(B, n)[1::2], data[1].view(B, n)[1::2])
    assert int(out[2].count_nonzero()) == 0
    s = 1  # one stripe through the reference chain
    arenas = [to_host(x[s * n:(s + 1) * n]) for x in data + parity]
    ref = oracle.decode(mat, k, m, m_d1, [a if (m_d1 >> i) & 1 else None for i, a in enumerate(arenas)])
    assert np.array_equal(ref[0], to_host(out[1][s * n:(s + 1) * n]))
    _assert_parity_matches_oracle(torch, oracle, mat, k, m, data, parity)  # the whole 1 GiB batch


def test_cfg4_rs42_64k_roundtrip(gpu, oracle):
    """BASELINE configs[3] (per GPU): RS(4,2), 64 KiB values x 16,384 stripes (1 GiB per
    shard): the whole batch's parity equals the oracle's, and a double erasure (D0, D3)
    rebuilt from both parities equals the data."""
    torch, ec = gpu
    k, m, n, B = 4, 2, 65536, 16384
    mat = ec.coding_matrix(k, m)
    g = torch.Generator(device="cuda").manual_seed(0xC0C70004)
    data = [torch.randint(0, 256, (B * n,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    parity = [torch.empty(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    with ec.Plan([(s * n, 0, n, 0) for s in range(B)]) as plan:
        ec.encode(k, m, mat, data, parity, plan)
        torch.cuda.synchronize()
    # double erasure (D0, D3) from both parities, in place of the lost arenas
    mask = 0b110110
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    with ec.Plan([(0, 0, B * n // 2, 0), (B * n // 2, 0, B * n // 2, 0)]) as plan:
        ec.decode(k, m, mat, [mask], data + parity, out, plan)
        torch.cuda.synchronize()
    assert torch.equal(out[0], data[0]) and torch.equal(out[3], data[3])
    _assert_parity_matches_oracle(torch, oracle, mat, k, m, data, parity)


def _assert_parity_matches_oracle(torch, oracle, mat, k, m, data, parity):
    """Whole-batch parity == the oracle's (its AVX2 restatement of GF-Complete's region
    multiply, pinned to the scalar oracle on a sample first), compared on the device."""
    hostd = [to_host(x) for x in data]
    probe, ref = np.zeros(2 * 4096 + 7, np.uint8), np.zeros(2 * 4096 + 7, np.uint8)
    for j in range(k):
        oracle.region_multiply_simd(hostd[j][:probe.size], mat[(k + m - 1) * k + j], probe)
        oracle.region_multiply(hostd[j][:ref.size].copy(), mat[(k + m - 1) * k + j], ref, 1)
    assert np.array_equal(probe, ref)
    for p in range(m):
        exp = np.zeros(hostd[0].size, np.uint8)
        for j in range(k):
            oracle.region_multiply_simd(hostd[j], mat[(k + p) * k + j], exp)
        assert torch.equal(parity[p], to_dev(torch, exp)), f"parity {p}"


# ------------------------------------------------------------------ batched drain (§8f 1)
@pytest.mark.parametrize("staging", [64 << 20, 64 << 10])
def test_drainer_matches_sequential_loop(gpu, oracle, engine, staging):
    """cec_drainer_apply == the reference's drain loop (process_rep_command one diff at
    a time, memcached.c:7762-7767), including overlapping and ragged updates."""
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(staging & 0xFFFF)
    arena = 1 << 20
    parity = rng.integers(0, 256, arena, dtype=np.uint8)
    dev = to_dev(torch, parity)
    ups = []
    for i in range(400):
        n = int(rng.integers(1, 9000)) if i % 5 else 4098
        addr = int(rng.integers(0, (arena - n) // 16)) * 16 + (3 if i % 37 == 0 else 0)
        ups.append((rng.integers(0, 256, n, dtype=np.uint8), addr, int(rng.integers(0, k))))
    lid_self = k + 1
    with ec.Drainer(k, m, mat, lid_self, staging_bytes=staging) as d:
        launches = d.apply(ups, dev)
        launches2 = d.apply([], dev)
    assert launches >= 2 and launches2 == 0  # overlaps force several waves
    for buf, addr, j in ups:
        v = parity[addr:addr + buf.size].copy()
        oracle.parity_apply(mat, k, lid_self, j, buf, v)
        parity[addr:addr + buf.size] = v
    assert np.array_equal(to_host(dev), parity)


@pytest.mark.parametrize("arena_kind", ["device", "registered_host"])
def test_drainer_small_windows(gpu, oracle, arena_kind):
    """Windows of 1 to ~60 diffs -- the small-window path (one pass of the caller's thread
    into mapped staging, no pack threads or uploads) and, at the edges, the pack path: each
    window, overlapping and ragged updates included, leaves the arena as the reference's
    drain loop (memcached.c:7762-7767), in HBM and in a registered host arena (its results
    fenced for the host on return: read without a device sync)."""
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0x5A11 + len(arena_kind))
    arena = 1 << 20
    parity = rng.integers(0, 256, arena, dtype=np.uint8)
    host = None
    if arena_kind == "device":
        dev = to_dev(torch, parity)
    else:
        host = parity.copy()
        dev = ec.host_register(host)
    lid_self = k
    try:
        with ec.Drainer(k, m, mat, lid_self, staging_bytes=1 << 20) as d:
            for n_ups, max_len in ((1, 16), (1, 4098), (5, 9000), (40, 3000), (60, 4400), (80, 4098),
                                   (200, 8000), (300, 8000)):
                ups = []
                for i in range(n_ups):
                    ln = int(rng.integers(1, max_len + 1))
                    if i % 7 == 3 and ups:  # on top of an earlier one: a second wave
                        addr = min(ups[-1][1] + 16, arena - ln)
                    else:
                        addr = int(rng.integers(0, (arena - ln) // 16)) * 16 + (5 if i % 11 == 10 else 0)
                    ups.append((rng.integers(0, 256, ln, dtype=np.uint8), addr, int(rng.integers(0, k))))
                small = sum((b.size + 15) // 16 * 16 for b, _, _ in ups) <= 1 << 20
                d.apply(ups, dev)
                for buf, addr, j in ups:
                    v = parity[addr:addr + buf.size].copy()
                    oracle.parity_apply(mat, k, lid_self, j, buf, v)
                    parity[addr:addr + buf.size] = v
                if host is not None:  # on return, no device sync
                    assert np.array_equal(host, parity), (n_ups, max_len)
                    if small:  # the small-window path's completion: fenced for the host
                        sync = ec.last_sync()
                        assert (sync["host_results"], sync["fenced"]) == (1, 1)
                else:
                    assert np.array_equal(to_host(dev), parity), (n_ups, max_len)
    finally:
        if host is not None:
            ec.host_unregister(host)


def test_drainer_full_size(gpu, oracle):
    """The batched drain at the bench's size: 65,536 pending 4 KiB
    diffs in pageable host memory, source shard uniform in {0,1,2}, addresses shuffled
    over a 256 MiB parity arena, applied by one cec_drainer_apply (64 MiB staging: several
    rounds) == the reference's sequential drain loop (memcached.c:4350 -> 7764) run by the
    oracle over the same diffs."""
    torch, ec = gpu
    k, m, n, N = 3, 2, 4096, 65536
    mat = ec.coding_matrix(k, m)
    lid_self = k + 1
    rng = np.random.default_rng(0xC0C70001)
    diffs = rng.integers(0, 256, N * n, dtype=np.uint8)
    src = rng.integers(0, k, N)
    addrs = rng.permutation(N).astype(np.uint64) * n
    parity0 = rng.integers(0, 256, N * n, dtype=np.uint8)
    parity = to_dev(torch, parity0)
    with ec.Drainer(k, m, mat, lid_self, staging_bytes=64 << 20) as d:
        launches = d.apply([(diffs[i * n:(i + 1) * n], int(addrs[i]), int(src[i])) for i in range(N)], parity)
    torch.cuda.synchronize()
    want = parity0.copy()
    oracle.bench_apply(diffs, np.arange(N, dtype=np.uint64) * n, addrs, np.full(N, n),
                       [mat[lid_self * k + int(j)] for j in src], want)
    assert launches >= 4  # 256 MiB of diffs through 64 MiB of staging
    assert torch.equal(parity, to_dev(torch, want))


def test_drainer_in_place_staging(gpu, oracle):
    """Diffs received straight into the drainer's pinned staging are applied without the
    pack copy (overlapping and ragged ones included), same bytes as the sequential loop."""
    torch, ec = gpu
    k, m = 4, 2
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(21)
    arena = 1 << 20
    parity = rng.integers(0, 256, arena, dtype=np.uint8)
    dev = to_dev(torch, parity)
    with ec.Drainer(k, m, mat, k, staging_bytes=1 << 20) as d:
        base, view = d.staging()
        assert view.size == 2 << 20
        ups, so = [], 0
        for i in range(300):
            n = int(rng.integers(1, 7000))
            addr = int(rng.integers(0, (arena - n) // 16)) * 16
            view[so:so + n] = rng.integers(0, 256, n, dtype=np.uint8)  # "recv" into staging
            ups.append((base + so, addr, int(rng.integers(0, k)), n))
            so = (so + n + 15) & ~15
        expect = [(view[u[0] - base:u[0] - base + u[3]].copy(), u[1], u[2]) for u in ups]
        d.apply(ups, dev)
    for buf, addr, j in expect:
        v = parity[addr:addr + buf.size].copy()
        oracle.parity_apply(mat, k, k, j, buf, v)
        parity[addr:addr + buf.size] = v
    assert np.array_equal(to_host(dev), parity)


def test_drainer_rejects_bad_updates(gpu):
    torch, ec = gpu
    mat = ec.coding_matrix(3, 2)
    dev = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    with ec.Drainer(3, 2, mat, 3, staging_bytes=8192) as d:
        with pytest.raises(ec.CecError):
            d.apply([(np.zeros(10000, np.uint8), 0, 0)], dev)  # larger than staging
        with pytest.raises(ec.CecError):
            d.apply([(np.zeros(16, np.uint8), 0, 3)], dev)  # src lid is a parity
    with pytest.raises(ec.CecError):
        ec.Drainer(3, 2, mat, 1)  # a data lid cannot drain


# ------------------------------------------------------------------ recovery sessions (§8f 2)
@pytest.mark.parametrize("host_inputs", [True, False])
def test_recovery_session_single_loss_with_updates(gpu, oracle, host_inputs):
    """D0 lost, leader P0 (mask {D1, D2, P0}); writes from D1/D2 land while the
    recovery is in flight (recovery.c:99-131); the rebuilt D0 equals the live data."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(8 + host_inputs)
    nunits, ub, ue = 96, 10, 73
    data = [rng.integers(0, 256, nunits * U, dtype=np.uint8) for _ in range(k)]
    parity = oracle.encode(mat, k, m, data)
    p0 = to_dev(torch, parity[0])
    mask = oracle.recovery_mask(k, m, 3, [0, 1, 1, 1, 1])
    lo, hi = ub * U, (ue + 1) * U

    def land_update(rec, s):  # a SET on data peer s: diff to the parity (+ fold)
        n = int(rng.integers(1, 9000))
        addr = int(rng.integers(lo - 5000, hi - n + 5000)) // 16 * 16
        addr = max(0, min(addr, nunits * U - n))
        new = rng.integers(0, 256, n, dtype=np.uint8)
        diff = oracle.set_diff(data[s][addr:addr + n].copy(), new)
        data[s][addr:addr + n] = new
        rec.fold_update(s, addr, diff if host_inputs else to_dev(torch, diff))
        ec.region_multiply(to_dev(torch, diff), mat[3 * k + s], n, p0.data_ptr() + addr, 1)  # memcached.c:7764
        torch.cuda.synchronize()

    with ec.Recovery(k, m, mat, 3, mask, ub, ue, p0) as rec:
        assert rec.nbytes == hi - lo and not rec.complete
        land_update(rec, 1)                      # before any peer: picked up at first touch
        units1 = data[1][lo:hi].copy()
        rec.add_peer(1, units1 if host_inputs else to_dev(torch, units1))
        land_update(rec, 1)                      # peer 1 already sent: no fold
        land_update(rec, 2)                      # peer 2 not yet: folded
        land_update(rec, 2)
        assert not rec.complete
        units2 = data[2][lo:hi].copy()
        rec.add_peer(2, units2 if host_inputs else to_dev(torch, units2))
        assert rec.complete
        with pytest.raises(ec.CecError):
            rec.add_peer(2, units2)              # recovery.c:75 asserts a peer applies once
        if host_inputs:
            out = np.zeros(hi - lo, np.uint8)
            rec.solve({}, {0: out})
        else:
            dout = torch.zeros(hi - lo, dtype=torch.uint8, device="cuda")
            rec.solve({}, {0: dout})
            out = to_host(dout)
    assert np.array_equal(out, data[0][lo:hi])


def test_recovery_sessions_double_loss_leader_solve(gpu, oracle):
    """D0 and D1 lost; P0 and P1 each build a residual from D2; the leader P0 solves with
    P1's residual shipped as host bytes (recover_units_gather) -> both shards rebuilt;
    residuals equal the reference chain (recovery_recover_units)."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    n = 40 * U
    data = [oracle.splitmix_bytes(0xC0C70005 + j, n) for j in range(k)]
    parity = oracle.encode(mat, k, m, data)
    pdev = [to_dev(torch, p) for p in parity]
    mask = 0b11100
    with ec.Recovery(k, m, mat, 3, mask, 0, 39, pdev[0]) as r0, \
         ec.Recovery(k, m, mat, 4, mask, 0, 39, pdev[1]) as r1:
        r0.add_peer(2, data[2])
        r1.add_peer(2, data[2])
        tmp = torch.empty(n, dtype=torch.uint8, device="cuda")
        res = {}
        for p, rec in ((3, r0), (4, r1)):
            ec.region_multiply(rec.residual, 1, n, tmp, 0)  # copy the device residual out
            torch.cuda.synchronize()
            res[p] = to_host(tmp)
            exp = np.empty(n, np.uint8)
            touched = [0]
            oracle.recover_units(mat, k, p, 2, parity[p - k], data[2], exp, touched)
            assert np.array_equal(res[p], exp), p
        res1 = res[4]
        out0, out1 = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
        r0.solve({4: res1}, {0: out0, 1: out1})
    assert np.array_equal(out0, data[0]) and np.array_equal(out1, data[1])


# ------------------------------------------------------------------ the drop-in symbols
def test_dropin_host_buffers(gpu, oracle):
    """galois_w08_region_multiply on pageable host memory at arbitrary alignment."""
    _, ec = gpu
    rng = np.random.default_rng(11)
    for n in [1, 2, 4095, 4098, 8194, 12289, 40000, 65537, 3 << 20]:
        for so, do in [(0, 0), (5, 9), (16, 3)]:
            for c in [1, 2, 245, 0]:
                buf = rng.integers(0, 256, n + 32, dtype=np.uint8)
                dst = rng.integers(0, 256, n + 32, dtype=np.uint8)
                exp = dst.copy()
                v = exp[do:do + n].copy()
                oracle.region_multiply(buf[so:so + n].copy(), c, v, 1)
                exp[do:do + n] = v
                ec.galois_w08_region_multiply(buf[so:], c, n, dst[do:], 1)
                bad = np.flatnonzero(dst != exp)
                assert bad.size == 0, (n, so, do, c, bad.size, bad[:8].tolist(), bad[-8:].tolist())
                if c:  # zero-copy: the waves release the mapped staging; staged: DMA + sync
                    rec = ec.last_sync()
                    want = (1, 1, 0) if n <= 256 << 10 else (1, 0, 1)
                    assert (rec["host_results"], rec["waves_released"], rec["fenced"]) == want, (n, rec)


def test_dropin_mixed_buffers(gpu, oracle):
    """One operand on the device and the other in pageable or pinned host memory, ragged
    and misaligned: each combination takes its own path (staged, zero-copy, in place over
    PCIe), and the host-side result must be complete when the call returns (the
    completion signal follows a system-scope release)."""
    torch, ec = gpu
    rng = np.random.default_rng(0x3B)
    for n in [4098, 9000, 300001]:
        a = rng.integers(0, 256, n + 16, dtype=np.uint8)
        b = rng.integers(0, 256, n + 16, dtype=np.uint8)
        exp = b.copy()
        v = exp[3:3 + n].copy()
        oracle.region_multiply(a[5:5 + n].copy(), 0x53, v, 1)
        exp[3:3 + n] = v
        # device source, pageable destination
        da = to_dev(torch, a)
        got = b.copy()
        ec.galois_w08_region_multiply(da[5:], 0x53, n, got[3:], 1)
        assert np.array_equal(got, exp), ("device -> pageable", n)
        # pageable source, device destination
        db = to_dev(torch, b)
        ec.galois_w08_region_multiply(a[5:], 0x53, n, db[3:], 1)
        assert np.array_equal(to_host(db), exp), ("pageable -> device", n)
        # pinned source and destination: in place, the kernel writes host memory
        pa = torch.from_numpy(a.copy()).pin_memory()
        pb = torch.from_numpy(b.copy()).pin_memory()
        ec.galois_w08_region_multiply(pa[5:], 0x53, n, pb[3:], 1)
        rec = ec.last_sync()
        assert (rec["host_results"], rec["waves_released"], rec["fenced"]) == (1, 1, 0), (n, rec)
        assert np.array_equal(pb.numpy(), exp), ("pinned -> pinned", n)


def _hip_lib(ec):
    """The HIP runtime already mapped into this process (torch's), via ctypes."""
    import ctypes

    rts = sorted(ec._hip_runtimes())
    assert len(rts) == 1, rts
    L = ctypes.CDLL(rts[0])
    L.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    L.hipHostFree.argtypes = [ctypes.c_void_p]
    L.hipMallocManaged.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    L.hipFree.argtypes = [ctypes.c_void_p]
    return L


HOST_KINDS = {  # hipHostMalloc flags (hip_runtime_api.h)
    "mapped_coherent": 0x2 | 0x40000000,  # the library's own zero-copy staging
    "coherent": 0x40000000,
    "default": 0x0,  # torch's pin_memory
    "noncoherent": 0x80000000,  # cached in the GPU's L2 on every box
}


@pytest.mark.parametrize("kind", sorted(HOST_KINDS) + ["managed"])
def test_dropin_host_result_visible_from_every_xcd(gpu, oracle, kind):
    """Round 2's stale-tile defect, box-independent: a drop-in call whose 65 tiles run on
    every XCD writes a destination the host reads on return, with no synchronisation.
    Round 2's completion signal wrote back only its own XCD's L2, which lost tiles only
    on boxes whose host mappings the L2 caches; non-coherent pinned memory is cached on
    every box, and managed memory is read by the host in place.  Every
    writing wave must release its own XCD's L2 (kSysRel) for all of them."""
    import ctypes

    torch, ec = gpu
    L = _hip_lib(ec)
    n = 65 * 4096 - 14  # 65 tiles, the last ragged: workgroups on all 8 XCDs
    p = ctypes.c_void_p()
    rc = (L.hipMallocManaged(ctypes.byref(p), n, 1) if kind == "managed"
          else L.hipHostMalloc(ctypes.byref(p), n, HOST_KINDS[kind]))
    assert rc == 0 and p.value, (kind, rc)
    try:
        dst = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p.value))
        rng = np.random.default_rng(0x5CA1)
        for rep in range(24):
            src = rng.integers(0, 256, n, dtype=np.uint8)
            dsrc = to_dev(torch, src)
            torch.cuda.synchronize()
            dst[:] = rng.integers(0, 256, n, dtype=np.uint8)
            exp = dst.copy()
            c = [1, 2, 245, 0x53][rep % 4]
            oracle.region_multiply(src, c, exp, 1)
            ec.galois_w08_region_multiply(dsrc, c, n, p.value, 1)
            bad = np.flatnonzero(dst != exp)  # read on return: no synchronize
            assert bad.size == 0, (kind, rep, c, bad.size, sorted(set((bad // 4096).tolist()))[:16])
            # the protocol itself, on any box (round 2's defect was a missing release that
            # only some boxes' host mappings exposed): every writing wave released its
            # XCD's L2, and no fence event was spent on top of it
            rec = ec.last_sync()
            assert (rec["host_results"], rec["waves_released"], rec["fenced"]) == (1, 1, 0), (kind, rec)
    finally:
        torch.cuda.synchronize()
        (L.hipFree if kind == "managed" else L.hipHostFree)(p)


def test_dropin_device_buffers(gpu, oracle):
    torch, ec = gpu
    a = oracle.splitmix_bytes(1, 10000)
    b = oracle.splitmix_bytes(2, 10000)
    exp = b.copy()
    oracle.region_multiply(a, 0x8E, exp, 1)
    da, db = to_dev(torch, a), to_dev(torch, b)
    ec.galois_w08_region_multiply(da, 0x8E, 10000, db, 1)
    rec = ec.last_sync()  # a device result: neither release nor fence is paid for
    assert (rec["host_results"], rec["waves_released"], rec["fenced"]) == (0, 0, 0), rec
    assert np.array_equal(to_host(db), exp)


def test_dropin_c_program(gpu, oracle, tmp_path):
    """A C program written against include/{galois,jerasure,reed_sol}.h and linked with
    -lJerasure (the shim) replays the reference's call chain; outputs vs the oracle."""
    from tests.dropin import run_dropin_case

    run_dropin_case(oracle, tmp_path)


def test_dropin_after_daemonize_fork(gpu, tmp_path):
    """memcached builds the matrix (memcached.c:6845) before it daemonizes with fork()
    (:6946-6955): the shim's host-only symbols must leave the GPU untouched so that the
    daemon child's first galois_w08_region_multiply can open it."""
    from tests.dropin import run_dropin_daemon

    assert "child 0 mismatches" in run_dropin_daemon(tmp_path)


def test_dropin_reentrant_threads(gpu, tmp_path):
    """8 pthreads call the drop-in concurrently (all four argument forms, sizes up to
    300 KB so both the zero-copy and the staged path run, odd alignments); each checks
    against its own scalar GF(2^8)."""
    from tests.dropin import run_dropin_threads

    out = run_dropin_threads(tmp_path, threads=8, iters=150)
    assert "0 mismatches" in out


def test_arena_allocator(gpu, oracle):
    """cec_arenas_alloc: count arenas at an odd-4 KiB stride, usable by every op."""
    import ctypes

    torch, ec = gpu
    for nbytes, want in [(1, 4096), (4096, 4096), (8192, 12288), (256 << 20, (256 << 20) + 4096)]:
        assert ec.arena_stride(nbytes) == want
    k, m, n = 3, 2, 3 * 4096
    arr = (ctypes.c_void_p * (k + m))()
    slab = ctypes.c_void_p()
    assert ec.lib().cec_arenas_alloc(k + m, n, arr, ctypes.byref(slab)) == 0
    stride = ec.arena_stride(n)
    assert [arr[i] - arr[0] for i in range(k + m)] == [i * stride for i in range(k + m)]
    host = [oracle.splitmix_bytes(70 + j, n) for j in range(k)]
    for j in range(k):
        src = to_dev(torch, host[j])
        ec.region_multiply(src, 1, n, arr[j], 0)  # copy into arena j
    mat = ec.coding_matrix(k, m)
    ec.encode_region(k, m, mat, [arr[j] for j in range(k)], [arr[k + p] for p in range(m)], n)
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, host)
    for p in range(m):
        got = torch.empty(n, dtype=torch.uint8, device="cuda")
        ec.region_multiply(arr[k + p], 1, n, got, 0)
        torch.cuda.synchronize()
        assert np.array_equal(to_host(got), exp[p])
    assert ec.lib().cec_arenas_free(slab) == 0
    views = ec.arena_tensors(4, 100)
    assert all(v.numel() == 100 for v in views)
    assert views[1].data_ptr() - views[0].data_ptr() == 4096


@pytest.mark.parametrize("shift", [0, 1, 2])
def test_forced_split_shift(gpu, oracle, shift):
    """Every workgroups-per-tile choice (1, 2, 4) is bit-exact on aligned, ragged and
    misaligned tiles, not only the one the automatic rule picks (cec_runtime.hip
    split_shift_for).  Child process: the library reads CEC_SPLIT_SHIFT once."""
    env = dict(os.environ, CEC_SPLIT_SHIFT=str(shift))
    r = subprocess.run(["python", os.path.join(ROOT, "tests", "split_case.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("env,expect", [({"CEC_STORE_POLICY": "nt"}, "nt:%d" % (512 << 20)),
                                        ({"CEC_STORE_POLICY": "wt"}, "wt:%d" % (512 << 20)),
                                        ({"CEC_WT_MAX_BYTES": "0"}, "auto:0")])
def test_store_policy_every_kernel_kind(gpu, oracle, env, expect):
    """Both store paths of every kernel kind are bit-exact: under the default
    policy the suite's small launches all take write-through stores, so the non-temporal
    path is forced here (CEC_STORE_POLICY=nt, and auto with a 0-byte write-through limit),
    and write-through pinned too.  Child process: the library reads the policy once."""
    e = {x: v for x, v in os.environ.items() if x not in ("CEC_STORE_POLICY", "CEC_WT_MAX_BYTES")}
    e.update(env, CEC_EXPECT_POLICY=expect)
    r = subprocess.run(["python", os.path.join(ROOT, "tests", "split_case.py")], env=e,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout[-2000:] + r.stderr[-2000:]


def test_pinned_host_arenas_zero_copy(gpu, oracle):
    """bench.py --e2e-zero-copy: pinned host buffers used as arenas by the batched ops
    (the kernels read and write them over PCIe); encode, then a decode of every mask
    reading the parity the encode just wrote to host memory, ragged values included."""
    torch, ec = gpu
    k, m = 3, 2
    rng = np.random.default_rng(77)
    lens = [4096] * 40 + [1, 17, 4098, 300, 65536 + 5]
    ext, arena, _ = make_extents(rng, lens)
    mat = ec.coding_matrix(k, m)
    host = [rng.integers(0, 256, arena, dtype=np.uint8) for _ in range(k)]

    def pin(a):
        return torch.from_numpy(a.copy()).pin_memory()

    data = [pin(h) for h in host]
    parity = [pin(np.full(arena, SENT, np.uint8)) for _ in range(m)]
    out = [pin(np.full(arena, SENT, np.uint8)) for _ in range(k)]
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    with ec.Plan([(o, 0, n, 0) for o, _, n, _ in ext]) as ep, \
         ec.Plan([(o, 0, n, i % len(masks)) for i, (o, _, n, _) in enumerate(ext)]) as dp:
        ec.encode(k, m, mat, data, parity, ep)
        ec.decode(k, m, mat, masks, data + parity, out, dp)
        torch.cuda.synchronize()
    exp = [np.full(arena, SENT, np.uint8) for _ in range(m)]
    for o, _, n, _ in ext:
        seg = oracle.encode(mat, k, m, [h[o:o + n].copy() for h in host])
        for p in range(m):
            exp[p][o:o + n] = seg[p]
    for p in range(m):
        assert np.array_equal(parity[p].numpy(), exp[p]), p
    for i, (o, _, n, _) in enumerate(ext):
        j = [x for x in range(k) if not (masks[i % len(masks)] >> x) & 1][0]
        assert np.array_equal(out[j].numpy()[o:o + n], host[j][o:o + n]), i


def test_registered_host_arena_zero_copy(gpu, oracle):
    """an arena left in malloc'd host memory, registered once with
    hipHostRegister(mapped), used through its device alias as the parity arena of
    cec_apply_diffs (the parity server's drain) and as the data arenas of cec_encode."""
    import ctypes

    torch, ec = gpu
    rt = sorted(ec._hip_runtimes())
    assert len(rt) == 1, rt
    hip = ctypes.CDLL(rt[0])
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    k, m, n, B = 3, 2, 4096, 64
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(5)
    def page_aligned(nbytes):
        raw = np.empty(nbytes + 4096, np.uint8)
        o = (-raw.ctypes.data) % 4096
        return raw[o:o + nbytes]

    arenas = []
    for _ in range(k + m):
        a = page_aligned(B * n)
        a[:] = rng.integers(0, 256, B * n, dtype=np.uint8)
        arenas.append(a)
    orig = [a.copy() for a in arenas]
    alias = []
    try:
        for a in arenas:
            assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 2) == 0  # hipHostRegisterMapped
            d = ctypes.c_void_p()
            assert hip.hipHostGetDevicePointer(ctypes.byref(d), a.ctypes.data, 0) == 0
            alias.append(d.value)
        with ec.Plan([(s * n, 0, n, 0) for s in range(B)]) as ep:
            ec.encode(k, m, mat, alias[:k], alias[k:], ep)
            torch.cuda.synchronize()
        exp = oracle.encode(mat, k, m, orig[:k])
        for p in range(m):
            assert np.array_equal(arenas[k + p], exp[p]), p
        # a drain of shipped diffs into the registered parity arena P1 (lid k + 1)
        diffs = rng.integers(0, 256, B * n, dtype=np.uint8)
        ddev = to_dev(torch, diffs)
        ext = [(s * n, s * n, n, s % k) for s in range(B)]
        want = arenas[k + 1].copy()
        for off, soff, ln, j in ext:
            w = want[off:off + ln].copy()
            oracle.parity_apply(mat, k, k + 1, j, diffs[soff:soff + ln].copy(), w)
            want[off:off + ln] = w
        with ec.Plan(ext) as ap:
            ec.apply_diffs(k, m, mat, k + 1, ddev, alias[k + 1], ap)
            torch.cuda.synchronize()
        assert np.array_equal(arenas[k + 1], want)
    finally:
        for a in arenas[:len(alias)]:
            hip.hipHostUnregister(a.ctypes.data)


def test_native_metric_harness(gpu, tmp_path):
    """tools/bench_native.c, the metric's step through the C-ABI alone (C99, no HIP
    header, no torch): 65,536 RS(3,2) stripes encoded and decoded with rotating
    erasures; it checks every rebuilt shard against its original itself.  Then its
    thread-per-GPU mode with two threads pinned to this one card (CEC_NATIVE_DEVICE):
    barrier-aligned start, max over threads, both batches verified."""
    import json

    exe = str(tmp_path / "bench_native")
    subprocess.run(["gcc", "-O2", "-std=c99", "-D_POSIX_C_SOURCE=200809L", "-Wall", "-Werror", "-pthread",
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tools", "bench_native.c"),
                    "-L", os.path.join(ROOT, "cocytus_amd"), "-lcocytus_ec",
                    "-Wl,-rpath," + os.path.join(ROOT, "cocytus_amd"), "-o", exe], check=True)
    r = subprocess.run([exe, "2", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    out = json.loads(r.stdout)
    assert out["verified"] is True and out["n_gpus"] == 1
    env = dict(os.environ, CEC_NATIVE_DEVICE="0")
    r = subprocess.run([exe, "2", "1", "2"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr + r.stdout
    out = json.loads(r.stdout)
    assert out["verified"] is True and out["n_gpus"] == 2


def test_bench_two_ranks_one_card_weak_and_strong(gpu):
    """bench.py --gpus 2 (the driver's multi-GPU entry point) with both ranks on this one
    card (gloo): one JSON line, n_gpus 2, the weak line verified and the fixed-batch
    `strong` record (32,768 stripes per rank) verified.  Short steps: this
    checks the path, not the rates (two ranks share one card)."""
    import json

    env = {x: v for x, v in os.environ.items()
           if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["CEC_BENCH_DEVICE"] = "0"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--also=", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["verified"] is True
    st = out["strong"]
    assert st["n_gpus"] == 2 and st["stripes_per_gpu"] == 32768 and st["verified"] is True
    assert st["value"] > 0
    # the per-rank evidence: both ranks on one card, so the line must NOT pass for a
    # 2-GPU run; each rank's own step times and identity are carried
    rk = out["ranks"]
    assert rk["world_size"] == 2 and rk["backend"] == "gloo" and rk["distinct_devices"] is False
    ids = [e["identity"] for e in rk["per_rank"]]
    assert ids[0]["uuid"] == ids[1]["uuid"] and ids[0]["pci"] == ids[1]["pci"] and ids[0]["arch"] == "gfx950"
    for e in rk["per_rank"]:
        assert e["weak"]["ms_per_step"] > 0 and e["weak"]["encode_ms"] > 0 and e["weak"]["decode_ms"] > 0
        assert e["strong"]["ms_per_step"] > 0 and e["strong"]["verified"] is True
    assert [e["strong"]["stripes"] for e in rk["per_rank"]] == [[0, 32768], [32768, 65536]]
    assert max(e["weak"]["ms_per_step"] for e in rk["per_rank"]) == pytest.approx(out["ms_per_step"], rel=1e-3)
    assert rk["slowest_rank_weak"] in (0, 1) and rk["slowest_rank_strong"] in (0, 1)


def test_cfg4_eight_rank_batches_one_card(gpu):
    """BASELINE configs[3] ("RS(4,2) parity encode, 64 KiB values, 8 x MI355X, independent
    batches sharded per GPU") through the driver's multi-GPU entry point with its 8 ranks
    on this one card (gloo, CEC_BENCH_DEVICE=0): each rank encodes its own 16,384-stripe
    batch (seeded per rank) and rebuilds a rotating lost shard of every stripe, checked
    byte for byte on the device; the line reports all 8 ranks verified, n_gpus 8, and,
    correctly, distinct_devices false.  (The rates are not scaling numbers: the ranks
    share one card.)"""
    import json

    env = {x: v for x, v in os.environ.items()
           if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["CEC_BENCH_DEVICE"] = "0"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--workload", "rs42_64k",
                        "--steps", "2", "--warmup", "1", "--also=", "--no-strong", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 8 and out["verified"] is True
    assert out["config"]["k"] == 4 and out["config"]["m"] == 2 and out["config"]["stripes_per_gpu"] == 16384
    rk = out["ranks"]
    assert rk["world_size"] == 8 and rk["distinct_devices"] is False
    assert [e["rank"] for e in rk["per_rank"]] == list(range(8))
    assert all(e["weak"]["verified"] for e in rk["per_rank"])


def test_bench_rccl_path_one_rank(gpu):
    """The N > 1 line's RCCL path on this one card: CEC_BENCH_PG=1 brings up a one-rank
    nccl (= RCCL) process group with the device bound (init_process_group(device_id=)),
    so the barriers, the all_reduce MAX over ranks and the all_gather of the per-rank
    evidence all run through RCCL as they do for the driver's N-GPU run (two ranks on one
    card is refused by RCCL, hence one)."""
    import json

    env = {x: v for x, v in os.environ.items()
           if x not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "CEC_BENCH_DEVICE")}
    env["CEC_BENCH_PG"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--also=rs32_diff_update,rs32_1m_recovery", "--no-cpu-baseline", "--dist-backend", "nccl"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 1 and out["verified"] is True
    rk = out["ranks"]
    assert rk["backend"] == "nccl" and rk["world_size"] == 1 and rk["distinct_devices"] is True
    e = rk["per_rank"][0]
    assert e["identity"]["arch"] == "gfx950" and e["weak"]["ms_per_step"] == pytest.approx(out["ms_per_step"], rel=1e-3)
    assert set(e["other_workloads"]) == {"rs32_diff_update", "rs32_1m_recovery"}


def test_graph_capture_replay(gpu, oracle):
    """An encode + decode step captured into a HIP graph (torch.cuda.graph) replays
    bit-exactly; the coefficient tables are cached by a warm-up call before capture."""
    torch, ec = gpu
    k, m, n, B = 3, 2, 4096, 512
    mat = ec.coding_matrix(k, m)
    host = [oracle.splitmix_bytes(0xC0C70002 + j, B * n) for j in range(k)]
    data = [to_dev(torch, h) for h in host]
    parity = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    ep = ec.Plan([(s * n, 0, n, 0) for s in range(B)])
    dp = ec.Plan([(s * n, 0, n, s % 6) for s in range(B)])
    ec.encode(k, m, mat, data, parity, ep)  # warm the pattern cache (no allocation in capture)
    ec.decode(k, m, mat, masks, data + parity, out, dp)
    torch.cuda.synchronize()
    for t in parity + out:
        t.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream()
        ec.encode(k, m, mat, data, parity, ep, s)
        ec.decode(k, m, mat, masks, data + parity, out, dp, s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, host)
    for p in range(m):
        assert np.array_equal(to_host(parity[p]), exp[p])
    for q, mk in enumerate(masks):
        j = [x for x in range(k) if not (mk >> x) & 1][0]
        sel = torch.arange(q, B, len(masks), device="cuda")
        assert torch.equal(out[j].view(B, n)[sel], data[j].view(B, n)[sel])
    ep.destroy()
    dp.destroy()


def test_edge_cases(gpu, oracle, engine):
    """Empty plans and zero-length extents, k+m at the limit, bad masks / patterns."""
    torch, ec = gpu
    k, m = 16, 8  # CEC_MAX_K, CEC_MAX_M
    mat = ec.coding_matrix(k, m)
    assert mat == oracle.big_vandermonde(k + m, k)
    n = 3 * 4096 + 5
    data = [oracle.splitmix_bytes(500 + j, n) for j in range(k)]
    ddev = [to_dev(torch, d) for d in data]
    pdev = [to_dev(torch, np.zeros(n, np.uint8)) for _ in range(m)]
    with ec.Plan([(0, 0, n, 0), (0, 0, 0, 0)]) as plan:  # a zero-length extent
        ec.encode(k, m, mat, ddev, pdev, plan)
        torch.cuda.synchronize()
    exp = oracle.encode(mat, k, m, data)
    for p in range(m):
        assert np.array_equal(to_host(pdev[p]), exp[p])
    # k = 16 decode of 8 lost data shards (max width: 16 inputs x 8 outputs)
    mask = sum(1 << x for x in list(range(8, 16)) + list(range(16, 24)))
    odev = [to_dev(torch, np.zeros(n, np.uint8)) for _ in range(k)]
    with ec.Plan([(0, 0, n, 0)]) as plan:
        ec.decode(k, m, mat, [mask], ddev + pdev, odev, plan)
        torch.cuda.synchronize()
    for j in range(8):
        assert np.array_equal(to_host(odev[j]), data[j]), j
    with ec.Plan([]) as empty:  # empty plan: every op is a no-op
        assert empty.num_tiles == 0
        ec.encode(k, m, mat, ddev, pdev, empty)
    with ec.Plan([(0, 0, 16, 1)]) as plan:
        with pytest.raises(ec.CecError):  # pattern index beyond the masks given
            ec.decode(3, 2, ec.coding_matrix(3, 2), [0b01110], ddev[:5], odev[:3], plan)
        with pytest.raises(ec.CecError):  # mask without k members
            ec.decode(3, 2, ec.coding_matrix(3, 2), [0b00011, 0b0111], ddev[:5], odev[:3], plan)
    with pytest.raises(ec.CecError):
        ec.encode_region(17, 2, [1] * 19 * 17, ddev[:17] + [ddev[0]], pdev[:2], 16)


# ------------------------------------------------------------------ randomized sweep
@pytest.mark.parametrize("seed", range(12))
def test_fuzz_random_plans(gpu, oracle, seed):
    """Random code, engine, extent sizes / offsets and arena base misalignment, for
    encode, diff-update and decode in one pass; every byte checked against the oracle."""
    torch, ec = gpu
    rng = np.random.default_rng(0xF022 + seed)
    k = int(rng.integers(2, 9))
    m = int(rng.integers(1, 5))
    default = ec.get_engine()
    ec.set_engine(ec.CEC_ENGINE_LDS if seed % 2 else ec.CEC_ENGINE_PERM)
    try:
        mat = ec.coding_matrix(k, m)
        kind = rng.choice(["small", "tiles", "large"])
        hi = {"small": 300, "tiles": 9000, "large": 200000}[kind]
        lens = [int(x) for x in rng.integers(0, hi, int(rng.integers(1, 40)))]
        ext, arena_len, stage_len = make_extents(rng, lens, unaligned_every=int(rng.integers(0, 5)))
        shift = int(rng.integers(0, 16)) if seed % 3 == 0 else 0  # misaligned arena bases

        def dev(a):
            buf = torch.zeros(a.size + shift, dtype=torch.uint8, device="cuda")
            view = buf[shift:]
            view.copy_(torch.from_numpy(np.ascontiguousarray(a)))
            return view

        data = [rng.integers(0, 256, arena_len, dtype=np.uint8) for _ in range(k)]
        ddev = [dev(d) for d in data]
        pdev = [dev(np.full(arena_len, SENT, np.uint8)) for _ in range(m)]
        with ec.Plan([tuple(e) for e in ext]) as plan:
            ec.encode(k, m, mat, ddev, pdev, plan)
            torch.cuda.synchronize()
        parity = [np.full(arena_len, SENT, np.uint8) for _ in range(m)]
        for off, _, n, _ in ext:
            if n:
                ps = oracle.encode(mat, k, m, [d[off:off + n].copy() for d in data])
                for p in range(m):
                    parity[p][off:off + n] = ps[p]
        for p in range(m):
            assert np.array_equal(to_host(pdev[p]), parity[p]), ("encode", p)
        # diff-update with install on a random source shard per extent
        for e in ext:
            e[3] = int(rng.integers(0, k))
        staging = rng.integers(0, 256, stage_len, dtype=np.uint8)
        with ec.Plan([tuple(e) for e in ext]) as plan:
            ec.diff_update(k, m, mat, ddev, dev(staging), pdev, True, plan)
            torch.cuda.synchronize()
        for off, soff, n, j in ext:
            if not n:
                continue
            old = data[j][off:off + n].copy()
            pv = [p[off:off + n].copy() for p in parity]
            oracle.diff_update(mat, k, m, j, old, staging[soff:soff + n].copy(), pv, True)
            data[j][off:off + n] = old
            for p in range(m):
                parity[p][off:off + n] = pv[p]
        for j in range(k):
            assert np.array_equal(to_host(ddev[j]), data[j]), ("diff_update data", j)
        for p in range(m):
            assert np.array_equal(to_host(pdev[p]), parity[p]), ("diff_update parity", p)
        # decode under a random mask per extent
        masks = list(all_masks(k, m))
        pick = rng.choice(len(masks), min(len(masks), 6), replace=False)
        masks = [masks[int(i)] for i in pick]
        for e in ext:
            e[3] = int(rng.integers(0, len(masks)))
        odev = [dev(np.full(arena_len, SENT, np.uint8)) for _ in range(k)]
        with ec.Plan([tuple(e) for e in ext]) as plan:
            ec.decode(k, m, mat, masks, ddev + pdev, odev, plan)
            torch.cuda.synchronize()
        out = [np.full(arena_len, SENT, np.uint8) for _ in range(k)]
        for off, _, n, q in ext:
            if not n:
                continue
            for j in range(k):
                if not (masks[q] >> j) & 1:
                    out[j][off:off + n] = data[j][off:off + n]
        for j in range(k):
            assert np.array_equal(to_host(odev[j]), out[j]), ("decode", j)
    finally:
        ec.set_engine(default)


# ------------------------------------------------------------------ reference allocator layout
def test_reference_allocator_layout(gpu, oracle, engine):
    """SETs placed by the reference's own allocator (tests/golden/ecalloc_layout.npz,
    from /root/reference/ecalloc.c after churn): per-shard fused diff-update with
    install, and the parity drain of the same diffs across shards (overlapping in the
    parity arena, memcached.c:7704-7717), each equal to the reference's chain."""
    torch, ec = gpu
    z = np.load(os.path.join(ROOT, "tests", "golden", "ecalloc_layout.npz"))
    sets = [tuple(int(x) for x in row) for row in z["sets"]]
    k, m = int(z["k"]), 2
    mat = ec.coding_matrix(k, m)
    arena = ((max(a + n for _, a, n in sets) + 4095) // 4096) * 4096
    rng = np.random.default_rng(0xA10)
    data = [rng.integers(0, 256, arena, dtype=np.uint8) for _ in range(k)]  # stale bytes
    parity = oracle.encode(mat, k, m, data)
    news, soff, ext = [], 0, {j: [] for j in range(k)}
    for j, a, n in sets:
        news.append(rng.integers(0, 256, n, dtype=np.uint8))
        ext[j].append((a, soff, n, j))
        soff = (soff + n + 15) & ~15
    staging = np.zeros(soff, np.uint8)
    so_of = {}
    for j in range(k):
        for a, so, n, _ in ext[j]:
            so_of[(j, a)] = so
    for (j, a, n), v in zip(sets, news):
        staging[so_of[(j, a)]:so_of[(j, a)] + n] = v
    ddev = [to_dev(torch, d) for d in data]
    pdev = [to_dev(torch, p) for p in parity]
    sdev = to_dev(torch, staging)
    p_drain = to_dev(torch, parity[1])
    # the shipped diffs (new ^ stale old bytes at the fresh address, memcached.c:2673-2681)
    diffs = [(oracle.set_diff(data[j][a:a + n].copy(), v), a, j) for (j, a, n), v in zip(sets, news)]
    for j in range(k):  # one launch per shard: its SETs never overlap each other
        with ec.Plan(ext[j]) as plan:
            ec.diff_update(k, m, mat, ddev, sdev, pdev, True, plan)
    with ec.Drainer(k, m, mat, k + 1, staging_bytes=8 << 20) as d:
        launches = d.apply(diffs, p_drain)
    torch.cuda.synchronize()
    assert launches >= 2  # cross-shard overlaps need several waves
    drained = parity[1].copy()
    for d_, a, j in diffs:  # the parity's drain loop, one diff at a time
        v = drained[a:a + d_.size].copy()
        oracle.parity_apply(mat, k, k + 1, j, d_, v)
        drained[a:a + d_.size] = v
    assert np.array_equal(to_host(p_drain), drained)
    for (j, a, n), v in zip(sets, news):  # the data-side chain, SET by SET
        old = data[j][a:a + n].copy()
        pv = [p[a:a + n].copy() for p in parity]
        oracle.diff_update(mat, k, m, j, old, v, pv, True)
        data[j][a:a + n] = old
        for p in range(m):
            parity[p][a:a + n] = pv[p]
    for j in range(k):
        assert np.array_equal(to_host(ddev[j]), data[j]), j
    for p in range(m):
        assert np.array_equal(to_host(pdev[p]), parity[p]), p
    assert np.array_equal(drained, parity[1])  # drain == per-shard fused update


def test_reference_microbenchmark_on_shim(gpu):
    """The reference's own micro-benchmark (microbenchmarks/galois_tp.c: one 512 MiB
    galois_w08_region_multiply from malloc'd memory), compiled unmodified against the
    shim's <galois.h> and linked -lJerasure (oracle/Makefile `ref`), runs to completion
    on the GPU.  Skips where oracle/_ref was not built (no /root/reference)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "galois_tp")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/galois_tp not built")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    parts = r.stdout.split()
    assert len(parts) == 4 and parts[1] == "s" and parts[3] == "ns", r.stdout


@pytest.mark.parametrize("kind", ["pageable", "pinned", "device", "pageable_in_device_out"])
def test_recovery_finish_matches_two_step(gpu, oracle, kind):
    """cec_recovery_finish (last peer + leader solve, pipelined in 16 MiB pieces) ==
    add_peer + solve: same rebuilt bytes, same residual, for every buffer kind; with a
    diff folded before the last peer (recovery.c:99-131)."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(sum(map(ord, kind)))
    nunits = 9 * 1024 + 37  # 36 MiB + 37 units: three pieces, the last one partial
    n = nunits * U
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    pdev = [to_dev(torch, p) for p in oracle.encode(mat, k, m, data)]
    mask = oracle.recovery_mask(k, m, 4, [1, 0, 1, 1, 1])  # D1 lost, leader P1 (inverse 1/245)

    def buf(a, what):
        if what == "device":
            return to_dev(torch, a)
        if what == "pinned":
            return torch.from_numpy(a.copy()).pin_memory()
        return a.copy()

    in_kind = {"pageable_in_device_out": "pageable"}.get(kind, kind)
    out_kind = {"pageable_in_device_out": "device"}.get(kind, kind)
    diff = rng.integers(0, 256, 5000, dtype=np.uint8)
    outs, resid = [], []
    for fused in (False, True):
        with ec.Recovery(k, m, mat, 4, mask, 0, nunits - 1, pdev[1]) as rec:
            rec.add_peer(0, buf(data[0], in_kind))
            assert rec.fold_update(2, 4096 * 7 + 16, diff) >= 1  # peer 2 not yet applied
            o = buf(np.zeros(n, np.uint8), out_kind)
            if fused:
                rec.finish(2, buf(data[2], in_kind), {}, {1: o})
            else:
                rec.add_peer(2, buf(data[2], in_kind))
                rec.solve({}, {1: o})
            sync = ec.last_sync()
            if out_kind == "pinned":  # the kernel wrote host memory: fenced before return
                assert sync["host_results"] == 1 and sync["fenced"] == 1, sync
            elif out_kind == "device":
                assert sync["host_results"] == 0 and sync["fenced"] == 0, sync
            assert rec.complete
            torch.cuda.synchronize()
            outs.append(o.cpu().numpy() if hasattr(o, "cpu") else o)
            tmp = torch.empty(n, dtype=torch.uint8, device="cuda")
            ec.region_multiply(rec.residual, 1, n, tmp, 0)
            torch.cuda.synchronize()
            resid.append(to_host(tmp))
    assert np.array_equal(outs[1], outs[0])
    assert np.array_equal(resid[1], resid[0])
    # the folded diff makes the rebuilt bytes differ from data[1] exactly where the
    # reference's would: D1' = D1 ^ inv * MATRIX(P1, D2) * diff over that piece
    exp = data[1].copy()
    v = np.zeros(5000, np.uint8)
    oracle.region_multiply(diff, oracle.gf_mul(oracle.gf_div(1, mat[4 * k + 1]), mat[4 * k + 2]), v, 1)
    exp[4096 * 7 + 16:4096 * 7 + 16 + 5000] ^= v
    assert np.array_equal(outs[1], exp)


@pytest.mark.parametrize("outs_kind", ["device", "one_pageable", "two_pageable"])
def test_recovery_finish_double_loss(gpu, oracle, outs_kind):
    """D0, D1 lost: P1 ships its residual; the leader P0 finishes with the last data peer
    D2 and rebuilds both shards in the same pass."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    nunits = 4 * 1024 + 3
    n = nunits * U
    data = [oracle.splitmix_bytes(0xC0C70105 + j, n) for j in range(k)]
    pdev = [to_dev(torch, p) for p in oracle.encode(mat, k, m, data)]
    mask = 0b11100
    with ec.Recovery(k, m, mat, 3, mask, 0, nunits - 1, pdev[0]) as r0, \
         ec.Recovery(k, m, mat, 4, mask, 0, nunits - 1, pdev[1]) as r1:
        r1.add_peer(2, data[2])
        res1 = torch.empty(n, dtype=torch.uint8, device="cuda")
        ec.region_multiply(r1.residual, 1, n, res1, 0)
        torch.cuda.synchronize()
        res1_host = to_host(res1)
        o0 = np.zeros(n, np.uint8) if outs_kind != "device" else torch.zeros(n, dtype=torch.uint8, device="cuda")
        o1 = np.zeros(n, np.uint8) if outs_kind == "two_pageable" else torch.zeros(n, dtype=torch.uint8, device="cuda")
        r0.finish(2, data[2], {4: res1_host}, {0: o0, 1: o1})
        torch.cuda.synchronize()
    got = [x.cpu().numpy() if hasattr(x, "cpu") else x for x in (o0, o1)]
    assert np.array_equal(got[0], data[0]) and np.array_equal(got[1], data[1])


def test_recovery_finish_rejects_early_peer(gpu, oracle):
    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    p = torch.zeros(8 * 4096, dtype=torch.uint8, device="cuda")
    mask = oracle.recovery_mask(k, m, 3, [0, 1, 1, 1, 1])
    with ec.Recovery(k, m, mat, 3, mask, 0, 7, p) as rec:
        with pytest.raises(ec.CecError):  # D2 still missing after D1
            rec.finish(1, np.zeros(8 * 4096, np.uint8), {}, {0: np.zeros(8 * 4096, np.uint8)})


# ------------------------------------------------------------------ recovery pool (§8f 2)
@pytest.mark.parametrize("engine_name", ["perm", "lds"])
@pytest.mark.parametrize("out_kind", ["device", "pinned", "host"])
def test_recovery_pool_idle_recoverer(gpu, oracle, engine_name, out_kind):
    """The idle recoverer's traffic (memcached.c:5712-5734): single-unit and short-range
    requests, a bounded window in flight, replies from D1 / D2 in random order, flushes at
    random points, SETs landing mid-recovery (fold_update, then the parity apply,
    memcached.c:7757-7764) on D1 / D2 and on lost D0 (its substitute forwards them under
    lid 0, which recovery.c:116-120 folds like any other), batched leader solves.  Every
    rebuilt unit of lost D0 equals the live data.  With `pinned`, the rebuilt shard's arena
    is pinned host memory and is read as soon as the last synchronous solve returns (no
    device sync): the pool then waits with the system-fence event.  With
    `host`, the rebuilt shard is a pageable host array (the unchanged server's sub_ecmem)
    and the solves go to the pool's own output (the _host calls), copied out per request
    as fill_completed_recovered_data does (memcached.c:7967-8000)."""
    torch, ec = gpu
    default = ec.get_engine()
    ec.set_engine(ec.CEC_ENGINE_PERM if engine_name == "perm" else ec.CEC_ENGINE_LDS)
    try:
        k, m, U = 3, 2, 4096
        mat = ec.coding_matrix(k, m)
        rng = np.random.default_rng(0x9001 + len(engine_name))
        nunits = 256
        data = [rng.integers(0, 256, nunits * U, dtype=np.uint8) for _ in range(k)]
        p0 = to_dev(torch, oracle.encode(mat, k, m, data)[0])
        host = out_kind == "host"
        out0 = (np.zeros(nunits * U, dtype=np.uint8) if host
                else torch.zeros(nunits * U, dtype=torch.uint8).pin_memory() if out_kind == "pinned"
                else torch.zeros(nunits * U, dtype=torch.uint8, device="cuda"))
        mask = oracle.recovery_mask(k, m, 3, [0, 1, 1, 1, 1])  # D0 lost, leader P0
        pending, done = {}, []  # id -> (ub, ue, peers left)
        ranges, rebuilt = {}, np.zeros(nunits, dtype=bool)  # id -> (ub, ue); units solved into out0

        def mark_solved():
            for i, (a, b) in ranges.items():
                if pool.solved(i):
                    rebuilt[a:b + 1] = True
                    if host:  # fill_completed_recovered_data from the pool's output
                        out0[a * U:(b + 1) * U] = pool.output(i)

        def flush_solve():
            if host:
                pool.flush_solve_host()
            else:
                pool.flush_solve([out0, None, None])

        def solve(ids):
            if host:
                pool.solve_host(ids)
            else:
                pool.solve(ids, [out0, None, None])

        def check_sync():  # a solve into pinned memory is fenced before it returns; HBM: not
            sync = ec.last_sync()
            want = (0, 0) if out_kind == "device" else (1, 1)
            assert (sync["host_results"], sync["fenced"]) == want, (out_kind, sync)

        next_unit, window = 0, 24
        with ec.RecoveryPool(k, m, mat, 3, p0, capacity_units=64) as pool:
            while next_unit < nunits or pending:
                while next_unit < nunits and len(pending) < window:
                    n = 1 if rng.random() < 0.7 else int(rng.integers(2, 5))
                    ub, ue = next_unit, min(nunits - 1, next_unit + n - 1)
                    try:
                        i = pool.begin(mask, ub, ue)
                        pending[i], ranges[i] = (ub, ue, [1, 2]), (ub, ue)
                    except ec.CecError as e:  # pool full: back off like the TOO_MANY check
                        assert e.code == ec.CEC_EFULL
                        break
                    next_unit = ue + 1
                rid = list(pending)[int(rng.integers(0, len(pending)))]
                ub, ue, left = pending[rid]
                peer = left.pop(int(rng.integers(0, len(left))))
                if rng.random() < 0.5:  # received straight into the pool's staging
                    addr, view = pool.staging(rid, peer)
                    view[:] = data[peer][ub * U:(ue + 1) * U]
                    pool.add_peer(rid, peer, addr)
                else:
                    pool.add_peer(rid, peer, data[peer][ub * U:(ue + 1) * U].copy())
                if rng.random() < 0.3:
                    if rng.random() < 0.5:
                        pool.flush()
                    else:  # the completed single-loss requests are rebuilt in the same pass
                        flush_solve()
                        check_sync()
                        mark_solved()
                if rng.random() < 0.25:  # a SET lands: on D1 / D2, or on lost D0 through its
                    # substitute, forwarded under lid 0 (memcached.c:7700, :7758)
                    j = int(rng.integers(0, 3))
                    ln = int(rng.integers(1, 9000))
                    addr = int(rng.integers(0, nunits * U - ln)) // 16 * 16
                    new = rng.integers(0, 256, ln, dtype=np.uint8)
                    diff = oracle.set_diff(data[j][addr:addr + ln].copy(), new)
                    data[j][addr:addr + ln] = new
                    pool.fold_update(j, addr, diff)
                    ec.region_multiply(to_dev(torch, diff), mat[3 * k + j], ln, p0.data_ptr() + addr, 1)
                    if j == 0:  # units already rebuilt: the substitute writes them itself
                        for u in range(addr // U, (addr + ln - 1) // U + 1):
                            if rebuilt[u]:
                                lo, hi = max(addr, u * U), min(addr + ln, (u + 1) * U)
                                out0[lo:hi] = (data[0][lo:hi] if host else
                                               torch.from_numpy(data[0][lo:hi].copy()).to(out0.device))
                    torch.cuda.synchronize()
                if not left:
                    assert pool.complete(rid)
                    del pending[rid]
                    if pool.solved(rid):
                        pool.end(rid)
                        del ranges[rid]
                    else:
                        done.append(rid)
                if done and (rng.random() < 0.3 or not pending):
                    solve(done)
                    check_sync()
                    for d in done:
                        assert pool.solved(d)
                        a, b = ranges.pop(d)
                        rebuilt[a:b + 1] = True
                        if host:
                            out0[a * U:(b + 1) * U] = pool.output(d)
                        pool.end(d)
                    done = []
            assert pool.active == 0
            if out_kind == "pinned":  # read on return of the last synchronous call
                assert np.array_equal(out0.numpy(), data[0])
        torch.cuda.synchronize()
        assert np.array_equal(out0 if host else to_host(out0), data[0])
    finally:
        ec.set_engine(default)


def test_recovery_pool_non_leader_residual_and_errors(gpu, oracle):
    """Double loss (D0, D1; mask {D2, P0, P1}): the non-leader P1's pooled residual equals
    recovery_recover_units (recovery.c:61-96); the pool refuses a multi-loss solve, a
    repeated peer, an incomplete solve and a request beyond its capacity."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    nunits = 32
    data = [oracle.splitmix_bytes(0xC0C70200 + j, nunits * U) for j in range(k)]
    parity = oracle.encode(mat, k, m, data)
    p1 = to_dev(torch, parity[1])
    with ec.RecoveryPool(k, m, mat, 4, p1, capacity_units=8) as pool:
        rid = pool.begin(0b11100, 5, 7)
        assert not pool.complete(rid)
        with pytest.raises(ec.CecError):
            pool.solve([rid], [torch.zeros(nunits * U, dtype=torch.uint8, device="cuda")] * 3)
        pool.add_peer(rid, 2, data[2][5 * U:8 * U].copy())
        with pytest.raises(ec.CecError):
            pool.add_peer(rid, 2, data[2][5 * U:8 * U].copy())
        assert pool.complete(rid)
        res = np.zeros(3 * U, np.uint8)
        pool.residual(rid, res)
        exp = np.empty(3 * U, np.uint8)
        oracle.recover_units(mat, k, 4, 2, parity[1][5 * U:8 * U].copy(), data[2][5 * U:8 * U].copy(), exp, [0])
        assert np.array_equal(res, exp)
        with pytest.raises(ec.CecError):  # two lost shards: the leader needs other residuals
            pool.solve([rid], [torch.zeros(nunits * U, dtype=torch.uint8, device="cuda")] * 3)
        with pytest.raises(ec.CecError) as ei:
            pool.begin(0b11100, 10, 15)  # 6 more units, 5 free
        assert ei.value.code == ec.CEC_EFULL
        pool.end(rid)
        assert pool.begin(0b11100, 10, 17) >= 0  # room again


@pytest.mark.parametrize("engine_name", ["perm", "lds"])
@pytest.mark.parametrize("capacity", [64, 12])
def test_recovery_pool_fold_updates_window(gpu, oracle, capacity, engine_name):
    """A drain window folded at once (cec_recovery_pool_fold_updates) equals the same
    updates folded one by one (cec_recovery_pool_fold_update, recovery.c:99-131) on a twin
    pool: 300 SET diffs of every data lid -- lost ones too -- crowded onto few units, so
    they meet in R and split into waves; requests untouched, touched, complete and
    partly fed.  capacity 12: the window has more tiles than the pool's tile buffer."""
    torch, ec = gpu
    default = ec.get_engine()
    ec.set_engine(ec.CEC_ENGINE_PERM if engine_name == "perm" else ec.CEC_ENGINE_LDS)
    k, m, U = 4, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0xF01D + capacity)
    nunits = 64
    data = [rng.integers(0, 256, nunits * U, dtype=np.uint8) for _ in range(k)]
    p0 = to_dev(torch, oracle.encode(mat, k, m, data)[0])
    mask = 0b010000 | 0b1110  # D0 lost, leader P0
    pools = [ec.RecoveryPool(k, m, mat, 4, p0, capacity_units=capacity) for _ in range(2)]
    try:
        ranges = [(2, 2), (3, 5), (8, 8), (9, 10), (20, 22)]
        rids = []
        for x, (ub, ue) in enumerate(ranges):
            ids = [pl.begin(mask, ub, ue) for pl in pools]
            assert ids[0] == ids[1]
            rids.append(ids[0])
            for j in [1, 2, 3][:x % 4]:  # 0..3 peers fed: untouched, partly fed, complete
                for pl in pools:
                    pl.add_peer(ids[0], j, data[j][ub * U:(ue + 1) * U].copy())
        window = []
        for _ in range(300):
            ln = int(rng.integers(1, 3 * U))
            addr = int(rng.integers(1 * U, 12 * U - ln)) if rng.random() < 0.8 else \
                int(rng.integers(0, nunits * U - ln))
            window.append((rng.integers(0, 256, ln, dtype=np.uint8), addr, int(rng.integers(0, k))))
        got = pools[0].fold_updates(window)
        want = [pools[1].fold_update(lid, addr, diff) for diff, addr, lid in window]
        assert got == want
        assert sum(got) > 60, "the window should mostly land on units under recovery"
        for x, (rid, (ub, ue)) in enumerate(zip(rids, ranges)):
            if x % 4 == 0:  # untouched: no residual yet (both pools fold nothing into it)
                continue
            a, b = np.zeros((ue - ub + 1) * U, np.uint8), np.zeros((ue - ub + 1) * U, np.uint8)
            pools[0].residual(rid, a)
            pools[1].residual(rid, b)
            assert np.array_equal(a, b), (ub, ue)
        assert pools[0].fold_updates([]) == []
    finally:
        for pl in pools:
            pl.destroy()
        ec.set_engine(default)


def test_recovery_pool_host_output_lifecycle(gpu, oracle):
    """The _host solves' output (what cocytus_recovery_pool.c hands fill_completed_recovered_
    data): none before a solve; after flush_solve_host the rebuilt units of a request it
    completes; a lost lid's diff folded afterwards (recovery.c:116-120) makes it stale --
    solved() and output() drop it -- and solve_host rebuilds the live bytes; a request the
    flush did not complete is solved by solve_host; ending a request drops its output."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0x0B7)
    nunits = 16
    data = [rng.integers(0, 256, nunits * U, dtype=np.uint8) for _ in range(k)]
    p0 = to_dev(torch, oracle.encode(mat, k, m, data)[0])
    mask = (1 << 3) | 0b110  # D0 lost, leader P0
    with ec.RecoveryPool(k, m, mat, 3, p0, capacity_units=8) as pool:
        a, b = pool.begin(mask, 2, 4), pool.begin(mask, 9, 9)
        assert pool.output(a) is None
        for j in (1, 2):
            pool.add_peer(a, j, data[j][2 * U:5 * U].copy())
        pool.add_peer(b, 1, data[1][9 * U:10 * U].copy())
        assert pool.flush_solve_host() == 1  # a completes in this flush, b does not
        assert pool.solved(a) and not pool.solved(b) and pool.output(b) is None
        assert np.array_equal(pool.output(a), data[0][2 * U:5 * U])
        # a SET on lost D0, forwarded by its substitute: folded into a's residual
        addr, ln = 3 * U + 100, 5000
        new = rng.integers(0, 256, ln, dtype=np.uint8)
        diff = oracle.set_diff(data[0][addr:addr + ln].copy(), new)
        data[0][addr:addr + ln] = new
        assert pool.fold_update(0, addr, diff) == 2  # units 3 and 4 of a
        ec.region_multiply(to_dev(torch, diff), mat[3 * k + 0], ln, p0.data_ptr() + addr, 1)
        torch.cuda.synchronize()
        assert not pool.solved(a) and pool.output(a) is None
        pool.add_peer(b, 2, data[2][9 * U:10 * U].copy())
        pool.flush()  # b's last reply folded, no solve
        assert not pool.solved(b)
        pool.solve_host([a, b])
        assert np.array_equal(pool.output(a), data[0][2 * U:5 * U])
        assert np.array_equal(pool.output(b), data[0][9 * U:10 * U])
        pool.end(a)
        assert pool.output(a) is None


def test_recovery_pool_add_peers_batch(gpu, oracle):
    """cec_recovery_pool_add_peers (a pass's replies in one call): a batch with a bad reply
    -- a peer twice for one request, a peer already applied, a parity lid, an ended request
    -- is refused and queues nothing (the next flush folds nothing); the good batch, mixing
    replies received in the pool's staging and copied from host buffers, rebuilds every
    request's bytes in one flush_solve_host, as add_peer one by one does."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0xADD5)
    nunits = 64
    data = [rng.integers(0, 256, nunits * U, dtype=np.uint8) for _ in range(k)]
    p1 = to_dev(torch, oracle.encode(mat, k, m, data)[1])
    mask = (1 << 4) | 0b101  # D1 lost, leader P1 (inverse 1/245)
    starts = [0, 3, 10, 11, 30, 50]
    with ec.RecoveryPool(k, m, mat, 4, p1, capacity_units=32) as pool:
        ended = pool.begin(mask, 60, 60)
        pool.end(ended)
        rids = [pool.begin(mask, s, s + 1) for s in starts]  # two units each
        pool.add_peer(rids[0], 0, data[0][0:2 * U].copy())  # D0 of the first already applied
        ids, lids, bufs = [], [], []
        for q, (rid, s) in enumerate(zip(rids, starts)):
            for j in (0, 2):
                if q == 0 and j == 0:
                    continue
                src = data[j][s * U:(s + 2) * U]
                if (q + j) % 2:  # received in place
                    addr, view = pool.staging(rid, j)
                    view[:] = src
                    bufs.append(addr)
                else:
                    bufs.append(src.copy())
                ids.append(rid)
                lids.append(j)
        for bad in ((ids + [ids[1]], lids + [lids[1]], bufs + [bufs[1]]),  # a pair twice
                    (ids + [rids[0]], lids + [0], bufs + [bufs[0]]),
                    (ids + [rids[2]], lids + [3], bufs + [bufs[0]]),
                    (ids + [ended], lids + [2], bufs + [bufs[0]])):
            with pytest.raises(ec.CecError):
                pool.add_peers(*bad)
        assert all(not pool.complete(r) for r in rids)  # nothing of a refused batch queued
        pool.add_peers(ids, lids, bufs)
        assert pool.flush_solve_host() == len(rids)
        for rid, s in zip(rids, starts):
            assert np.array_equal(pool.output(rid), data[1][s * U:(s + 2) * U]), s
        pool.add_peers([], [], [])  # an empty pass


def test_recovery_pool_misuse_is_refused(gpu, oracle):
    """Stale and bad handles on the pool's calls (what a server bug would send): an ended or
    never-begun id, a repeated end, a reply or a solve for an ended request, a window with a
    data lid out of range -- each refused (CecError / None), nothing crashes, and a live
    request next to them still rebuilds its bytes."""
    torch, ec = gpu
    k, m, U = 3, 2, 4096
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(0xBAD)
    data = [rng.integers(0, 256, 8 * U, dtype=np.uint8) for _ in range(k)]
    p0 = to_dev(torch, oracle.encode(mat, k, m, data)[0])
    mask = (1 << 3) | 0b110
    with ec.RecoveryPool(k, m, mat, 3, p0, capacity_units=4) as pool:
        dead, live = pool.begin(mask, 0, 0), pool.begin(mask, 5, 5)
        pool.end(dead)
        for bad in (dead, 7, -1, 1 << 20):
            with pytest.raises(ec.CecError):
                pool.end(bad)
            with pytest.raises(ec.CecError):
                pool.add_peer(bad, 1, data[1][:U].copy())
            with pytest.raises(ec.CecError):
                pool.solve_host([bad])
            assert pool.output(bad) is None and not pool.solved(bad) and not pool.complete(bad)
        with pytest.raises(ec.CecError):
            pool.fold_updates([(np.zeros(16, np.uint8), 0, k)])  # data lid k: out of range
        with pytest.raises(ec.CecError):
            pool.add_peer(live, 3, data[1][5 * U:6 * U].copy())  # a parity lid is no data peer
        for j in (1, 2):
            pool.add_peer(live, j, data[j][5 * U:6 * U].copy())
        with pytest.raises(ec.CecError):
            pool.solve_host([live, live])  # listed twice
        pool.solve_host([live])
        assert np.array_equal(pool.output(live), data[0][5 * U:6 * U])
        assert pool.active == 1


def test_batched_bindings_c_program(gpu, oracle, tmp_path):
    """The batched bindings from a C99 program (cec_encode_region, cec_diff_update,
    cec_drainer_apply, cec_recovery_pool) vs the reference's chains."""
    from tests.dropin import run_batched_case

    run_batched_case(oracle, tmp_path)
