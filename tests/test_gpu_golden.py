"""GPU vs the COMMITTED golden fixtures (tests/golden/*.npz, frozen oracle bytes with a
sha256 manifest): every fixture is replayed through the HIP path (C-ABI), both GF
engines, and compared byte for byte with the frozen outputs -- not with a live oracle,
so a regression in the oracle and the kernels at once cannot hide.  Plus the whole
BASELINE configs[1] batch (65,536 x 4 KiB RS(3,2) stripes) compared with the oracle's
parity, not a sample.

Parity is unpinned (see oracle/gf8_ref.h and tests/golden/make_golden.py): the fixtures
freeze the restatement of Jerasure 2.x / GF-Complete that tests/test_oracle.py checks
against every independent known answer available.
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(params=["perm", "lds"])
def engine(request, gpu):
    torch, ec = gpu
    default = ec.get_engine()
    ec.set_engine(ec.CEC_ENGINE_PERM if request.param == "perm" else ec.CEC_ENGINE_LDS)
    yield request.param
    ec.set_engine(default)


def load(name):
    path = os.path.join(GOLD, name)
    with open(os.path.join(GOLD, "manifest.json")) as f:
        want = json.load(f)["files"][name]["sha256"]
    with open(path, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == want, f"{name} differs from its manifest"
    return np.load(path)


def dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def host(t):
    return t.cpu().numpy()


def test_golden_region_multiply(gpu, engine):
    """galois_w08_region_multiply(src, c, n, r2, add=1) for every frozen (c, n): the
    device form (cec_region_multiply) and the drop-in symbol on host buffers."""
    torch, ec = gpu
    z = load("region_multiply.npz")
    cases = sorted({k.rsplit("_", 1)[0] for k in z.keys()})
    assert len(cases) == 42
    for case in cases:
        c = int(case.split("_")[0][1:])
        src, r2, out = z[case + "_src"], z[case + "_r2"], z[case + "_out"]
        n = src.size
        ds, dd = dev(torch, src), dev(torch, r2)
        ec.region_multiply(ds, c, n, dd, 1)
        torch.cuda.synchronize()
        assert np.array_equal(host(dd), out), case
        h = r2.copy()
        ec.galois_w08_region_multiply(src.copy(), c, n, h, 1)
        assert np.array_equal(h, out), case + " (drop-in, host buffers)"


@pytest.mark.parametrize("name,k,m", [("encode_rs32.npz", 3, 2), ("encode_rs42.npz", 4, 2),
                                      ("encode_rs63.npz", 6, 3)])
def test_golden_encode(gpu, engine, name, k, m):
    torch, ec = gpu
    z = load(name)
    mat = ec.coding_matrix(k, m)
    assert mat == z["matrix"].tolist()
    n = z["data0"].size
    data = [dev(torch, z[f"data{j}"]) for j in range(k)]
    par = [torch.full((n,), 0xA5, dtype=torch.uint8, device="cuda") for _ in range(m)]
    with ec.Plan([(0, 0, n, 0)]) as plan:
        ec.encode(k, m, mat, data, par, plan)
        torch.cuda.synchronize()
    for p in range(m):
        assert np.array_equal(host(par[p]), z[f"parity{p}"]), f"parity {p}"
    par2 = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    ec.encode_region(k, m, mat, data, par2, n)
    torch.cuda.synchronize()
    for p in range(m):
        assert np.array_equal(host(par2[p]), z[f"parity{p}"]), f"parity {p} (region)"


def test_golden_diff_update(gpu, engine):
    """The per-SET chain (memcached.c:2681 diff, :7764 parity apply per parity, :5666
    install) for a SET to each shard j, fused in one cec_diff_update launch."""
    torch, ec = gpu
    z = load("diff_update_rs32.npz")
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    assert mat == z["matrix"].tolist()
    n = z["j0_old"].size
    for j in range(k):
        data = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(k)]
        data[j] = dev(torch, z[f"j{j}_old"])
        par = [dev(torch, z[f"j{j}_parity{p}_before"]) for p in range(m)]
        new = dev(torch, z[f"j{j}_new"])
        with ec.Plan([(0, 0, n, j)]) as plan:
            ec.diff_update(k, m, mat, data, new, par, True, plan)
            torch.cuda.synchronize()
        for p in range(m):
            assert np.array_equal(host(par[p]), z[f"j{j}_parity{p}_after"]), (j, p)
        assert np.array_equal(host(data[j]), z[f"j{j}_new"])
        # the unfused chain through the device ops: diff, then one apply per parity
        par = [dev(torch, z[f"j{j}_parity{p}_before"]) for p in range(m)]
        data[j] = dev(torch, z[f"j{j}_old"])
        diff = torch.empty(n, dtype=torch.uint8, device="cuda")
        with ec.Plan([(0, 0, n, j)]) as plan:
            ec.set_diff(k, data, new, diff, plan)
            for p in range(m):
                ec.apply_diffs(k, m, mat, k + p, diff, par[p], plan)
            torch.cuda.synchronize()
        for p in range(m):
            assert np.array_equal(host(par[p]), z[f"j{j}_parity{p}_after"]), (j, p, "chain")


@pytest.mark.parametrize("name,k,m", [("decode_rs32.npz", 3, 2), ("decode_rs42.npz", 4, 2)])
def test_golden_decode(gpu, engine, name, k, m):
    """Every frozen single and double erasure: the fused cec_decode (all masks in one
    plan) and, per mask, the reference's two steps (residual per participating parity,
    then the leader solve)."""
    torch, ec = gpu
    z = load(name)
    mat = ec.coding_matrix(k, m)
    assert mat == z["matrix"].tolist()
    n = z["arena0"].size
    masks = z["masks"].tolist()
    arenas = [dev(torch, z[f"arena{i}"]) for i in range(k + m)]
    B = len(masks)
    # stripe q of a B-stripe batch carries mask q: tile the frozen arenas B times
    big = [a.repeat(B) for a in arenas]
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    with ec.Plan([(q * n, 0, n, q) for q in range(B)]) as plan:
        ec.decode(k, m, mat, masks, big, out, plan)
        torch.cuda.synchronize()
    checked = 0
    for q, mask in enumerate(masks):
        for j in range(k):
            key = f"mask{mask}_lost{j}"
            if (mask >> j) & 1:
                continue
            assert np.array_equal(host(out[j][q * n:(q + 1) * n]), z[key]), key
            checked += 1
    assert checked == sum(1 for x in z.keys() if x.startswith("mask") and "_lost" in x)
    for mask in masks:  # two-step chain
        pars = [p for p in range(k, k + m) if (mask >> p) & 1]
        res = [None] * (k + m)
        with ec.Plan([(0, 0, n, 0)]) as plan:
            for p in pars:
                res[p] = torch.empty(n, dtype=torch.uint8, device="cuda")
                ec.residual(k, m, mat, p, mask, arenas, res[p], plan)
            o = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(k)]
            ec.solve(k, m, mat, mask, res, o, plan)
            torch.cuda.synchronize()
        for j in range(k):
            if not (mask >> j) & 1:
                assert np.array_equal(host(o[j]), z[f"mask{mask}_lost{j}"]), (mask, j, "two-step")


def test_cfg2_full_batch_parity_vs_oracle(gpu, oracle):
    """BASELINE configs[1] in full: RS(3,2) parity of all 65,536 x 4 KiB stripes equals
    the oracle's (its AVX2 restatement of GF-Complete's region multiply, checked against
    the scalar oracle first), then the rotating single-shard decode rebuilds every lost
    stripe."""
    torch, ec = gpu
    k, m, n, B = 3, 2, 4096, 65536
    mat = ec.coding_matrix(k, m)
    hostd = [oracle.splitmix_bytes(0xC0C70002 + j, B * n) for j in range(k)]
    probe = np.zeros(4096 * 3, np.uint8)
    ref = probe.copy()
    for j in range(k):  # the SIMD restatement == the scalar oracle on a sample
        oracle.region_multiply_simd(hostd[j][:probe.size], mat[(k + 1) * k + j], probe)
        oracle.region_multiply(hostd[j][:ref.size].copy(), mat[(k + 1) * k + j], ref, 1)
    assert np.array_equal(probe, ref)
    exp = [np.zeros(B * n, np.uint8) for _ in range(m)]
    for p in range(m):
        for j in range(k):
            oracle.region_multiply_simd(hostd[j], mat[(k + p) * k + j], exp[p])
    data = [dev(torch, h) for h in hostd]
    parity = [torch.empty(B * n, dtype=torch.uint8, device="cuda") for _ in range(m)]
    out = [torch.zeros(B * n, dtype=torch.uint8, device="cuda") for _ in range(k)]
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    with ec.Plan([(s * n, 0, n, 0) for s in range(B)]) as ep, \
         ec.Plan([(s * n, 0, n, s % len(masks)) for s in range(B)]) as dp:
        ec.encode(k, m, mat, data, parity, ep)
        ec.decode(k, m, mat, masks, data + parity, out, dp)
        torch.cuda.synchronize()
    for p in range(m):
        assert np.array_equal(host(parity[p]), exp[p]), f"parity {p}"
    lost_of = [[j for j in range(k) if not (mk >> j) & 1][0] for mk in masks]
    for q, j in enumerate(lost_of):
        sel = torch.arange(q, B, len(masks), device="cuda")
        assert torch.equal(out[j].view(B, n)[sel], data[j].view(B, n)[sel]), f"mask {q}"


@pytest.fixture(scope="module")
def cfg3_batch(gpu, oracle):
    """BASELINE configs[2] at its stated size: bench.layout("rs32_mixed") -- 8,432 RS(3,2)
    values, log-uniform 256 B - 1 MiB, ~1 GiB per shard, starts 16-B aligned
    (ecalloc.c:176) -- with random data (generated on the device, seeded), the oracle's
    parity of every value (AVX2 restatement, pinned to the scalar oracle on a sample), and
    per arena byte the data shard the rotating decode rebuilds there (-1: the alignment
    gaps between values, which no op may write)."""
    import bench

    torch, ec = gpu
    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    stripes, arena = bench.layout("rs32_mixed")
    assert len(stripes) == 8432 and sum(ln for _, ln in stripes) >= 1 << 30
    g = torch.Generator(device="cuda").manual_seed(0xC0C70003)
    data = [torch.randint(0, 256, (arena,), dtype=torch.uint8, device="cuda", generator=g) for _ in range(k)]
    hostd = [d.cpu().numpy() for d in data]
    probe, ref = np.zeros(3 * 4096 + 5, np.uint8), np.zeros(3 * 4096 + 5, np.uint8)
    for j in range(k):  # the SIMD restatement == the scalar oracle on a sample
        oracle.region_multiply_simd(hostd[j][:probe.size], mat[(k + 1) * k + j], probe)
        oracle.region_multiply(hostd[j][:ref.size].copy(), mat[(k + 1) * k + j], ref, 1)
    assert np.array_equal(probe, ref)
    masks = [ec.recovery_mask(k, m, k + p, [int(i != j) for i in range(k + m)])
             for p in range(m) for j in range(k)]
    lost_of = [[j for j in range(k) if not (mk >> j) & 1][0] for mk in masks]
    label = np.full(arena, -1, np.int8)
    for s, (o, ln) in enumerate(stripes):
        label[o:o + ln] = lost_of[s % len(masks)]
    exp = []
    for p in range(m):
        e = np.zeros(arena, np.uint8)
        for j in range(k):
            oracle.region_multiply_simd(hostd[j], mat[(k + p) * k + j], e)
        e[label < 0] = 0  # gaps: never written (parity arena starts zeroed)
        exp.append(dev(torch, e))
    del hostd
    return {"k": k, "m": m, "mat": mat, "stripes": stripes, "arena": arena, "data": data, "masks": masks,
            "label": dev(torch, label), "exp": exp}


@pytest.mark.parametrize("engine_name", ["auto", "perm", "lds"])
def test_cfg3_mixed_full_size(gpu, cfg3_batch, engine_name):
    """BASELINE configs[2] ("RS(3,2) encode + single-shard decode, mixed 256 B-1 MiB
    values") at the size the bench runs it (bench.layout("rs32_mixed"), ~1 GiB per
    shard): the whole batch's parity equals the oracle's byte for byte, and the rotating
    single-shard decode (masks as start_recovery builds them, memcached.c:8136-8151;
    residual + leader solve, recovery.c:61-96, memcached.c:7842-7922) rebuilds every
    value's lost shard byte for byte and writes nothing else.  Under AUTO (the default;
    PERM encode, LDS decode for this mean extent, as cec_last_engine reports), PERM and
    LDS."""
    torch, ec = gpu
    c = cfg3_batch
    k, m, mat, stripes, arena = c["k"], c["m"], c["mat"], c["stripes"], c["arena"]
    default = ec.get_engine()
    ec.set_engine({"auto": ec.CEC_ENGINE_AUTO, "perm": ec.CEC_ENGINE_PERM, "lds": ec.CEC_ENGINE_LDS}[engine_name])
    try:
        parity = [torch.zeros(arena, dtype=torch.uint8, device="cuda") for _ in range(m)]
        out = [torch.zeros(arena, dtype=torch.uint8, device="cuda") for _ in range(k)]
        with ec.Plan([(o, 0, ln, 0) for o, ln in stripes]) as ep, \
             ec.Plan([(o, 0, ln, s % len(c["masks"])) for s, (o, ln) in enumerate(stripes)]) as dp:
            ec.encode(k, m, mat, c["data"], parity, ep)
            ran_enc = ec.last_engine()
            ec.decode(k, m, mat, c["masks"], c["data"] + parity, out, dp)
            ran_dec = ec.last_engine()
            torch.cuda.synchronize()
    finally:
        ec.set_engine(default)
    if engine_name == "auto":
        assert (ran_enc, ran_dec) == (ec.CEC_ENGINE_PERM, ec.CEC_ENGINE_LDS)
    for p in range(m):
        assert torch.equal(parity[p], c["exp"][p]), f"parity {p}"
    for j in range(k):
        want = torch.where(c["label"] == j, c["data"][j], torch.zeros_like(c["data"][j]))
        assert torch.equal(out[j], want), f"rebuilt shard {j}"
