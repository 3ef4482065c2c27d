"""CPU tests of the oracle itself (oracle/gf8_ref.c): pinned against every independent
known answer available -- the field defined from scratch in pure Python (carry-less
multiply mod 0x11D) and through sympy's GF(2)[x] arithmetic, a second implementation of
the big-Vandermonde construction, SURVEY.md §8c's restated matrices, the invariants of
Jerasure's big-Vandermonde distribution matrix -- plus round trips of the reference's
call chains and the committed golden fixtures.  (Jerasure itself is unavailable:
parity unpinned.)"""
from __future__ import annotations

import hashlib
import itertools
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def clmul_mod(a: int, b: int, poly: int = 0x11D) -> int:
    """GF(2^8) multiply from the definition: shift-and-add, reduce by the polynomial."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= poly
    return r


def py_matmul(A, B, n, k, p):
    C = [0] * (n * p)
    for i in range(n):
        for j in range(p):
            acc = 0
            for x in range(k):
                acc ^= clmul_mod(A[i * k + x], B[x * p + j])
            C[i * p + j] = acc
    return C


def test_field_against_definition(oracle):
    for a in range(256):
        for b in range(0, 256, 3):
            assert oracle.gf_mul(a, b) == clmul_mod(a, b)
    assert oracle.gf_exp(8) == 0x1D and oracle.gf_mul(2, 0x80) == 0x1D
    seen = {oracle.gf_exp(i) for i in range(255)}
    assert len(seen) == 255 and 0 not in seen  # 2 generates GF(2^8)*
    for a in range(1, 256):
        assert oracle.gf_exp(oracle.gf_log(a)) == a
        assert oracle.gf_mul(a, oracle.gf_div(1, a)) == 1
    assert oracle.gf_div(5, 0) == -1


def _poly(a: int) -> list[int]:
    """GF(2)[x] coefficient list (highest degree first) of the bit pattern a."""
    return [int(b) for b in bin(a)[2:]] if a else []


def _int(f) -> int:
    return int("".join(str(int(c)) for c in f), 2) if f else 0


def test_field_against_sympy(oracle):
    """The field through a third-party implementation: sympy's GF(p)[x] arithmetic
    (galoistools), product modulo x^8+x^4+x^3+x^2+1 for every pair of bytes, the
    polynomial irreducible and x (= 2) of order 255, so the log / antilog tables the
    reference's w = 8 region multiply is built from exist and are the oracle's."""
    from sympy import ZZ
    from sympy.polys import galoistools as gt

    P = _poly(0x11D)
    assert gt.gf_irreducible_p(P, 2, ZZ)
    x = _poly(2)
    assert _int(gt.gf_pow_mod(x, 255, P, 2, ZZ)) == 1
    for q in (3, 5, 17):  # 255 = 3 * 5 * 17: x has full order
        assert _int(gt.gf_pow_mod(x, 255 // q, P, 2, ZZ)) != 1
    for i in range(255):
        assert _int(gt.gf_pow_mod(x, i, P, 2, ZZ)) == oracle.gf_exp(i)
    for a in range(256):
        fa = _poly(a)
        for b in range(256):
            got = _int(gt.gf_rem(gt.gf_mul(fa, _poly(b), 2, ZZ), P, 2, ZZ))
            assert oracle.gf_mul(a, b) == got, (a, b)


def _jerasure_big_vandermonde(rows: int, cols: int) -> list[int]:
    """Jerasure 2.x reed_sol_big_vandermonde_distribution_matrix(rows, cols, 8), written
    again from its published algorithm with the from-scratch field above (a second
    implementation to check the C oracle's, not the library itself):
    the extended Vandermonde matrix (row 0 = e_0, row rows-1 = e_{cols-1}, row i = powers
    of i), column operations to the identity on top, then coding columns scaled so row
    `cols` is all ones, then coding rows scaled so column 0 is all ones."""
    def inv(a):
        return next(b for b in range(1, 256) if clmul_mod(a, b) == 1)

    def pw(a, e):
        r = 1
        for _ in range(e):
            r = clmul_mod(r, a)
        return r

    d = [[0] * cols for _ in range(rows)]
    d[0][0] = 1
    d[rows - 1][cols - 1] = 1
    for i in range(1, rows - 1):
        for j in range(cols):
            d[i][j] = pw(i, j)
    for i in range(1, cols):
        j = next(r for r in range(i, rows) if d[r][i])
        if j != i:
            d[i], d[j] = d[j], d[i]
        if d[i][i] != 1:
            t = inv(d[i][i])
            for r in range(rows):
                d[r][i] = clmul_mod(t, d[r][i])
        for j in range(cols):
            t = d[i][j]
            if j != i and t:
                for r in range(rows):
                    d[r][j] ^= clmul_mod(t, d[r][i])
    for j in range(cols):
        t = d[cols][j]
        if t != 1:
            t = inv(t)
            for r in range(cols, rows):
                d[r][j] = clmul_mod(t, d[r][j])
    for r in range(cols + 1, rows):
        t = d[r][0]
        if t != 1:
            t = inv(t)
            for j in range(cols):
                d[r][j] = clmul_mod(d[r][j], t)
    return [v for row in d for v in row]


@pytest.mark.parametrize("k,m", [(2, 1), (3, 2), (4, 2), (6, 3), (8, 4), (10, 4), (12, 4), (16, 8)])
def test_big_vandermonde_second_implementation(oracle, k, m):
    got = oracle.big_vandermonde(k + m, k)
    assert got == _jerasure_big_vandermonde(k + m, k)


@pytest.mark.parametrize("c", [0, 1, 2, 3, 0x80, 0x8E, 244, 245, 255])
def test_region_multiply_semantics(oracle, c):
    rng = np.random.default_rng(c)
    src = rng.integers(0, 256, 1000, dtype=np.uint8)
    r2 = rng.integers(0, 256, 1000, dtype=np.uint8)
    prod = np.array([clmul_mod(c, int(x)) for x in src], np.uint8)
    a = r2.copy()
    oracle.region_multiply(src, c, a, 1)
    assert np.array_equal(a, r2 ^ prod)
    b = r2.copy()
    oracle.region_multiply(src, c, b, 0)
    assert np.array_equal(b, prod)
    s = src.copy()
    oracle.region_multiply(s, c, None, 0)
    assert np.array_equal(s, prod)


def test_simd_baseline_equals_scalar(oracle):
    rng = np.random.default_rng(1)
    for n in [0, 1, 31, 32, 33, 4096, 4098, 100003]:
        for c in [0, 1, 2, 245, 255]:
            src = rng.integers(0, 256, n, dtype=np.uint8)
            r2 = rng.integers(0, 256, n, dtype=np.uint8)
            a, b = r2.copy(), r2.copy()
            oracle.region_multiply(src, c, a, 1)
            if n:
                oracle.region_multiply_simd(src, c, b)
            assert np.array_equal(a, b)


def test_cpu_baseline_server_loops(oracle):
    """bench.py's 1-thread CPU legs of the server placements against the scalar oracle:
    the SET-diff loop (memcached.c:2676-2681) gives value ^ old per SET; the recovery chain
    (recovery.c:72-94 + memcached.c:7853-7922) gives inv * (parity ^ sum c_p * reply_p) per
    request -- which is the lost shard's bytes when the parity is the code's."""
    rng = np.random.default_rng(11)
    n, size, stride = 50, 4098, 4112
    ecmem = rng.integers(0, 256, n * stride, dtype=np.uint8)
    values = rng.integers(0, 256, n * stride, dtype=np.uint8)
    vo = rng.permutation(n).astype(np.uint64) * stride
    ad = rng.permutation(n).astype(np.uint64) * stride
    do = np.arange(n, dtype=np.uint64) * stride
    diffs = np.zeros(n * stride, np.uint8)
    assert oracle.bench_set_diffs(values, vo, ecmem, ad, np.full(n, size), diffs, do) >= 0
    for i in range(n):
        exp = oracle.set_diff(ecmem[int(ad[i]):int(ad[i]) + size].copy(), values[int(vo[i]):int(vo[i]) + size].copy())
        assert np.array_equal(diffs[int(do[i]):int(do[i]) + size], exp)
    k, m, U, self_lid, lost = 3, 2, 4096, 4, 1
    mat = oracle.big_vandermonde(k + m, k)
    nunits = 40
    data = [rng.integers(0, 256, nunits * U, dtype=np.uint8) for _ in range(k)]
    ecm = oracle.encode(mat, k, m, data)[1]  # this parity's arena: P1
    inv = oracle.gf_div(1, mat[self_lid * k + lost])
    for units, starts in ((8, [3]), (1, [0, 7, 39, 12])):
        replies = [data[p][s * U:(s + units) * U].copy() for s in starts for p in (0, 2)]
        t, outs = oracle.bench_recover_requests(ecm, starts, units, replies, 2,
                                                [mat[self_lid * k + 0], mat[self_lid * k + 2]], inv)
        assert t >= 0
        for s, o in zip(starts, outs):
            assert np.array_equal(o, data[lost][s * U:(s + units) * U]), (units, s)


def test_known_matrices(oracle):
    # restated answers of the survey's own (separate) restatement
    assert oracle.big_vandermonde(5, 3)[9:] == [1, 1, 1, 1, 245, 244]
    assert oracle.big_vandermonde(6, 4)[16:] == [1, 1, 1, 1, 1, 70, 143, 200]
    assert oracle.big_vandermonde(3, 3) is None
    ev = oracle.extended_vandermonde(5, 3)
    assert ev == [1, 0, 0, 1, 1, 1, 1, 2, 4, 1, 3, 5, 0, 0, 1]


@pytest.mark.parametrize("k,m", [(1, 1), (2, 2), (3, 2), (4, 2), (6, 3), (10, 4), (4, 4), (8, 8), (16, 16)])
def test_matrix_invariants(oracle, k, m):
    mat = oracle.big_vandermonde(k + m, k)
    for i in range(k):
        assert mat[i * k:(i + 1) * k] == [int(i == j) for j in range(k)]  # systematic
    assert mat[k * k:(k + 1) * k] == [1] * k  # first parity row all ones (XOR parity)
    for r in range(k, k + m):
        assert mat[r * k] == 1  # first column all ones
    if k + m <= 9:  # MDS: every k x k submatrix invertible
        for rows in itertools.combinations(range(k + m), k):
            sub = [mat[r * k + c] for r in rows for c in range(k)]
            rc, inv = oracle.invert(list(sub), k)
            assert rc == 0, rows
            assert py_matmul(sub, inv, k, k, k) == [int(i == j) for i in range(k) for j in range(k)]


def test_invert_singular(oracle):
    assert oracle.invert([1, 2, 2, 4], 2)[0] == -1  # row 2 = 2 * row 1
    assert oracle.invert([0, 0, 0, 0], 2)[0] == -1
    rc, inv = oracle.invert([0, 1, 1, 0], 2)  # needs a row swap
    assert rc == 0 and inv == [0, 1, 1, 0]


@pytest.mark.parametrize("k,m", [(3, 2), (4, 2), (6, 3)])
def test_encode_erase_decode_all_patterns(oracle, k, m):
    mat = oracle.big_vandermonde(k + m, k)
    n = 4099
    data = [oracle.splitmix_bytes(100 + j, n) for j in range(k)]
    par = oracle.encode(mat, k, m, data)
    arenas = data + par
    for lids in itertools.combinations(range(k + m), k):
        mask = sum(1 << x for x in lids)
        lost = [j for j in range(k) if not (mask >> j) & 1]
        out = oracle.decode(mat, k, m, mask, [a if (mask >> i) & 1 else None for i, a in enumerate(arenas)])
        assert len(out) == len(lost)
        for x, j in enumerate(lost):
            assert np.array_equal(out[x], data[j])


def test_encode_is_linear(oracle):
    k, m, n = 4, 2, 777
    mat = oracle.big_vandermonde(k + m, k)
    a = [oracle.splitmix_bytes(j, n) for j in range(k)]
    b = [oracle.splitmix_bytes(50 + j, n) for j in range(k)]
    pa, pb = oracle.encode(mat, k, m, a), oracle.encode(mat, k, m, b)
    pab = oracle.encode(mat, k, m, [x ^ y for x, y in zip(a, b)])
    for p in range(m):
        assert np.array_equal(pab[p], pa[p] ^ pb[p])


def test_diff_update_chain_equals_reencode(oracle):
    k, m, n = 3, 2, 512
    mat = oracle.big_vandermonde(k + m, k)
    rng = np.random.default_rng(2)
    data = [np.zeros(n, np.uint8) for _ in range(k)]
    par = [np.zeros(n, np.uint8) for _ in range(m)]  # fresh arenas are zero (mmap)
    for _ in range(200):
        j = int(rng.integers(0, k))
        off = int(rng.integers(0, n // 16)) * 16
        ln = int(rng.integers(1, n - off + 1))
        old = data[j][off:off + ln].copy()
        pv = [p[off:off + ln].copy() for p in par]
        oracle.diff_update(mat, k, m, j, old, rng.integers(0, 256, ln, dtype=np.uint8), pv, True)
        data[j][off:off + ln] = old
        for p in range(m):
            par[p][off:off + ln] = pv[p]
    enc = oracle.encode(mat, k, m, data)
    for p in range(m):
        assert np.array_equal(enc[p], par[p])


def test_recovery_with_concurrent_updates(oracle):
    """recovery.c:99-131: diffs landing during recovery are folded into in-flight
    residuals only for peers that have not contributed yet; the residual always ends
    equal to P_final ^ sum c * D_final over the mask's data peers."""
    k, m, U = 3, 2, 4096
    mat = oracle.big_vandermonde(k + m, k)
    rng = np.random.default_rng(4)
    for trial in range(20):
        data = [rng.integers(0, 256, U, dtype=np.uint8) for _ in range(k)]
        par = oracle.encode(mat, k, m, data)
        self_lid, mask = 3, 0b01011  # D2 lost, leader P0, survivors D0, D1
        peers = [0, 1]
        res = np.empty(U, np.uint8)
        touched = [0]
        contributed = set()
        events = ["c0", "c1", "u0", "u1", "u0"]
        rng.shuffle(events)
        for ev in events:
            s = int(ev[1])
            if ev[0] == "c" and s not in contributed:
                oracle.recover_units(mat, k, self_lid, s, par[0], data[s], res, touched)
                contributed.add(s)
            elif ev[0] == "u":  # SET on data peer s: diff to the parity (+ residual if needed)
                new = rng.integers(0, 256, U, dtype=np.uint8)
                diff = oracle.set_diff(data[s], new)
                data[s] = new
                if touched[0] and s not in contributed:
                    oracle.try_update_unit(mat, k, self_lid, s, diff, res)
                oracle.parity_apply(mat, k, self_lid, s, diff, par[0])
        for s in peers:
            if s not in contributed:
                oracle.recover_units(mat, k, self_lid, s, par[0], data[s], res, touched)
        exp = par[0].copy()
        for s in peers:
            oracle.region_multiply(data[s], mat[self_lid * k + s], exp, 1)
        assert np.array_equal(res, exp), (trial, events)


def test_recovery_mask(oracle):
    assert oracle.recovery_mask(3, 2, 3, [1, 1, 1, 1, 1]) == 0b01011
    assert oracle.recovery_mask(3, 2, 3, [0, 1, 1, 1, 1]) == 0b01110
    assert oracle.recovery_mask(3, 2, 4, [1, 0, 1, 0, 1]) == 0b10101
    assert oracle.recovery_mask(3, 2, 3, [0, 0, 1, 1, 1]) == 0b11100
    assert oracle.recovery_mask(3, 2, 3, [0, 0, 0, 1, 0]) == 0


def test_golden_manifest(oracle):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)
    for name, meta in man["files"].items():
        with open(os.path.join(GOLDEN, name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == meta["sha256"], name
    for key, mat in man["matrices"].items():
        k, m = map(int, key.split(","))
        assert oracle.big_vandermonde(k + m, k) == mat


def test_golden_recomputed_by_oracle(oracle):
    z = np.load(os.path.join(GOLDEN, "region_multiply.npz"))
    for key in z.files:
        if key.endswith("_src"):
            base = key[:-4]
            c = int(base.split("_")[0][1:])
            r2 = z[base + "_r2"].copy()
            oracle.region_multiply(z[key].copy(), c, r2, 1)
            assert np.array_equal(r2, z[base + "_out"]), base
    for name, (k, m) in [("encode_rs32.npz", (3, 2)), ("encode_rs42.npz", (4, 2)), ("encode_rs63.npz", (6, 3))]:
        z = np.load(os.path.join(GOLDEN, name))
        par = oracle.encode(list(z["matrix"]), k, m, [z[f"data{j}"] for j in range(k)])
        for p in range(m):
            assert np.array_equal(par[p], z[f"parity{p}"])
    for name, (k, m) in [("decode_rs32.npz", (3, 2)), ("decode_rs42.npz", (4, 2))]:
        z = np.load(os.path.join(GOLDEN, name))
        arenas = [z[f"arena{i}"] for i in range(k + m)]
        for mask in z["masks"]:
            mask = int(mask)
            out = oracle.decode(list(z["matrix"]), k, m, mask,
                                [a if (mask >> i) & 1 else None for i, a in enumerate(arenas)])
            lost = [j for j in range(k) if not (mask >> j) & 1]
            for x, j in enumerate(lost):
                assert np.array_equal(out[x], z[f"mask{mask}_lost{j}"])


def test_oracle_vs_system_jerasure(oracle):
    """Pin the oracle against a real Jerasure 2.x when the machine has one (SURVEY §8c:
    'cross-checked against real libJerasure if the box has it').  This image has
    none, so this skips and the oracle stays 'parity unpinned' (DESIGN.md §2)."""
    from oracle import jerasure_probe

    lib, where = jerasure_probe.load()
    if lib is None:
        pytest.skip(where)
    for k, m in [(3, 2), (4, 2), (6, 3)]:
        mat = jerasure_probe.matrix(lib, k, m)
        assert mat == oracle.big_vandermonde(k + m, k), (k, m, where)
        data = [oracle.splitmix_bytes(0xC0C70001 + j, 4096 + 7) for j in range(k)]
        ref = jerasure_probe.encode(lib, mat, k, m, data)
        ours = oracle.encode(mat, k, m, data)
        for p in range(m):
            assert np.array_equal(ref[p], ours[p]), (k, m, p, where)


def test_jerasure_probe_rejects_the_shim():
    """The probe must never return the repository's own libJerasure.so symlink."""
    from oracle import jerasure_probe

    for p in jerasure_probe.candidates():
        assert not os.path.realpath(p).startswith(jerasure_probe.ROOT + os.sep), p


def _ecalloc_fixture():
    z = np.load(os.path.join(GOLDEN, "ecalloc_layout.npz"))
    return [tuple(int(x) for x in row) for row in z["sets"]], int(z["seed"]), int(z["k"])


def test_ecalloc_fixture_matches_reference():
    """tests/golden/ecalloc_layout.npz is what the reference's own allocator
    (/root/reference/ecalloc.c, built into oracle/_ref) hands out for that SET trace."""
    from oracle import ecalloc_ref

    if not ecalloc_ref.available():
        pytest.skip("oracle/_ref/libecalloc_ref.so not built (needs /root/reference)")
    sets, seed, k = _ecalloc_fixture()
    assert ecalloc_ref.set_trace(seed, k) == sets


def test_ecalloc_layout_contract():
    """The address contract the kernels rely on: 16-B aligned
    starts (ecalloc.c:176), no overlap within one shard's batch, and -- because each
    lid has its own allocator -- overlaps ACROSS shards in the parity arena."""
    sets, _, k = _ecalloc_fixture()
    assert all(a % 16 == 0 for _, a, _ in sets)
    cross = 0
    for j in range(k):
        r = sorted((a, a + n) for jj, a, n in sets if jj == j)
        assert all(r[i][0] >= r[i - 1][1] for i in range(1, len(r))), j
    allr = sorted((a, a + n, j) for j, a, n in sets)
    for i in range(1, len(allr)):
        cross += allr[i][0] < allr[i - 1][1]
    assert cross > 0
