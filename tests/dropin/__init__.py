"""Drop-in check: a C program against include/{galois,jerasure,reed_sol}.h linked as
-lJerasure (libJerasure.so -> libcocytus_ec.so) vs the oracle on the same inputs."""
from __future__ import annotations

import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
# tools/asan.sh points these at a host-ASan/UBSan build of the library and compiles
# the programs with the matching clang runtime (CEC_DROPIN_CC / CEC_DROPIN_CFLAGS).
LIBDIR = os.environ.get("CEC_DROPIN_LIBDIR") or os.path.join(ROOT, "cocytus_amd")
CC = os.environ.get("CEC_DROPIN_CC") or "gcc"
XFLAGS = os.environ.get("CEC_DROPIN_CFLAGS", "").split()


def build_dropin(out_dir: str) -> str:
    exe = os.path.join(out_dir, "dropin_main")
    subprocess.run(
        [CC, "-O1", "-std=gnu11", "-I", os.path.join(ROOT, "include"),
         os.path.join(HERE, "dropin_main.c"), "-L", LIBDIR, "-lJerasure",
         f"-Wl,-rpath,{LIBDIR}", *XFLAGS, "-o", exe],
        check=True,
    )
    return exe


def run_dropin_threads(tmp_path, threads=8, iters=200) -> str:
    exe = os.path.join(str(tmp_path), "dropin_threads")
    subprocess.run(
        [CC, "-O1", "-std=gnu11", "-I", os.path.join(ROOT, "include"),
         os.path.join(HERE, "dropin_threads.c"), "-L", LIBDIR, "-lJerasure", "-lpthread",
         f"-Wl,-rpath,{LIBDIR}", *XFLAGS, "-o", exe],
        check=True,
    )
    r = subprocess.run([exe, str(threads), str(iters)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:] + r.stdout
    return r.stdout


def run_dropin_case(oracle, tmp_path, K=3, M=2, seed=0xC0C70001) -> None:
    rng = np.random.default_rng(seed)
    arena = 64 * 4096
    nsets = 300
    sets, vals = [], []
    for _ in range(nsets):  # SETs may overlap: the chain is sequential, like the server
        n = int(rng.integers(1, 6000)) + 2          # vlen + "\r\n"
        addr = int(rng.integers(0, (arena - n) // 16)) * 16  # ecalloc.c:176
        sets.append((int(rng.integers(0, K)), addr, n))
        vals.append(rng.integers(0, 256, n, dtype=np.uint8))
    mask = oracle.recovery_mask(K, M, K + 1, [1, 0, 1, 0, 1][: K + M])  # D1, P0 lost; leader P1
    ub, ue = 3, 40
    inp = tmp_path / "in.bin"
    with open(inp, "wb") as f:
        f.write(np.array([K, M, arena, nsets, ub, ue, mask], np.int32).tobytes())
        f.write(np.array(sets, np.int32).tobytes())
        for v in vals:
            f.write(v.tobytes())
    exe = build_dropin(str(tmp_path))
    outp = tmp_path / "out.bin"
    r = subprocess.run([exe, str(inp), str(outp)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr + r.stdout
    got = np.fromfile(outp, np.uint8)

    mat = oracle.big_vandermonde(K + M, K)
    data = [np.zeros(arena, np.uint8) for _ in range(K)]
    parity = [np.zeros(arena, np.uint8) for _ in range(M)]
    for (j, addr, n), v in zip(sets, vals):
        old = data[j][addr:addr + n].copy()
        pv = [p[addr:addr + n].copy() for p in parity]
        oracle.diff_update(mat, K, M, j, old, v, pv, True)
        data[j][addr:addr + n] = old
        for p in range(M):
            parity[p][addr:addr + n] = pv[p]
    lo, hi = ub * 4096, (ue + 1) * 4096
    arenas = [a[lo:hi].copy() if (mask >> i) & 1 else None for i, a in enumerate(data + parity)]
    rec = oracle.decode(mat, K, M, mask, arenas)
    exp = np.concatenate(data + parity + rec)
    assert got.size == exp.size
    assert np.array_equal(got, exp)
    assert np.array_equal(rec[0], data[1][lo:hi])  # the rebuilt shard is D1


def run_batched_case(oracle, tmp_path, K=3, M=2, units=24, seed=0xC0C70B47) -> None:
    """tests/dropin/batched_main.c (the batched bindings from C, no HIP header) vs the
    reference's chains restated by the oracle: encode, per-SET diff-update with install,
    the parity drain loop, and the idle recoverer's single-unit recoveries of D0."""
    rng = np.random.default_rng(seed)
    U = 4096
    A = units * U
    data = [rng.integers(0, 256, A, dtype=np.uint8) for _ in range(K)]
    sets, vals, taken = [], [], [[] for _ in range(K)]
    while len(sets) < 60:  # SETs never overlap within a shard; across shards they may
        j = int(rng.integers(0, K))
        n = int(rng.integers(1, 6000)) + 2
        addr = int(rng.integers(0, (A - n) // 16)) * 16
        if any(addr < e and s < addr + n for s, e in taken[j]):
            continue
        taken[j].append((addr, addr + n))
        sets.append((j, addr, n))
        vals.append(rng.integers(0, 256, n, dtype=np.uint8))
    inp = tmp_path / "batched_in.bin"
    with open(inp, "wb") as f:
        f.write(np.array([K, M, units, len(sets)], np.int32).tobytes())
        f.write(np.array(sets, np.int32).tobytes())
        for d in data:
            f.write(d.tobytes())
        for v in vals:
            f.write(v.tobytes())
    exe = os.path.join(str(tmp_path), "batched_main")
    subprocess.run(
        [CC, "-O1", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
         os.path.join(HERE, "batched_main.c"), "-L", LIBDIR, "-lcocytus_ec",
         f"-Wl,-rpath,{LIBDIR}", *XFLAGS, "-o", exe],
        check=True,
    )
    outp = tmp_path / "batched_out.bin"
    r = subprocess.run([exe, str(inp), str(outp)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stderr + r.stdout
    got = np.fromfile(outp, np.uint8).reshape(-1, A)

    mat = oracle.big_vandermonde(K + M, K)
    parity = oracle.encode(mat, K, M, data)
    drained = parity[1].copy()
    stale = [d.copy() for d in data]
    for (j, addr, n), v in zip(sets, vals):  # the data side, SET by SET
        old = data[j][addr:addr + n].copy()
        pv = [p[addr:addr + n].copy() for p in parity]
        oracle.diff_update(mat, K, M, j, old, v, pv, True)
        data[j][addr:addr + n] = old
        for p in range(M):
            parity[p][addr:addr + n] = pv[p]
    for (j, addr, n), v in zip(sets, vals):  # the parity's drain loop, one diff at a time
        diff = oracle.set_diff(stale[j][addr:addr + n].copy(), v)
        w = drained[addr:addr + n].copy()
        oracle.parity_apply(mat, K, K + 1, j, diff, w)
        drained[addr:addr + n] = w
    exp = parity + data + [drained, data[0]]
    assert got.shape[0] == len(exp)
    for i, e in enumerate(exp):
        assert np.array_equal(got[i], e), i


def run_dropin_daemon(tmp_path) -> str:
    """tests/dropin/dropin_daemon.c: matrix + inversion, fork() (memcached's daemonize),
    then the first region multiplies in the child; returns the child's report."""
    exe = os.path.join(str(tmp_path), "dropin_daemon")
    subprocess.run(
        [CC, "-O1", "-std=gnu11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
         os.path.join(HERE, "dropin_daemon.c"), "-L", LIBDIR, "-lJerasure",
         f"-Wl,-rpath,{LIBDIR}", *XFLAGS, "-o", exe],
        check=True,
    )
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stderr[-2000:]}\n{r.stdout}"
    return r.stdout


def run_cache_threads(tmp_path, threads=8, iters=60, limit=6) -> dict:
    """tests/dropin/cache_threads.c: the coefficient-table cache (capped at `limit`
    sets), the idle-buffer cache and the stream trackers under concurrent use; every
    result checked by a round-trip property inside the program."""
    import json

    exe = os.path.join(str(tmp_path), "cache_threads")
    subprocess.run(
        [CC, "-O1", "-std=gnu11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
         os.path.join(HERE, "cache_threads.c"), "-L", LIBDIR, "-lJerasure", "-lpthread",
         f"-Wl,-rpath,{LIBDIR}", *XFLAGS, "-o", exe],
        check=True,
    )
    r = subprocess.run([exe, str(threads), str(iters), str(limit)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stderr[-3000:]}\n{r.stdout}"
    return json.loads(r.stdout.strip().splitlines()[-1])
