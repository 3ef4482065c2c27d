"""The server glue of integration/ (cocytus_drain.c: the parity process's drain loops,
memcached.c:4231/4322/4350/8068 -> process_rep_command :7739-7798, batched onto one
cec_drainer_apply) driven over the server's own queue type: oracle/_ref/glue_drain is
built (oracle/Makefile `ref`) from the glue and tests/glue/drain_main.c against the
reference's rep_queue.h where it lies.  Skips where it was not built (no /root/reference
when the tree was built).

CPU: which queued diffs a drain call takes (the xid window, ring order and wrap, the
item's nbytes rather than the buffer's capacity, a missing xid, more than cap).
GPU: the parity arena after cocytus_drain_gf equals the reference's sequential loop
(one region multiply per non-vetoed xid, in xid order) computed by the oracle.
"""
from __future__ import annotations

import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "oracle", "_ref", "glue_drain")


def _need_exe():
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/glue_drain not built (make -C oracle ref)")


def write_input(path, *, lid, self_lid, k, m, ring, tail, entries, done, stable, cap, arena=0, parity=None):
    """entries: [(xid, addr, bytes, vnbytes, veto)] at ring indices tail, tail+1, ..."""
    with open(path, "wb") as f:
        tail32 = tail - (1 << 32) if tail >= 1 << 31 else tail  # the driver reads it as uint32
        f.write(struct.pack("<9i", lid, self_lid, k, m, ring, tail32, len(entries), arena, cap))
        f.write(struct.pack("<2Q", done, stable))
        for xid, addr, val, vn, veto in entries:
            f.write(struct.pack("<2Q3i", xid, addr, len(val), vn, veto))
        for _, _, val, _, _ in entries:
            f.write(bytes(val))
        if parity is not None:
            f.write(parity.tobytes())


def run(mode, tmp_path, **kw):
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    write_input(inp, **kw)
    r = subprocess.run([EXE, mode, str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r, out


def collect(tmp_path, **kw):
    _, out = run("collect", tmp_path, **kw)
    lines = out.read_text().split("\n")
    if lines[0].startswith("rc "):
        return int(lines[0].split()[1])
    return [tuple(int(v) for v in ln.split()) for ln in lines if ln]


def test_collect_window_ring_and_lengths(tmp_path):
    """Entries with done_xid < xid <= stable_xid, in xid order, walking the ring [tail,
    head) across its wrap; len = the item's nbytes, not the buffer's vnbytes (which may be
    up to twice as large, memcached.c:7727-7731); src_lid = the peer."""
    _need_exe()
    rng = np.random.default_rng(3)
    ents = []
    for i in range(60):  # xids 101..160, ring of 64 entries starting near its end
        n = int(rng.integers(1, 300))
        ents.append((101 + i, 16 * int(rng.integers(0, 1 << 16)), rng.integers(0, 256, n, dtype=np.uint8),
                     n + int(rng.integers(0, n + 1)), 0))
    got = collect(tmp_path, lid=2, self_lid=4, k=3, m=2, ring=64, tail=50, entries=ents, done=110,
                  stable=150, cap=64)
    want = [(e, ents[e][1], len(ents[e][2]), 2) for e in range(60) if 110 < ents[e][0] <= 150]
    assert got == want and len(got) == 40
    # nothing pending: no update
    assert collect(tmp_path, lid=2, self_lid=4, k=3, m=2, ring=64, tail=50, entries=ents, done=150,
                   stable=150, cap=64) == []


def test_collect_refuses_gaps_and_overflow(tmp_path):
    """A missing xid of the window is refused (process_rep_command asserts its entry
    exists), and a window wider than the caller's scratch is CEC_EFULL (drain it in
    several calls); a repeated xid resolves to its first entry, as rep_queue_find."""
    _need_exe()
    v = np.arange(8, dtype=np.uint8)
    ents = [(x, 16 * x, v, 8, 0) for x in (1, 2, 3, 5, 6)]
    assert collect(tmp_path, lid=0, self_lid=3, k=3, m=2, ring=8, tail=0, entries=ents, done=0, stable=6,
                   cap=16) == -1  # CEC_EINVAL: xid 4 missing
    assert collect(tmp_path, lid=0, self_lid=3, k=3, m=2, ring=8, tail=0, entries=ents, done=0, stable=3,
                   cap=2) == -7  # CEC_EFULL
    dup = [(1, 16, v, 8, 0), (2, 32, v, 8, 0), (2, 48, v, 8, 0), (3, 64, v, 8, 0)]
    got = collect(tmp_path, lid=1, self_lid=3, k=3, m=2, ring=8, tail=6, entries=dup, done=0, stable=3, cap=8)
    assert [(a, n) for _, a, n, _ in got] == [(16, 8), (32, 8), (64, 8)]


def _drain_case(rng, count=3000, arena=4 << 20, max_len=20 << 10):
    ents = []
    for i in range(count):
        n = int(rng.integers(1, max_len))
        addr = 16 * int(rng.integers(0, (arena - n) // 16))
        ents.append((1000 + i, addr, rng.integers(0, 256, n, dtype=np.uint8), n + int(rng.integers(0, 64)),
                     int(rng.random() < 0.1)))
    return ents


def _drain_model(oracle, ents, parity, done, stable, k, lid, self_lid):
    c = oracle.big_vandermonde(k + 2, k)[self_lid * k + lid]
    want = parity.copy()
    applied = vetoed = 0
    for xid, addr, val, _, veto in ents:  # already in xid order
        if not done < xid <= stable:
            continue
        if veto:
            vetoed += 1
            continue
        oracle.region_multiply(val.copy(), c, want[addr:addr + len(val)], 1)
        applied += 1
    return want, applied, vetoed


@pytest.mark.gpu
def test_drain_gf_into_registered_host_arena(gpu, oracle, tmp_path):
    """The placement the unchanged server runs (ecmem in host memory, read by recovery.c:81
    and sent by memcached.c:4282 from the host): the arena registered once with
    cec_host_register and drained by cocytus_drain_gf through its device alias -- the same
    bytes as the sequential loop, in the host arena itself when the call returns."""
    _need_exe()
    k, m, lid, self_lid = 3, 2, 2, 3
    arena = 4 << 20
    rng = np.random.default_rng(12)
    ents = _drain_case(rng, 1500)
    parity = rng.integers(0, 256, arena, dtype=np.uint8)
    done, stable = 1000 + 100, 1000 + 1400
    r, out = run("apply_host", tmp_path, lid=lid, self_lid=self_lid, k=k, m=m, ring=2048, tail=100, entries=ents,
                 done=done, stable=stable, cap=2048, arena=arena, parity=parity)
    want, applied, vetoed = _drain_model(oracle, ents, parity, done, stable, k, lid, self_lid)
    assert np.array_equal(np.fromfile(out, dtype=np.uint8), want)
    assert r.stdout.split()[:4] == ["applied", str(applied), "vetoed", str(vetoed)], r.stdout


@pytest.mark.gpu
def test_drain_refused_window_runs_no_fold(gpu, oracle, tmp_path):
    """the recovery fold has side effects, so a window the apply would refuse
    (here a diff larger than the drainer's staging) is refused before ANY fold runs
    (cec_drainer_validate first): rc CEC_EINVAL, zero hook calls, the arena untouched."""
    _need_exe()
    rng = np.random.default_rng(4)
    ents = [(1 + i, 16 * i * 512, rng.integers(0, 256, n, dtype=np.uint8), n, 0)
            for i, n in enumerate([100, 4000, 5000, 300])]          # xid 3: 5000 B > 4096
    parity = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    r, out = run("apply4k", tmp_path, lid=0, self_lid=3, k=3, m=2, ring=8, tail=0, entries=ents, done=0, stable=4,
                 cap=8, arena=1 << 20, parity=parity)
    assert r.stdout.split() == ["rc", "-1", "hooks", "0"], r.stdout
    assert np.array_equal(np.fromfile(out, dtype=np.uint8), parity)


@pytest.mark.gpu
def test_drain_gf_matches_sequential_loop(gpu, oracle, tmp_path):
    """cocytus_drain_gf over 3,000 queued diffs of one data peer (random lengths 1 B -
    20 KiB at 16-B-aligned, overlapping addresses of a 4 MiB parity arena; 10 % vetoed by
    the recovery hook; a window in the middle of the ring, across its wrap) leaves the
    device parity arena equal to the reference's loop: for each xid in order, if the fold
    lets it through, parity[addr..] ^= MATRIX(self, lid) * diff (memcached.c:7758-7767),
    computed by the oracle."""
    _need_exe()
    k, m, lid, self_lid = 3, 2, 1, 4
    arena = 4 << 20
    rng = np.random.default_rng(11)
    ents = []
    for i in range(3000):
        n = int(rng.integers(1, 20 << 10))
        addr = 16 * int(rng.integers(0, (arena - n) // 16))
        ents.append((1000 + i, addr, rng.integers(0, 256, n, dtype=np.uint8), n + int(rng.integers(0, 64)),
                     int(rng.random() < 0.1)))
    parity = rng.integers(0, 256, arena, dtype=np.uint8)
    done, stable = 1000 + 200, 1000 + 2800
    r, out = run("apply", tmp_path, lid=lid, self_lid=self_lid, k=k, m=m, ring=4096, tail=3000, entries=ents,
                 done=done, stable=stable, cap=4096, arena=arena, parity=parity)
    got = np.fromfile(out, dtype=np.uint8)
    c = oracle.big_vandermonde(k + m, k)[self_lid * k + lid]
    want = parity.copy()
    applied = vetoed = 0
    for xid, addr, val, _, veto in ents:  # already in xid order
        if not done < xid <= stable:
            continue
        if veto:
            vetoed += 1
            continue
        oracle.region_multiply(val.copy(), c, want[addr:addr + len(val)], 1)
        applied += 1
    assert np.array_equal(got, want)
    words = r.stdout.split()
    assert words[:4] == ["applied", str(applied), "vetoed", str(vetoed)], r.stdout
    assert int(words[5]) >= 2  # overlapping diffs went to separate waves


def test_collect_under_asan_ubsan(tmp_path):
    """The glue's host walk of the ring under AddressSanitizer + UBSan (gcc), over the
    same cases as above: no out-of-bounds access, no undefined behaviour."""
    ref = "/root/reference/rep_queue.h"
    if not os.path.exists(ref):
        pytest.skip("the reference's rep_queue.h is not here")
    exe = tmp_path / "glue_drain_asan"
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"),
                    "-I", os.path.dirname(ref), "-o", str(exe), os.path.join(ROOT, "tests", "glue", "drain_main.c"),
                    os.path.join(ROOT, "integration", "cocytus_drain.c"), "-I", os.path.join(ROOT, "oracle"),
                    "-L", os.path.join(ROOT, "cocytus_amd"), "-lcocytus_ec", "-L", os.path.join(ROOT, "oracle"),
                    "-lgf8ref", "-Wl,-rpath," + os.path.join(ROOT, "cocytus_amd"),
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle")], check=True)
    global EXE
    saved, EXE = EXE, str(exe)
    os.environ["ASAN_OPTIONS"] = "detect_leaks=0"
    try:
        test_collect_window_ring_and_lengths(tmp_path)
        test_collect_refuses_gaps_and_overflow(tmp_path)
    finally:
        EXE = saved
        os.environ.pop("ASAN_OPTIONS", None)


def _collect_model(ents, tail, ring, done, stable, cap):
    """What the drain loop would process (rep_queue_find per xid, memcached.c:7747):
    per xid of (done, stable], the first entry in ring order [tail, head) with it."""
    n = stable - done
    if n <= 0:
        return []
    if n > cap:
        return -7
    first = {}
    for e, ent in enumerate(ents):
        first.setdefault(ent[0], e)
    out = []
    for x in range(done + 1, stable + 1):
        if x not in first:
            return -1
        e = first[x]
        out.append((e, ents[e][1], len(ents[e][2]), 3))
    return out


@pytest.mark.parametrize("seed", range(24))
def test_collect_random_rings(tmp_path, seed):
    """Random queues against a model of the reference's per-xid loop: ring sizes 1-64,
    tails anywhere rep_queue_add leaves them (below twice the ring: it rebases both indices
    by cap once tail passes cap, rep_queue.c:51-55), xids ascending with gaps and repeats,
    windows inside, across and beyond the queued xids, scratch caps below and above the
    window."""
    _need_exe()
    rng = np.random.default_rng(1000 + seed)
    ring = int(rng.integers(1, 65))
    count = int(rng.integers(0, ring + 1))
    tail = int(rng.choice([0, rng.integers(0, ring), rng.integers(ring, 2 * ring)]))
    x, ents = int(rng.integers(0, 50)), []
    for _ in range(count):
        x += int(rng.choice([0, 1, 1, 1, 2]))  # repeats and gaps
        n = int(rng.integers(1, 40))
        ents.append((x, 16 * int(rng.integers(0, 4096)), rng.integers(0, 256, n, dtype=np.uint8), n, 0))
    lo = int(rng.integers(0, x + 3))
    done, stable = lo, lo + int(rng.integers(0, 12))
    cap = int(rng.integers(0, 16))
    got = collect(tmp_path, lid=3, self_lid=4, k=3, m=2, ring=ring, tail=tail, entries=ents, done=done,
                  stable=stable, cap=cap)
    assert got == _collect_model(ents, tail, ring, done, stable, cap), (ring, tail, done, stable, cap)
