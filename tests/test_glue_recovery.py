"""The recovery glue of integration/ (cocytus_recovery.c: recovery_recover_units,
recovery_try_update_unit and complete_recovery_bottom_half's arithmetic batched onto
cec_region_multiply_batch) driven over the server's own types: oracle/_ref/glue_recovery is
built (oracle/Makefile `ref`) from the glue and tests/glue/recovery_main.c against the
reference's recovery.h / ecmem.h / const.h / rep_queue.h where they lie.  Skips where it was
not built (no /root/reference when the tree was built).

The model below restates the reference's per-unit code (recovery.c:61-131,
memcached.c:7842-7922, process_rep_command :7758-7767) on numpy buffers with the oracle's
region multiply, one call per unit, in the reference's order.

CPU: the deferred path (no GPU until the flush): flags, touch_flags, the return values of
the try-update walk, the first-touch copies and the exact list of folds the flush will run,
on hand-written and random scripts; the reference's assertions as refused calls.
GPU: the immediate and the deferred paths leave every unit byte, flag and solve output equal
to the model; a drain window during recovery folds and applies as process_rep_command.
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (tools/asan.sh runs these tests through a sanitizer build of the same driver)
EXE = os.environ.get("CEC_GLUE_RECOVERY_EXE") or os.path.join(ROOT, "oracle", "_ref", "glue_recovery")
U = 4096
F_UPDATE, F_RECOVERED = 1 << 30, 1 << 31


def _need_exe():
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/glue_recovery not built (make -C oracle ref)")


def fnv(b: np.ndarray) -> str:
    h = 1469598103934665603
    for x in b.tobytes():
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


class Model:
    """recovery.c / memcached.c on numpy, one region multiply per unit (the oracle's)."""

    def __init__(self, oracle, heap, k, m, self_lid, nunits):
        self.o, self.heap, self.k, self.m, self.self_lid, self.n = oracle, heap, k, m, self_lid, nunits
        self.mat = oracle.big_vandermonde(k + m, k)
        self.flags = [0] * nunits
        self.data: list[np.ndarray | None] = [None] * nunits
        self.touch = [np.zeros(nunits, np.uint8) for _ in range(k + m)]
        self.sub = None
        self.queue = []      # deferred folds: (src, dst, base, len, multby, add)
        self.queue_src = []  # ... and their source bytes
        self.solves = []     # outputs in op order
        self.pending_solves = []

    def c(self, row, col):
        return self.mat[row * self.k + col]

    def _fold(self, src: np.ndarray, c, unit, off, src_desc, defer):
        if defer:
            self.queue.append((src_desc, f"u:{unit}:{off}", "-", src.size, c, 1))
            self.queue_src.append(src.copy())
        else:
            self.o.region_multiply(src.copy(), c, self.data[unit][off:off + src.size], 1)

    def recover(self, peer, ub, ue, off, defer=False):
        for i in range(ub, ue + 1):                      # recovery.c:72-78 (asserts)
            f = self.flags[i]
            if f & F_RECOVERED or f & (1 << peer) or (not f & F_UPDATE) != (self.data[i] is None):
                return -1
        c = self.c(self.self_lid, peer)
        for i in range(ub, ue + 1):
            if not self.flags[i] & F_UPDATE:             # first touch :76-86
                self.data[i] = self.heap[i * U:(i + 1) * U].copy()
                self.flags[i] |= F_UPDATE | (1 << self.self_lid)
            self.flags[i] |= 1 << peer                   # :89
            s = off + (i - ub) * U
            self._fold(self.heap[s:s + U], c, i, 0, f"h:{s}", defer)   # :91
        return 0

    def try_update(self, peer, addr, size, off, defer=False):
        ret, pos, c = 0, 0, self.c(self.self_lid, peer)   # recovery.c:99-131
        while size > 0:
            o = addr % U
            base = addr - o
            ln = min(U - o, size)
            size -= ln
            self.touch[peer][base // U] = 1
            if self.sub is None or self.sub[base // U] != 2:
                ret += 1
            f = self.flags[base // U]
            if not f & F_RECOVERED and f & F_UPDATE and not f & (1 << peer):
                piece = self.heap[off + pos:off + pos + ln]
                self._fold(piece, c, base // U, o, "k:" + fnv(piece), defer)
            addr += ln
            pos += ln
        return ret

    def solve(self, ub, ue, mask, dfp):
        k, m = self.k, self.m
        lost = [j for j in range(k) if not mask >> j & 1]
        pars = [i for i in range(k, k + m) if mask >> i & 1]
        if len(lost) != len(pars):
            return -1, 0
        if not lost:
            return 0, 0
        C = []
        for p in pars:
            if p == self.self_lid:
                if any(self.data[i] is None for i in range(ub, ue + 1)):
                    return -1, 0
                C.append(np.concatenate([self.data[i] for i in range(ub, ue + 1)]))
            else:
                if dfp[p] < 0:
                    return -1, 0
                C.append(self.heap[dfp[p]:dfp[p] + (ue - ub + 1) * U].copy())
        out = self.o.bottom_half(self.mat, k, m, mask, C)
        if out is None:
            return -2, 0
        return 0, out


class Script:
    def __init__(self, k, m, self_lid, nunits):
        self.lines = [f"init {k} {m} {self_lid} {nunits}"]

    def add(self, *words):
        self.lines.append(" ".join(str(w) for w in words))


def run_script(tmp_path, script: Script, heap: np.ndarray, nunits, k, m):
    sp, hp, out = tmp_path / "script.txt", tmp_path / "heap.bin", tmp_path / "out"
    sp.write_text("\n".join(script.lines) + "\n")
    heap.tofile(hp)
    err = tmp_path / "stderr.txt"
    with open(err, "w") as ef:  # (a file, so a stuck driver still shows what it printed)
        proc = subprocess.Popen([EXE, str(sp), str(hp), str(out)], stdout=subprocess.DEVNULL, stderr=ef)
        try:  # below the tests' own 120 s limit
            rc = proc.wait(timeout=90)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
            done = (tmp_path / "out.log").read_text() if (tmp_path / "out.log").exists() else ""
            raise AssertionError(f"{EXE} did not finish in 90 s; ops done: {done[-2000:]!r}; "
                                 f"stderr: {err.read_text()[-4000:]!r}") from None
    r = subprocess.CompletedProcess(proc.args, rc, None, err.read_text())
    assert r.returncode == 0, r.stderr
    log = (tmp_path / "out.log").read_text().split("\n")
    raw = np.fromfile(tmp_path / "out.units", dtype=np.uint8)
    flags, data, p = [], [], 0
    for _ in range(nunits):
        flags.append(int(raw[p:p + 4].view(np.uint32)[0]))
        present = raw[p + 4]
        p += 5
        if present:
            data.append(raw[p:p + U].copy())
            p += U
        else:
            data.append(None)
    touch = [raw[p + l * nunits:p + (l + 1) * nunits] for l in range(k + m)]
    p += (k + m) * nunits
    arena = raw[p:p + nunits * U]
    solves = np.fromfile(tmp_path / "out.solves", dtype=np.uint8)
    return [ln for ln in log if ln], flags, data, touch, arena, solves


def check_state(model: Model, flags, data, touch, bytes_too=True):
    assert flags == model.flags
    for i in range(model.n):
        assert (data[i] is None) == (model.data[i] is None), i
        if bytes_too and data[i] is not None:
            assert np.array_equal(data[i], model.data[i]), f"unit {i}"
    for l in range(model.k + model.m):
        assert np.array_equal(touch[l], model.touch[l]), f"touch_flags of lid {l}"


def jobs_from_log(log):
    out = []
    for ln in log:
        w = ln.split()
        if w[0] == "J" and w[1] == "fold":
            out.append((w[2], w[3], w[4], int(w[5]), int(w[6]), int(w[7])))
    return out


# ----------------------------------------------------------------- CPU: the deferred path
def _setup(oracle, k=3, m=2, self_lid=4, nunits=64, seed=0, extra=8 << 20):
    rng = np.random.default_rng(seed)
    heap = rng.integers(0, 256, nunits * U + extra, dtype=np.uint8)
    # (the model works on its own copy: its drains change the arena the script starts from)
    return rng, heap, Model(oracle, heap.copy(), k, m, self_lid, nunits), Script(k, m, self_lid, nunits)


def test_defer_flags_first_touch_and_queue(oracle, tmp_path):
    """Hand-written recovery: two data peers' replies over overlapping unit ranges (first
    touch vs already touched), SET diffs during recovery crossing unit boundaries at
    unaligned addresses (from a peer already applied: skipped; from one not yet applied:
    folded), a recovered unit and sub_flags == 2 units (not counted by the return value).
    Everything before the flush -- flags, first-touch copies, touch_flags, returns and the
    fold list -- equals the model."""
    _need_exe()
    k, m, s, n = 3, 2, 4, 64
    rng, heap, mod, sc = _setup(oracle, k, m, s, n)
    base = n * U
    ops = [("flag", 20, F_RECOVERED | F_UPDATE, base + 7 * U), ("sub", 9, 2), ("sub", 10, 2),
           ("D", 0, 4, 11, base), ("D", 1, 8, 15, base + 16 * U),
           ("t", 2, 4 * U + 100, 3 * U, base + 40 * U), ("t", 0, 10 * U + 16, 5000, base + 48 * U),
           ("t", 1, 19 * U + 4000, 200, base + 52 * U), ("t", 2, 30 * U, 16, base + 53 * U)]
    got_ret = []
    for op in ops:
        sc.add(*op)
        if op[0] == "flag":
            mod.flags[op[1]] = op[2]
            mod.data[op[1]] = heap[op[3]:op[3] + U].copy()
        elif op[0] == "sub":
            mod.sub = mod.sub if mod.sub is not None else np.zeros(n, np.uint8)
            mod.sub[op[1]] = op[2]
        elif op[0] == "D":
            got_ret.append(("D", mod.recover(op[1], op[2], op[3], op[4], defer=True)))
        else:
            got_ret.append(("t", mod.try_update(op[1], op[2], op[3], op[4], defer=True)))
    sc.add("P")
    log, flags, data, touch, _, _ = run_script(tmp_path, sc, heap, n, k, m)
    assert [(ln.split()[0], int(ln.split()[1])) for ln in log if ln[0] in "Dt"] == got_ret
    # pieces per unit crossed; unit 10 (sub_flags == 2) is not counted (recovery.c:113)
    assert [r for op, r in got_ret if op == "t"] == [4, 1, 2, 1]
    check_state(mod, flags, data, touch)   # first-touch copies = the parity units (folds still queued)
    assert jobs_from_log(log) == mod.queue
    p = [ln for ln in log if ln.startswith("P ")][0].split()
    assert int(p[2]) == len(mod.queue) and int(p[3]) == 0


def test_defer_refuses_what_the_reference_asserts(oracle, tmp_path):
    """recovery.c:72-78 assert: a recovered unit, a peer applied twice, an untouched unit that
    holds data.  The glue refuses the whole call (CEC_EINVAL) and changes nothing -- not
    even the units of the range before the offending one."""
    _need_exe()
    k, m, s, n = 3, 2, 3, 32
    rng, heap, mod, sc = _setup(oracle, k, m, s, n, seed=1)
    base = n * U
    sc.add("D", 0, 0, 3, base)
    mod.recover(0, 0, 3, base, defer=True)
    sc.add("flag", 6, F_RECOVERED, -1)
    mod.flags[6] = F_RECOVERED
    sc.add("flag", 12, 0, base)                 # data without UPDATE
    mod.flags[12], mod.data[12] = 0, heap[base:base + U].copy()
    for bad in [("D", 0, 2, 5, base), ("D", 1, 4, 7, base), ("D", 1, 10, 13, base), ("D", 5, 0, 0, base),
                ("D", 1, 5, 4, base)]:
        sc.add(*bad)
    sc.add("D", 1, 0, 1, base + 8 * U)          # still fine afterwards
    mod.recover(1, 0, 1, base + 8 * U, defer=True)
    sc.add("P")
    log, flags, data, touch, _, _ = run_script(tmp_path, sc, heap, n, k, m)
    rcs = [int(ln.split()[1]) for ln in log if ln.startswith("D ")]
    assert rcs == [0, -1, -1, -1, -1, -1, 0]
    check_state(mod, flags, data, touch)
    assert jobs_from_log(log) == mod.queue


def test_try_update_refusal_changes_nothing(oracle, tmp_path):
    """A unit with UPDATE set and no data (the reference would dereference NULL at
    recovery.c:123): a try-update that would fold into it is refused (CEC_EINVAL) before
    anything changes -- in a window, even when the offending update is the third, the
    earlier updates' touch_flags, need[] and the fold queue stay as they were; the same for
    the single-update calls, deferred and immediate (refused before any GPU pass)."""
    _need_exe()
    k, m, s, n = 3, 2, 4, 32
    rng, heap, mod, sc = _setup(oracle, k, m, s, n, seed=5)
    base = n * U
    sc.add("D", 0, 0, 7, base)                   # units 0..7 touched (first touch, D0 in)
    mod.recover(0, 0, 7, base, defer=True)
    sc.add("flag", 20, F_UPDATE, -1)             # UPDATE without data
    mod.flags[20] = F_UPDATE
    window = [(1, 1 * U + 64, 300, base + 9 * U), (2, 3 * U, 2 * U, base + 10 * U),
              (1, 19 * U + 4000, 200, base + 12 * U), (2, 5 * U, 100, base + 13 * U)]
    for op in ("w", "W"):
        sc.add(op, len(window))
        for w in window:
            sc.add(*w)
    sc.add("t", 2, 20 * U + 8, 64, base + 14 * U)
    sc.add("T", 1, 19 * U + 4090, 20, base + 14 * U)
    sc.add("P")
    log, flags, data, touch, _, _ = run_script(tmp_path, sc, heap, n, k, m)
    lines = [ln.split() for ln in log]
    assert [ln for ln in lines if ln[0] in "wW"] == [["w", "-1", "0", "0", "0", "0"], ["W", "-1", "0", "0", "0", "0"]]
    assert [ln for ln in lines if ln[0] in "tT"] == [["t", "-1"], ["T", "-1"]]
    check_state(mod, flags, data, touch)         # no touch_flags byte written by the refusals
    assert jobs_from_log(log) == mod.queue       # only the reply's folds queued


def _random_script(oracle, seed, k, m, s, n, gpu_ops=False):
    """Random ranges / diffs / flags: replies of every data peer (each unit at most once
    per peer, as the protocol delivers), SET diffs of any lid at any address and size,
    sub_flags, recovered units; deferred (and, with gpu_ops, immediate) forms mixed."""
    rng, heap, mod, sc = _setup(oracle, k, m, s, n, seed=seed)
    base = n * U
    applied = {p: set() for p in range(k)}
    for _ in range(int(rng.integers(10, 30))):
        r = rng.random()
        if r < 0.35:
            p = int(rng.integers(0, k))
            ub = int(rng.integers(0, n - 1))
            ue = min(n - 1, ub + int(rng.integers(0, 8)))
            off = base + int(rng.integers(0, (8 << 20) - (ue - ub + 1) * U) // 16) * 16
            imm = gpu_ops and rng.random() < 0.5
            sc.add("R" if imm else "D", p, ub, ue, off)
            mod.recover(p, ub, ue, off, defer=not imm)
        elif r < 0.75:
            p = int(rng.integers(0, k))
            size = int(rng.integers(1, 3 * U))
            addr = int(rng.integers(0, n * U - size))
            off = base + int(rng.integers(0, (8 << 20) - size))
            imm = gpu_ops and rng.random() < 0.5
            sc.add("T" if imm else "t", p, addr, size, off)
            mod.try_update(p, addr, size, off, defer=not imm)
        elif r < 0.85:
            cnt = int(rng.integers(1, 6))
            imm = gpu_ops and rng.random() < 0.5
            sc.add("W" if imm else "w", cnt)
            for _ in range(cnt):
                p = int(rng.integers(0, k))
                size = int(rng.integers(1, 2 * U))
                addr = int(rng.integers(0, n * U - size))
                off = base + int(rng.integers(0, (8 << 20) - size))
                sc.add(p, addr, size, off)
                mod.try_update(p, addr, size, off, defer=not imm)
        elif r < 0.93:
            i = int(rng.integers(0, n))
            v = int(rng.choice([0, 1, 2]))
            sc.add("sub", i, v)
            mod.sub = mod.sub if mod.sub is not None else np.zeros(n, np.uint8)
            mod.sub[i] = v
        else:
            i = int(rng.integers(0, n))
            if mod.data[i] is None and mod.flags[i] == 0:
                sc.add("flag", i, F_RECOVERED, -1)
                mod.flags[i] = F_RECOVERED
    return heap, mod, sc


@pytest.mark.parametrize("seed", range(12))
def test_defer_random_scripts(oracle, tmp_path, seed):
    """Random recovery traffic, deferred: flags, touch_flags, returns, first-touch copies
    and the queued fold list equal the model's (no GPU: nothing is flushed)."""
    _need_exe()
    heap, mod, sc = _random_script(oracle, seed, 3, 2, 3 + seed % 2, 48)
    sc.add("P")
    log, flags, data, touch, _, _ = run_script(tmp_path, sc, heap, 48, 3, 2)
    check_state(mod, flags, data, touch)
    assert jobs_from_log(log) == mod.queue


def test_glue_recovery_under_asan_ubsan(oracle, tmp_path):
    """The glue's host logic (flag walk, queues, owned copies, solve job building) under
    AddressSanitizer + UBSan (gcc), over the CPU scripts above."""
    ref = "/root/reference/recovery.h"
    if not os.path.exists(ref):
        pytest.skip("the reference's recovery.h is not here")
    exe = tmp_path / "glue_recovery_asan"
    subprocess.run(["gcc", "-O1", "-g", "-std=gnu11", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"),
                    "-I", os.path.dirname(ref), "-o", str(exe), os.path.join(ROOT, "tests", "glue", "recovery_main.c"),
                    os.path.join(ROOT, "integration", "cocytus_recovery.c"),
                    os.path.join(ROOT, "integration", "cocytus_drain.c"),
                    os.path.join(ROOT, "integration", "cocytus_set.c"), "-L", os.path.join(ROOT, "cocytus_amd"),
                    "-lcocytus_ec", "-Wl,-rpath," + os.path.join(ROOT, "cocytus_amd")], check=True)
    global EXE
    saved, EXE = EXE, str(exe)
    os.environ["ASAN_OPTIONS"] = "detect_leaks=1"
    try:
        for sub in ("a", "b", "c"):
            d = tmp_path / sub
            d.mkdir()
        test_defer_flags_first_touch_and_queue(oracle, tmp_path / "a")
        test_defer_refuses_what_the_reference_asserts(oracle, tmp_path / "b")
        test_defer_random_scripts(oracle, tmp_path / "c", 3)
    finally:
        EXE = saved
        os.environ.pop("ASAN_OPTIONS", None)


# ----------------------------------------------------------------- GPU: the bytes
def _solve_masks(rng, k, m, s):
    """Every loss count 1..m with this parity in the mask (start_recovery's masks: this
    leader + the other parities it needs + the surviving data lids), and masks without
    this parity (start_fast_recovery's) where enough other parities exist."""
    masks = []
    others = [p for p in range(k, k + m) if p != s]
    for n_lost in range(1, m + 1):
        lost = set(int(x) for x in rng.choice(k, n_lost, replace=False))
        pars = [s] + [int(x) for x in rng.choice(others, n_lost - 1, replace=False)]
        masks.append(sum(1 << p for p in pars) | sum(1 << j for j in range(k) if j not in lost))
    for n_lost in range(1, len(others) + 1):
        lost = set(int(x) for x in rng.choice(k, n_lost, replace=False))
        pars = [int(x) for x in rng.choice(others, n_lost, replace=False)]
        masks.append(sum(1 << p for p in pars) | sum(1 << j for j in range(k) if j not in lost))
    return masks


def _solve_ops(rng, mod, sc, n, k, m, s, deferred):
    """Leader solves over ranges made complete first (every data lid of the mask applied)
    for every mask of _solve_masks, on unit ranges of 1-4 units: C from this parity's units
    and the other parities' residuals (data_from_parity), as memcached.c:7868-7922."""
    base = n * U
    want = []
    for q, mk in enumerate(_solve_masks(rng, k, m, s)):
        ub = 4 * q
        ue = ub + int(rng.integers(0, 4))
        assert ue < n
        dfp = [-1] * (k + m)
        for p in range(k, k + m):
            if mk >> p & 1 and p != s:
                dfp[p] = base + int(rng.integers(0, (8 << 20) - (ue - ub + 1) * U))
        if mk >> s & 1:  # make the range complete on this parity first: every data lid of the mask
            for j in range(k):
                if mk >> j & 1:
                    todo = [i for i in range(ub, ue + 1) if not mod.flags[i] & (1 << j)]
                    if any(mod.flags[i] & F_RECOVERED for i in todo):
                        continue
                    for i in todo:
                        off = base + int(rng.integers(0, (8 << 20) - U))
                        sc.add("D" if deferred else "R", j, i, i, off)
                        mod.recover(j, i, i, off, defer=False)
        sc.add("Q" if deferred else "S", ub, ue, mk, *dfp)
        rc, out = mod.solve(ub, ue, mk, dfp)
        want.append((rc, out))
    return want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_glue_bytes_match_reference_chain(gpu, oracle, tmp_path, seed):
    """Immediate and deferred forms mixed (R/T/W and D/t/w, a flush at the end), then
    leader solves for every loss count up to m: every unit byte, flag, touch flag and solve
    output equals the reference's per-unit chain run by the model.  RS(3,2) (seeds 0-3),
    RS(4,2) (4-5) and RS(6,3) (6-7), this parity rotating over the parity lids."""
    _need_exe()
    k, m = ([(3, 2)] * 4 + [(4, 2)] * 2 + [(6, 3)] * 2)[seed]
    s, n = k + seed % m, 48
    heap, mod, sc = _random_script(oracle, seed, k, m, s, n, gpu_ops=True)
    sc.add("F")
    _apply_model_queue(mod)
    rng = np.random.default_rng(100 + seed)
    deferred = seed % 2 == 1
    want = _solve_ops(rng, mod, sc, n, k, m, s, deferred)
    if deferred:
        sc.add("F")
    log, flags, data, touch, _, solves = run_script(tmp_path, sc, heap, n, k, m)
    check_state(mod, flags, data, touch)
    rcs = [(int(ln.split()[1]), int(ln.split()[2])) for ln in log if ln[0] in "SQ"]
    assert [r for r, _ in rcs] == [w[0] for w in want]
    outs = np.concatenate([o for rc, out in want if rc == 0 and out for o in out]) if any(
        rc == 0 and out for rc, out in want) else np.zeros(0, np.uint8)
    assert np.array_equal(solves, outs)
    assert all(int(ln.split()[1]) >= 0 for ln in log if ln.startswith("F "))


def _apply_model_queue(mod: Model):
    """The flush, in the model: every queued fold, in queue order."""
    for (_, dst_desc, _, ln, c, _), src in zip(mod.queue, mod.queue_src):
        _, unit, off = dst_desc.split(":")
        mod.o.region_multiply(src.copy(), c, mod.data[int(unit)][int(off):int(off) + ln], 1)
    mod.queue.clear()
    mod.queue_src.clear()


@pytest.mark.gpu
@pytest.mark.parametrize("defer", [0, 1])
def test_drain_during_recovery_folds_then_applies(gpu, oracle, tmp_path, defer):
    """A parity draining SET diffs while a recovery is in flight (process_rep_command,
    memcached.c:7739-7767: recovery_try_update_unit, then the parity multiply if it says
    so): cocytus_drain_gf with the recovery glue's fold hook, over the server's
    rep_queue.h, into the parity arena kept in host memory (registered with
    cec_host_register: the unchanged server's ecmem) -- the folds of the whole window in one
    batch (or queued: defer), the apply in one.  Units, flags, touch_flags and the arena
    equal the per-xid chain."""
    _need_exe()
    k, m, s, n = 3, 2, 4, 64
    rng, heap, mod, sc = _setup(oracle, k, m, s, n, seed=40 + defer)
    base = n * U
    for p, ub, ue in ((0, 0, 31), (1, 0, 15), (2, 40, 47)):
        off = base + int(rng.integers(0, (4 << 20) // 16)) * 16
        sc.add("R", p, ub, ue, off)
        assert mod.recover(p, ub, ue, off) == 0
    sc.add("sub", 5, 2)
    mod.sub = np.zeros(n, np.uint8)
    mod.sub[5] = 2
    for lid in (1, 2, 0):
        cnt = 150
        sc.add("Z", lid, cnt, defer)
        c = mod.c(s, lid)
        for _ in range(cnt):
            size = int(rng.integers(1, 6000))
            addr = 16 * int(rng.integers(0, (n * U - size) // 16))
            off = base + (4 << 20) + int(rng.integers(0, (4 << 20) - size))
            sc.add(addr, size, off)
            if mod.try_update(lid, addr, size, off, defer=bool(defer)):   # :7758-7767
                oracle.region_multiply(mod.heap[off:off + size].copy(), c, mod.heap[addr:addr + size], 1)
    if defer:
        sc.add("F")
        _apply_model_queue(mod)
    log, flags, data, touch, arena, _ = run_script(tmp_path, sc, heap, n, k, m)
    z = [int(ln.split()[1]) for ln in log if ln.startswith("Z ")]
    assert all(v > 0 for v in z), log
    check_state(mod, flags, data, touch)
    assert np.array_equal(arena, mod.heap[:n * U])


@pytest.mark.gpu
def test_set_diffs_batch(gpu, oracle, tmp_path):
    """The data side (integration/cocytus_set.c): complete_nread's diff of every SET of a
    pass (memcached.c:2664-2681: diff = new value, then ^= 1 * the old bytes at the value's
    new arena address), in one batch -- the diffs equal the reference's per-SET chain
    (values of 1 B - 20 KiB, CRLF-ragged lengths, 16-B aligned addresses as ecalloc.c:176
    gives, some reusing the same old bytes)."""
    _need_exe()
    k, m, s, n = 3, 2, 3, 2048
    rng, heap, mod, sc = _setup(oracle, k, m, s, n, seed=77)
    base = n * U
    sets = []
    for _ in range(600):
        size = int(rng.integers(1, 20 << 10)) + 2
        addr = 16 * int(rng.integers(0, (n * U - size) // 16))
        off = base + int(rng.integers(0, (8 << 20) - size))
        sets.append((addr, size, off))
    sc.add("V", len(sets))
    for addr, size, off in sets:
        sc.add(addr, size, off)
    log, _, _, _, _, diffs = run_script(tmp_path, sc, heap, n, k, m)
    assert "V 0" in log
    want = []
    for addr, size, off in sets:
        d = heap[off:off + size].copy()                                   # memcpy(diff, c->vbuf)
        oracle.region_multiply(heap[addr:addr + size].copy(), 1, d, 1)    # ^= 1 * ecmem[addr]
        want.append(d)
    assert np.array_equal(diffs, np.concatenate(want))


SIM = os.path.join(ROOT, "oracle", "_ref", "glue_cluster_sim")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("defer", [0, 1, 2])
@pytest.mark.parametrize("code", ["", "63"])
def test_cluster_sim_rebuilds_the_lost_shard(gpu, seed, defer, code):
    """An RS(3,2) group in one process through all the glue (tests/glue/cluster_sim.c): SET
    diffs from every data process queued at both parities and drained through the recovery
    fold hook into registered host arenas; a data process lost mid-stream; the leader
    parity rebuilds every unit range while the survivors keep writing (each reply applied
    after that peer's queue is drained, drains folding at random moments, immediate or
    deferred, or -- defer 2 -- on the pool placement, cocytus_recovery_pool.c).  RS(3,2)
    and RS(6,3) (code "63"), 1..M data lids lost: every parity of
    start_recovery's mask folds the replies and the non-leaders ship their units to the
    leader (data_from_parity).  Every rebuilt range equals the bytes the lost shards held --
    a truth that needs no oracle -- and the parities end as the code of the data."""
    exe = SIM + code
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built (make -C oracle ref)")
    r = subprocess.run([exe, str(seed), str(defer)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr
    m = 3 if code == "63" else 2
    assert f"lost {1 + seed % m} data lids" in r.stdout, r.stdout  # every loss count over the seeds


@pytest.mark.gpu
@pytest.mark.parametrize("defer", [0, 2])
def test_cluster_sim_control_breaks_without_the_drain(gpu, defer):
    """The same simulation with the protocol broken on purpose -- each reply applied before
    that peer's queued diffs are drained (skipping recover_units_reply's drain,
    memcached.c:4311-4316) -- must rebuild wrong bytes: the check above detects a wrong fold."""
    if not os.path.exists(SIM):
        pytest.skip("oracle/_ref/glue_cluster_sim not built (make -C oracle ref)")
    r = subprocess.run([SIM, "0", str(defer), "1", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "differ" in r.stdout, r.stdout + r.stderr
