"""The recovery glue's pool placement (integration/cocytus_recovery_pool.c: the idle
recoverer's requests coalesced onto a cec_recovery_pool, residuals in HBM, one launch per
event-loop pass) driven over the server's own types by oracle/_ref/glue_rpool
(tests/glue/rpool_main.c, built by oracle/Makefile `ref` against the reference's
recovery.h / rep_queue.h where they lie).  Skips where it was not built.

The model is test_glue_recovery's restatement of recovery.c:61-131 and memcached.c:
7842-7922 (one oracle region multiply per unit, in the reference's order), with the
request bookkeeping of recovery_req_add / recovery_req_remove (recovery.c:190-238).  Every
op's return value, every unit flag and touch flag, the parity arena after the drains,
every residual a non-leader would send and every solve output equal the model's.
"""
from __future__ import annotations

import os
import subprocess

import numpy as np
import pytest

from tests.test_glue_recovery import Model, U

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.environ.get("CEC_GLUE_RPOOL_EXE") or os.path.join(ROOT, "oracle", "_ref", "glue_rpool")
EXTRA = 8 << 20


def _need_exe():
    if not os.path.exists(EXE):
        pytest.skip("oracle/_ref/glue_rpool not built (make -C oracle ref)")


def run(tmp_path, lines, heap, nunits, k, m):
    sp, hp, out = tmp_path / "script.txt", tmp_path / "heap.bin", tmp_path / "out"
    sp.write_text("\n".join(lines) + "\n")
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
    log = [ln for ln in (tmp_path / "out.log").read_text().split("\n") if ln]
    raw = np.fromfile(tmp_path / "out.units", dtype=np.uint8)
    flags = [int(x) for x in raw[:4 * nunits].view(np.uint32)]
    p = 4 * nunits
    touch = [raw[p + l * nunits:p + (l + 1) * nunits] for l in range(k + m)]
    p += (k + m) * nunits
    arena = raw[p:p + nunits * U]
    return log, flags, touch, arena, np.fromfile(tmp_path / "out.solves", dtype=np.uint8)


def _masks(k, m, s, rng):
    """start_recovery's masks (this parity + the parities it needs + the surviving data
    lids) for every loss count, and start_fast_recovery's (this parity not in the mask)."""
    others = [p for p in range(k, k + m) if p != s]
    out = []
    for n_lost in range(1, m + 1):
        lost = set(int(x) for x in rng.choice(k, n_lost, replace=False))
        pars = [s] + [int(x) for x in rng.choice(others, n_lost - 1, replace=False)]
        out.append(sum(1 << p for p in pars) | sum(1 << j for j in range(k) if j not in lost))
    lost = set(int(x) for x in rng.choice(k, 1, replace=False))
    out.append((1 << others[0]) | sum(1 << j for j in range(k) if j not in lost))
    return out


class Sim:
    """The script and the model side by side."""

    def __init__(self, oracle, k, m, s, nunits, qcap, cap, seed):
        self.rng = np.random.default_rng(seed)
        self.heap = self.rng.integers(0, 256, nunits * U + EXTRA, dtype=np.uint8)
        self.mod = Model(oracle, self.heap.copy(), k, m, s, nunits)
        self.k, self.m, self.s, self.n, self.qcap = k, m, s, nunits, qcap
        self.lines = [f"init {k} {m} {s} {nunits} {qcap} {cap}"]
        self.want_log: list[str] = []
        self.want_out: list[np.ndarray] = []
        self.active = {}   # qi -> dict(ub, ue, mask, replied, solved)
        self.queued = []   # qi with a solve queued, in order
        self.o = oracle

    def off(self, nbytes):
        return self.n * U + int(self.rng.integers(0, EXTRA - nbytes))

    def data_lids(self, mask):
        return [j for j in range(self.k) if mask >> j & 1]

    def complete(self, r):
        return set(self.data_lids(r["mask"])) <= r["replied"]

    # ---- ops
    def begin(self, qi, ub, ue, mask):
        self.lines.append(f"B {qi} {ub} {ue} {mask}")
        self.want_log.append("B 0")
        self.active[qi] = dict(ub=ub, ue=ue, mask=mask, replied=set(), solved=False, dfp=None)

    def reply(self, qi, peer, staged):
        r = self.active[qi]
        off = self.off((r["ue"] - r["ub"] + 1) * U)
        op = "r" if staged else "R"
        self.lines.append(f"{op} {qi} {peer} {off}")
        self.want_log.append(f"{op} {self.mod.recover(peer, r['ub'], r['ue'], off)}")
        r["replied"].add(peer)

    def set_diff(self, peer, addr, size):
        off = self.off(size)
        self.lines.append(f"T {peer} {addr} {size} {off}")
        self.want_log.append(f"T {self.mod.try_update(peer, addr, size, off)}")

    def window(self, ups):
        self.lines.append(f"W {len(ups)}")
        need = []
        for peer, addr, size in ups:
            off = self.off(size)
            self.lines.append(f"{peer} {addr} {size} {off}")
            need.append(self.mod.try_update(peer, addr, size, off))
        self.want_log.append("W 0 " + " ".join(str(x) for x in need))

    def drain(self, lid, ups):
        """process_rep_command per xid (memcached.c:7758-7767): fold, then the apply."""
        self.lines.append(f"Z {lid} {len(ups)}")
        c, applied = self.mod.c(self.s, lid), 0
        for addr, size in ups:
            off = self.off(size)
            self.lines.append(f"{addr} {size} {off}")
            if self.mod.try_update(lid, addr, size, off):
                self.o.region_multiply(self.mod.heap[off:off + size].copy(), c, self.mod.heap[addr:addr + size], 1)
                applied += 1
        self.want_log.append(f"Z {applied}")

    def residual(self, qi):
        r = self.active[qi]
        self.lines.append(f"X {qi}")
        self.want_log.append("X 0")
        self.want_out.append(np.concatenate([self.mod.data[i] for i in range(r["ub"], r["ue"] + 1)]))

    def solve(self, qi):
        r = self.active[qi]
        dfp = [-1] * (self.k + self.m)
        for p in range(self.k, self.k + self.m):
            if r["mask"] >> p & 1 and p != self.s:
                dfp[p] = self.off((r["ue"] - r["ub"] + 1) * U)
        self.lines.append(f"S {qi} " + " ".join(str(x) for x in dfp))
        n_lost = sum(1 for j in range(self.k) if not r["mask"] >> j & 1)
        self.want_log.append(f"S 0 {n_lost}")
        r["solved"], r["dfp"] = True, dfp
        self.queued.append(qi)

    def flush(self):
        self.lines.append("F")
        self.want_log.append(f"F {len(self.queued)}")
        for qi in self.queued:  # the bottom half at the flush, over the residual as it is then
            r = self.active[qi]
            rc, out = self.mod.solve(r["ub"], r["ue"], r["mask"], r["dfp"])
            assert rc == 0
            self.want_out.extend(out)
        self.queued = []

    def end(self, qi):
        r = self.active.pop(qi)
        self.lines.append(f"E {qi}")
        self.want_log.append("E 0")
        for i in range(r["ub"], r["ue"] + 1):  # recovery_req_remove (recovery.c:200-205)
            self.mod.flags[i] = 0
            self.mod.data[i] = None
        if qi in self.queued:
            self.queued.remove(qi)

    def sub(self, i, v):
        self.lines.append(f"sub {i} {v}")
        self.mod.sub = self.mod.sub if self.mod.sub is not None else np.zeros(self.n, np.uint8)
        self.mod.sub[i] = v

    # ---- random traffic
    def free_range(self, width):
        busy = np.zeros(self.n, bool)
        for r in self.active.values():
            busy[r["ub"]:r["ue"] + 1] = True
        for _ in range(20):
            ub = int(self.rng.integers(0, self.n - width + 1))
            if not busy[ub:ub + width].any() and all(self.mod.flags[i] == 0 for i in range(ub, ub + width)):
                return ub
        return None

    def random_update(self):
        size = int(self.rng.integers(1, 2 * U))
        return int(self.rng.integers(0, self.k)), int(self.rng.integers(0, self.n * U - size)), size

    def step(self, masks):
        x = self.rng.random()
        free_q = [q for q in range(self.qcap) if q not in self.active]
        if x < 0.2 and free_q:
            width = 1 if self.rng.random() < 0.7 else int(self.rng.integers(2, 5))
            ub = self.free_range(width)
            if ub is not None:
                self.begin(free_q[int(self.rng.integers(0, len(free_q)))], ub, ub + width - 1,
                           masks[int(self.rng.integers(0, len(masks)))])
        elif x < 0.5:
            cand = [(q, j) for q, r in self.active.items() if r["mask"] >> self.s & 1 and not r["solved"]
                    for j in self.data_lids(r["mask"]) if j not in r["replied"]]
            if cand:
                q, j = cand[int(self.rng.integers(0, len(cand)))]
                self.reply(q, j, self.rng.random() < 0.5)
        elif x < 0.62:
            self.set_diff(*self.random_update())
        elif x < 0.67:
            self.window([self.random_update() for _ in range(int(self.rng.integers(1, 6)))])
        elif x < 0.72:
            lid = int(self.rng.integers(0, self.k))
            ups = []
            for _ in range(int(self.rng.integers(1, 12))):
                size = int(self.rng.integers(1, 6000))
                ups.append((16 * int(self.rng.integers(0, (self.n * U - size) // 16)), size))
            self.drain(lid, ups)
        elif x < 0.8:
            cand = [q for q, r in self.active.items() if not r["solved"] and
                    (not r["mask"] >> self.s & 1 or self.complete(r))]
            if cand:
                self.solve(cand[int(self.rng.integers(0, len(cand)))])
        elif x < 0.85:
            cand = [q for q, r in self.active.items() if r["mask"] >> self.s & 1 and self.complete(r)]
            if cand:
                self.residual(cand[int(self.rng.integers(0, len(cand)))])
        elif x < 0.92:
            self.flush()
        elif x < 0.97:
            cand = [q for q, r in self.active.items() if r["solved"] and q not in self.queued]
            if not cand and self.active and self.rng.random() < 0.3:  # an abort (restart_failed_recovery)
                cand = [q for q in self.active if q not in self.queued]
            if cand:
                self.end(cand[int(self.rng.integers(0, len(cand)))])
        else:
            self.sub(int(self.rng.integers(0, self.n)), int(self.rng.choice([0, 1, 2])))


def check(sim: Sim, tmp_path):
    log, flags, touch, arena, outs = run(tmp_path, sim.lines, sim.heap, sim.n, sim.k, sim.m)
    assert log == sim.want_log
    assert flags == sim.mod.flags
    for l in range(sim.k + sim.m):
        assert np.array_equal(touch[l], sim.mod.touch[l]), f"touch_flags of lid {l}"
    assert np.array_equal(arena, sim.mod.heap[:sim.n * U])
    want = np.concatenate(sim.want_out) if sim.want_out else np.zeros(0, np.uint8)
    assert outs.size == want.size
    assert np.array_equal(outs, want)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_rpool_random_traffic_matches_reference_chain(gpu, oracle, tmp_path, seed):
    """Random recovery traffic on the pool placement: requests begun over free unit ranges
    (single units mostly, as the idle recoverer; every loss count; masks without this
    parity), replies copied or received in place, SET diffs of every data lid (lost ones
    too: recovery.c:116-120 folds them) alone, in windows and in drain windows that apply to
    the registered host arena right after, non-leader residuals, leader solves at the
    flush, requests ended or aborted.  RS(3,2) (seeds 0-3), RS(4,2) (4-5), RS(6,3) (6-7)."""
    _need_exe()
    k, m = ([(3, 2)] * 4 + [(4, 2)] * 2 + [(6, 3)] * 2)[seed]
    s = k + seed % m
    sim = Sim(oracle, k, m, s, 64, 16, 40, seed=500 + seed)
    masks = _masks(k, m, s, sim.rng)
    for _ in range(220):
        sim.step(masks)
    sim.flush()
    for qi in list(sim.active):
        if sim.active[qi]["mask"] >> s & 1 and sim.complete(sim.active[qi]):
            sim.residual(qi)
    check(sim, tmp_path)
    assert sum(1 for ln in sim.lines if ln.startswith("S ")) >= 3, "too few solves to mean anything"


@pytest.mark.gpu
def test_rpool_idle_recoverer_shape(gpu, oracle, tmp_path):
    """The idle recoverer's pass (memcached.c:5712-5734): 85 single-unit requests in flight
    (TOO_MANY_RECOVERY, const.h:27), both surviving data peers' replies, SETs landing
    between (lost D1's too, forwarded by its substitute), 85 leader solves and ONE flush,
    then fill + recovery_req_remove; twice over (slots reused).  Outputs equal the model."""
    _need_exe()
    k, m, s = 3, 2, 4
    sim = Sim(oracle, k, m, s, 256, 96, 96, seed=9)
    mask = (1 << s) | 1 | 4  # D1 lost, leader P1 (start_recovery's mask)
    for rnd in range(2):
        qs = list(range(85))
        units = sim.rng.permutation(256)[:85]
        for q, u in zip(qs, units):
            sim.begin(q, int(u), int(u), mask)
        for j in (0, 2):
            for q in qs:
                sim.reply(q, j, (q + j) % 2 == 0)
                if q % 17 == 0:
                    sim.set_diff(*sim.random_update())
        for q in qs:
            sim.solve(q)
        sim.flush()
        for q in qs:
            sim.end(q)
    check(sim, tmp_path)


@pytest.mark.gpu
def test_rpool_refusals(gpu, oracle, tmp_path):
    """The reference's assert()s and this placement's own rules, refused before anything
    changes: a peer applied twice (recovery.c:74), a recovered unit (:72), a request begun
    twice, a reply for a request without slots, a solve of an incomplete request or twice,
    a pool too full for the request (CEC_EFULL)."""
    _need_exe()
    k, m, s = 3, 2, 3
    sim = Sim(oracle, k, m, s, 64, 8, 8, seed=3)
    mask = (1 << s) | 2 | 4  # D0 lost, leader P0
    sim.begin(0, 0, 1, mask)
    sim.reply(0, 1, False)
    L = sim.lines
    L.append(f"R 0 1 {sim.off(2 * U)}")           # peer 1 again
    sim.want_log.append("R -1")
    L.append("b 0")                                # begun twice
    sim.want_log.append("b -1")
    L.append("S 0 -1 -1 -1 -1 -1")                 # incomplete: peer 2 missing
    sim.want_log.append("S -1 -1")
    sim.begin(1, 20, 20, mask)
    L.append(f"flag 21 {1 << 31}")
    sim.mod.flags[21] = 1 << 31
    sim.begin(2, 21, 21, mask)
    L.append(f"R 2 1 {sim.off(U)}")                 # a recovered unit
    sim.want_log.append("R -1")
    L.append(f"B 3 30 39 {mask}")                   # 10 units: 2 + 1 + 1 in use of 8
    sim.want_log.append("B -7")
    fast = (1 << (s + 1)) | 2 | 4                   # this parity not in the mask
    sim.begin(4, 50, 50, fast)
    L.append(f"R 4 1 {sim.off(U)}")
    sim.want_log.append("R -1")
    sim.reply(0, 2, True)
    sim.solve(0)
    L.append("S 0 -1 -1 -1 -1 -1")                  # queued already
    sim.want_log.append("S -1 -1")
    sim.flush()
    for q in (0, 1, 2, 4):                          # (E of request 2 resets unit 21's flag)
        sim.end(q)
    check(sim, tmp_path)


DRB = os.path.join(ROOT, "oracle", "_ref", "glue_drain_recovery_bench")


@pytest.mark.gpu
def test_drain_during_recovery_four_paths_agree(gpu):
    """tests/glue/drain_recovery_bench.c at a small size: a drain window during recovery
    (process_rep_command's fold, then the apply) through the host-batch glue, the pool glue,
    the unchanged per-xid loop on the drop-in and on the restated CPU multiply leaves the same
    arena and the same units in all four (its "verified"), half the diffs on units under
    recovery."""
    if not os.path.exists(DRB):
        pytest.skip("oracle/_ref/glue_drain_recovery_bench not built (make -C oracle ref)")
    r = subprocess.run([DRB, "512", "4098", "64", "0.5", "1"], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    import json

    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["verified"] is True and line["aimed_at_recovering_units"] == 256

