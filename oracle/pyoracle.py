"""ctypes wrapper of oracle/libgf8ref.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker (or the timed CPU baseline).  PARITY UNPINNED: see
gf8_ref.h -- the reference's Jerasure/GF-Complete is not available to run.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgf8ref.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_ip = ctypes.POINTER(ctypes.c_int)
_i = ctypes.c_int
_l = ctypes.c_long
_u32 = ctypes.c_uint32
_vpp = ctypes.POINTER(ctypes.c_void_p)

_SIGS = {
    "ref_gf_mul": ([_i, _i], _i),
    "ref_gf_div": ([_i, _i], _i),
    "ref_gf_exp": ([_i], _i),
    "ref_gf_log": ([_i], _i),
    "ref_region_multiply": ([ctypes.c_void_p, _i, _l, ctypes.c_void_p, _i], None),
    "ref_extended_vandermonde": ([_i, _i], _ip),
    "ref_big_vandermonde": ([_i, _i], _ip),
    "ref_invert_matrix": ([_ip, _ip, _i], _i),
    "ref_set_diff": ([ctypes.c_void_p, ctypes.c_void_p, _l, ctypes.c_void_p], None),
    "ref_parity_apply": ([_ip, _i, _i, _i, ctypes.c_void_p, _l, ctypes.c_void_p], None),
    "ref_diff_update": ([_ip, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p, _l, _vpp, _i], None),
    "ref_encode": ([_ip, _i, _i, _vpp, _vpp, _l], None),
    "ref_recovery_mask": ([_i, _i, _i, _ip], _u32),
    "ref_recover_units": ([_ip, _i, _i, _i, ctypes.c_void_p, ctypes.c_void_p, _l, ctypes.c_void_p, _ip], None),
    "ref_try_update_unit": ([_ip, _i, _i, _i, ctypes.c_void_p, _l, ctypes.c_void_p], None),
    "ref_bottom_half": ([_ip, _i, _i, _u32, _vpp, _l, _vpp], _i),
    "ref_decode": ([_ip, _i, _i, _u32, _vpp, _l, _vpp], _i),
    "ref_region_multiply_simd": ([ctypes.c_void_p, _i, _l, ctypes.c_void_p], None),
    "ref_simd_available": ([], _i),
    "ref_bench_encode_decode": ([_i, _i, _l, _l, _i, _i, _i], ctypes.c_double),
    "ref_bench_encode_decode_samples": ([_i, _i, _l, _l, _i, _i, _i, _i, ctypes.POINTER(ctypes.c_double)], _i),
    "ref_bench_encode_decode_sizes": ([_i, _i, _l, ctypes.c_void_p, _l, _i, _i, _i, _i,
                                       ctypes.POINTER(ctypes.c_double)], _i),
    "ref_bench_apply": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_void_p, _i, ctypes.c_void_p], ctypes.c_double),
    "ref_bench_recover": ([ctypes.c_void_p, _vpp, ctypes.c_void_p, _i, _i, _l, ctypes.c_void_p,
                           ctypes.c_void_p], ctypes.c_double),
    "ref_bench_set_diffs": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, _i, ctypes.c_void_p, ctypes.c_void_p], ctypes.c_double),
    "ref_bench_recover_requests": ([ctypes.c_void_p, ctypes.c_void_p, _i, _i, _vpp, _i, ctypes.c_void_p, _i,
                                    _vpp], ctypes.c_double),
}

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        for n, (a, r) in _SIGS.items():
            f = getattr(L, n)
            f.argtypes = a
            f.restype = r
        libc = ctypes.CDLL(None)
        libc.free.argtypes = [ctypes.c_void_p]
        L._free = libc.free
        _lib = L
    return _lib


def _p(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def _arr(xs):
    return (ctypes.c_void_p * len(xs))(*[_p(x) for x in xs])


def _mat(matrix):
    return (ctypes.c_int * len(matrix))(*[int(v) for v in matrix])


def gf_mul(a: int, b: int) -> int:
    return lib().ref_gf_mul(a, b)


def gf_div(a: int, b: int) -> int:
    return lib().ref_gf_div(a, b)


def gf_exp(i: int) -> int:
    return lib().ref_gf_exp(i)


def gf_log(a: int) -> int:
    return lib().ref_gf_log(a)


def region_multiply(region: np.ndarray, multby: int, r2: np.ndarray | None, add: int = 1) -> None:
    n = region.size if r2 is None else min(region.size, r2.size)
    lib().ref_region_multiply(_p(region), multby, n, _p(r2), add)


def _take_matrix(p, n) -> list[int] | None:
    if not p:
        return None
    out = [p[i] for i in range(n)]
    lib()._free(ctypes.cast(p, ctypes.c_void_p))
    return out


def big_vandermonde(rows: int, cols: int) -> list[int] | None:
    return _take_matrix(lib().ref_big_vandermonde(rows, cols), rows * cols)


def extended_vandermonde(rows: int, cols: int) -> list[int] | None:
    return _take_matrix(lib().ref_extended_vandermonde(rows, cols), rows * cols)


def invert(mat: list[int], n: int) -> tuple[int, list[int]]:
    a = _mat(mat)
    inv = (ctypes.c_int * (n * n))()
    rc = lib().ref_invert_matrix(a, inv, n)
    return rc, list(inv)


def set_diff(old: np.ndarray, new: np.ndarray) -> np.ndarray:
    d = np.empty_like(new)
    lib().ref_set_diff(_p(old), _p(new), new.size, _p(d))
    return d


def parity_apply(matrix, k, lid_self, lid_src, diff: np.ndarray, parity: np.ndarray) -> None:
    lib().ref_parity_apply(_mat(matrix), k, lid_self, lid_src, _p(diff), diff.size, _p(parity))


def diff_update(matrix, k, m, j, old: np.ndarray, new: np.ndarray, parity: list, install: bool) -> None:
    lib().ref_diff_update(_mat(matrix), k, m, j, _p(old), _p(new), new.size, _arr(parity), int(install))


def encode(matrix, k: int, m: int, data: list[np.ndarray]) -> list[np.ndarray]:
    n = data[0].size
    par = [np.zeros(n, np.uint8) for _ in range(m)]
    lib().ref_encode(_mat(matrix), k, m, _arr(data), _arr(par), n)
    return par


def recovery_mask(k: int, m: int, leader: int, connected: list[int]) -> int:
    return lib().ref_recovery_mask(k, m, leader, (ctypes.c_int * (k + m))(*connected))


def recover_units(matrix, k, lid_self, peer, own_parity, peer_data, residual, touched: list[int]) -> None:
    t = ctypes.c_int(touched[0])
    lib().ref_recover_units(_mat(matrix), k, lid_self, peer, _p(own_parity), _p(peer_data),
                            peer_data.size, _p(residual), ctypes.byref(t))
    touched[0] = t.value


def try_update_unit(matrix, k, lid_self, peer, diff: np.ndarray, residual_view: np.ndarray) -> None:
    lib().ref_try_update_unit(_mat(matrix), k, lid_self, peer, _p(diff), diff.size, _p(residual_view))


def bottom_half(matrix, k, m, mask, C: list[np.ndarray]) -> list[np.ndarray] | None:
    nbuf = C[0].size
    n_lost = sum(1 for j in range(k) if not (mask >> j) & 1)
    out = [np.empty(nbuf, np.uint8) for _ in range(n_lost)]
    r = lib().ref_bottom_half(_mat(matrix), k, m, mask, _arr(C), nbuf, _arr(out))
    return None if r < 0 else out


def decode(matrix, k, m, mask, arenas: list) -> list[np.ndarray] | None:
    n = next(a.size for a in arenas if a is not None)
    n_lost = sum(1 for j in range(k) if not (mask >> j) & 1)
    out = [np.empty(n, np.uint8) for _ in range(n_lost)]
    r = lib().ref_decode(_mat(matrix), k, m, mask, _arr(arenas), n, _arr(out))
    return None if r < 0 else out


def region_multiply_simd(region: np.ndarray, multby: int, r2: np.ndarray) -> None:
    lib().ref_region_multiply_simd(_p(region), multby, region.size, _p(r2))


def simd_available() -> bool:
    return bool(lib().ref_simd_available())


def bench_encode_decode(k, m, n, nstripes, threads, reps=1, do_decode=True) -> float:
    return lib().ref_bench_encode_decode(k, m, n, nstripes, threads, reps, int(do_decode))


def bench_encode_decode_samples(k, m, n, nstripes, threads, reps, samples, do_decode=True) -> list[float]:
    """Seconds of each of `samples` passes (reps repetitions each) over one filled batch."""
    t = (ctypes.c_double * samples)()
    if lib().ref_bench_encode_decode_samples(k, m, n, nstripes, threads, reps, int(do_decode), samples, t):
        raise ValueError("ref_bench_encode_decode_samples: bad arguments")
    return list(t)


def bench_encode_decode_sizes(k, m, lens, threads, reps, samples, do_decode=True) -> list[float]:
    """bench_encode_decode_samples over stripes of the given lengths (mixed value sizes)."""
    ln = np.ascontiguousarray(lens, np.int64)
    t = (ctypes.c_double * samples)()
    if lib().ref_bench_encode_decode_sizes(k, m, 0, ln.ctypes.data, len(ln), threads, reps, int(do_decode),
                                           samples, t):
        raise ValueError("ref_bench_encode_decode_sizes: bad arguments")
    return list(t)


def bench_apply(stage: np.ndarray, soffs, addrs, lens, coefs, parity: np.ndarray) -> float:
    """The reference's single-threaded drain loop over packed diffs; seconds."""
    so = np.ascontiguousarray(soffs, np.uint64)
    ad = np.ascontiguousarray(addrs, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint32)
    cf = np.ascontiguousarray(coefs, np.int32)
    return lib().ref_bench_apply(_p(stage), so.ctypes.data, ad.ctypes.data, ln.ctypes.data,
                                 cf.ctypes.data, len(ln), _p(parity))


def bench_recover(parity: np.ndarray, peers: list, coefs, inv: int) -> tuple[float, np.ndarray]:
    """The reference's one-parity recovery chain (residual + leader solve); (s, out)."""
    n = parity.size
    res = np.empty(n, np.uint8)
    out = np.empty(n, np.uint8)
    cf = np.ascontiguousarray(coefs, np.int32)
    t = lib().ref_bench_recover(_p(parity), _arr(peers), cf.ctypes.data, len(peers), inv, n,
                                _p(res), _p(out))
    return t, out


def bench_set_diffs(values: np.ndarray, voffs, ecmem: np.ndarray, addrs, lens, diffs: np.ndarray,
                    doffs) -> float:
    """The reference's SET-diff loop (memcpy + XOR with the old bytes per SET, one thread)
    over values / diffs packed at the given offsets; seconds."""
    vo = np.ascontiguousarray(voffs, np.uint64)
    ad = np.ascontiguousarray(addrs, np.uint64)
    ln = np.ascontiguousarray(lens, np.uint32)
    do = np.ascontiguousarray(doffs, np.uint64)
    return lib().ref_bench_set_diffs(_p(values), vo.ctypes.data, _p(ecmem), ad.ctypes.data, ln.ctypes.data,
                                     len(ln), _p(diffs), do.ctypes.data)


def bench_recover_requests(ecmem: np.ndarray, starts, units: int, replies: list, npeers: int, coefs,
                           inv: int) -> tuple[float, list]:
    """The reference's recovery of len(starts) single-loss requests led by this parity
    (per-unit folds with malloc'd units, then the bottom half), one thread; replies[q *
    npeers + p].  Returns (seconds, [rebuilt bytes per request])."""
    st = np.ascontiguousarray(starts, np.int32)
    cf = np.ascontiguousarray(coefs, np.int32)
    outs = [np.empty(units * 4096, np.uint8) for _ in range(len(st))]
    t = lib().ref_bench_recover_requests(_p(ecmem), st.ctypes.data, len(st), units, _arr(replies), npeers,
                                         cf.ctypes.data, inv, _arr(outs))
    return t, outs


def splitmix_bytes(seed: int, n: int) -> np.ndarray:
    """Deterministic uniform bytes (splitmix64), the synthetic input of SURVEY §8d."""
    words = (n + 7) // 8
    idx = np.arange(1, words + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:n].copy()
