"""Probe for a system Jerasure 2.x / GF-Complete (TEST INFRASTRUCTURE, never product).

SURVEY.md §8(c)/§8(d): the reference links a bare `-lJerasure`
(/root/reference/Makefile.am:46,49); neither Jerasure nor GF-Complete is vendored in
/root/reference or installed in this image, so the oracle is "parity unpinned".  This
module looks for a system copy anyway (here and on the GPU box).  When one exists it
is used to pin the oracle (tests/test_oracle.py::test_oracle_vs_system_jerasure) and
bench.py reports it; when none exists both say so.

Our own shim (cocytus_amd/libJerasure.so -> libcocytus_ec.so) exports the same
symbols, so anything that resolves inside this repository is rejected: a probe that
found the shim would pin the product against itself.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_DIRS = ["/usr/lib", "/usr/lib64", "/usr/local/lib", "/usr/local/lib64",
         "/usr/lib/x86_64-linux-gnu", "/opt/rocm/lib"]


def candidates() -> list[str]:
    """Paths of system libJerasure shared objects (the repository's shim excluded)."""
    found = []
    name = ctypes.util.find_library("Jerasure")
    if name:
        found.append(name)
    for d in _DIRS:
        found.extend(sorted(glob.glob(os.path.join(d, "libJerasure.so*"))))
    out = []
    for p in found:
        real = os.path.realpath(p) if os.path.isabs(p) else p
        if os.path.isabs(real) and real.startswith(ROOT + os.sep):
            continue
        if real not in out:
            out.append(real)
    return out


def load():
    """(CDLL, path) of the first loadable system Jerasure, or (None, reason)."""
    for p in candidates():
        try:
            lib = ctypes.CDLL(p)
        except OSError:
            continue
        try:
            path = os.path.realpath(p)
            if path.startswith(ROOT + os.sep):
                continue
            lib.galois_w08_region_multiply.restype = None
            lib.galois_w08_region_multiply.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                                       ctypes.c_void_p, ctypes.c_int]
            lib.reed_sol_big_vandermonde_distribution_matrix.restype = ctypes.POINTER(ctypes.c_int)
            lib.reed_sol_big_vandermonde_distribution_matrix.argtypes = [ctypes.c_int] * 3
        except AttributeError:
            continue
        return lib, path
    return None, "no system libJerasure (searched find_library and " + ", ".join(_DIRS) + ")"


def matrix(lib, k: int, m: int) -> list[int]:
    """reed_sol_big_vandermonde_distribution_matrix(k+m, k, 8) as called at memcached.c:6845."""
    p = lib.reed_sol_big_vandermonde_distribution_matrix(k + m, k, 8)
    return [p[i] for i in range((k + m) * k)]


def encode(lib, mat: list[int], k: int, m: int, data):
    """Parity the way the reference accumulates it: one region multiply-XOR per
    (parity, data shard), memcached.c:2681 -> 7764 (numpy uint8 arrays)."""
    import numpy as np

    n = len(data[0])
    out = []
    for p in range(m):
        acc = np.zeros(n, np.uint8)
        for j in range(k):
            src = np.ascontiguousarray(data[j])
            lib.galois_w08_region_multiply(src.ctypes.data, mat[(k + p) * k + j], n, acc.ctypes.data, 1)
        out.append(acc)
    return out
