"""The reference's own arena allocator, run here -- TEST INFRASTRUCTURE ONLY.

oracle/_ref/libecalloc_ref.so is /root/reference/ecalloc.c + avltree.c, unmodified,
behind oracle/ecalloc_shim.c (`make -C oracle ref`; only where /root/reference exists).
It produces value addresses exactly as a Cocytus data server does:

  * every SET allocates the value's new space, ecmem_alloc(&ecmem, it->nbytes)
    (memcached.c:2667), with nbytes = vlen + 2 (memcached.c:3610) rounded up to 16
    bytes by ec_alloc (ecalloc.c:176);
  * replacing a key frees the old value's space afterwards (store_item,
    memcached.c:2888-2889);
  * each data shard lid has its own allocator, and the parity replays it per lid
    (memcached.c:7704-7717), so parity byte a covers byte a of every shard: SETs of
    different shards can overlap in the parity arena.

The layout is frozen in tests/golden/ecalloc_layout.npz (tests/golden/make_ecalloc_layout.py),
so the GPU tests need neither /root/reference nor this library.
"""
from __future__ import annotations

import ctypes
import math
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_ref", "libecalloc_ref.so")
_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"{LIB_PATH} not built (make -C oracle ref, needs /root/reference)")
        L = ctypes.CDLL(LIB_PATH)
        L.ref_ecalloc_create.restype = ctypes.c_void_p
        L.ref_ecalloc_create.argtypes = [ctypes.c_uint64]
        L.ref_ec_alloc.restype = ctypes.c_uint64
        L.ref_ec_alloc.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.ref_ec_free.restype = None
        L.ref_ec_free.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.ref_ec_used.restype = ctypes.c_uint64
        L.ref_ec_used.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


def set_trace(seed: int, k: int, arena: int = 64 << 20, keys: int = 1500, churn: int = 6000,
              batch: int = 400, vmin: int = 254, vmax: int = 65534):
    """Per data shard j: the final batch of `batch` SETs on distinct keys after a
    warm-up (every key SET once) and `churn` replacing SETs; values log-uniform in
    [vmin, vmax] bytes.  Returns [(j, addr, nbytes)] in SET order."""
    L = lib()
    rng = random.Random(seed)
    lo, hi = math.log(vmin), math.log(vmax)
    out = []
    for j in range(k):
        a = L.ref_ecalloc_create(arena)
        live = {}

        def set_key(key):
            nbytes = int(math.exp(rng.uniform(lo, hi))) + 2  # vlen + "\r\n"
            addr = L.ref_ec_alloc(a, nbytes)
            old = live.get(key)
            live[key] = addr
            if old is not None:
                L.ref_ec_free(a, old)  # store_item frees the replaced value
            return addr, nbytes

        for key in range(keys):
            set_key(key)
        for _ in range(churn):
            set_key(rng.randrange(keys))
        for key in rng.sample(range(keys), batch):
            addr, nbytes = set_key(key)
            out.append((j, addr, nbytes))
    return out
