"""Python mirror of libcocytus_ec.so (include/cocytus_ec.h + the Jerasure drop-in).

Thin ctypes bindings: the product is the C-ABI library; this module only marshals
arguments and raises on error.  There is no Python or CPU implementation of any
region arithmetic here -- if the shared library (or a gfx950 GPU) is missing, calls
fail loudly.

Device memory is passed as integer device pointers; anything with ``data_ptr()``
(torch tensors) is accepted too.  When torch is used in the same process, import it
BEFORE calling :func:`lib` so that both share one HIP runtime (checked).
"""
from __future__ import annotations

import ctypes
import os
from typing import Iterable, Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
# CEC_LIB_PATH: load another build of the library (A/B measurement of two builds)
LIB_PATH = os.environ.get("CEC_LIB_PATH") or os.path.join(HERE, "libcocytus_ec.so")

CEC_OK = 0
CEC_EINVAL = -1
CEC_ESINGULAR = -2
CEC_EHIP = -3
CEC_ENOMEM = -4
CEC_EOVERLAP = -5
CEC_ENODEV = -6
CEC_EFULL = -7
CEC_ENGINE_PERM = 0
CEC_ENGINE_LDS = 1
CEC_ENGINE_AUTO = 2  # default: LDS for decodes of values >= 64 KiB, PERM for the rest (cocytus_ec.h)
CEC_MAX_K = 16
CEC_MAX_M = 8
UNIT_SIZE = 4096

_STATUS = {
    CEC_EINVAL: "CEC_EINVAL",
    CEC_ESINGULAR: "CEC_ESINGULAR",
    CEC_EHIP: "CEC_EHIP",
    CEC_ENOMEM: "CEC_ENOMEM",
    CEC_EOVERLAP: "CEC_EOVERLAP",
    CEC_ENODEV: "CEC_ENODEV",
}


class CecError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{_STATUS.get(code, code)}: {msg}")
        self.code = code


class Extent(ctypes.Structure):
    """cec_extent: one value of a batch (off: arena offset, src_off: staging offset)."""

    _fields_ = [
        ("off", ctypes.c_uint64),
        ("src_off", ctypes.c_uint64),
        ("len", ctypes.c_uint32),
        ("pattern", ctypes.c_uint32),
    ]


class HostUpdate(ctypes.Structure):
    """cec_host_update: one pending rep_queue_item (diff in host memory)."""

    _fields_ = [
        ("buf", ctypes.c_void_p),
        ("addr", ctypes.c_uint64),
        ("len", ctypes.c_uint32),
        ("src_lid", ctypes.c_uint32),
    ]


class RegionJob(ctypes.Structure):
    """cec_region_job: one galois_w08_region_multiply call of a host-memory batch."""

    _fields_ = [
        ("src", ctypes.c_void_p),
        ("dst", ctypes.c_void_p),
        ("base", ctypes.c_void_p),
        ("len", ctypes.c_uint32),
        ("multby", ctypes.c_int32),
        ("add", ctypes.c_int32),
    ]


class BatchStats(ctypes.Structure):
    """cec_batch_stats: the thread's last cec_region_multiply_batch."""
    _fields_ = [("launches", ctypes.c_int), ("rounds", ctypes.c_int), ("plan_us", ctypes.c_float),
                ("pack_us", ctypes.c_float), ("gpu_us", ctypes.c_float), ("unpack_us", ctypes.c_float),
                ("in_place_launches", ctypes.c_int)]


class CacheInfo(ctypes.Structure):
    """cec_cache_info: the coefficient-table cache and the idle-buffer caches."""

    _fields_ = [(n, ctypes.c_uint64) for n in (
        "pattern_entries", "pattern_bytes", "pattern_uploads", "pattern_evictions",
        "pattern_entry_limit", "device_cached_bytes", "pinned_cached_bytes")]


class SyncRecord(ctypes.Structure):
    """cec_sync_record (cocytus_ec.h): how the thread's last synchronous call made its
    results visible to the host."""
    _fields_ = [("seq", ctypes.c_uint64), ("host_results", ctypes.c_int),
                ("waves_released", ctypes.c_int), ("fenced", ctypes.c_int)]


_vp = ctypes.c_void_p
_i = ctypes.c_int
_u32 = ctypes.c_uint32
_ip = ctypes.POINTER(ctypes.c_int)
_pp = ctypes.POINTER(ctypes.c_void_p)

_SIGS = {
    "cec_version": ([], ctypes.c_char_p),
    "cec_last_error": ([], ctypes.c_char_p),
    "cec_device_check": ([], _i),
    "cec_set_engine": ([_i], _i),
    "cec_get_engine": ([], _i),
    "cec_last_engine": ([], _i),
    "cec_internal_check_launch_layout": ([_i, _ip, _i, _ip, _i, _pp, _i], _i),
    "cec_internal_store_policy": ([ctypes.POINTER(ctypes.c_uint64)], _i),
    "cec_internal_fail_launch": ([_i], _i),
    "cec_plan_release_stream": ([_vp, _vp], _i),
    "cec_plan_tracked_streams": ([_vp], _i),
    "cec_drainer_release_stream": ([_vp, _vp], _i),
    "cec_recovery_release_stream": ([_vp, _vp], _i),
    "cec_recovery_pool_release_stream": ([_vp, _vp], _i),
    "cec_set_waves_per_cu": ([_i], _i),
    "cec_get_waves_per_cu": ([], _i),
    "cec_plan_create": ([ctypes.POINTER(_vp), ctypes.POINTER(Extent), _i, _vp], _i),
    "cec_plan_destroy": ([_vp], _i),
    "cec_plan_num_extents": ([_vp], _i),
    "cec_plan_num_tiles": ([_vp], ctypes.c_int64),
    "cec_plan_total_bytes": ([_vp], ctypes.c_uint64),
    "cec_region_multiply": ([_vp, _i, ctypes.c_size_t, _vp, _i, _vp], _i),
    "cec_encode": ([_i, _i, _ip, _pp, _pp, _vp, _vp], _i),
    "cec_encode_region": ([_i, _i, _ip, _pp, _pp, ctypes.c_size_t, _vp], _i),
    "cec_diff_update": ([_i, _i, _ip, _pp, _vp, _pp, _i, _vp, _vp], _i),
    "cec_set_diff": ([_i, _pp, _vp, _vp, _vp, _vp], _i),
    "cec_apply_diffs": ([_i, _i, _ip, _i, _vp, _vp, _vp, _vp], _i),
    "cec_residual": ([_i, _i, _ip, _i, _u32, _pp, _vp, _vp, _vp], _i),
    "cec_solve": ([_i, _i, _ip, _u32, _pp, _pp, _vp, _vp], _i),
    "cec_decode": ([_i, _i, _ip, ctypes.POINTER(_u32), _i, _pp, _pp, _vp, _vp], _i),
    "cec_recovery_mask": ([_i, _i, _i, _ip], _u32),
    "cec_arena_stride": ([ctypes.c_size_t], ctypes.c_size_t),
    "cec_arenas_alloc": ([_i, ctypes.c_size_t, _pp, ctypes.POINTER(_vp)], _i),
    "cec_arenas_free": ([_vp], _i),
    "cec_drainer_create": ([ctypes.POINTER(_vp), _i, _i, _ip, _i, ctypes.c_size_t], _i),
    "cec_drainer_destroy": ([_vp], _i),
    "cec_drainer_apply": ([_vp, ctypes.POINTER(HostUpdate), _i, _vp, _vp], _i),
    "cec_drainer_last_launches": ([_vp], _i),
    "cec_drainer_validate": ([_vp, ctypes.POINTER(HostUpdate), _i], _i),
    "cec_region_multiply_batch": ([ctypes.POINTER(RegionJob), _i, _vp], _i),
    "cec_region_multiply_batch_stats": ([ctypes.POINTER(BatchStats)], _i),
    "cec_drainer_staging": ([_vp, ctypes.POINTER(ctypes.c_size_t)], ctypes.POINTER(ctypes.c_uint8)),
    "cec_recovery_create": ([ctypes.POINTER(_vp), _i, _i, _ip, _i, _u32, _i, _i, _vp, _vp], _i),
    "cec_recovery_destroy": ([_vp], _i),
    "cec_recovery_add_peer": ([_vp, _i, _vp, _vp], _i),
    "cec_recovery_fold_update": ([_vp, _i, ctypes.c_uint64, _vp, _u32, _vp], _i),
    "cec_recovery_complete": ([_vp], _i),
    "cec_recovery_residual": ([_vp], _vp),
    "cec_recovery_bytes": ([_vp], ctypes.c_uint64),
    "cec_recovery_solve": ([_vp, _pp, _pp, _vp], _i),
    "cec_recovery_finish": ([_vp, _i, _vp, _pp, _pp, _vp], _i),
    "cec_recovery_pool_create": ([ctypes.POINTER(_vp), _i, _i, _ip, _i, _vp, _i], _i),
    "cec_recovery_pool_destroy": ([_vp], _i),
    "cec_recovery_pool_begin": ([_vp, _u32, _i, _i], _i),
    "cec_recovery_pool_add_peer": ([_vp, _i, _i, _vp], _i),
    "cec_recovery_pool_add_peers": ([_vp, _ip, _ip, _pp, _i], _i),
    "cec_recovery_pool_flush": ([_vp, _vp], _i),
    "cec_recovery_pool_flush_solve": ([_vp, _pp, _vp], _i),
    "cec_recovery_pool_solved": ([_vp, _i], _i),
    "cec_recovery_pool_flush_solve_host": ([_vp, _vp], _i),
    "cec_recovery_pool_solve_host": ([_vp, _ip, _i, _vp], _i),
    "cec_recovery_pool_output": ([_vp, _i, ctypes.POINTER(ctypes.c_size_t)], _vp),
    "cec_recovery_pool_staging": ([_vp, _i, _i, ctypes.POINTER(ctypes.c_size_t)], _vp),
    "cec_recovery_pool_complete": ([_vp, _i], _i),
    "cec_recovery_pool_fold_update": ([_vp, _i, ctypes.c_uint64, _vp, _u32, _vp], _i),
    "cec_recovery_pool_fold_updates": ([_vp, _vp, _i, _ip, _vp], _i),
    "cec_recovery_pool_solve": ([_vp, _ip, _i, _pp, _vp], _i),
    "cec_recovery_pool_residual": ([_vp, _i, _vp, _vp], _i),
    "cec_recovery_pool_end": ([_vp, _i], _i),
    "cec_recovery_pool_active": ([_vp], _i),
    "cec_cache_get_info": ([ctypes.POINTER(CacheInfo)], _i),
    "cec_last_sync": ([ctypes.POINTER(SyncRecord)], _i),
    "cec_cache_set_pattern_limit": ([_i], _i),
    "cec_cache_trim": ([], _i),
    "cec_event_create": ([ctypes.POINTER(_vp)], _i),
    "cec_event_destroy": ([_vp], _i),
    "cec_event_record": ([_vp, _vp], _i),
    "cec_event_elapsed_ms": ([_vp, _vp, ctypes.POINTER(ctypes.c_float)], _i),
    "cec_stream_synchronize": ([_vp], _i),
    "cec_host_register": ([_vp, ctypes.c_size_t, ctypes.POINTER(_vp)], _i),
    "cec_host_unregister": ([_vp], _i),
    "cec_copy": ([_vp, _vp, ctypes.c_size_t, _vp], _i),
    "cec_device_count": ([ctypes.POINTER(_i)], _i),
    "cec_set_device": ([_i], _i),
    "cec_stream_create": ([ctypes.POINTER(_vp)], _i),
    "cec_stream_destroy": ([_vp], _i),
    "galois_w08_region_multiply": ([_vp, _i, _i, _vp, _i], None),
    "galois_single_multiply": ([_i, _i, _i], _i),
    "galois_single_divide": ([_i, _i, _i], _i),
    "galois_inverse": ([_i, _i], _i),
    "reed_sol_big_vandermonde_distribution_matrix": ([_i, _i, _i], _ip),
    "reed_sol_extended_vandermonde_matrix": ([_i, _i, _i], _ip),
    "jerasure_invert_matrix": ([_ip, _ip, _i, _i], _i),
    "jerasure_matrix_multiply": ([_ip, _ip, _i, _i, _i, _i, _i], _ip),
}

_lib = None


def _hip_runtimes() -> set[str]:
    """Distinct libamdhip64 files mapped into this process."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return paths


def lib() -> ctypes.CDLL:
    """Load libcocytus_ec.so (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} is missing: build it with `python cocytus_amd/build.py` "
            "(there is no CPU fallback)"
        )
    L = ctypes.CDLL(LIB_PATH)
    for name, (args, res) in _SIGS.items():
        if os.environ.get("CEC_LIB_PATH") and not hasattr(L, name):
            continue  # an older build under A/B measurement: bind what it has
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [_vp]
    L._free = libc.free
    rts = _hip_runtimes()
    if len(rts) > 1:
        raise RuntimeError(
            "two HIP runtimes are mapped (%s): import torch before loading cocytus_amd" % sorted(rts)
        )
    _lib = L
    return L


def kernel_code_id(path: str | None = None) -> str | None:
    """Identity of the library's device code: sha256 (16 hex digits) of its gfx950 code
    object disassembled (llvm-objdump), one block per kernel sorted by name, addresses
    and encodings dropped -- so host-only changes and a different link order of the same
    kernels keep the id, and any change to a kernel's instructions changes it.  Nothing
    is loaded.  None if the file or llvm-objdump is missing."""
    import hashlib
    import re
    import shutil
    import subprocess
    import tempfile

    path = path or LIB_PATH
    objdump = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin", "llvm-objdump")
    if not (os.path.exists(path) and os.path.exists(objdump)):
        return None
    with tempfile.TemporaryDirectory() as d:
        so = os.path.join(d, "lib.so")
        shutil.copy(os.path.realpath(path), so)
        if subprocess.run([objdump, "--offloading", so], cwd=d, capture_output=True).returncode:
            return None
        cos = sorted(f for f in os.listdir(d) if f.endswith("gfx950"))
        if len(cos) != 1:
            return None
        r = subprocess.run([objdump, "-d", os.path.join(d, cos[0])], capture_output=True, text=True)
        if r.returncode:
            return None
    funcs, cur = {}, None
    for line in r.stdout.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
        elif cur is not None and line.startswith("\t"):
            ins = line.split("//")[0].strip()
            if ins:
                cur.append(ins)
    if not funcs:
        return None
    h = hashlib.sha256()
    for name in sorted(funcs):
        h.update(name.encode() + b"\n" + "\n".join(funcs[name]).encode() + b"\n\n")
    return h.hexdigest()[:16]


def _check(rc: int) -> None:
    if rc != CEC_OK:
        raise CecError(rc, lib().cec_last_error().decode(errors="replace"))


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "__index__") and not hasattr(x, "data_ptr"):  # numpy integers
        return x.__index__()
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    raise TypeError(f"cannot take a device pointer of {type(x)!r}")


def _stream(s) -> int:
    if s is None:
        return 0
    if isinstance(s, int):
        return s
    if hasattr(s, "cuda_stream"):
        return int(s.cuda_stream)
    raise TypeError(f"not a stream: {type(s)!r}")


def _ptr_array(xs: Iterable) -> ctypes.Array:
    xs = list(xs)
    return (ctypes.c_void_p * len(xs))(*[_ptr(x) or None for x in xs])


def _int_array(xs: Sequence[int]) -> ctypes.Array:
    return (ctypes.c_int * len(xs))(*[int(v) for v in xs])


# ------------------------------------------------------------------ runtime
def version() -> str:
    return lib().cec_version().decode()


def device_check() -> int:
    return lib().cec_device_check()


def set_engine(engine: int) -> None:
    _check(lib().cec_set_engine(engine))


def get_engine() -> int:
    return lib().cec_get_engine()


def last_engine() -> int:
    """cec_last_engine: the engine (CEC_ENGINE_PERM / _LDS) this thread's last op ran
    with, AUTO resolved; -1 before the first op."""
    return lib().cec_last_engine()


def check_launch_layout(narrow: bool, in_slots, out_slots, bases) -> int:
    """cec_internal_check_launch_layout (test hook, host only): CEC_OK or CEC_EINVAL."""
    return lib().cec_internal_check_launch_layout(int(bool(narrow)), _int_array(in_slots), len(in_slots),
                                                  _int_array(out_slots), len(out_slots), _ptr_array(bases),
                                                  len(bases))


def store_policy() -> tuple[str, int]:
    """cec_internal_store_policy: ('auto' | 'nt' | 'wt', auto's write-through limit)."""
    v = ctypes.c_uint64()
    p = lib().cec_internal_store_policy(ctypes.byref(v))
    return {0: "auto", 1: "nt", 2: "wt"}[p], int(v.value)


def fail_launch(after: int) -> None:
    """cec_internal_fail_launch (test hook): the thread's launch number `after` (0-based)
    fails with CEC_EHIP; -1 disarms."""
    _check(lib().cec_internal_fail_launch(after))


def set_waves_per_cu(waves: int) -> None:
    _check(lib().cec_set_waves_per_cu(waves))



def get_waves_per_cu() -> int:
    return lib().cec_get_waves_per_cu()


def cache_info() -> dict:
    """cec_cache_get_info for the current device, as a dict."""
    ci = CacheInfo()
    _check(lib().cec_cache_get_info(ctypes.byref(ci)))
    return {n: int(getattr(ci, n)) for n, _ in CacheInfo._fields_}


def last_sync() -> dict:
    """cec_last_sync: the calling thread's last synchronous completion, as a dict."""
    r = SyncRecord()
    _check(lib().cec_last_sync(ctypes.byref(r)))
    return {n: int(getattr(r, n)) for n, _ in SyncRecord._fields_}


def cache_set_pattern_limit(entries: int) -> None:
    _check(lib().cec_cache_set_pattern_limit(entries))


def cache_trim() -> None:
    _check(lib().cec_cache_trim())


def arena_stride(nbytes: int) -> int:
    """cec_arena_stride: the HBM-friendly distance between arena bases (odd x 4 KiB)."""
    return int(lib().cec_arena_stride(nbytes))


def arena_tensors(count: int, nbytes: int, device="cuda"):
    """count uint8 torch views of nbytes each, carved from one allocation at
    cec_arena_stride(nbytes) -- the layout of cec_arenas_alloc, owned by torch."""
    import torch

    stride = arena_stride(nbytes)
    slab = torch.empty(stride * count, dtype=torch.uint8, device=device)
    return [slab[i * stride:i * stride + nbytes] for i in range(count)]


class Plan:
    """A device-resident batch of extents (cec_plan)."""

    def __init__(self, extents: Sequence[tuple] | ctypes.Array, stream=None):
        if isinstance(extents, ctypes.Array):
            arr = extents
        else:
            arr = (Extent * len(extents))(*[Extent(*e) for e in extents])
        self._h = ctypes.c_void_p()
        _check(lib().cec_plan_create(ctypes.byref(self._h), arr, len(arr), _vp(_stream(stream))))

    @property
    def handle(self) -> ctypes.c_void_p:
        if not self._h:
            raise ValueError("plan destroyed")
        return self._h

    @property
    def num_extents(self) -> int:
        return lib().cec_plan_num_extents(self.handle)

    @property
    def num_tiles(self) -> int:
        return lib().cec_plan_num_tiles(self.handle)

    @property
    def total_bytes(self) -> int:
        return lib().cec_plan_total_bytes(self.handle)

    def release_stream(self, stream) -> None:
        """cec_plan_release_stream: call before destroying a stream this plan was used on."""
        _check(lib().cec_plan_release_stream(self.handle, _stream(stream)))

    @property
    def tracked_streams(self) -> int:
        return lib().cec_plan_tracked_streams(self.handle)

    def destroy(self) -> None:
        if self._h:
            _check(lib().cec_plan_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            if self._h and _lib is not None:
                _lib.cec_plan_destroy(self._h)
        except Exception:
            pass


def extents_array(rows: Iterable[tuple]) -> ctypes.Array:
    rows = list(rows)
    return (Extent * len(rows))(*[Extent(*r) for r in rows])


# ------------------------------------------------------------------ ops
def region_multiply(src, multby: int, nbytes: int, dst, add: int = 1, stream=None) -> None:
    _check(lib().cec_region_multiply(_ptr(src), multby, nbytes, _ptr(dst) or None, add, _stream(stream)))


def encode(k, m, matrix, data, parity, plan: Plan, stream=None) -> None:
    _check(lib().cec_encode(k, m, _int_array(matrix), _ptr_array(data), _ptr_array(parity),
                            plan.handle, _stream(stream)))


def encode_region(k, m, matrix, data, parity, length: int, stream=None) -> None:
    _check(lib().cec_encode_region(k, m, _int_array(matrix), _ptr_array(data), _ptr_array(parity),
                                   length, _stream(stream)))


def diff_update(k, m, matrix, data, staging, parity, install: bool, plan: Plan, stream=None) -> None:
    _check(lib().cec_diff_update(k, m, _int_array(matrix), _ptr_array(data), _ptr(staging),
                                 _ptr_array(parity), int(bool(install)), plan.handle, _stream(stream)))


def set_diff(k, data, staging, diff, plan: Plan, stream=None) -> None:
    _check(lib().cec_set_diff(k, _ptr_array(data), _ptr(staging), _ptr(diff), plan.handle,
                              _stream(stream)))


def apply_diffs(k, m, matrix, lid_self, diffs, parity, plan: Plan, stream=None) -> None:
    _check(lib().cec_apply_diffs(k, m, _int_array(matrix), lid_self, _ptr(diffs), _ptr(parity),
                                 plan.handle, _stream(stream)))


def residual(k, m, matrix, lid_self, mask, arenas, out, plan: Plan, stream=None) -> None:
    _check(lib().cec_residual(k, m, _int_array(matrix), lid_self, mask, _ptr_array(arenas), _ptr(out),
                              plan.handle, _stream(stream)))


def solve(k, m, matrix, mask, residuals, out, plan: Plan, stream=None) -> None:
    _check(lib().cec_solve(k, m, _int_array(matrix), mask, _ptr_array(residuals), _ptr_array(out),
                           plan.handle, _stream(stream)))


def decode(k, m, matrix, masks: Sequence[int], arenas, out, plan: Plan, stream=None) -> None:
    marr = (ctypes.c_uint32 * len(masks))(*[int(x) for x in masks])
    _check(lib().cec_decode(k, m, _int_array(matrix), marr, len(masks), _ptr_array(arenas),
                            _ptr_array(out), plan.handle, _stream(stream)))


def recovery_mask(k: int, m: int, leader_lid: int, connected: Sequence[int]) -> int:
    return lib().cec_recovery_mask(k, m, leader_lid, _int_array(connected))


def host_updates(updates) -> ctypes.Array:
    """[(host buffer (numpy / bytearray / pointer), addr, src_lid[, len])] -> cec_host_update[]."""
    arr = (HostUpdate * len(updates))()
    for i, u in enumerate(updates):
        buf, addr, src = u[0], u[1], u[2]
        n = u[3] if len(u) > 3 else (buf.nbytes if hasattr(buf, "nbytes") else len(buf))
        arr[i] = HostUpdate(_host_or_dev(buf), addr, n, src)
    return arr


class Drainer:
    """cec_drainer: batched deferred-commit drain of a parity process (§8f rank 1)."""

    def __init__(self, k: int, m: int, matrix, lid_self: int, staging_bytes: int = 64 << 20):
        self._h = ctypes.c_void_p()
        _check(lib().cec_drainer_create(ctypes.byref(self._h), k, m, _int_array(matrix), lid_self,
                                        staging_bytes))

    def apply(self, updates, parity, stream=None) -> int:
        """updates: a host_updates() array, or [(host buffer, addr, src_lid[, len])]
        (the caller keeps the buffers alive).  Returns the launches used."""
        arr = updates if isinstance(updates, ctypes.Array) else host_updates(updates)
        _check(lib().cec_drainer_apply(self._h, arr, len(arr), _ptr(parity), _stream(stream)))
        return lib().cec_drainer_last_launches(self._h)

    def staging(self):
        """(address, numpy uint8 view) of the drainer's pinned staging area: diffs
        received straight into it are applied without a pack copy."""
        import numpy as np

        cap = ctypes.c_size_t()
        p = lib().cec_drainer_staging(self._h, ctypes.byref(cap))
        addr = ctypes.cast(p, ctypes.c_void_p).value
        return addr, np.ctypeslib.as_array((ctypes.c_uint8 * cap.value).from_address(addr))

    def release_stream(self, stream) -> None:
        _check(lib().cec_drainer_release_stream(self._h, _stream(stream)))

    def destroy(self) -> None:
        if self._h:
            _check(lib().cec_drainer_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            if self._h and _lib is not None:
                _lib.cec_drainer_destroy(self._h)
        except Exception:
            pass


class Recovery:
    """cec_recovery: one online-recovery request on a participating parity (§8f rank 2).

    Buffers may be host (numpy / bytearray) or device (tensor / int pointer)."""

    def __init__(self, k, m, matrix, lid_self, mask, unit_begin, unit_end, parity_arena, stream=None):
        self.k, self.m = k, m
        self._h = ctypes.c_void_p()
        _check(lib().cec_recovery_create(ctypes.byref(self._h), k, m, _int_array(matrix), lid_self, mask,
                                         unit_begin, unit_end, _ptr(parity_arena), _stream(stream)))

    def add_peer(self, peer_lid: int, units, stream=None) -> None:
        _check(lib().cec_recovery_add_peer(self._h, peer_lid, _host_or_dev(units), _stream(stream)))

    def fold_update(self, peer_lid: int, addr: int, diff, stream=None) -> int:
        n = diff.nbytes if hasattr(diff, "nbytes") else len(diff)
        rc = lib().cec_recovery_fold_update(self._h, peer_lid, addr, _host_or_dev(diff), n, _stream(stream))
        if rc < 0:
            _check(rc)
        return rc

    @property
    def complete(self) -> bool:
        return bool(lib().cec_recovery_complete(self._h))

    @property
    def residual(self) -> int:
        return int(lib().cec_recovery_residual(self._h) or 0)

    @property
    def nbytes(self) -> int:
        return int(lib().cec_recovery_bytes(self._h))

    def solve(self, peer_residuals: dict, out: dict, stream=None) -> None:
        """peer_residuals / out: {lid: buffer} (host or device)."""
        pr = (ctypes.c_void_p * (self.k + self.m))(*[_host_or_dev(peer_residuals.get(i)) or None
                                                     for i in range(self.k + self.m)])
        oo = (ctypes.c_void_p * self.k)(*[_host_or_dev(out.get(j)) or None for j in range(self.k)])
        _check(lib().cec_recovery_solve(self._h, pr, oo, _stream(stream)))

    def finish(self, peer_lid: int, units, peer_residuals: dict, out: dict, stream=None) -> None:
        """add_peer(peer_lid, units) + solve(peer_residuals, out) in one pipelined pass."""
        pr = (ctypes.c_void_p * (self.k + self.m))(*[_host_or_dev(peer_residuals.get(i)) or None
                                                     for i in range(self.k + self.m)])
        oo = (ctypes.c_void_p * self.k)(*[_host_or_dev(out.get(j)) or None for j in range(self.k)])
        _check(lib().cec_recovery_finish(self._h, peer_lid, _host_or_dev(units), pr, oo, _stream(stream)))

    def release_stream(self, stream) -> None:
        _check(lib().cec_recovery_release_stream(self._h, _stream(stream)))

    def destroy(self) -> None:
        if self._h:
            _check(lib().cec_recovery_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            if self._h and _lib is not None:
                _lib.cec_recovery_destroy(self._h)
        except Exception:
            pass


class RecoveryPool:
    """cec_recovery_pool: many small in-flight recovery requests of one parity, their
    replies folded in one launch per flush (the idle recoverer, §8f rank 2)."""

    def __init__(self, k, m, matrix, lid_self, parity_arena, capacity_units=1024):
        self.k, self.m = k, m
        self._h = ctypes.c_void_p()
        _check(lib().cec_recovery_pool_create(ctypes.byref(self._h), k, m, _int_array(matrix), lid_self,
                                              _ptr(parity_arena), capacity_units))

    def begin(self, mask: int, unit_begin: int, unit_end: int) -> int:
        rc = lib().cec_recovery_pool_begin(self._h, mask, unit_begin, unit_end)
        if rc < 0:
            _check(rc)
        return rc

    def add_peer(self, rid: int, peer_lid: int, units) -> None:
        """units: host / device buffer, or the address from staging() (no copy)."""
        ptr = units if isinstance(units, int) else _host_or_dev(units)
        _check(lib().cec_recovery_pool_add_peer(self._h, rid, peer_lid, ptr))

    def add_peers(self, ids, peer_lids=None, units=None) -> None:
        """n replies in one call (cec_recovery_pool_add_peers): lists of request ids, data
        peer lids and buffers / staging addresses, or one pool_replies() tuple built ahead."""
        ia, pa, ua, n = ids if peer_lids is None else pool_replies(ids, peer_lids, units)
        _check(lib().cec_recovery_pool_add_peers(self._h, ia, pa, ua, n))

    def staging(self, rid: int, peer_lid: int):
        """(address, numpy uint8 view) where peer_lid's reply for rid may be received in place."""
        import numpy as np

        n = ctypes.c_size_t()
        addr = lib().cec_recovery_pool_staging(self._h, rid, peer_lid, ctypes.byref(n))
        if not addr:
            _check(CEC_EINVAL)
        return addr, np.ctypeslib.as_array((ctypes.c_uint8 * n.value).from_address(addr))

    def flush(self, stream=None) -> int:
        rc = lib().cec_recovery_pool_flush(self._h, _stream(stream))
        if rc < 0:
            _check(rc)
        return rc

    def flush_solve(self, out_arenas, stream=None) -> int:
        """flush(), also solving every single-loss request it completes into out_arenas."""
        oo = (ctypes.c_void_p * self.k)(*[_ptr(out_arenas[j]) if j < len(out_arenas) and
                                          out_arenas[j] is not None else None for j in range(self.k)])
        rc = lib().cec_recovery_pool_flush_solve(self._h, oo, _stream(stream))
        if rc < 0:
            _check(rc)
        return rc

    def flush_solve_host(self, stream=None) -> int:
        """flush(), also solving every single-loss request it completes into the pool's
        own host output (read with output())."""
        rc = lib().cec_recovery_pool_flush_solve_host(self._h, _stream(stream))
        if rc < 0:
            _check(rc)
        return rc

    def solve_host(self, rids, stream=None) -> None:
        ids = (ctypes.c_int * len(rids))(*rids)
        _check(lib().cec_recovery_pool_solve_host(self._h, ids, len(rids), _stream(stream)))

    def output(self, rid: int):
        """numpy uint8 view of rid's rebuilt units after a _host solve, or None."""
        import numpy as np

        n = ctypes.c_size_t()
        addr = lib().cec_recovery_pool_output(self._h, rid, ctypes.byref(n))
        if not addr:
            return None
        return np.ctypeslib.as_array((ctypes.c_uint8 * n.value).from_address(addr))

    def solved(self, rid: int) -> bool:
        return bool(lib().cec_recovery_pool_solved(self._h, rid))

    def complete(self, rid: int) -> bool:
        return bool(lib().cec_recovery_pool_complete(self._h, rid))

    def fold_update(self, peer_lid: int, addr: int, diff, stream=None) -> int:
        n = diff.nbytes if hasattr(diff, "nbytes") else len(diff)
        rc = lib().cec_recovery_pool_fold_update(self._h, peer_lid, addr, _host_or_dev(diff), n, _stream(stream))
        if rc < 0:
            _check(rc)
        return rc

    def fold_updates(self, updates, stream=None):
        """updates: [(host diff, addr, peer_lid)] (host_updates' form), one drain window,
        folded as fold_update per update.  Returns the units folded per update."""
        arr = host_updates(updates) if updates else (HostUpdate * 1)()
        units = (ctypes.c_int * max(len(updates), 1))()
        rc = lib().cec_recovery_pool_fold_updates(self._h, arr, len(updates), units, _stream(stream))
        if rc < 0:
            _check(rc)
        return [units[i] for i in range(len(updates))]

    def solve(self, rids, out_arenas, stream=None) -> None:
        """out_arenas: k device arenas by data lid (None where not lost)."""
        ids = (ctypes.c_int * len(rids))(*rids)
        oo = (ctypes.c_void_p * self.k)(*[_ptr(out_arenas[j]) if j < len(out_arenas) and
                                          out_arenas[j] is not None else None for j in range(self.k)])
        _check(lib().cec_recovery_pool_solve(self._h, ids, len(rids), oo, _stream(stream)))

    def residual(self, rid: int, dst, stream=None) -> None:
        _check(lib().cec_recovery_pool_residual(self._h, rid, _host_or_dev(dst), _stream(stream)))

    def end(self, rid: int) -> None:
        _check(lib().cec_recovery_pool_end(self._h, rid))

    @property
    def active(self) -> int:
        return int(lib().cec_recovery_pool_active(self._h))

    def release_stream(self, stream) -> None:
        _check(lib().cec_recovery_pool_release_stream(self._h, _stream(stream)))

    def destroy(self) -> None:
        if self._h:
            _check(lib().cec_recovery_pool_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.destroy()

    def __del__(self):
        try:
            if self._h and _lib is not None:
                _lib.cec_recovery_pool_destroy(self._h)
        except Exception:
            pass


def pool_replies(ids, peer_lids, units) -> tuple:
    """The argument arrays of cec_recovery_pool_add_peers (units: buffers or addresses)."""
    n = len(ids)
    ua = (ctypes.c_void_p * max(n, 1))(*[u if isinstance(u, int) else _host_or_dev(u) for u in units])
    return _int_array(ids), _int_array(peer_lids), ua, n


class Event:
    def __init__(self):
        self._e = ctypes.c_void_p()
        _check(lib().cec_event_create(ctypes.byref(self._e)))

    def record(self, stream=None) -> None:
        _check(lib().cec_event_record(self._e, _stream(stream)))

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _check(lib().cec_event_elapsed_ms(self._e, end._e, ctypes.byref(ms)))
        return float(ms.value)

    def __del__(self):
        try:
            if self._e and _lib is not None:
                _lib.cec_event_destroy(self._e)
        except Exception:
            pass


def stream_synchronize(stream=None) -> None:
    _check(lib().cec_stream_synchronize(_stream(stream)))


# ------------------------------------------------------------------ Jerasure drop-in
def galois_w08_region_multiply(region, multby: int, nbytes: int, r2, add: int) -> None:
    """The drop-in symbol itself (host or device buffers; synchronous; aborts on error).

    region / r2: device pointers (int / tensor) or writable host buffers (bytearray,
    numpy arrays) -- host buffers are passed by address.
    """
    lib().galois_w08_region_multiply(_host_or_dev(region), multby, nbytes, _host_or_dev(r2), add)


def region_jobs(jobs) -> ctypes.Array:
    """A cec_region_job array of (src, dst, base, len, multby, add) tuples, built once (a
    batch re-run with the same jobs passes the array itself)."""
    arr = (RegionJob * len(jobs))()
    for i, (src, dst, base, n, c, add) in enumerate(jobs):
        arr[i] = RegionJob(_host_or_dev(src), _host_or_dev(dst), _host_or_dev(base), n, c, add)
    return arr


def region_multiply_batch(jobs, stream=None) -> tuple[int, int]:
    """cec_region_multiply_batch over host buffers.  jobs: (src, dst, base, len, multby,
    add) with src / dst / base as host addresses (int), numpy arrays, bytearrays or None
    (or a region_jobs() array).
    Returns (kernel launches, staging rounds) of the call."""
    arr = jobs if isinstance(jobs, ctypes.Array) else region_jobs(jobs)
    _check(lib().cec_region_multiply_batch(arr, len(arr), _stream(stream)))
    st = batch_stats()
    return st["launches"], st["rounds"]


def host_register(buf) -> int:
    """cec_host_register of a host buffer (numpy array / bytearray / address, nbytes from
    the array): returns its device alias.  Unregister with host_unregister(buf)."""
    addr = _host_or_dev(buf)
    n = buf.nbytes if hasattr(buf, "nbytes") else len(buf)
    alias = ctypes.c_void_p()
    _check(lib().cec_host_register(addr, n, ctypes.byref(alias)))
    return alias.value


def host_unregister(buf) -> None:
    _check(lib().cec_host_unregister(_host_or_dev(buf)))


def batch_stats() -> dict:
    st = BatchStats()
    _check(lib().cec_region_multiply_batch_stats(ctypes.byref(st)))
    return {f: getattr(st, f) for f, _ in BatchStats._fields_}


def _host_or_dev(x):
    if x is None:
        return None
    if isinstance(x, (bytearray, memoryview)):
        return ctypes.addressof(ctypes.c_char.from_buffer(x))
    if hasattr(x, "ctypes") and hasattr(x, "dtype"):  # numpy
        return x.ctypes.data
    return _ptr(x)


def galois_single_multiply(a: int, b: int, w: int = 8) -> int:
    return lib().galois_single_multiply(a, b, w)


def galois_single_divide(a: int, b: int, w: int = 8) -> int:
    return lib().galois_single_divide(a, b, w)


def reed_sol_big_vandermonde_distribution_matrix(rows: int, cols: int, w: int = 8) -> list[int] | None:
    p = lib().reed_sol_big_vandermonde_distribution_matrix(rows, cols, w)
    if not p:
        return None
    out = [p[i] for i in range(rows * cols)]
    lib()._free(ctypes.cast(p, ctypes.c_void_p))
    return out


def jerasure_invert_matrix(mat: Sequence[int], rows: int, w: int = 8) -> tuple[int, list[int]]:
    a = _int_array(mat)
    inv = (ctypes.c_int * (rows * rows))()
    rc = lib().jerasure_invert_matrix(a, inv, rows, w)
    return rc, list(inv)


def coding_matrix(k: int, m: int) -> list[int]:
    """MATRIX of memcached.c:6845: reed_sol_big_vandermonde_distribution_matrix(k+m, k, 8)."""
    mat = reed_sol_big_vandermonde_distribution_matrix(k + m, k, 8)
    if mat is None:
        raise CecError(CEC_EINVAL, f"no coding matrix for k={k} m={m}")
    return mat
