"""Build libcocytus_ec.so (HIP, gfx950) in-tree.

The library is the product: the C-ABI of include/*.h.  It is compiled with hipcc
for gfx950 only (no dual CUDA/HIP path, no hipify) and written next to this file so
it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libcocytus_ec.so")
JERASURE_LINK = os.path.join(HERE, "libJerasure.so")
SOURCES = [os.path.join(CSRC, "cec_runtime.hip")]
DEPS = SOURCES + [os.path.join(CSRC, f) for f in ("cec_kernels.hpp", "gf256.hpp", "cec_cache.inc", "cec_drain.inc", "cec_recovery.inc", "cec_pool.inc", "cec_hostbatch.inc")] + [
    os.path.join(ROOT, "include", f) for f in ("cocytus_ec.h", "galois.h", "jerasure.h", "reed_sol.h")
]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def hipcc_cmd(out: str = LIB, extra: list[str] | None = None) -> list[str]:
    return [
        os.path.join(ROCM, "bin", "hipcc"),
        "--offload-arch=gfx950",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-fvisibility=hidden",
        "-mcode-object-version=5",
        "-Wall",
        "-Wno-unused-function",
        "-I" + os.path.join(ROOT, "include"),
        f"-Wl,-rpath,{ROCM}/lib",
        "-o",
        out,
        *SOURCES,
        *(extra or []),
    ]


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False, verbose: bool = True) -> str:
    if force or needs_build():
        cmd = hipcc_cmd()
        if verbose:
            print("[cocytus_amd] " + " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
    if os.path.lexists(JERASURE_LINK):
        os.remove(JERASURE_LINK)
    os.symlink(os.path.basename(LIB), JERASURE_LINK)  # -lJerasure drop-in name
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
