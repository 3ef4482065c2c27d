"""cocytus_amd -- MI355X-native erasure-coding path for Cocytus (SJTU-IPADS/cocytus).

The product is ``libcocytus_ec.so`` (HIP kernels for gfx950 behind a C-ABI that is a
drop-in for the three Jerasure symbols Cocytus links, plus a batched device API);
:mod:`cocytus_amd.ec` is its Python mirror.  See DESIGN.md and INTEGRATION.md.
"""
from . import ec  # noqa: F401

__all__ = ["ec"]
