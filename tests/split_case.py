"""Parity of every launch shape under a pinned workgroups-per-tile choice or store policy.

Run as a child process by tests/test_gpu_parity.py::test_forced_split_shift with
CEC_SPLIT_SHIFT set, and by ::test_store_policy_every_kernel_kind with CEC_STORE_POLICY /
CEC_WT_MAX_BYTES set (the library reads them once per process; CEC_EXPECT_POLICY names
the policy the child must see).  Covers every kernel kind -- the narrow 1 x 1 kernels
(region multiply), exact shapes (encode, decode, diff-update) and the capacity kernel
(RS(12,4): 12 inputs) -- on aligned full tiles, ragged / misaligned tiles, RMW outputs
and the implicit region, against the oracle, both engines.  Prints "OK" on success;
any mismatch raises.
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    import torch

    torch.cuda.set_device(0)
    torch.empty(1, device="cuda")
    from cocytus_amd import ec

    assert ec.device_check() == ec.CEC_OK, ec.lib().cec_last_error()
    want = os.environ.get("CEC_EXPECT_POLICY")
    if want:
        policy, limit = ec.store_policy()
        assert f"{policy}:{limit}" == want, (policy, limit, want)
    for engine in (ec.CEC_ENGINE_LDS, ec.CEC_ENGINE_PERM):  # both GF engines per split
        ec.set_engine(engine)
        check(torch, ec)
    print("OK")


def check(torch, ec) -> None:
    from oracle import pyoracle

    k, m = 3, 2
    mat = ec.coding_matrix(k, m)
    rng = np.random.default_rng(int(os.environ.get("CEC_SPLIT_SHIFT", "9")) + 17)

    def dev(a):
        return torch.from_numpy(np.ascontiguousarray(a)).cuda()

    # aligned full 4 KiB tiles, then ragged 16-B-aligned extents, then misaligned ones
    lens = [4096] * 8 + [1, 17, 255, 4097, 8195, 65536 + 16, 100003]
    ext, off = [], 0
    for i, n in enumerate(lens):
        o = off + (1 + i % 15 if i >= 12 else 0)
        ext.append((o, 0, n, 0))
        off = (o + n + 127) & ~127 if i < 8 else (o + n + 15) & ~15
    size = off + 64
    host = [rng.integers(0, 256, size, dtype=np.uint8) for _ in range(k)]
    data = [dev(h) for h in host]
    parity = [torch.zeros(size, dtype=torch.uint8, device="cuda") for _ in range(m)]
    exp = [np.zeros(size, np.uint8) for _ in range(m)]
    full = pyoracle.encode(mat, k, m, host)
    for o, _, n, _ in ext:
        for p in range(m):
            exp[p][o:o + n] = full[p][o:o + n]
    for sub in (ext[:8], ext):  # the all-aligned plan and the mixed plan
        with ec.Plan(sub) as pl:
            ec.encode(k, m, mat, data, parity, pl)
    torch.cuda.synchronize()
    for p in range(m):
        assert np.array_equal(parity[p].cpu().numpy(), exp[p]), f"encode parity {p}"

    # decode every single-data-loss mask over the mixed plan
    masks = [ec.recovery_mask(k, m, k, [int(i != j) for i in range(k + m)]) for j in range(k)]
    out = [torch.zeros(size, dtype=torch.uint8, device="cuda") for _ in range(k)]
    dext = [(o, s, n, e % len(masks)) for e, (o, s, n, _) in enumerate(ext)]
    with ec.Plan(dext) as dp:
        ec.decode(k, m, mat, masks, data + parity, out, dp)
    torch.cuda.synchronize()
    for e, (o, _, n, pi) in enumerate(dext):
        j = [x for x in range(k) if not (masks[pi] >> x) & 1][0]
        assert np.array_equal(out[j][o:o + n].cpu().numpy(), host[j][o:o + n]), f"decode ext {e}"

    # diff-update with install (RMW outputs) on aligned and ragged extents
    new = rng.integers(0, 256, size, dtype=np.uint8)
    uext = [(o, o, n, 1) for (o, _, n, _) in (ext[0], ext[3], ext[9], ext[13])]
    with ec.Plan(uext) as up:
        ec.diff_update(k, m, mat, data, dev(new), parity, True, up)
    torch.cuda.synchronize()
    for o, _, n, _ in uext:
        old = host[1][o:o + n].copy()
        pv = [x[o:o + n].copy() for x in exp]
        pyoracle.diff_update(mat, k, m, 1, old, new[o:o + n].copy(), pv, True)
        for p in range(m):
            assert np.array_equal(parity[p][o:o + n].cpu().numpy(), pv[p]), f"diff parity {p} @{o}"
        assert np.array_equal(data[1][o:o + n].cpu().numpy(), new[o:o + n]), f"install @{o}"

    # implicit region multiply-XOR, aligned and 1-byte-misaligned bases
    for shift in (0, 1):
        n = 3 * 4096 + 77
        src = rng.integers(0, 256, n + 1, dtype=np.uint8)
        dst = rng.integers(0, 256, n + 1, dtype=np.uint8)
        ds, dd = dev(src), dev(dst)
        ec.region_multiply(ds[shift:], 0x53, n, dd[shift:], 1)
        torch.cuda.synchronize()
        want = dst.copy()
        pyoracle.region_multiply(src[shift:shift + n].copy(), 0x53, want[shift:shift + n], 1)
        assert np.array_equal(dd.cpu().numpy(), want), f"region shift {shift}"

    # the capacity (generic) kernel: RS(12, 4), 12 inputs > the exact shapes' 8
    k2, m2 = 12, 4
    mat2 = ec.coding_matrix(k2, m2)
    n2 = 5 * 4096 + 333
    host2 = [rng.integers(0, 256, n2, dtype=np.uint8) for _ in range(k2)]
    par2 = [torch.zeros(n2, dtype=torch.uint8, device="cuda") for _ in range(m2)]
    with ec.Plan([(0, 0, 4 * 4096, 0), (4 * 4096 + 16, 0, 4096 + 300, 0)]) as gp:
        ec.encode(k2, m2, mat2, [dev(h) for h in host2], par2, gp)
    torch.cuda.synchronize()
    full2 = pyoracle.encode(mat2, k2, m2, host2)
    for p in range(m2):
        got = par2[p].cpu().numpy()
        assert np.array_equal(got[:4 * 4096], full2[p][:4 * 4096]), f"generic parity {p}"
        assert np.array_equal(got[4 * 4096 + 16:n2 - 17], full2[p][4 * 4096 + 16:n2 - 17]), f"generic parity {p}"


if __name__ == "__main__":
    main()
