#!/usr/bin/env python3
"""Generate the committed golden fixtures from the oracle (oracle/libgf8ref.so).

PARITY UNPINNED: the reference's arithmetic (Jerasure 2.x + GF-Complete) is not in
/root/reference nor installed, and the reference holds no EC vectors; these fixtures
freeze the oracle's restatement (cross-checked in tests/test_oracle.py against
independent known answers) so that every later build is compared with the same bytes.

Run:  python tests/golden/make_golden.py      (writes tests/golden/*.npz + manifest.json)
"""
from __future__ import annotations

import hashlib
import itertools
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import pyoracle as O  # noqa: E402

COEFS = [0, 1, 2, 0x80, 244, 245, 255]
SIZES = [1, 15, 16, 17, 4096, 4098]


def region_fixture():
    arrs = {}
    seed = 0xC0C70001
    for c in COEFS:
        for n in SIZES:
            src = O.splitmix_bytes(seed, n)
            r2 = O.splitmix_bytes(seed + 1, n)
            exp = r2.copy()
            O.region_multiply(src, c, exp, 1)
            arrs[f"c{c}_n{n}_src"] = src
            arrs[f"c{c}_n{n}_r2"] = r2
            arrs[f"c{c}_n{n}_out"] = exp
            seed += 2
    return arrs


def encode_fixture(k, m, n):
    mat = O.big_vandermonde(k + m, k)
    data = [O.splitmix_bytes(0xC0C70002 + 17 * j + k, n) for j in range(k)]
    par = O.encode(mat, k, m, data)
    arrs = {"matrix": np.array(mat, np.int32)}
    for j in range(k):
        arrs[f"data{j}"] = data[j]
    for p in range(m):
        arrs[f"parity{p}"] = par[p]
    return arrs


def diff_fixture(k=3, m=2, n=4098):
    mat = O.big_vandermonde(k + m, k)
    arrs = {"matrix": np.array(mat, np.int32)}
    for j in range(k):
        data = [O.splitmix_bytes(0xC0C70003 + 31 * x + j, n) for x in range(k)]
        par = O.encode(mat, k, m, data)
        new = O.splitmix_bytes(0xC0C70103 + j, n)
        old = data[j].copy()
        pv = [p.copy() for p in par]
        O.diff_update(mat, k, m, j, old, new, pv, True)
        arrs[f"j{j}_old"] = data[j]
        arrs[f"j{j}_new"] = new
        for p in range(m):
            arrs[f"j{j}_parity{p}_before"] = par[p]
            arrs[f"j{j}_parity{p}_after"] = pv[p]
    return arrs


def decode_fixture(k, m, n):
    mat = O.big_vandermonde(k + m, k)
    data = [O.splitmix_bytes(0xC0C70005 + 13 * j + k, n) for j in range(k)]
    par = O.encode(mat, k, m, data)
    arenas = data + par
    arrs = {"matrix": np.array(mat, np.int32)}
    for i, a in enumerate(arenas):
        arrs[f"arena{i}"] = a
    masks = []
    for lids in itertools.combinations(range(k + m), k):
        mask = sum(1 << x for x in lids)
        if mask == (1 << k) - 1:
            continue
        lost = [j for j in range(k) if not (mask >> j) & 1]
        if len(lost) > 2:
            continue  # single and double erasures
        out = O.decode(mat, k, m, mask, [a if (mask >> i) & 1 else None for i, a in enumerate(arenas)])
        for x, j in enumerate(lost):
            assert np.array_equal(out[x], data[j])
            arrs[f"mask{mask}_lost{j}"] = out[x]
        masks.append(mask)
    arrs["masks"] = np.array(masks, np.uint32)
    return arrs


FIXTURES = {
    "region_multiply.npz": (region_fixture, "galois_w08_region_multiply(src, c, n, r2, 1) for c in "
                            f"{COEFS}, n in {SIZES}: r2 ^= c*src"),
    "encode_rs32.npz": (lambda: encode_fixture(3, 2, 4096 + 2), "RS(3,2) stripe encode, n = 4098"),
    "encode_rs42.npz": (lambda: encode_fixture(4, 2, 4096), "RS(4,2) stripe encode, n = 4096"),
    "encode_rs63.npz": (lambda: encode_fixture(6, 3, 1000), "RS(6,3) stripe encode, n = 1000"),
    "diff_update_rs32.npz": (diff_fixture, "RS(3,2) per-SET diff-update chain with install, j in 0..2"),
    "decode_rs32.npz": (lambda: decode_fixture(3, 2, 4096), "RS(3,2) decode, every single/double erasure mask"),
    "decode_rs42.npz": (lambda: decode_fixture(4, 2, 2048), "RS(4,2) decode, every single/double erasure mask"),
}


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def main():
    manifest = {"generator": "python tests/golden/make_golden.py (oracle/libgf8ref.so)",
                "parity": "unpinned (Jerasure/GF-Complete unavailable; oracle restatement)",
                "field": "GF(2^8), poly 0x11D, generator 2", "files": {},
                "matrices": {f"{k},{m}": O.big_vandermonde(k + m, k)
                             for k, m in [(3, 2), (4, 2), (6, 3), (10, 4)]}}
    for name, (fn, desc) in FIXTURES.items():
        path = os.path.join(HERE, name)
        arrs = fn()
        np.savez(path, **arrs)
        manifest["files"][name] = {"sha256": sha256(path), "what": desc, "arrays": len(arrs)}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(FIXTURES), "fixtures")


if __name__ == "__main__":
    main()
