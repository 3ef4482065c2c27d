#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/ (committed evidence).

Per workload and per cocytus kernel: average duration (kernel-trace pass), HBM
traffic per launch from FETCH_SIZE / WRITE_SIZE (separate --pmc passes) with the
gfx950 corrections of MI355X_MICROARCH.md §HBM: values are KiB; FETCH_SIZE counts
half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B streaming stores.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGO = {  # algorithmic bytes per launch: (encode, decode)
    "rs32_4k": ((3 + 2) * 4096 * 65536, (3 + 1) * 4096 * 65536),
    "rs42_64k": ((4 + 2) * 65536 * 16384, (4 + 1) * 65536 * 16384),
    "rs32_1m": ((3 + 2) * (1 << 20) * 1024, (3 + 1) * (1 << 20) * 1024),
}
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (layout() of the mixed workload; no torch at import)

_MIXED = sum(n for _, n in bench.layout("rs32_mixed")[0])
ALGO["rs32_mixed"] = ((3 + 2) * _MIXED, (3 + 1) * _MIXED)
# the fused diff-update + install (a4): read old, new, 2 parities; write 2 parities + D
ALGO["rs32_diff_update"] = ((2 + 2 * 2 + 1) * 4096 * 65536, None)
SHAPES = {"rs32_4k": ("<3, 2,", "<3, 1,"), "rs42_64k": ("<4, 2,", "<4, 1,"), "rs32_1m": ("<3, 2,", "<3, 1,"),
          "rs32_mixed": ("<3, 2,", "<3, 1,"), "rs32_diff_update": ("<2, 3,", None)}
OPS = {"rs32_diff_update": ("diff_update", None)}  # op names of (first, second) shape


def sources_sha256() -> str:
    """sha256 (16 hex digits) of the library's sources (cocytus_amd/csrc/*, include/*) when
    the summary is written, for the record; bench.py keys on kernel_code_id (the device
    code the counters measured), which host-only edits leave unchanged."""
    import hashlib

    h = hashlib.sha256()
    for d in ("cocytus_amd/csrc", "include"):
        for name in sorted(os.listdir(os.path.join(ROOT, d))):
            with open(os.path.join(ROOT, d, name), "rb") as f:
                h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def one(path_glob):
    c = glob.glob(path_glob, recursive=True)
    return c[0] if c else None


def kernel_rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(out, rnd, engine="perm"):
    summary, traffic, lines = {}, {}, []
    for w in ALGO:
        stats = one(f"{out}/trace_{w}/**/run_kernel_stats.csv")
        if not stats:
            continue
        enc_key, dec_key = SHAPES[w]
        res = {}
        for r in kernel_rows(stats):
            name = r["Name"]
            if "combine_kernel" not in name:
                continue
            ops = OPS.get(w, ("encode", "decode"))
            if enc_key in name:
                op = ops[0]
            elif dec_key and dec_key in name:
                op = ops[1]
            else:
                continue  # set-up kernels of the run (e.g. the diff-update's initial encode)
            res[op] = {"kernel": name, "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
        for counter, kind in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
            cc = one(f"{out}/{kind}_{w}/**/run_counter_collection.csv")
            if not cc:
                continue
            acc = {}
            for r in kernel_rows(cc):
                name = r.get("Kernel_Name", "")
                if "combine_kernel" not in name or r.get("Counter_Name") != counter:
                    continue
                ops = OPS.get(w, ("encode", "decode"))
                if enc_key in name:
                    op = ops[0]
                elif dec_key and dec_key in name:
                    op = ops[1]
                else:
                    continue
                acc.setdefault(op, {})
                d = r.get("Dispatch_Id", r.get("Correlation_Id"))
                acc[op][d] = acc[op].get(d, 0.0) + float(r["Counter_Value"])
            for op, per in acc.items():
                vals = list(per.values())
                res.setdefault(op, {})[counter + "_KiB_raw"] = sum(vals) / len(vals)
        ops = OPS.get(w, ("encode", "decode"))
        for op, algo in ((ops[0], ALGO[w][0]), (ops[1], ALGO[w][1])):
            e = res.get(op) if op else None
            if not e or "avg_ns" not in e or algo is None:
                continue
            e["algorithmic_bytes"] = algo
            e["achieved_GBps"] = algo / e["avg_ns"]
            e["frac_of_8TBps"] = e["achieved_GBps"] / 8000.0
            if "FETCH_SIZE_KiB_raw" in e and "WRITE_SIZE_KiB_raw" in e:
                rd = 2 * e["FETCH_SIZE_KiB_raw"] * 1024  # gfx950: FETCH_SIZE is half of a wide read
                wr = e["WRITE_SIZE_KiB_raw"] * 1024
                e["hbm_read_bytes"] = rd
                e["hbm_write_bytes"] = wr
                e["hbm_bytes"] = rd + wr
                e["traffic_over_algorithmic"] = (rd + wr) / algo
        summary[w] = res
        traffic[w] = {f"{op}_hbm_bytes_per_launch": res[op].get("hbm_bytes") for op in ops if op and op in res}
        for op in [o for o in ops if o]:
            e = res.get(op, {})
            if "avg_ns" in e:
                lines.append(f"| {w} | {op} | {e['avg_ns'] / 1e3:.1f} | {e['achieved_GBps']:.0f} | "
                             f"{e['frac_of_8TBps']:.3f} | {e.get('hbm_bytes', float('nan')) / 2**20:.1f} | "
                             f"{e['algorithmic_bytes'] / 2**20:.1f} | {e.get('traffic_over_algorithmic', float('nan')):.3f} |")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    with open(os.path.join(prof, f"{rnd}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # bench.py's `traffic` per engine: pmc_traffic.json (PERM), pmc_traffic_lds.json.
    # `_build` ties the bytes to the kernels they measured: bench.py reports them only
    # while the library it loads has the same device code (traffic_stale otherwise).
    from cocytus_amd import ec

    traffic["_build"] = {"kernel_code_id": ec.kernel_code_id(), "sources_sha256": sources_sha256(),
                         "round": rnd, "engine": engine}
    with open(os.path.join(prof, "pmc_traffic.json" if engine == "perm" else f"pmc_traffic_{engine}.json"),
              "w") as f:
        json.dump(traffic, f, indent=1)
    md = [f"# rocprofv3 summary ({rnd}, engine {engine})", "",
          f"bench.py --steps 10 --warmup 2 --no-strong --engine {engine} per workload "
          "(rs32_diff_update: --also=rs32_diff_update, only its",
          "<2, 3, ..., 2> kernel counted); durations from --kernel-trace --stats;",
          "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB, gfx950 correction), separate --pmc passes.", "",
          "| workload | op | avg us | algorithmic GB/s | frac of 8 TB/s | HBM MiB/launch (PMC) | algorithmic MiB | PMC/algo |",
          "|---|---|---|---|---|---|---|---|", *lines, ""]
    with open(os.path.join(prof, f"{rnd}_summary.md"), "w") as f:
        f.write("\n".join(md))
    for w in ALGO:  # keep the raw stats csv next to the summary
        s = one(f"{out}/trace_{w}/**/run_kernel_stats.csv")
        if s:
            shutil.copy(s, os.path.join(prof, f"{rnd}_{w}_kernel_stats.csv"))
    print("\n".join(md))


if __name__ == "__main__":
    a = sys.argv[1:]
    eng = "perm"
    if "--engine" in a:
        i = a.index("--engine")
        eng = a[i + 1]
        del a[i:i + 2]
    main(a[0], a[1], eng)
