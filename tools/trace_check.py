#!/usr/bin/env python3
"""Check a bench line's roofline against rocprofv3's kernel trace of the SAME run.

    python tools/trace_check.py <rocprof -d dir> <bench line .jsonl> [out.json]

`tools/r06_calls.sh` runs the driver's exact command (`python bench.py`, no flags) under
`rocprofv3 --kernel-trace --stats`.  The line's `roofline.launch_ms` / `decode_roofline.
launch_ms` are the average HIP-event times of its timed whole-batch encode / decode
launches; here the same launches are picked out of the trace -- for each op, the first
(warmup + steps) dispatches of its kernel (encode: combine_kernel<K, M, engine>, the
rotating single-shard decode: combine_kernel<K, 1, engine>, the engine the line says
ran) with the whole batch's grid (256 work-items per 4 KiB tile), in start order (the
metric's workload runs first; later whole-batch dispatches of that kernel belong to other
workloads), the last `steps` of them timed -- and their average duration is compared with
the line's.  The trace may be gzip'd (run_kernel_trace.csv.gz).
"""
from __future__ import annotations

import csv
import glob
import gzip
import json
import os
import statistics
import sys


def main(prof_dir, line_path, out_path=None):
    line = json.loads([ln for ln in open(line_path) if ln.startswith("{")][-1])
    traces = glob.glob(os.path.join(prof_dir, "**", "run_kernel_trace.csv*"), recursive=True)
    stats = glob.glob(os.path.join(prof_dir, "**", "run_kernel_stats.csv"), recursive=True)
    assert traces, f"no run_kernel_trace.csv under {prof_dir}"
    opener = gzip.open if traces[0].endswith(".gz") else open
    with opener(traces[0], "rt") as f:
        rows = list(csv.DictReader(f))
    # the warmups the bench actually ran (it runs at least one even under --warmup 0)
    steps, warm = line["steps"], line.get("warmup_run", max(1, line["warmup"]))
    k, m = line["config"]["k"], line["config"]["m"]
    tiles = line["config"]["stripes_per_gpu"] * line["config"]["value_bytes"] // 4096
    whole = tiles * 256  # one 4 KiB tile = 256 lanes (in 1, 2 or 4 workgroups): the whole batch
    ran = line["config"]["engine"]  # "... (ran: encode PERM, decode PERM, ..."

    def engine_of(op):
        return "LdsEngine" if f"{op} LDS" in ran else "PermEngine"

    def grid(r):
        return int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)

    # encode: combine_kernel<K, M, ...>; decode (one lost shard): combine_kernel<K, 1, ...>
    out = {"command": "python bench.py (the driver's command, no flags) under rocprofv3 --kernel-trace --stats",
           "whole_batch_grid_work_items": whole, "tiles": tiles, "line_value": line["value"],
           "line_kernel_code_id": line["roofline"].get("kernel_code_id"),
           "stats_csv": os.path.relpath(stats[0], prof_dir) if stats else None}
    for op, outs, rl in (("encode", m, line["roofline"]), ("decode", 1, line["decode_roofline"])):
        eng = engine_of(op)
        sig = f"combine_kernel<{k}, {outs}, cec::{eng}"
        disp = sorted((r for r in rows if sig in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
        # the metric's workload runs first: its warm + steps whole-batch dispatches; later
        # ones of the same kernel and grid belong to other workloads
        batch = [r for r in disp if grid(r) == whole][: warm + steps]
        timed = batch[warm:]
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
        avg = sum(durs) / len(durs)
        ev = rl["launch_ms"]
        nbytes = rl["algorithmic_bytes_per_launch"]
        out[op] = {
            "kernel": timed[0]["Kernel_Name"], "dispatches_timed": len(durs), "warmup_dispatches_skipped": warm,
            "trace_avg_ms": round(avg, 5), "trace_median_ms": round(statistics.median(durs), 5),
            "line_event_avg_ms": ev, "event_over_trace": round(ev / avg, 4),
            "trace_frac_of_8TBps": round(nbytes / (avg * 1e-3) / 8e12, 4), "line_frac": rl["frac"],
        }
    # (round-5 keys, for the records that quote them)
    out.update({x: out["encode"][x] for x in ("kernel", "dispatches_timed", "warmup_dispatches_skipped",
                                               "trace_avg_ms", "trace_median_ms", "line_event_avg_ms",
                                               "event_over_trace", "trace_frac_of_8TBps", "line_frac")})
    print(json.dumps(out, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1)
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
