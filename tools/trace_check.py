#!/usr/bin/env python3
"""Check a bench line's roofline against rocprofv3's kernel trace of the SAME run.

    python tools/trace_check.py <rocprof -d dir> <bench line .jsonl> [out.json]

`tools/r04_calls.sh g` runs the driver's exact command (`python bench.py`, no flags) under
`rocprofv3 --kernel-trace --stats`.  The line's `roofline.launch_ms` is the average
HIP-event time of its timed whole-batch encode launches; here the same launches are
picked out of the trace -- the first (warmup + steps) dispatches of the line's encode
kernel with the whole batch's grid (256 work-items per 4 KiB tile), in start order (the metric's workload runs first;
later whole-batch dispatches of that kernel belong to other workloads), the last `steps`
of them timed -- and their average duration is compared with the line's.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys


def main(prof_dir, line_path, out_path=None):
    line = json.loads([ln for ln in open(line_path) if ln.startswith("{")][-1])
    traces = glob.glob(os.path.join(prof_dir, "**", "run_kernel_trace.csv"), recursive=True)
    stats = glob.glob(os.path.join(prof_dir, "**", "run_kernel_stats.csv"), recursive=True)
    assert traces, f"no run_kernel_trace.csv under {prof_dir}"
    rows = list(csv.DictReader(open(traces[0])))
    # the warmups the bench actually ran (it runs at least one even under --warmup 0)
    steps, warm = line["steps"], line.get("warmup_run", max(1, line["warmup"]))
    k, m = line["config"]["k"], line["config"]["m"]
    eng = "PermEngine" if "PermEngine" in line["roofline"]["kernel"] else "LdsEngine"
    tiles = line["config"]["stripes_per_gpu"] * line["config"]["value_bytes"] // 4096

    def is_encode(r):
        n = r["Kernel_Name"]
        return "combine_kernel<" in n and f"<{k}, {m}, cec::{eng}" in n

    def grid(r):
        return int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)

    enc = sorted((r for r in rows if is_encode(r)), key=lambda r: int(r["Start_Timestamp"]))
    whole = tiles * 256  # one 4 KiB tile = 256 lanes (in 1, 2 or 4 workgroups): the whole batch
    batch = [r for r in enc if grid(r) == whole][: warm + steps]
    timed = batch[warm:]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
    avg = sum(durs) / len(durs)
    ev = line["roofline"]["launch_ms"]
    nbytes = line["roofline"]["algorithmic_bytes_per_launch"]
    out = {
        "command": "python bench.py (the driver's command, no flags) under rocprofv3 --kernel-trace --stats",
        "kernel": timed[0]["Kernel_Name"],
        "whole_batch_grid_work_items": whole, "tiles": tiles,
        "dispatches_timed": len(durs), "warmup_dispatches_skipped": warm,
        "trace_avg_ms": round(avg, 5), "trace_median_ms": round(statistics.median(durs), 5),
        "line_event_avg_ms": ev, "event_over_trace": round(ev / avg, 4),
        "trace_frac_of_8TBps": round(nbytes / (avg * 1e-3) / 8e12, 4), "line_frac": line["roofline"]["frac"],
        "line_value": line["value"], "line_kernel_code_id": line["roofline"].get("kernel_code_id"),
        "stats_csv": os.path.relpath(stats[0], prof_dir) if stats else None,
    }
    print(json.dumps(out, indent=1))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(out, f, indent=1)
    return out


if __name__ == "__main__":
    main(*sys.argv[1:])
