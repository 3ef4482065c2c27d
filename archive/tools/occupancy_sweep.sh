#!/bin/bash
# tools/occupancy_sweep.sh -- bench.py (metric + other workloads) and bench.py --ops
# under CEC_WAVES_PER_CU caps (run ON the GPU box).  Results: gpurun_out/occ/.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/occ
mkdir -p "$OUT"
cd "$R"
for r in ${ROUNDS:-1}; do
  for w in ${CAPS:-0 8 10 12 16 24}; do
    CEC_WAVES_PER_CU=$w timeout -k 10 200 python bench.py --no-cpu-baseline \
        | sed "s/^/{\"waves_per_cu\": $w, \"line\": /; s/\$/}/" >> "$OUT/bench.jsonl"
    [ -n "${NO_OPS:-}" ] || CEC_WAVES_PER_CU=$w timeout -k 10 200 python bench.py --ops \
        | sed "s/^/{\"waves_per_cu\": $w, \"line\": /; s/\$/}/" >> "$OUT/ops.jsonl"
    echo "cap $w done" >&2
  done
done
echo done > "$OUT/DONE"
