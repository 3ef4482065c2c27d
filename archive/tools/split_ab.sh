#!/bin/bash
# tools/split_ab.sh -- A/B of the workgroups-per-tile choice (CEC_SPLIT_SHIFT 0/1/2 and
# the automatic rule) on the bench workloads, interleaved, one box (run ON the GPU box
# through gpurun).  Lines land in gpurun_out/split_ab/ab.jsonl.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/split_ab
mkdir -p "$OUT"
cd "$R"
SPLITS=${SPLITS:-"auto 0 1 2"}
ROUNDS=${ROUNDS:-2}
WORKLOADS=${WORKLOADS:-"rs32_4k rs32_mixed rs42_64k rs32_1m"}
for r in $(seq "$ROUNDS"); do
  for s in $SPLITS; do
    for w in $WORKLOADS; do
      if [ "$s" = auto ]; then env=""; else env="CEC_SPLIT_SHIFT=$s"; fi
      env $env timeout -k 10 200 python bench.py --no-cpu-baseline --also= --workload "$w" \
        | sed "s/^/{\"split\": \"$s\", \"round\": $r, \"line\": /; s/\$/}/" >> "$OUT/ab.jsonl"
    done
  done
done
echo done > "$OUT/DONE"
