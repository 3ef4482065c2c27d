#!/bin/bash
# tools/dropin_ab.sh -- per-call drop-in cost, this build vs tools/ab/prev (a previous
# build's libcocytus_ec.so + libJerasure.so), interleaved in separate processes on one
# box (run ON the GPU box).  Lines land in gpurun_out/dropin_ab/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/dropin_ab
mkdir -p "$OUT"
: > "$OUT/ab.txt"
for rep in $(seq 1 ${REPS:-3}); do
  for v in cur prev; do
    if [ "$v" = prev ]; then LP=$R/tools/ab/prev; else LP=; fi
    b=$(LD_LIBRARY_PATH=$LP timeout -k 10 120 "$R/tools/dropin_breakdown.bin") || exit 1
    l=$(LD_LIBRARY_PATH=$LP timeout -k 10 120 "$R/tools/dropin_latency.bin" | tr '\n' ' ') || exit 1
    echo "$v $rep $b $l" >> "$OUT/ab.txt"
  done
done
