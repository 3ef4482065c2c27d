#!/bin/bash
# tools/profile_round.sh ROUND -- rocprofv3 evidence for the bench command (run ON the GPU box).
#   pass 1: --kernel-trace --stats      (per-kernel average duration)
#   pass 2: --pmc FETCH_SIZE            (HBM read bytes; separate pass: TCC slots)
#   pass 3: --pmc WRITE_SIZE            (HBM write bytes)
# then tools/pmc_summary.py writes profiles/ROUND_* and profiles/pmc_traffic.json.
set -euo pipefail
ROUND=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$ROUND
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# --no-strong: the strong-scaling shares launch the same kernels at smaller sizes, which
# would mix into the per-kernel averages.  PROF_ENGINE=lds profiles the LDS engine (its
# summary keeps profiles/pmc_traffic.json, the default engine's, untouched).
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-strong --engine ${PROF_ENGINE:-perm}"
for W in ${PROF_WORKLOADS:-rs32_4k rs32_mixed rs42_64k rs32_1m rs32_diff_update}; do
  if [ "$W" = rs32_diff_update ]; then WA="--workload rs32_4k --also=rs32_diff_update"; else WA="--workload $W --also="; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_$W" -o run --output-format csv \
      -- python3 "$R/bench.py" $ARGS $WA > "$OUT/bench_trace_$W.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_$W" -o run --output-format csv \
      -- python3 "$R/bench.py" $ARGS $WA > "$OUT/bench_fetch_$W.log" 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write_$W" -o run --output-format csv \
      -- python3 "$R/bench.py" $ARGS $WA > "$OUT/bench_write_$W.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" "$OUT" "$ROUND" ${PROF_ENGINE:+--engine $PROF_ENGINE}
