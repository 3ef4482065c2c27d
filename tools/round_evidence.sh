#!/bin/bash
# tools/round_evidence.sh ROUND -- every measurement DESIGN.md quotes, on one box, one call
# (run ON the GPU box through gpurun; build first, here: python -c 'import __graft_entry__ as g;
# g.build()' && make -C tools).  Results land in gpurun_out/evidence_ROUND/; copy what is
# quoted into profiles/ROUND_evidence/ here, and run tools/pmc_summary.py on the merged
# gpurun_out/prof_ROUND.
set -euo pipefail
ROUND=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/evidence_$ROUND
mkdir -p "$OUT"
cd "$R"
B="timeout -k 10 300 python bench.py"
BW="$B --also="  # one workload per line
$B                                     > "$OUT/bench_default.jsonl" 2> "$OUT/bench_default.err"
$BW --no-cpu-baseline --engine lds      > "$OUT/bench_lds.jsonl"     2> "$OUT/bench_lds.err"
$BW --no-cpu-baseline --workload rs32_mixed > "$OUT/bench_mixed.jsonl" 2> "$OUT/bench_mixed.err"
$BW --no-cpu-baseline --workload rs42_64k   > "$OUT/bench_rs42.jsonl"  2> "$OUT/bench_rs42.err"
$BW --no-cpu-baseline --workload rs32_1m    > "$OUT/bench_1m.jsonl"    2> "$OUT/bench_1m.err"
$B --e2e                               > "$OUT/bench_e2e.jsonl"     2> "$OUT/bench_e2e.err"
$B --e2e --e2e-zero-copy               > "$OUT/bench_e2e_zc.jsonl"  2> "$OUT/bench_e2e_zc.err"
$B --drain --steps 5 --warmup 2        > "$OUT/bench_drain.jsonl"   2> "$OUT/bench_drain.err"
$B --recovery --steps 5                > "$OUT/bench_recovery.jsonl" 2> "$OUT/bench_recovery.err"
$B --ops --engine perm                 > "$OUT/bench_ops.jsonl"     2> "$OUT/bench_ops.err"
$B --ops --engine lds                  > "$OUT/bench_ops_lds.jsonl" 2> "$OUT/bench_ops_lds.err"
timeout -k 10 200 tools/hbm_mix.bin arena random 64  > "$OUT/hbm_mix.txt" 2>&1
timeout -k 10 200 tools/hbm_mix.bin arena random 256 >> "$OUT/hbm_mix.txt" 2>&1
timeout -k 10 200 tools/dropin_latency.bin > "$OUT/dropin_latency.jsonl" 2>&1
timeout -k 10 200 tools/pool_bench.bin     > "$OUT/pool_bench.jsonl" 2>&1
# the drain loop at the server level, over the real rep_queue (oracle/_ref, built here)
if [ -x oracle/_ref/glue_drain ]; then
  timeout -k 10 200 oracle/_ref/glue_drain bench 65536 4098 > "$OUT/glue_drain_bench.jsonl" 2>&1
fi
timeout -k 10 200 tools/launch_latency.bin > "$OUT/launch_latency.txt" 2>&1
timeout -k 10 200 tools/bench_native.bin 20 3 > "$OUT/bench_native.jsonl" 2>&1
for b in 32768 16384 8192; do  # the strong-scaling shares with no Python in the loop
  CEC_NATIVE_STRIPES=$b timeout -k 10 200 tools/bench_native.bin 20 3 >> "$OUT/bench_native_shares.jsonl" 2>&1
done
CEC_NATIVE_DEVICE=0 timeout -k 10 200 tools/bench_native.bin 20 3 2 > "$OUT/bench_native_2threads_one_card.jsonl" 2>&1
CEC_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 > "$OUT/bench_gloo2_one_card.jsonl" 2> "$OUT/bench_gloo2.err"
# the driver's N: 8 ranks on one card (gloo), the weak line and the fixed-batch split
CEC_BENCH_WATCHDOG=60 CEC_BENCH_DEVICE=0 timeout -k 10 500 python bench.py --gpus 8 --also= \
    > "$OUT/bench_gloo8_one_card.jsonl" 2> "$OUT/bench_gloo8.err"
# configs[3] as stated (RS(4,2) 64 KiB, 8 independent rank batches), its 8 ranks on one card
CEC_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus 8 --workload rs42_64k --also= --no-strong \
    --no-cpu-baseline > "$OUT/bench_gloo8_rs42_one_card.jsonl" 2> "$OUT/bench_gloo8_rs42.err"
# the N > 1 line's RCCL collectives on a one-rank communicator
CEC_BENCH_PG=1 timeout -k 10 300 python bench.py --dist-backend nccl --no-cpu-baseline \
    > "$OUT/bench_rccl_one_rank.jsonl" 2> "$OUT/bench_rccl_one_rank.err"
timeout -k 10 120 tools/xcd_visibility_probe.bin 64 200 > "$OUT/xcd_visibility.jsonl" 2>&1
timeout -k 10 120 tools/small_batch_probe.bin 20 > "$OUT/small_batch_probe.jsonl" 2>&1
timeout -k 10 200 python tools/du_probe.py > "$OUT/du_probe.json" 2>/dev/null
timeout -k 10 200 python tools/decode_probe.py > "$OUT/decode_probe.txt" 2>/dev/null
[ -n "${EVID_NO_PROF:-}" ] || bash tools/profile_round.sh "$ROUND" > "$OUT/profile.log" 2>&1
[ -n "${EVID_NO_PROF:-}" ] || PROF_ENGINE=lds PROF_WORKLOADS="rs32_4k rs32_diff_update" \
    bash tools/profile_round.sh "${ROUND}_lds" > "$OUT/profile_lds.log" 2>&1
echo done > "$OUT/DONE"
