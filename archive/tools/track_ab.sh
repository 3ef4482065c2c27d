#!/bin/bash
# A/B of the bench step between library builds / runtime knobs (one GPU box), each in
# its own process, interleaved: VARIANTS="name:ENV=V,ENV2=V ..." (r01 = round-1 build).
set -u
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/track_ab.jsonl}
reps=${REPS:-2}
: > "$out"
for rep in $(seq $reps); do
  for spec in $VARIANTS; do
    name=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
    envargs=$(echo "$envs" | tr ',' ' ')
    env $envargs timeout -k 10 120 python bench.py --also= --no-cpu-baseline --steps 50 ${BENCH_ARGS:-} > /tmp/ab.json || exit 1
    python3 -c "
import json,sys; d=json.load(open('/tmp/ab.json'))
print(json.dumps({'variant': '$name', 'rep': $rep, 'value': d['value'], 'ms_per_step': d['ms_per_step'],
 'enc_ms': d['roofline']['launch_ms'], 'dec_ms': d['decode_roofline']['launch_ms']}))" >> "$out"
  done
done
cat "$out"
