#!/bin/bash
# rocprofv3 kernel durations of the bench step: round-1 build vs this build (tracking
# off / ext).  Writes gpurun_out/prof_<variant>/ and a one-line summary per variant.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for v in r01 off ext; do
  if [ "$v" = r01 ]; then export CEC_LIB_PATH=tools/ab/libcocytus_ec_r01.so; unset CEC_TRACK
  else unset CEC_LIB_PATH; export CEC_TRACK=$v; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$v -o run -- \
      python3 bench.py --also= --no-cpu-baseline --steps 50 > gpurun_out/prof_$v.json 2> gpurun_out/prof_$v.err || exit 1
done
unset CEC_LIB_PATH CEC_TRACK
for v in r01 off ext; do
  f=$(find gpurun_out/prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v: $(cat gpurun_out/prof_$v.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["launch_ms"], d["decode_roofline"]["launch_ms"])')"
  grep combine "$f" | cut -c1-300
done
