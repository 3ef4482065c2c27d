#!/bin/bash
# Round-5 GPU calls (run on the box by gpurun from the repo root).  Usage: bash tools/r05_calls.sh <case>
#   d  host batch + glue tests, the glue benches (recovery, SET diffs, drain in both placements)
set -o pipefail
case "$1" in
d)
    out=gpurun_out/r05d; mkdir -p $out
    timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_hostbatch.py \
        tests/test_glue.py tests/test_glue_recovery.py > $out/pytest.log 2>&1 || exit 1
    timeout -k 10 120 oracle/_ref/glue_recovery_bench 15 > $out/recovery_bench.jsonl 2>&1 || exit 2
    timeout -k 10 200 oracle/_ref/glue_recovery_bench set 65536 4098 5 > $out/set_bench.jsonl 2>&1 || exit 3
    timeout -k 10 120 oracle/_ref/glue_drain bench 65536 4098 64 host > $out/drain_host.jsonl 2>&1 || exit 4
    timeout -k 10 120 python -u tools/hostbatch_bench.py 20 > $out/hostbatch_bench.jsonl 2>&1 || exit 5
    ;;
*) echo "unknown case $1"; exit 9 ;;
esac
