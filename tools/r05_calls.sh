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
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 6
    ;;
e)  # host code under ASan + UBSan and TSan, incl. the round-5 glue and host batch (built here:
    # tools/asan.sh build + glue, tools/tsan.sh build + glue; .gpurunignore lets tools/asan and
    # tools/tsan travel for this call only)
    out=gpurun_out/r05e; mkdir -p $out
    timeout -k 10 900 bash tools/asan.sh run > $out/asan.txt 2>&1 || exit 1
    timeout -k 10 900 bash tools/tsan.sh run > $out/tsan.txt 2>&1 || exit 2
    ;;
*) echo "unknown case $1"; exit 9 ;;
esac
