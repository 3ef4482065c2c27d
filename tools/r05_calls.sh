#!/bin/bash
# Round-5 GPU calls (run on the box by gpurun from the repo root).  Usage: bash tools/r05_calls.sh <case>
#   d  host batch + glue tests, the glue benches (recovery, SET diffs, drain in both placements)
#   i  the recovery glue's pool placement (tests + bench)
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
f)  # the final tree as the driver runs it: smoke, the whole GPU suite (incl. the one-rank
    # RCCL path and configs[3]'s eight rank batches on one card), the default line
    out=gpurun_out/r05f; mkdir -p $out
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
    timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
    timeout -k 10 300 python -u bench.py > $out/bench_default.jsonl 2> $out/bench_default.err || exit 3
    ;;
g)  # rocprofv3 --kernel-trace --stats of the driver's exact command (python bench.py, no
    # flags) with its line, for tools/trace_check.py
    out=$GRAFT_REPO_ROOT/gpurun_out/r05g; mkdir -p $out
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r05_default" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" > $out/bench_default.jsonl 2> $out/bench_default.err
    ;;
h)  # where the host batch's GPU time goes: kernel durations of the recovery shapes
    out=$GRAFT_REPO_ROOT/gpurun_out/r05h; mkdir -p $out
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$out/prof" -o run --output-format csv \
        -- python3 "$GRAFT_REPO_ROOT/tools/hostbatch_bench.py" 5 > $out/hostbatch_bench.jsonl 2> $out/err.log
    ;;
i)  # the pool placement of the recovery glue: its tests, the pool's own tests, the bench shapes
    out=gpurun_out/r05i; mkdir -p $out
    timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_glue_rpool.py \
        tests/test_gpu_parity.py tests/test_glue_recovery.py -k "rpool or recovery_pool or cluster_sim" > $out/pytest.log 2>&1 || exit 1
    timeout -k 10 120 oracle/_ref/glue_recovery_bench 15 > $out/recovery_bench.jsonl 2>&1 || exit 2
    ;;
*) echo "unknown case $1"; exit 9 ;;
esac
