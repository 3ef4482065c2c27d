#!/bin/bash
# Round-6 GPU calls (run on the box by gpurun from the repo root).  Usage: bash tools/r06_calls.sh <case>
#   a  the changed paths' GPU tests (host batch, pool, drainer, glue) + smoke + the default line
#      with the server-placement entries
#   f  the final tree as the driver runs it: smoke, the whole GPU suite, the default line
#   g  rocprofv3 --kernel-trace --stats of the driver's exact command (python bench.py, no
#      flags) with its line, for tools/trace_check.py (encode and decode dispatches)
#   z  f, then g
set -o pipefail
case "$1" in
a)
    out=gpurun_out/r06a; mkdir -p $out
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
    timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_hostbatch.py \
        tests/test_glue.py tests/test_glue_recovery.py tests/test_glue_rpool.py tests/test_gpu_parity.py \
        -k "hostbatch or glue or rpool or recovery_pool or drain or set_diffs or batch or cluster_sim" \
        > $out/pytest.log 2>&1 || exit 2
    timeout -k 10 400 python -u bench.py > $out/bench_default.jsonl 2> $out/bench_default.err || exit 3
    ;;
f)
    out=gpurun_out/r06f; mkdir -p $out
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
    timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
    rc=$?; echo "pytest rc=$rc"; [ $rc -gt 1 ] && exit $rc
    timeout -k 10 400 python -u bench.py > $out/bench_default.jsonl 2> $out/bench_default.err || exit 3
    ;;
g)
    out=$GRAFT_REPO_ROOT/gpurun_out/r06g; mkdir -p $out
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r06_default" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" > $out/bench_default.jsonl 2> $out/bench_default.err
    ;;
z)  # f then g in one call (one box acquisition): the final tree's evidence set
    bash tools/r06_calls.sh f || exit $?
    bash tools/r06_calls.sh g || exit $?
    ;;
*) echo "unknown case $1"; exit 9 ;;
esac
