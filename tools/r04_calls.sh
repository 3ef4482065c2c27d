#!/bin/bash
# Round-4 gpurun calls, one case per call: `gpurun -- bash tools/r04_calls.sh <letter>`.
# Each GPU step runs under its own timeout; a step that faults, aborts or times out
# ends the call (rc > 1; pytest's rc 1 = failed tests, which the call reports and goes on).
# The letter names the gpurun_out/r04<letter>/ directory the call wrote, whose kept files
# are under profiles/r04_evidence/.
call=$1
mkdir -p gpurun_out/r04$call
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r04$call/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
case "$call" in
a)
  # this round's new GPU tests first (configs[2] at full size, AUTO's choices, released
  # streams, both store policies on every kernel kind, the 2-rank line's evidence), then
  # the whole GPU suite, then the default bench line
  run new_tests 900 $PYT -m gpu tests/test_gpu_golden.py::test_cfg3_mixed_full_size \
      tests/test_gpu_runtime.py::test_auto_engine_choices tests/test_gpu_runtime.py::test_release_stream_keeps_tracking_bounded \
      tests/test_gpu_parity.py::test_store_policy_every_kernel_kind tests/test_gpu_parity.py::test_bench_two_ranks_one_card_weak_and_strong
  run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  run bench_default 300 python -u bench.py
  ;;
b)
  # every DESIGN §5 number from one box (no profiles: call c)
  EVID_NO_PROF=1 timeout -k 10 1100 bash tools/round_evidence.sh r04
  ;;
c)
  # rocprofv3 on this round's kernels: kernel-trace stats and the FETCH_SIZE / WRITE_SIZE
  # passes per workload, PERM (profiles/pmc_traffic.json) and LDS (pmc_traffic_lds.json,
  # the workloads whose decode AUTO runs with it), each summary stamped with the kernels'
  # code id (bench.py reports traffic only for the kernels it measured)
  timeout -k 10 560 bash tools/profile_round.sh r04 > gpurun_out/r04c/profile.log 2>&1 && \
  PROF_ENGINE=lds PROF_WORKLOADS="rs32_4k rs32_mixed rs42_64k rs32_1m rs32_diff_update" \
      timeout -k 10 560 bash tools/profile_round.sh r04_lds > gpurun_out/r04c/profile_lds.log 2>&1
  ;;
d)
  # the one-rank RCCL path of the N > 1 line, the 2-rank one-card line, then the suite
  run rccl_tests 600 $PYT -m gpu tests/test_gpu_parity.py::test_bench_rccl_path_one_rank \
      tests/test_gpu_parity.py::test_bench_two_ranks_one_card_weak_and_strong \
      tests/test_gpu_parity.py::test_cfg4_eight_rank_batches_one_card
  run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  # host code under ASan + UBSan and TSan (built here: tools/asan.sh build, tools/tsan.sh
  # build; .gpurunignore lets tools/asan and tools/tsan travel for this call only)
  if [ -f tools/asan/libcocytus_ec.so ] && [ -f tools/tsan/libcocytus_ec.so ]; then
    run asan 600 bash tools/asan.sh run
    run tsan 600 bash tools/tsan.sh run
  fi
  ;;
e)
  # whole-batch oracle parity for configs[3] and configs[4], then the suite
  run cfg_tests 600 $PYT -m gpu tests/test_gpu_parity.py::test_cfg4_rs42_64k_roundtrip \
      tests/test_gpu_parity.py::test_cfg5_1mib_decode_d0_p0_and_d1_p1 tests/test_gpu_runtime.py::test_release_stream_refused_while_capturing
  run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  ;;
f)
  # AUTO's final rule (LDS only for decodes of values >= 64 KiB), the suite, then the
  # round's canonical evidence set on the final build (no profiles: kernels unchanged)
  run auto_tests 600 $PYT -m gpu tests/test_gpu_runtime.py::test_auto_engine_choices \
      tests/test_gpu_golden.py::test_cfg3_mixed_full_size tests/test_glue.py
  run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  EVID_NO_PROF=1 timeout -k 10 900 bash tools/round_evidence.sh r04f
  ;;
g)
  # rocprofv3 --kernel-trace --stats of the driver's exact command (python bench.py, no
  # flags) with its line, so the line's encode launch time can be checked against the
  # trace's whole-batch encode dispatches of the same run (tools/trace_check.py)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_default" -o run \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/r04g/bench_default.jsonl" \
      2> "$GRAFT_REPO_ROOT/gpurun_out/r04g/bench_default.err"
  ;;
h)
  # the final tree as the driver runs it: smoke, the GPU suite, the default line
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
  run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  run bench_default 300 python -u bench.py
  ;;
i)
  # the diff-update at the bench's size under each engine
  run du_tests 600 $PYT -m gpu tests/test_gpu_parity.py::test_diff_update_full_size tests/test_gpu_parity.py::test_drainer_full_size
  ;;
j)
  # the drain loop at the server level over the real rep_queue: the glue vs the unchanged
  # per-xid loop through the drop-in (4098 B = a 4 KiB value + CRLF, memcached.c:3610)
  run glue_bench 300 oracle/_ref/glue_drain bench 65536 4098
  run glue_bench_4k 300 oracle/_ref/glue_drain bench 65536 4096
  run glue_bench_256 300 oracle/_ref/glue_drain bench 65536 4098 256
  ;;
k)
  # the default line with the other configs' CPU baselines
  run bench_default 400 python -u bench.py
  ;;
l)
  # the drain's radix-sorted wave colouring: every drain test, then the drain lines
  run drain_tests 600 $PYT -m gpu -k "drainer or glue or batched_bindings or registered_host or release_stream" tests
  run bench_drain 300 python -u bench.py --drain --steps 5 --warmup 2
  run glue_bench 300 oracle/_ref/glue_drain bench 65536 4098
  run glue_bench_4k 300 oracle/_ref/glue_drain bench 65536 4096
  ;;
m)
  # the final host code: the GPU suite, then ASan + UBSan and TSan (sanitizer builds travel
  # for this call only)
  run pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
  run asan 600 bash tools/asan.sh run
  run tsan 600 bash tools/tsan.sh run
  ;;
esac
