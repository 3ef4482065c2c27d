#!/bin/bash
# Round-3 gpurun calls, one case per call: `gpurun -- bash tools/r03_calls.sh <letter>`.
# Each GPU step runs under its own timeout; a step that faults, aborts or times out
# ends the call. The letter names the gpurun_out/r03<letter>/ directory the call wrote,
# whose kept files are under profiles/r03_evidence/.
call=$1
mkdir -p gpurun_out/r03$call
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03$call/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
case "$call" in
b)
  # round-3 GPU step list (one call): full GPU suite, the stale-tile precondition probe and
  # negative control, the small-batch fixed-cost probe, the diff-update early-install A/B
  run pytest 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  run xcdvis 120 tools/xcd_visibility_probe.bin 64 200
  run prefix_neg 300 env CEC_LIB_PATH=tools/prefix_build/libcocytus_ec.so python -u -m pytest tests/test_gpu_parity.py -k visible_from_every_xcd -q --timeout 120 --timeout-method thread
  run smallbatch 120 tools/small_batch_probe.bin 20
  for i in 1 2 3; do
    run du_new_$i 200 python -u bench.py --also=rs32_diff_update --no-strong --no-cpu-baseline
    run du_old_$i 200 env CEC_LIB_PATH=tools/ab_du/libcocytus_ec.so python -u bench.py --also=rs32_diff_update --no-strong --no-cpu-baseline
  done
  ;;
c)
  # round-3 GPU steps: store-policy A/B on the strong-scaling shares, GPU suite under
  # forced write-through and under the default policy, box record for the stale-tile probe
  run xcdvis 120 tools/xcd_visibility_probe.bin 64 200
  run pytest_wt 700 env CEC_STORE_POLICY=wt python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  for i in 1 2 3; do
    for p in nt wt auto; do
      run bench_${p}_$i 200 env CEC_STORE_POLICY=$p python -u bench.py --also= --no-cpu-baseline
    done
  done
  run pytest_auto 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
  ;;
e)
  # round-3 GPU steps: uniform-stream launches (kFlagUniform) -- GPU suite, then A/B against
  # the previous build (tools/ab_prev) on the metric and its strong-scaling shares, and --ops
  run xcdvis 120 tools/xcd_visibility_probe.bin 64 200
  run pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  for i in 1 2 3; do
    run bench_new_$i 200 python -u bench.py --also= --no-cpu-baseline
    run bench_prev_$i 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u bench.py --also= --no-cpu-baseline
  done
  run ops_new 200 python -u bench.py --ops
  run ops_prev 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u bench.py --ops
  ;;
f)
  # round-3 evidence on the final kernels: GPU suite, then every DESIGN §5 number (no profiles)
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f/pytest.log 2>&1 && \
  EVID_NO_PROF=1 bash tools/round_evidence.sh r03
  ;;
g)
  # round-3 GPU steps: LDS-engine A/B -- this build (no write-through branch in the staged
  # kernels) vs the branch (tools/ab_lds_wt) vs the build before the store policy (tools/ab_lds_pre)
  B="python -u bench.py --engine lds --also= --no-cpu-baseline --no-strong"
  for i in 1 2 3; do
    run lds_new_$i 200 $B
    run lds_wt_$i 200 env CEC_LIB_PATH=tools/ab_lds_wt/libcocytus_ec.so $B
    run lds_pre_$i 200 env CEC_LIB_PATH=tools/ab_lds_pre/libcocytus_ec.so $B
  done
  run pytest_lds 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lds or golden or fuzz"
  ;;
h)
  # round-3 evidence on the final kernels (after the LDS fix): GPU suite, then every DESIGN §5 number (no profiles)
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h/pytest.log 2>&1 && \
  EVID_NO_PROF=1 bash tools/round_evidence.sh r03
  ;;
i)
  # round-3 rocprofv3 evidence on the final kernels: kernel-trace + FETCH_SIZE / WRITE_SIZE
  # passes per workload, default (PERM) engine, then the LDS engine for the metric and the
  # diff-update
  bash tools/profile_round.sh r03 || exit $?
  PROF_ENGINE=lds PROF_WORKLOADS="rs32_4k rs32_diff_update" bash tools/profile_round.sh r03_lds || exit $?
  ;;
j)
  # round-3 sanitizer runs on the final host code (pool tables, launch checks, cache changes)
  timeout -k 10 600 bash tools/asan.sh run > gpurun_out/r03j/asan.txt 2>&1 && \
  timeout -k 10 600 bash tools/tsan.sh run > gpurun_out/r03j/tsan.txt 2>&1
  ;;
k)
  # round-3: the two-rank bench test, and the decode shape ceiling in the bench's arena order
  # beside the library's decode in the same call
  run pytest2 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "two_ranks or edge_cases or extent_pattern"
  run hbm_mix 200 tools/hbm_mix.bin arena random 64
  run decode_probe 200 python -u tools/decode_probe.py
  run hbm_mix_b 200 tools/hbm_mix.bin arena random 64
  ;;
l)
  # round-3: workgroups per tile (CEC_SPLIT_SHIFT) at the strong-scaling shares
  for i in 1 2; do
    for sh in 2 1 0; do
      run split${sh}_$i 200 env CEC_SPLIT_SHIFT=$sh python -u bench.py --also= --no-cpu-baseline
    done
  done
  ;;
m)
  # round-3: occupancy floor of 8 waves per SIMD for the small exact PERM kernels
  # (tools/ab_occ, -DCEC_WAVES_PER_EU=8: encode 3x2 68 -> 64 VGPRs) vs this build
  for i in 1 2 3; do
    run cur_$i 200 python -u bench.py --also= --no-cpu-baseline
    run occ_$i 200 env CEC_LIB_PATH=tools/ab_occ/libcocytus_ec.so python -u bench.py --also= --no-cpu-baseline
  done
  ;;
n)
  # round-3: the metric's step through the C-ABI alone at the strong-scaling shares
  for i in 1 2; do
    for b in 65536 32768 16384 8192; do
      CEC_NATIVE_STRIPES=$b timeout -k 10 200 tools/bench_native.bin 20 3 >> gpurun_out/r03n/native_shares.jsonl 2>&1 || exit $?
    done
  done
  ;;
o)
  # round-3: where a small encode launch's fixed cost goes (tile list / GF multiply / neither)
  for b in 8192 65536 8192; do
    ENCODE_GAP_STRIPES=$b timeout -k 10 200 python -u tools/encode_gap.py >> gpurun_out/r03o/encode_gap.txt 2>&1 || exit $?
  done
  timeout -k 10 120 tools/small_batch_probe.bin 20 > gpurun_out/r03o/small_batch_probe.jsonl 2>&1
  ;;
p)
  # round-3: LDS engine, workgroups per tile (its rotating decode stages product rows per
  # workgroup: 768 B per 1 KiB quarter-tile with s = 2)
  for i in 1 2; do
    for sh in 2 1 0; do
      run lds_s${sh}_$i 200 env CEC_SPLIT_SHIFT=$sh python -u bench.py --engine lds --also= --no-cpu-baseline --no-strong
    done
  done
  ;;
q)
  # round-3 final check on the final tree, as the driver runs it: GPU suite, smoke, default bench
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1 && \
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q/smoke.log 2>&1 && \
  timeout -k 10 600 python -u bench.py > gpurun_out/r03q/bench_default.jsonl 2> gpurun_out/r03q/bench_default.err
  ;;
r)
  # round-3: does a kernel's code size cost a small launch (instruction-cache warm-up)?
  timeout -k 10 200 tools/small_batch_probe.bin 20 > gpurun_out/r03r/small_batch_probe_v3.jsonl 2>&1
  ;;
s)
  # round-3: the bare stream with 64-bit vector addresses (what the code-size variant's
  # hot path compiled to) against the scalar-base form the library uses
  timeout -k 10 200 tools/small_batch_probe.bin 20 > gpurun_out/r03s/small_batch_probe_vaddr2.jsonl 2>&1
  ;;
t)
  # round-3 (second session): the completion-protocol assertions (cec_last_sync) in the GPU
  # suite on a fresh build, smoke, and the default bench line
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03t/pytest.log 2>&1 && \
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03t/smoke.log 2>&1 && \
  timeout -k 10 600 python -u bench.py > gpurun_out/r03t/bench_default.jsonl 2> gpurun_out/r03t/bench_default.err
  ;;
u)
  # round-3 (second session): LDS engine, two 128-lane workgroups per tile for launches
  # staging >= 3 product rows (the rotating decode), else four 64-lane (the encode):
  # LDS-engine GPU tests, then the LDS line + diff-update and --ops against the previous
  # choice pinned by CEC_SPLIT_SHIFT=2
  run pytest_lds 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "lds or golden or fuzz or decode"
  B="python -u bench.py --engine lds --also=rs32_diff_update --no-cpu-baseline --no-strong"
  for i in 1 2 3; do
    run lds_new_$i 200 $B
    run lds_s2_$i 200 env CEC_SPLIT_SHIFT=2 $B
  done
  run ops_new 200 python -u bench.py --ops --engine lds
  run ops_s2 200 env CEC_SPLIT_SHIFT=2 python -u bench.py --ops --engine lds
  ;;
v)
  # round-3 (second session): load policy at the strong-scaling shares (memory-side cache
  # reuse between the encode and the decode), bare XOR streams with write-through stores
  timeout -k 10 200 tools/small_batch_probe.bin 20 loads > gpurun_out/r03v/small_batch_loads.jsonl 2>&1
  ;;
w)
  # round-3 (second session): kernel-argument size and the slot-table chain at the
  # strong-scaling shares (the library's argument form on the bare stream)
  timeout -k 10 200 tools/small_batch_probe.bin 20 kernarg > gpurun_out/r03w/small_batch_kernarg.jsonl 2>&1
  ;;
x)
  # round-3 (second session): arena size at the strong-scaling shares -- share-sized arenas
  # (32 MiB + 4 KiB apart at 8,192 stripes) against arenas of the whole batch's size (the
  # bare-stream probe's spacing, 256 MiB + 4 KiB), same build, interleaved
  for i in 1 2 3; do
    run share_$i 200 python -u bench.py --also= --no-cpu-baseline
    run batch_$i 200 env CEC_BENCH_SHARE_ARENA=batch python -u bench.py --also= --no-cpu-baseline
  done
  ;;
y)
  # round-3 (second session): LDS engine, full aligned tiles stage their product rows
  # before the stream loads (the LDS write and barrier under the HBM latency) -- LDS GPU
  # tests, then the LDS line + diff-update against the previous build (tools/ab_prev)
  run pytest_lds 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "lds or golden or fuzz or decode"
  B="python -u bench.py --engine lds --also=rs32_diff_update --no-cpu-baseline --no-strong"
  for i in 1 2 3; do
    run lds_new_$i 200 $B
    run lds_prev_$i 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so $B
  done
  run ops_new 200 python -u bench.py --ops --engine lds
  run ops_prev 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u bench.py --ops --engine lds
  ;;
z)
  # round-3 (second session): early row staging restricted to the diff-update shapes --
  # LDS GPU tests, then the LDS line + diff-update against the previous build
  run pytest_lds 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "lds or golden or fuzz or diff"
  B="python -u bench.py --engine lds --also=rs32_diff_update --no-cpu-baseline --no-strong"
  for i in 1 2 3; do
    run lds_new_$i 200 $B
    run lds_prev_$i 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so $B
  done
  run ops_new 200 python -u bench.py --ops --engine lds
  run ops_prev 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u bench.py --ops --engine lds
  ;;
final2|final3)
  # round-3 (second session) evidence on the final build: GPU suite, then every DESIGN §5
  # number (no profiles; those are call final2p)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03$call/pytest.log 2>&1 && \
  EVID_NO_PROF=1 bash tools/round_evidence.sh r03$call
  ;;
final2p)
  # round-3 (second session) rocprofv3 on the final build: kernel trace + FETCH / WRITE passes
  bash tools/profile_round.sh r03s2 || exit $?
  PROF_ENGINE=lds PROF_WORKLOADS="rs32_4k rs32_diff_update" bash tools/profile_round.sh r03s2_lds || exit $?
  ;;
san2|san3)
  # round-3 (second session) sanitizer reruns on the final host code (cec_last_sync)
  timeout -k 10 600 bash tools/asan.sh run > gpurun_out/r03$call/asan.txt 2>&1 && \
  timeout -k 10 600 bash tools/tsan.sh run > gpurun_out/r03$call/tsan.txt 2>&1
  ;;
rec)
  # round-3 (second session): configs[4] as stated (fixed-mask recovery decode, 1 MiB values)
  run rec1 200 python -u bench.py --also=rs32_1m_recovery --no-cpu-baseline --no-strong
  run rec2 200 python -u bench.py --also=rs32_1m_recovery --no-cpu-baseline --no-strong --engine lds
  run pytest2 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "two_ranks"
  ;;
q2|q3|q4|q5|q6|q7)
  # round-3 (second session) final check on the final tree, as the driver runs it
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03$call/pytest.log 2>&1 && \
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03$call/smoke.log 2>&1 && \
  s0=$SECONDS && timeout -k 10 600 python -u bench.py > gpurun_out/r03$call/bench_default.jsonl 2> gpurun_out/r03$call/bench_default.err && echo "bench wall $((SECONDS - s0)) s" > gpurun_out/r03$call/bench_wall.txt
  ;;
du2)
  # round-3 (second session): the pool test's per-call completion checks, the default line
  # with the LDS diff-update beside the default engine's
  run pytest_pool 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "pool or two_ranks"
  run bench 300 python -u bench.py
  ;;
eng)
  # round-3 (second session): the engine read once per op -- the concurrent engine-switch
  # test on this build, then on the previous build (tools/ab_prev, engine read twice; a
  # mismatch gives wrong bytes, never a fault: LDS reads past the allocation return 0)
  run pytest_eng 300 python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 240 --timeout-method thread -k "engine_switch"
  timeout -k 10 300 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 240 --timeout-method thread -k "engine_switch" > gpurun_out/r03eng/pytest_eng_prev.log 2>&1; echo "prev rc=$?"
  run pytest_rt 600 python -u -m pytest tests/test_gpu_runtime.py tests/test_gpu_golden.py -x -q --timeout 240 --timeout-method thread
  ;;
engprev)
  # the negative control of case eng alone (tools/ab_prev uploaded for this call)
  timeout -k 10 300 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u -m pytest tests/test_gpu_runtime.py -x -q --timeout 240 --timeout-method thread -k "engine_switch" > gpurun_out/r03engprev/pytest_eng_prev.log 2>&1; echo "prev rc=$?"
  ;;
fixdec)
  # round-3 (second session): engine per op for the fixed-mask decode (one recovery mask for
  # the whole batch: configs[4], --ops' decode) -- PERM vs LDS, interleaved, three rounds
  for i in 1 2 3; do
    run rec_perm_$i 200 python -u bench.py --also=rs32_1m_recovery --no-cpu-baseline --no-strong --engine perm
    run rec_lds_$i 200 python -u bench.py --also=rs32_1m_recovery --no-cpu-baseline --no-strong --engine lds
    run ops_perm_$i 200 python -u bench.py --ops --engine perm
    run ops_lds_$i 200 python -u bench.py --ops --engine lds
  done
  ;;
delay)
  # round-3 (second session): what the LDS engine adds between a wave's loads and stores,
  # on bare XOR streams (the fixed-mask decode ran 5 % faster with two staged rows)
  timeout -k 10 200 tools/delay_probe.bin 1024 > gpurun_out/r03delay/delay_1g.jsonl 2>&1 && \
  timeout -k 10 200 tools/delay_probe.bin 256 > gpurun_out/r03delay/delay_256m.jsonl 2>&1
  ;;
occ)
  # round-3 (second session): is the LDS engine's fixed-mask decode lead an occupancy
  # effect (76 VGPRs: 6 waves / SIMD against PERM's 8)?  PERM with the occupancy cap
  # (CEC_WAVES_PER_CU = waves per CU) against LDS uncapped, configs[4] decode + --ops
  for i in 1 2; do
    for w in 0 16 24 28; do
      run rec_perm_w${w}_$i 200 env CEC_WAVES_PER_CU=$w python -u bench.py --also=rs32_1m_recovery --no-cpu-baseline --no-strong --engine perm
    done
    run rec_lds_$i 200 python -u bench.py --also=rs32_1m_recovery --no-cpu-baseline --no-strong --engine lds
  done
  ;;
occ2)
  # round-3 (second session): occupancy cap per op -- the diff-update (PERM and LDS) and the
  # metric's rotating decode at 16 / 20 / 24 / 28 waves per CU against uncapped
  for i in 1 2; do
    for w in 0 16 20 24 28; do
      run du_w${w}_$i 200 env CEC_WAVES_PER_CU=$w python -u bench.py --also=rs32_diff_update,rs32_diff_update_perm --no-cpu-baseline --no-strong
    done
  done
  ;;
gloo)
  # round-3 (second session): the default line with every workload at 2 ranks and the new
  # ones at 8 ranks, all on this one card (gloo): the driver's multi-GPU path end to end
  CEC_BENCH_DEVICE=0 timeout -k 10 400 python -u bench.py --gpus 2 > gpurun_out/r03gloo/gloo2.jsonl 2> gpurun_out/r03gloo/gloo2.err && \
  CEC_BENCH_WATCHDOG=60 CEC_BENCH_DEVICE=0 timeout -k 10 500 python -u bench.py --gpus 8 --also=rs32_1m_recovery,rs32_diff_update,rs32_diff_update_perm \
      > gpurun_out/r03gloo/gloo8.jsonl 2> gpurun_out/r03gloo/gloo8.err
  ;;
profrec)
  # round-3 (second session): rocprofv3 for the configs[4] recovery decode under AUTO (the
  # LDS engine's 3 x 1 kernel; the metric's kernels in the same process are PERM)
  O=$GRAFT_REPO_ROOT/gpurun_out/r03profrec; R=$GRAFT_REPO_ROOT
  cd /tmp && export TMPDIR=/tmp
  A="--steps 10 --warmup 2 --no-cpu-baseline --no-strong --also=rs32_1m_recovery"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py $A > $O/trace.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py $A > $O/fetch.log 2>&1 && \
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py $A > $O/write.log 2>&1
  ;;
engw|engw2|engw3)
  # round-3 (second session): PERM vs LDS on the other device-resident workloads (encode +
  # rotating decode), interleaved, two rounds
  for i in 1 2; do
    for w in rs32_4k rs32_1m rs42_64k rs32_mixed; do
      run ${w}_perm_$i 200 python -u bench.py --workload $w --also= --no-cpu-baseline --no-strong --engine perm
      run ${w}_lds_$i 200 python -u bench.py --workload $w --also= --no-cpu-baseline --no-strong --engine lds
    done
  done
  ;;
proflds)
  # round-3 (second session): rocprofv3 for the LDS engine on the larger-value workloads
  # (what AUTO runs there): kernel trace + FETCH / WRITE passes
  PROF_ENGINE=lds PROF_WORKLOADS="rs32_1m rs42_64k rs32_mixed" bash tools/profile_round.sh r03s2_lds_large || exit $?
  ;;
*) echo "usage: bash tools/r03_calls.sh <b|c|e|...|r>" >&2; exit 2 ;;
esac
