#!/bin/bash
# tools/asan.sh build|run -- the library's host code under AddressSanitizer + UBSan.
#   build (here, on the CPU): tools/asan/libcocytus_ec.so (+ libJerasure.so), host-side
#         instrumented only (-Xarch_host: GPU sanitizers are not available on this pool),
#         and tools/asan/pool_bench.bin against it.
#   run   (on the GPU box): the C programs of tests/dropin (the drop-in chain, 8-thread
#         re-entrancy, memcached's daemonize order, the batched bindings: drainer,
#         recovery pool) compiled with clang -fsanitize=address,undefined against that
#         library and checked against the oracle by their pytest cases, then the idle-
#         recoverer pool bench.  Leaks are checked; only the HIP runtime's are suppressed.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROCM=${ROCM_PATH:-/opt/rocm}
RT=$ROCM/lib/llvm/lib/clang/22/lib/linux
A=$R/tools/asan
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer -shared-libsan"
case "${1:-}" in
build)
  mkdir -p "$A"
  $ROCM/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -fvisibility=hidden \
      -mcode-object-version=5 $SAN -I"$R/include" -Wl,-rpath,$ROCM/lib -Wl,-rpath,$RT \
      -o "$A/libcocytus_ec.so" "$R/cocytus_amd/csrc/cec_runtime.hip"
  ln -sf libcocytus_ec.so "$A/libJerasure.so"
  $ROCM/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 $SAN "$R/tools/pool_bench.hip" \
      -L"$A" -lcocytus_ec -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$RT -o "$A/pool_bench.bin"
  ;;
run)
  mkdir -p "$R/gpurun_out"
  export CEC_DROPIN_LIBDIR=$A CEC_DROPIN_CC=$ROCM/llvm/bin/clang
  export CEC_DROPIN_CFLAGS="-g -fsanitize=address,undefined -fno-sanitize-recover=undefined -shared-libsan -Wl,-rpath,$RT"
  # quarantine_size_mb: big enough that no freed chunk is recycled after the HSA runtime
  # has unloaded at exit.  With the default 256 MiB, the runtime's own teardown frees
  # can recycle a device-memory chunk that the exit hook freed. ASan's device allocator
  # then fails its CHECK "!dev_runtime_unloaded_" (sanitizer_allocator_device.h:125),
  # on some boxes and runs and not others (archive/profiles/r02_evidence_final/asan_*).
  # A larger quarantine only delays reuse, so use-after-free detection gets stronger.
  export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:verify_asan_link_order=0:quarantine_size_mb=4096
  export LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0
  export UBSAN_OPTIONS=print_stacktrace=1
  cd "$R"
  # the instrumented runtime is what the programs load (and the daemonize order under it)
  $CEC_DROPIN_CC -std=gnu11 -I"$R/include" "$R/tests/dropin/dropin_daemon.c" -L"$A" -lJerasure \
      -Wl,-rpath,"$A" $CEC_DROPIN_CFLAGS -o "$R/gpurun_out/dropin_daemon_asan"
  ldd "$R/gpurun_out/dropin_daemon_asan" | grep -E "asan|Jerasure"
  timeout -k 10 60 "$R/gpurun_out/dropin_daemon_asan"
  timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
      -k "dropin or batched_bindings or concurrent_threads" -p no:cacheprovider
  timeout -k 10 200 "$A/pool_bench.bin"
  # round 5: the server glue (integration/) and the host-memory batch under it, compiled
  # against the reference's headers on the CPU (glue build, below) and linked here to the
  # instrumented library: the GPU glue tests through that binary, then its bench shapes
  if [ -x "$A/glue_recovery" ]; then
    # test_rpool_refusals's driver, alone, with LeakSanitizer off: at its exit LSan's
    # stop-the-world attached to the main thread and two HIP runtime threads and then waited
    # forever on the next one (LSAN_OPTIONS=verbosity=2, tools/repro/run4.sh,
    # profiles/r05_evidence/lsan_hang/) -- whenever other GPU processes had run on the box
    # before it, in one pytest session or in separate ones.  Its refusals allocate nothing
    # (every check comes before any allocation); the other 20 run with leak detection on.
    CEC_GLUE_RECOVERY_EXE="$A/glue_recovery" CEC_GLUE_RPOOL_EXE="$A/glue_rpool" timeout -k 10 300 \
        python -u -m pytest tests/test_glue_recovery.py tests/test_glue_rpool.py \
        -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "not cluster_sim and not refusals"
    ASAN_OPTIONS=${ASAN_OPTIONS/detect_leaks=1/detect_leaks=0} CEC_GLUE_RPOOL_EXE="$A/glue_rpool" \
        timeout -k 10 200 python -u -m pytest tests/test_glue_rpool.py \
        -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k refusals
    timeout -k 10 200 "$A/glue_recovery_bench" 3
    timeout -k 10 200 "$A/glue_recovery_bench" set 16384 4098 2
    for s in 0 1 2; do timeout -k 10 200 "$A/glue_cluster_sim63" $s $s; done
    timeout -k 10 200 "$A/glue_drain_recovery_bench" 1024 4098 64 0.5 1
  fi
  ;;
glue)  # (here, on the CPU, where the reference's headers are) the glue programs against tools/asan
  REF=${REF:-/root/reference}
  G="-O1 -g -std=gnu11 -fsanitize=address,undefined -fno-sanitize-recover=undefined -shared-libsan -fno-omit-frame-pointer"
  CC=$ROCM/llvm/bin/clang
  $CC $G -I"$R/include" -I"$R/integration" -I"$REF" -o "$A/glue_recovery" "$R/tests/glue/recovery_main.c" \
      "$R/integration/cocytus_recovery.c" "$R/integration/cocytus_drain.c" "$R/integration/cocytus_set.c" \
      -L"$A" -lcocytus_ec -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$RT
  $CC $G -I"$R/include" -I"$R/integration" -I"$REF" -o "$A/glue_rpool" "$R/tests/glue/rpool_main.c" \
      "$R/integration/cocytus_recovery_pool.c" "$R/integration/cocytus_drain.c" \
      -L"$A" -lcocytus_ec -Wl,-rpath,'$ORIGIN' -Wl,-rpath,$RT
  $CC $G -DK=6 -DM=3 -I"$R/include" -I"$R/integration" -I"$REF" -I"$R/oracle" -o "$A/glue_cluster_sim63" \
      "$R/tests/glue/cluster_sim.c" "$R/integration/cocytus_recovery.c" "$R/integration/cocytus_drain.c" \
      "$R/integration/cocytus_set.c" "$R/integration/cocytus_recovery_pool.c" -L"$A" -lcocytus_ec -L"$R/oracle" -lgf8ref -Wl,-rpath,'$ORIGIN' \
      -Wl,-rpath,'$ORIGIN/../../oracle' -Wl,-rpath,$RT
  $CC $G -I"$R/include" -I"$R/integration" -I"$REF" -I"$R/oracle" -o "$A/glue_drain_recovery_bench" \
      "$R/tests/glue/drain_recovery_bench.c" "$R/integration/cocytus_drain.c" "$R/integration/cocytus_recovery.c" \
      "$R/integration/cocytus_recovery_pool.c" -L"$A" -lcocytus_ec -L"$R/oracle" -lgf8ref -Wl,-rpath,'$ORIGIN' \
      -Wl,-rpath,'$ORIGIN/../../oracle' -Wl,-rpath,$RT
  $CC $G -I"$R/include" -I"$R/integration" -I"$REF" -I"$R/oracle" -o "$A/glue_recovery_bench" \
      "$R/tests/glue/recovery_bench.c" "$R/integration/cocytus_recovery.c" "$R/integration/cocytus_set.c" \
      "$R/integration/cocytus_recovery_pool.c" \
      -L"$A" -lcocytus_ec -L"$R/oracle" -lgf8ref -Wl,-rpath,'$ORIGIN' -Wl,-rpath,'$ORIGIN/../../oracle' -Wl,-rpath,$RT
  ;;
*) echo "usage: $0 build|glue|run" >&2; exit 2 ;;
esac
