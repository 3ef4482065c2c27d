#!/bin/bash
# tools/tsan.sh build|run -- the library's host threads under ThreadSanitizer: the
# drop-in's per-thread contexts (8 pthreads calling galois_w08_region_multiply at once)
# and the drainer's pack pool (the batched bindings).  Host-only instrumentation
# (-Xarch_host); the static TSan runtime comes with the clang-built test programs.
#   build: here, on the CPU.   run: on the GPU box.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROCM=${ROCM_PATH:-/opt/rocm}
T=$R/tools/tsan
case "${1:-}" in
build)
  mkdir -p "$T"
  $ROCM/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -fvisibility=hidden \
      -mcode-object-version=5 -Xarch_host -fsanitize=thread -Xarch_host -fno-omit-frame-pointer \
      -I"$R/include" -Wl,-rpath,$ROCM/lib -o "$T/libcocytus_ec.so" "$R/cocytus_amd/csrc/cec_runtime.hip"
  ln -sf libcocytus_ec.so "$T/libJerasure.so"
  ;;
run)
  export CEC_DROPIN_LIBDIR=$T CEC_DROPIN_CC=$ROCM/llvm/bin/clang
  # the C programs link clang's C++ interceptors too (function-local statics and
  # operator new/delete inside the library are then understood)
  RT=$ROCM/lib/llvm/lib/clang/22/lib/linux
  export CEC_DROPIN_CFLAGS="-g -fsanitize=thread -Wl,--whole-archive $RT/libclang_rt.tsan_cxx-x86_64.a -Wl,--no-whole-archive -lstdc++"
  export TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:suppressions=$R/tools/tsan_supp.txt"
  cd "$R"
  timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
      -k "dropin_c_program or reentrant_threads or batched_bindings or concurrent_threads" -p no:cacheprovider
  # round 5: the host-memory batch's pack pool and pipelined rounds, through the glue bench
  if [ -x "$T/glue_recovery_bench" ]; then
    timeout -k 10 300 "$T/glue_recovery_bench" set 16384 4098 2
    timeout -k 10 300 "$T/glue_recovery_bench" 2
  fi
  ;;
glue)  # (here, on the CPU) the glue bench against tools/tsan
  REF=${REF:-/root/reference}
  RT=$ROCM/lib/llvm/lib/clang/22/lib/linux
  $ROCM/llvm/bin/clang -O1 -g -std=gnu11 -fsanitize=thread -I"$R/include" -I"$R/integration" -I"$REF" -I"$R/oracle" \
      -o "$T/glue_recovery_bench" "$R/tests/glue/recovery_bench.c" "$R/integration/cocytus_recovery.c" \
      "$R/integration/cocytus_set.c" "$R/integration/cocytus_recovery_pool.c" -L"$T" -lcocytus_ec -L"$R/oracle" -lgf8ref -Wl,-rpath,'$ORIGIN' \
      -Wl,-rpath,'$ORIGIN/../../oracle' -Wl,--whole-archive $RT/libclang_rt.tsan_cxx-x86_64.a -Wl,--no-whole-archive -lstdc++
  ;;
*) echo "usage: $0 build|glue|run" >&2; exit 2 ;;
esac
