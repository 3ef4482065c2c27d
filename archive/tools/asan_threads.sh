#!/bin/bash
# Diagnosis: tests/dropin/cache_threads.c under host ASan + UBSan with its full report
# (the pytest case keeps only the tail).  GPU box, after `tools/asan.sh build`.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROCM=${ROCM_PATH:-/opt/rocm}
A=${ASAN_DIR:-$R/tools/asan}
RT=$ROCM/lib/llvm/lib/clang/22/lib/linux
O=$R/gpurun_out/asan_threads${ASAN_TAG:-}
mkdir -p "$O"
$ROCM/llvm/bin/clang -O1 -std=gnu11 -Wall -Werror -I "$R/include" "$R/tests/dropin/cache_threads.c" \
    -L "$A" -lJerasure -lpthread -Wl,-rpath,"$A" -g -fsanitize=address,undefined \
    -fno-sanitize-recover=undefined -shared-libsan -Wl,-rpath,$RT -o "$O/cache_threads" || exit 1
export LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0
export UBSAN_OPTIONS=print_stacktrace=1
for i in $(seq 1 ${RUNS:-2}); do
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:verify_asan_link_order=0${ASAN_EXTRA:-} \
      timeout -k 10 200 "$O/cache_threads" 8 60 6 > "$O/out_$i.txt" 2> "$O/err_$i.txt"
  echo "run=$i rc=$?" >> "$O/summary.txt"
done
