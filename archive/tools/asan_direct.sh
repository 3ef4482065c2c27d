#!/bin/bash
# Diagnosis of an ASan exit-time hang: the batched-bindings C program's pytest case
# under host ASan, with and without the exit-time leak check.  GPU box, after
# `tools/asan.sh build`.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROCM=${ROCM_PATH:-/opt/rocm}
A=$R/tools/asan
RT=$ROCM/lib/llvm/lib/clang/22/lib/linux
O=$R/gpurun_out/asan_direct
mkdir -p "$O"
export CEC_DROPIN_LIBDIR=$A CEC_DROPIN_CC=$ROCM/llvm/bin/clang
export CEC_DROPIN_CFLAGS="-g -fsanitize=address,undefined -fno-sanitize-recover=undefined -shared-libsan -Wl,-rpath,$RT"
export LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0
export UBSAN_OPTIONS=print_stacktrace=1
cd $R
for leaks in 0 1; do
  t0=$(date +%s%N)
  ASAN_OPTIONS=detect_leaks=$leaks:abort_on_error=0:verify_asan_link_order=0 timeout -k 10 150 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "batched_bindings or concurrent_threads or reentrant" -p no:cacheprovider > $O/batched_l$leaks.txt 2>&1
  echo "leaks=$leaks rc=$? ms=$(( ($(date +%s%N) - t0) / 1000000 ))" >> $O/summary4.txt
done
