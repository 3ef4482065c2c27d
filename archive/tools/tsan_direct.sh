#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
ROCM=/opt/rocm
T=$R/tools/tsan
RT=$ROCM/lib/llvm/lib/clang/22/lib/linux
$ROCM/llvm/bin/clang -O1 -std=gnu11 -I$R/include $R/tests/dropin/dropin_threads.c -L$T -lJerasure -lpthread -Wl,-rpath,$T -g -fsanitize=thread -Wl,--whole-archive $RT/libclang_rt.tsan_cxx-x86_64.a -Wl,--no-whole-archive -lstdc++ -o $R/gpurun_out/dt_tsan
TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:suppressions=$R/tools/tsan_supp.txt" timeout -k 10 200 $R/gpurun_out/dt_tsan 8 150 > $R/gpurun_out/dt_tsan.out 2> $R/gpurun_out/dt_tsan.err
echo rc=$?
