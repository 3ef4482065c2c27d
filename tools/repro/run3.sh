# the glue part of tools/asan.sh run, twice: as is, then with LSan's exit-time leak check off
R=${GRAFT_REPO_ROOT:-$(pwd)}
RT=/opt/rocm/lib/llvm/lib/clang/22/lib/linux
A=$R/tools/asan
export LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0
export UBSAN_OPTIONS=print_stacktrace=1
mkdir -p $R/gpurun_out/repro3
cd $R
for leaks in 1 0; do
  ASAN_OPTIONS=detect_leaks=$leaks:abort_on_error=0:verify_asan_link_order=0:quarantine_size_mb=4096 \
  CEC_GLUE_RECOVERY_EXE="$A/glue_recovery" CEC_GLUE_RPOOL_EXE="$A/glue_rpool" timeout -k 10 300 \
      python -u -m pytest tests/test_glue_recovery.py tests/test_glue_rpool.py \
      -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "not cluster_sim" \
      > $R/gpurun_out/repro3/leaks$leaks.txt 2>&1
  echo "rc=$?" >> $R/gpurun_out/repro3/leaks$leaks.txt
done
