# test_rpool_refusals under the ASan build after the other glue tests, LeakSanitizer verbose
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$R/tools/asan
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:verify_asan_link_order=0:quarantine_size_mb=4096
export UBSAN_OPTIONS=print_stacktrace=1
mkdir -p $R/gpurun_out/repro4
cd $R
LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0 \
CEC_GLUE_RECOVERY_EXE="$A/glue_recovery" CEC_GLUE_RPOOL_EXE="$A/glue_rpool" timeout -k 10 300 \
    python -u -m pytest tests/test_glue_recovery.py tests/test_glue_rpool.py \
    -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "not cluster_sim and not refusals and not four_paths" \
    > $R/gpurun_out/repro4/others.txt 2>&1
LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0:verbosity=2:log_threads=1 \
CEC_GLUE_RPOOL_EXE="$A/glue_rpool" timeout -k 10 200 python -u -m pytest tests/test_glue_rpool.py \
    -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -k refusals --basetemp=$R/gpurun_out/repro4/tmp \
    > $R/gpurun_out/repro4/refusals.txt 2>&1
echo "rc=$?" >> $R/gpurun_out/repro4/refusals.txt
ps -eLo pid,tid,stat,wchan:32,comm 2>/dev/null | grep -i "glue_rpool" > $R/gpurun_out/repro4/ps.txt || true
