# test_rpool_refusals alone through pytest under the ASan build (as tools/asan.sh run sets it up)
R=${GRAFT_REPO_ROOT:-$(pwd)}
RT=/opt/rocm/lib/llvm/lib/clang/22/lib/linux
A=$R/tools/asan
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=0:verify_asan_link_order=0:quarantine_size_mb=4096
export LSAN_OPTIONS=suppressions=$R/tools/asan_lsan.supp:print_suppressions=0
export UBSAN_OPTIONS=print_stacktrace=1
mkdir -p $R/gpurun_out/repro2
cd $R
CEC_GLUE_RPOOL_EXE="$A/glue_rpool" timeout -k 10 200 python -u -m pytest tests/test_glue_rpool.py -m gpu -v \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k refusals --basetemp=$R/gpurun_out/repro2/tmp \
    > $R/gpurun_out/repro2/pytest.txt 2>&1
echo "rc=$?" >> $R/gpurun_out/repro2/pytest.txt
