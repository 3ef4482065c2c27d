# round-3 GPU step list (one call): full GPU suite, the stale-tile precondition probe and
# negative control, the small-batch fixed-cost probe, the diff-update early-install A/B
mkdir -p gpurun_out/r03b
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03b/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
run pytest 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
run xcdvis 120 tools/xcd_visibility_probe.bin 64 200
run prefix_neg 300 env CEC_LIB_PATH=tools/prefix_build/libcocytus_ec.so python -u -m pytest tests/test_gpu_parity.py -k visible_from_every_xcd -q --timeout 120 --timeout-method thread
run smallbatch 120 tools/small_batch_probe.bin 20
for i in 1 2 3; do
  run du_new_$i 200 python -u bench.py --also=rs32_diff_update --no-strong --no-cpu-baseline
  run du_old_$i 200 env CEC_LIB_PATH=tools/ab_du/libcocytus_ec.so python -u bench.py --also=rs32_diff_update --no-strong --no-cpu-baseline
done
