# round-3 GPU steps: uniform-stream launches (kFlagUniform) -- GPU suite, then A/B against
# the previous build (tools/ab_prev) on the metric and its strong-scaling shares, and --ops
mkdir -p gpurun_out/r03e
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03e/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
run xcdvis 120 tools/xcd_visibility_probe.bin 64 200
run pytest 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
for i in 1 2 3; do
  run bench_new_$i 200 python -u bench.py --also= --no-cpu-baseline
  run bench_prev_$i 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u bench.py --also= --no-cpu-baseline
done
run ops_new 200 python -u bench.py --ops
run ops_prev 200 env CEC_LIB_PATH=tools/ab_prev/libcocytus_ec.so python -u bench.py --ops
