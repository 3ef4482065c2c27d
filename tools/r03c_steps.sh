# round-3 GPU steps: store-policy A/B on the strong-scaling shares, GPU suite under
# forced write-through and under the default policy, box record for the stale-tile probe
mkdir -p gpurun_out/r03c
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03c/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
run xcdvis 120 tools/xcd_visibility_probe.bin 64 200
run pytest_wt 700 env CEC_STORE_POLICY=wt python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
for i in 1 2 3; do
  for p in nt wt auto; do
    run bench_${p}_$i 200 env CEC_STORE_POLICY=$p python -u bench.py --also= --no-cpu-baseline
  done
done
run pytest_auto 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
