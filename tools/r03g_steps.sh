# round-3 GPU steps: LDS-engine A/B -- this build (no write-through branch in the staged
# kernels) vs the branch (tools/ab_lds_wt) vs the build before the store policy (tools/ab_lds_pre)
mkdir -p gpurun_out/r03g
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03g/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
B="python -u bench.py --engine lds --also= --no-cpu-baseline --no-strong"
for i in 1 2 3; do
  run lds_new_$i 200 $B
  run lds_wt_$i 200 env CEC_LIB_PATH=tools/ab_lds_wt/libcocytus_ec.so $B
  run lds_pre_$i 200 env CEC_LIB_PATH=tools/ab_lds_pre/libcocytus_ec.so $B
done
run pytest_lds 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lds or golden or fuzz"
