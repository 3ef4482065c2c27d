# round-3: occupancy floor of 8 waves per SIMD for the small exact PERM kernels
# (tools/ab_occ, -DCEC_WAVES_PER_EU=8: encode 3x2 68 -> 64 VGPRs) vs this build
mkdir -p gpurun_out/r03m
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03m/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
for i in 1 2 3; do
  run cur_$i 200 python -u bench.py --also= --no-cpu-baseline
  run occ_$i 200 env CEC_LIB_PATH=tools/ab_occ/libcocytus_ec.so python -u bench.py --also= --no-cpu-baseline
done
