# round-3: workgroups per tile (CEC_SPLIT_SHIFT) at the strong-scaling shares
mkdir -p gpurun_out/r03l
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03l/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
for i in 1 2; do
  for sh in 2 1 0; do
    run split${sh}_$i 200 env CEC_SPLIT_SHIFT=$sh python -u bench.py --also= --no-cpu-baseline
  done
done
