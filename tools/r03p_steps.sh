# round-3: LDS engine, workgroups per tile (its rotating decode stages product rows per
# workgroup: 768 B per 1 KiB quarter-tile with s = 2)
mkdir -p gpurun_out/r03p
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03p/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
for i in 1 2; do
  for sh in 2 1 0; do
    run lds_s${sh}_$i 200 env CEC_SPLIT_SHIFT=$sh python -u bench.py --engine lds --also= --no-cpu-baseline --no-strong
  done
done
