# round-3: the metric's step through the C-ABI alone at the strong-scaling shares
mkdir -p gpurun_out/r03n
for i in 1 2; do
  for b in 65536 32768 16384 8192; do
    CEC_NATIVE_STRIPES=$b timeout -k 10 200 tools/bench_native.bin 20 3 >> gpurun_out/r03n/native_shares.jsonl 2>&1 || exit $?
  done
done
