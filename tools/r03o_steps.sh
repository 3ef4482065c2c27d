# round-3: where a small encode launch's fixed cost goes (tile list / GF multiply / neither)
mkdir -p gpurun_out/r03o
for b in 8192 65536 8192; do
  ENCODE_GAP_STRIPES=$b timeout -k 10 200 python -u tools/encode_gap.py >> gpurun_out/r03o/encode_gap.txt 2>&1 || exit $?
done
timeout -k 10 120 tools/small_batch_probe.bin 20 > gpurun_out/r03o/small_batch_probe.jsonl 2>&1
