# round-3: does a kernel's code size cost a small launch (instruction-cache warm-up)?
mkdir -p gpurun_out/r03r
timeout -k 10 200 tools/small_batch_probe.bin 20 > gpurun_out/r03r/small_batch_probe_v3.jsonl 2>&1
