# round-3 sanitizer runs on the final host code (pool tables, launch checks, cache changes)
mkdir -p gpurun_out/r03j
timeout -k 10 600 bash tools/asan.sh run > gpurun_out/r03j/asan.txt 2>&1 && \
timeout -k 10 600 bash tools/tsan.sh run > gpurun_out/r03j/tsan.txt 2>&1
