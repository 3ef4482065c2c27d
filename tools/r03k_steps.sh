# round-3: the two-rank bench test, and the decode shape ceiling in the bench's arena order
# beside the library's decode in the same call
mkdir -p gpurun_out/r03k
run() { name=$1; shift; timeout -k 10 "$@" > gpurun_out/r03k/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
run pytest2 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "two_ranks or edge_cases or extent_pattern"
run hbm_mix 200 tools/hbm_mix.bin arena random 64
run decode_probe 200 python -u tools/decode_probe.py
run hbm_mix_b 200 tools/hbm_mix.bin arena random 64
