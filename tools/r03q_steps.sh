# round-3 final check on the final tree, as the driver runs it: GPU suite, smoke, default bench
mkdir -p gpurun_out/r03q
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r03q/bench_default.jsonl 2> gpurun_out/r03q/bench_default.err
