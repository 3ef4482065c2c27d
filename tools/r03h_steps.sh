# round-3 evidence on the final kernels (after the LDS fix): GPU suite, then every DESIGN §5 number (no profiles)
mkdir -p gpurun_out/r03h
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h/pytest.log 2>&1 && \
EVID_NO_PROF=1 bash tools/round_evidence.sh r03
