set -o pipefail
out=gpurun_out/r06m; mkdir -p $out
timeout -k 10 300 env CEC_BENCH_DEVICE=0 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-strong --no-cpu-baseline \
    --also=drain_host_ecmem,recovery_pool_host,set_diffs_host > $out/two_ranks_one_card.jsonl 2> $out/two_ranks.err || exit 1
timeout -k 10 300 env CEC_BENCH_PG=1 python -u bench.py --steps 3 --warmup 1 --no-strong \
    --also=drain_host_ecmem,recovery_pool_host,set_diffs_host > $out/one_rank_rccl.jsonl 2> $out/one_rank_rccl.err || exit 2
