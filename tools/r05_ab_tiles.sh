# tools/r05_ab_tiles.sh -- the recovery pool's tile list in mapped pinned memory (read by the
# kernel in place) against the upload ahead of each launch (tools/ab_old/libcocytus_ec.so:
# the previous commit's library, built here from `git archive HEAD`), same box, alternating;
# then the recovery glue bench on the new library.  (The old library lacks
# cec_recovery_pool_fold_updates, which the glue bench links: it runs on the new one only.)
set -o pipefail
out=gpurun_out/r05k; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_glue_rpool.py \
    tests/test_gpu_parity.py tests/test_glue_recovery.py -k "rpool or recovery_pool or cluster_sim" > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 tools/pool_bench.bin > $out/pool_new_$r.jsonl 2>&1 || exit 2
  LD_LIBRARY_PATH=$PWD/tools/ab_old timeout -k 10 200 tools/pool_bench.bin > $out/pool_old_$r.jsonl 2>&1 || exit 3
  timeout -k 10 120 oracle/_ref/glue_recovery_bench 15 > $out/rec_new_$r.jsonl 2>&1 || exit 4
done
